#!/bin/bash
# Hot-chain diagnosis: NFLX wave trace (busiest wave's time split), the isolated one-wave chain,
# and the same chain beside background waves in one launch.
set -o pipefail
O=gpurun_out/diag
mkdir -p $O
CFGS=${CFGS:-NFLX} bash tools/gpurun_systrace.sh > $O/systrace.txt 2>&1 || { echo "systrace failed"; tail -5 $O/systrace.txt; exit 1; }
cat $O/systrace.txt
timeout -k 10 300 python tools/chain_bench.py 128 100000 > $O/chain.log 2>&1 || { echo "chain failed"; tail -5 $O/chain.log; exit 1; }
grep substep $O/chain.log
[ -n "${NO_INTERF:-}" ] && exit 0
timeout -k 10 300 python tools/interference_bench.py > $O/interf.log 2>&1 || { echo "interf failed"; tail -5 $O/interf.log; exit 1; }
grep substep $O/interf.log
