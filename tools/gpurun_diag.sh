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
MFHIP_WAVE_TRACE=$O/wt_chain.txt timeout -k 10 300 python tools/chain_bench.py 128 100000 chain > $O/chain_wt.log 2>&1 || { echo "chain trace failed"; tail -5 $O/chain_wt.log; exit 1; }
python tools/sys_trace.py $O/wt_chain.txt | grep -A1 "superstep 0"
for bg in 0 2000000; do
  timeout -k 10 300 python tools/det_chain_bench.py 128 30000 $bg > $O/det_chain_$bg.log 2>&1 || { echo "det chain failed"; tail -5 $O/det_chain_$bg.log; exit 1; }
  tail -1 $O/det_chain_$bg.log
done
[ -n "${NO_INTERF:-}" ] && exit 0
timeout -k 10 300 python tools/interference_bench.py > $O/interf.log 2>&1 || { echo "interf failed"; tail -5 $O/interf.log; exit 1; }
grep substep $O/interf.log
