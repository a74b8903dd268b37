#!/bin/bash
# Round-3: per-phase shader cycles of the deterministic sweep's hot chain (experiment builds with
# MFHIP_DET_PROBE: lib_probe = one-lane fold, lib_probe_bc = 64-lane broadcast fold).
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
for L in lib_probe lib_probe_bc; do
  MFHIP_LIB=$PWD/large-scale-recommendation_amd/$L/libmfhip.so timeout -k 10 300 python tools/det_chain_bench.py 128 30000 0 > $O/chain_$L.log 2>&1 || { echo "chain $L failed"; tail -3 $O/chain_$L.log; exit 1; }
  echo "== $L"; grep "det probe" $O/chain_$L.log | tail -2; tail -1 $O/chain_$L.log
done
