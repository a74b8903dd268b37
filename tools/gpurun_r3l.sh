#!/bin/bash
# Round-3: systolic wave traces (cells, hand-off gaps, placement) for ML20M and NFLX.
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
for cfg in ML20M NFLX; do
  MFHIP_WAVE_TRACE=$O/wt_$cfg.txt timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/bench_$cfg.log 2>&1 || { echo "trace $cfg failed"; tail -3 $O/bench_$cfg.log; exit 1; }
  python tools/sys_trace.py $O/wt_$cfg.txt > $O/trace_$cfg.txt 2>&1 || { echo "sys_trace $cfg failed"; tail -3 $O/trace_$cfg.txt; exit 1; }
  echo "== $cfg"; head -4 $O/trace_$cfg.txt; grep -A2 "superstep [0-2]:" $O/trace_$cfg.txt
done
