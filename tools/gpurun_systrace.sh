#!/bin/bash
# Per-cell wave trace of the systolic fast sweep (MFHIP_WAVE_TRACE) for NFLX and ML20M, summarised by
# tools/sys_trace.py: per-kind cell cost, hand-off gaps, each superstep's busiest wave.
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-NFLX ML20M}; do
  MFHIP_WAVE_TRACE=gpurun_out/wt_$cfg.txt timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 \
    --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 ${ARGS:-} > gpurun_out/st_$cfg.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench $cfg rc=$rc"; tail -3 gpurun_out/st_$cfg.log; exit $rc; }
  python tools/sys_trace.py gpurun_out/wt_$cfg.txt > gpurun_out/st_$cfg.txt 2>&1
  echo "== $cfg"; cat gpurun_out/st_$cfg.txt
done
