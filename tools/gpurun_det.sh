#!/bin/bash
# Deterministic-mode persistent sweep on the GPU box: parity tests, then the det bench on ML20M
# and NFLX.  Run via gpurun from the repo root.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_configs.py -x -v --timeout 300 \
  --timeout-method thread -k "deterministic or golden or oracle or shard or resume or snapshot or learning or online" \
  > gpurun_out/pytest_det.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
for cfg in ML20M NFLX; do
  timeout -k 10 300 python bench.py --mode det --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --online-batches 0 \
    > gpurun_out/bench_det_$cfg.log 2> gpurun_out/bench_det_$cfg.err
  rc=$?; echo "bench det $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
