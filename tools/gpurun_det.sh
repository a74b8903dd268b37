#!/bin/bash
# Deterministic-mode persistent sweep on the GPU box: parity tests, then ML20M det bench with the
# persistent sweep and with the per-level launches (A/B).  Run via gpurun from the repo root.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py -x -v --timeout 300 --timeout-method thread \
  -k "deterministic or golden or oracle or shard or resume or snapshot or learning" > gpurun_out/pytest_det.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode det --config ML20M --steps 3 --warmup 1 --no-cpu-baseline --online-batches 0 \
  > gpurun_out/bench_det_ML20M.log 2> gpurun_out/bench_det_ML20M.err
rc=$?; echo "bench det rc=$rc"; [ $rc -ne 0 ] && exit $rc
MFHIP_DET_KERNEL=level timeout -k 10 300 python bench.py --mode det --config ML20M --steps 2 --warmup 1 --no-cpu-baseline \
  --online-batches 0 > gpurun_out/bench_det_ML20M_level.log 2> gpurun_out/bench_det_ML20M_level.err
echo "bench level rc=$?"
