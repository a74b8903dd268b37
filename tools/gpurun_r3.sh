#!/bin/bash
# Round-3 GPU check: the GPU parity suite (one process, per-test timeout), then the default bench
# line.  Output under gpurun_out/r3/.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "PASSED|FAILED|ERROR" $O/pytest_gpu.log | tail -5; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
grep -h "online f32\|fast .* vs oracle" $O/pytest_gpu.log || true
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
tail -c 2500 $O/bench.json
