# GPU check: parity tests, chain microbenchmark, NFLX bench (no CPU baseline).
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/chain_bench.py 128 100000 > gpurun_out/chain.log 2>&1 || { echo "chain failed"; tail -5 gpurun_out/chain.log; exit 1; }
grep substep gpurun_out/chain.log
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_nocpu.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_nocpu.log; exit 1; }
tail -1 gpurun_out/bench_nocpu.log
