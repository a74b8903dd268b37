# GPU check: the GPU test suite, then NFLX and ML20M bench lines with prepare-phase timings.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for cfg in NFLX ML20M ${EXTRA_CFGS:-}; do
  MFHIP_TIMING=1 timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline --online-batches 0 --det-epochs 0 > gpurun_out/bench_t_$cfg.json 2> gpurun_out/bench_t_$cfg.err || { echo "bench $cfg failed"; tail -5 gpurun_out/bench_t_$cfg.err; exit 1; }
  echo "== $cfg"; grep mfhip gpurun_out/bench_t_$cfg.err; python -c "import json,sys; d=json.load(open('gpurun_out/bench_t_$cfg.json')); print(d['value'], d['ms_per_step'], d['rmse'], d.get('rmse_rel'), d['setup_s'])"
done
