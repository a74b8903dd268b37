# Device-built fast schedule: equality with the host plan, the GPU suite, prepare timings.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dsgd.py -m gpu -x -v --timeout 200 --timeout-method thread -k device_plan > gpurun_out/devplan_test.log 2>&1 || { echo "device plan test failed"; tail -30 gpurun_out/devplan_test.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/devplan_test.log | tail -5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in NFLX ML20M ${EXTRA_CFGS:-}; do
  MFHIP_TIMING=1 timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline --online-batches 0 --det-epochs 0 > gpurun_out/bench_t_$cfg.json 2> gpurun_out/bench_t_$cfg.err || { echo "bench $cfg failed"; tail -5 gpurun_out/bench_t_$cfg.err; exit 1; }
  echo "== $cfg"; grep mfhip gpurun_out/bench_t_$cfg.err | grep -v "thread time"; python -c "import json,sys; d=json.load(open('gpurun_out/bench_t_$cfg.json')); print(d['value'], d['ms_per_step'], d['rmse'], d.get('rmse_rel'), d['config']['pad_records'], d['setup_s'])"
done
MFHIP_TIMING=1 timeout -k 10 400 python bench.py --config NFLX --steps 2 --no-cpu-baseline --no-profile --det-epochs 0 --online-batches 4 > gpurun_out/onl.json 2> gpurun_out/onl.err || { echo "online bench failed"; tail -5 gpurun_out/onl.err; exit 1; }
grep "online:" gpurun_out/onl.err | tail -6
python -c "import json; d=json.load(open('gpurun_out/onl.json')); print('online', d['online']['value'], d['online']['min'])"
