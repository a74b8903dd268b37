# Online leg A/B (NFLX model): level replay vs one-launch sweep, plus the online GPU tests
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_online.py > gpurun_out/online_tests.log 2>&1 || { tail -30 gpurun_out/online_tests.log; exit 1; }
tail -2 gpurun_out/online_tests.log
for K in ${KERNELS:-level sweep level sweep}; do
  MFHIP_ONLINE_KERNEL=$K MFHIP_TIMING=${TIMING:-0} timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --det-epochs 0 > gpurun_out/online_$K.log 2> gpurun_out/online_$K.err || { echo FAIL $K; tail -5 gpurun_out/online_$K.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/online_$K.log').read().strip().splitlines()[-1]); o=d['online']; print('$K', round(o['value']/1e6,2), o.get('launches_median'))"
done
