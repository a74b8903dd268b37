# A/B: systolic wave placement (MFHIP_SYS_PLACE=1: heavy waves paired with light ones per CU) vs default.
mkdir -p gpurun_out
MFHIP_SYS_PLACE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "systolic or schedule or fast_rmse" > gpurun_out/place_tests.log 2>&1 || { echo "place tests failed"; tail -20 gpurun_out/place_tests.log; exit 1; }
tail -1 gpurun_out/place_tests.log
for cfg in NFLX ML20M; do
  for pl in 0 1 0 1; do
    if [ $pl = 1 ]; then export MFHIP_SYS_PLACE=1; else unset MFHIP_SYS_PLACE; fi
    timeout -k 10 300 python bench.py --config $cfg --steps 9 --no-cpu-baseline --online-batches 0 --det-epochs 0 --no-profile > gpurun_out/place.json 2> gpurun_out/place.err || { echo "bench failed"; tail -5 gpurun_out/place.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/place.json')); print('$cfg place=$pl', d['ms_per_step'], round(d['value']/1e6), d['rmse'])"
  done
done
