set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
for cfg in "0 1" "-128 1" "-128 1000000000" "-96 1" "-192 1"; do
  set -- $cfg
  MFHIP_PRIO_LEN=$2 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fast-waves $1 > gpurun_out/sw.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/sw.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); c=d['config']; print('$cfg', round(d['value']/1e6,1), d['ms_per_step'], c['groups'], c['pad_records'], d['roofline']['frac'], d['rmse'])"
done
