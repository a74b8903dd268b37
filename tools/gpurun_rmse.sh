# RMSE of fast mode under both blockings at a given NFLX scale (10 epochs).
mkdir -p gpurun_out
for sc in ${SCALES:-0.25 1.0}; do
  for bl in balanced reference; do
    timeout -k 10 300 python bench.py --steps 9 --warmup 1 --no-cpu-baseline --scale $sc --blocking $bl > gpurun_out/rm.log 2>&1 || { echo FAIL; tail -3 gpurun_out/rm.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/rm.log').read().strip().splitlines()[-1]); print('$sc $bl', d['rmse'], round(d['value']/1e6), d['ms_per_step'])"
  done
done
