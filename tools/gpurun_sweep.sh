# Sweep rotation groups G (and the priority threshold) on the NFLX bench; one line per config.
set -o pipefail
mkdir -p gpurun_out
for cfg in ${SWEEP:-"0 1" "-64 1" "-80 1" "-96 1" "-112 1" "-144 1" "-160 1" "0 1000000000"}; do
  set -- $cfg
  MFHIP_PRIO_LEN=$2 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --fast-waves $1 > gpurun_out/sw.log 2>&1 || { echo "FAIL $cfg"; tail -3 gpurun_out/sw.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); c=d['config']; print('$cfg', round(d['value']/1e6,1), d['ms_per_step'], c['groups'], c['pad_records'], d['roofline']['frac'], d['rmse'])"
done
