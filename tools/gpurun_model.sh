# A/B the systolic per-block group model constants (MFHIP_SYS_MODEL="cell,pair,run") on NFLX
mkdir -p gpurun_out
for M in ${MODELS:-2600,265,186}; do
  MFHIP_SYS_MODEL=$M timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile ${ARGS:-} > gpurun_out/m.log 2>&1 || { echo FAIL $M; tail -3 gpurun_out/m.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/m.log').read().strip().splitlines()[-1]); print('$M', round(d['value']/1e6), d['ms_per_step'], d['config']['groups'])"
done
