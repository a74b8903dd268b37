# Hot-item replica sweep on NFLX: CONFIGS="split:waves ..." (waves '' = default budget)
mkdir -p gpurun_out
for C in ${CONFIGS:-0: 8192: 4096: 2048:}; do
  S=${C%%:*}; W=${C#*:}
  if [ -n "$W" ]; then export MFHIP_SYS_WAVES=$W; else unset MFHIP_SYS_WAVES; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-9} --warmup 1 --no-cpu-baseline --no-profile --item-split $S ${ARGS:-} > gpurun_out/split_${S}_${W}.log 2>&1 || { echo "FAIL $C"; tail -5 gpurun_out/split_${S}_${W}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/split_${S}_${W}.log').read().strip().splitlines()[-1]); print('$C', round(d['value']/1e6), d['ms_per_step'], d['rmse'], d['config']['groups'])"
done
