# pair kernel: rotation groups G sweep (NFLX k=128, no per-launch events)
mkdir -p gpurun_out
for G in ${GS:-96 128 160 192}; do
  MFHIP_FAST_KERNEL=${KERNEL:-pair} timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --fast-waves -$G > gpurun_out/b_$G.log 2>&1 || { echo FAIL; tail -3 gpurun_out/b_$G.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b_$G.log').read().strip().splitlines()[-1]); print('G $G', round(d['value']/1e6), d['ms_per_step'], d['config']['pad_records'], d['rmse'])"
done
