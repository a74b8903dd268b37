#!/bin/bash
# Uniform rotation groups G (fast_waves = -G) on one config: ms per epoch per G.
mkdir -p gpurun_out
for G in ${GS:-64 128}; do
  timeout -k 10 300 python bench.py --config ${CFG:-NFLX} --steps 4 --warmup 1 --fast-waves -$G \
    --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > gpurun_out/g.log 2>&1 \
    || { echo FAIL $G; tail -3 gpurun_out/g.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/g.log').read().strip().splitlines()[-1]); print('${CFG:-NFLX}', 'G=$G', round(d['value']/1e6), d['ms_per_step'], d['config']['groups'], d['rmse'])"
done
