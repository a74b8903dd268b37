#!/bin/bash
# Sweep the systolic sweep's wave budget (MFHIP_SYS_WAVES) and cell-cost model (MFHIP_SYS_MODEL)
# on one config: ms per epoch and the mean rotation groups per rating block.
mkdir -p gpurun_out
for W in ${WAVES:-1024}; do
  for M in ${MODELS:-6000,300,186}; do
    MFHIP_SYS_WAVES=$W MFHIP_SYS_MODEL=$M timeout -k 10 300 python bench.py --config ${CFG:-NFLX} --steps 4 --warmup 1 \
      --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > gpurun_out/g.log 2>&1 \
      || { echo FAIL $W $M; tail -3 gpurun_out/g.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/g.log').read().strip().splitlines()[-1]); print('${CFG:-NFLX}', '$W', '$M', round(d['value']/1e6), d['ms_per_step'], d['config']['groups'], d['rmse'])"
  done
done
