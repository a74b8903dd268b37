#!/bin/bash
# A/B of environment knobs on the bench line: AB="ENV1=a ENV2=b|ENV1=c" (variants split on '|'),
# each run REPS times alternating, CFG (NFLX) and BARGS extra bench args.  Prints ms/epoch per run.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
IFS='|' read -ra VARS <<< "${AB:-}"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VARS[@]}"; do
    tag=$(echo "$v" | tr ' =' '_-')
    env $v timeout -k 10 300 python bench.py --config ${CFG:-NFLX} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-profile \
      --online-batches 0 --det-epochs 0 ${BARGS:-} > $O/$tag.json 2> $O/$tag.err || { echo "run [$v] failed"; tail -3 $O/$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('[$v]', d['ms_per_step'], 'ms', round(d['value']/1e9,3), 'Gups rmse', d['rmse'], 'rel', d['rmse_rel'])"
  done
done
