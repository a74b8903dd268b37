#!/bin/bash
# Group-model constants (MFHIP_SYS_MODEL="cell_ns,pair_ns,run_pair_ns", experiments build) on one
# config, alternated twice:  CONFIG=ML20M bash tools/ab_model.sh <out> <lib> name=c,p,r ...
set -o pipefail
O=gpurun_out/${1:?out dir}; L=${2:?lib}; shift 2
mkdir -p $O
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; M=${spec#*=}
    MFHIP_SYS_MODEL=$M MFHIP_LIB=$L timeout -k 10 300 python bench.py --config ${CONFIG:-ML20M} --steps 5 --no-cpu-baseline --online-batches 0 --det-epochs 0 --block-update-reps 0 --no-profile > $O/b_${name}_$rep.json 2> $O/b_${name}_$rep.err || { echo bench failed $name; tail -5 $O/b_${name}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${name}_$rep.json').read().strip().splitlines()[-1])
print('$name', '$M', d['ms_per_step'], 'ms/epoch', round(d['value']/1e9,3), 'G/s rmse_rel', d.get('rmse_rel'), 'groups', d['config'].get('groups'))"
  done
done
