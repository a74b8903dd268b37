#!/bin/bash
# ML20M (fast, k = 64) epoch time for several library builds (MFHIP_LIB), alternated twice:
#   bash tools/ab_ml20m.sh <out> name=path/libmfhip.so[@MFHIP_TEST knobs] ...
set -o pipefail
O=gpurun_out/${1:?out dir}; shift
mkdir -p $O
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; L=${spec#*=}; K=
    case $L in *@*) K=${L#*@}; L=${L%%@*};; esac
    MFHIP_TEST=$K MFHIP_LIB=$L timeout -k 10 300 python bench.py --config ${CONFIG:-ML20M} --steps 5 --no-cpu-baseline --online-batches 0 --det-epochs 0 --block-update-reps 0 --no-profile > $O/b_${name}_$rep.json 2> $O/b_${name}_$rep.err || { echo bench failed $name; tail -5 $O/b_${name}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${name}_$rep.json').read().strip().splitlines()[-1])
print('$name', d['ms_per_step'], 'ms/epoch', round(d['value']/1e9,3), 'G/s rmse_rel', d.get('rmse_rel'), 'groups', d['config'].get('groups', d.get('groups')))"
  done
done
