#!/bin/bash
# Online 1M-rating NFLX batches (bench.py online leg) under MFHIP_TEST knob sets, alternated twice:
#   bash tools/ab_online.sh <out> name=knobs ...   (knobs may be empty: the defaults)
set -o pipefail
O=gpurun_out/${1:?out dir}; shift
mkdir -p $O
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; K=${spec#*=}
    MFHIP_TEST=$K timeout -k 10 300 python bench.py --steps 1 --no-cpu-baseline --det-epochs 0 --ml20m-epochs 0 --block-update-reps 0 --online-batches 5 --no-profile > $O/b_${name}_$rep.json 2> $O/b_${name}_$rep.err || { echo bench failed $name; tail -5 $O/b_${name}_$rep.err; exit 1; }
    python3 - "$O/b_${name}_$rep.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["online"]
print(sys.argv[2], " ".join(f"{k} {round(v['value'] / 1e6)} M/s kernel {v['kernel_ms_median']} ms" for k, v in d.items() if isinstance(v, dict) and "value" in v))
PY
  done
done
