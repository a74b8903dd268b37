#!/bin/bash
# Hot-item replicas: averaged join vs keep-one join, NFLX and ML20M, bench lines with RMSE.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/split2; mkdir -p $O; cd $R
LEAN="--no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 --steps 5 --warmup 1"
run() { local name=$1 cfg=$2 split=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $cfg --item-split $split $LEAN > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['ms_per_step'], 'ms', 'rmse', d['rmse'], 'rel', d.get('rmse_rel'), 'G', d['config']['groups'])"; }
for cfg in NFLX ML20M; do
  for sp in 8192 2048; do
    run ${cfg}_mean_$sp $cfg $sp MFHIP_SPLIT_JOIN=mean
    run ${cfg}_keep_$sp $cfg $sp MFHIP_SPLIT_JOIN=keep
  done
done
