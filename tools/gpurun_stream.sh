#!/bin/bash
# Stream sweep on one MI355X: its GPU tests, then bench lines for the stream kernel at several
# (G, K) next to the systolic per-cell kernel, ML20M and NFLX.  Output under gpurun_out/stream/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stream
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py -x -v --timeout 120 --timeout-method thread -k "stream" > $O/pytest.log 2>&1 || { echo "stream tests failed"; tail -30 $O/pytest.log; exit 1; }
  echo "tests: $(tail -1 $O/pytest.log)"
fi
LEAN="--no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 --steps 5 --warmup 1"
run() {  # name config env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg $LEAN > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['ms_per_step'], 'ms', '%.3e'%d['value'], 'rmse', d['rmse'], d.get('rmse_rel'), 'pads', d['config']['pad_records'], 'prep', d['setup_s']['prepare'])"
}
for cfg in ${CONFIGS:-ML20M NFLX}; do
  run ${cfg}_sys $cfg MFHIP_STREAM=0
  IFS=';' read -ra LIST <<< "${GKRS:-64 2 3 4;128 2 3 4;128 4 3 4}"  # "G K ring period;..."
  for GKR in "${LIST[@]}"; do
    set -- $GKR
    run ${cfg}_stream_G$1_K$2_R$3_P$4 $cfg MFHIP_STREAM=1 MFHIP_STREAM_G=$1 MFHIP_STREAM_K=$2 MFHIP_STREAM_RING=$3 MFHIP_STREAM_PUB=$4 MFHIP_STREAM_STATS=1
    grep "stream waits" $O/${cfg}_stream_G$1_K$2_R$3_P$4.err | tail -2
  done
done
