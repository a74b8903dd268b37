#!/bin/bash
# Round-3: the deterministic sweep and online sweep with the one-lane fold (seq_fold.hpp) and the
# det sweep's exact wait counts, against the HEAD build (lib_base): bit-exact GPU tests, the
# isolated hot chain, the det bench leg with its f64 online leg, the fast line's f32 online leg.
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_online.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for L in lib_np lib lib_np lib; do
  export MFHIP_LIB=$PWD/large-scale-recommendation_amd/$L/libmfhip.so
  timeout -k 10 300 python tools/det_chain_bench.py 128 30000 0 > $O/chain_$L.log 2>&1 || { echo "chain $L failed"; tail -3 $O/chain_$L.log; exit 1; }
  echo "$L $(tail -1 $O/chain_$L.log)"
done
for L in lib_np lib; do
  export MFHIP_LIB=$PWD/large-scale-recommendation_amd/$L/libmfhip.so
  timeout -k 10 400 python bench.py --mode det --steps 2 --warmup 1 --no-cpu-baseline --no-profile --online-batches 5 --det-epochs 0 > $O/det_$L.json 2> $O/det_$L.err || { echo "det bench $L failed"; tail -3 $O/det_$L.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/det_$L.json').read().strip().splitlines()[-1]); print('$L det', d['ms_per_step'], 'ms', round(d['value']/1e6,1), 'Mups rmse', d['rmse'], 'ref', d['rmse_ref'], 'online f64', d['online']['f32']['value'] if d.get('online') else None)"
  timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 5 --det-epochs 0 > $O/fast_$L.json 2> $O/fast_$L.err || { echo "fast bench $L failed"; tail -3 $O/fast_$L.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/fast_$L.json').read().strip().splitlines()[-1]); print('$L online f32', d['online']['f32']['value'], d['online']['f32']['min'], d['online']['f32']['max'])"
done
