#!/bin/bash
# Round-3: item-row operations only at run boundaries (MFHIP_ITEM_BRANCH build, lib_ib) vs lib.
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
MFHIP_LIB=$PWD/large-scale-recommendation_amd/lib_ib/libmfhip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py -m gpu -x -q --timeout 300 --timeout-method thread -k "systolic or fast or schedule" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in NFLX ML20M; do
  LIBS="lib lib_ib lib lib_ib" ARGS="--config $cfg --online-batches 0 --det-epochs 0" bash tools/gpurun_libcmp.sh || exit 1
done
