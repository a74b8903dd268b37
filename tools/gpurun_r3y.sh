#!/bin/bash
# Round-3: PRE = 2 (the next cell's record chunks loaded with the current cell's first ring rows):
# systolic tests under it, then A/B against each config's default (NFLX PRE = 1, ML20M PRE = 0).
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
MFHIP_CELL_PRELOAD=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "systolic or fast or schedule or ring or pair" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB="MFHIP_CELL_PRELOAD=1|MFHIP_CELL_PRELOAD=2" REPS=3 bash tools/gpurun_ab.sh
CFG=ML20M AB="MFHIP_CELL_PRELOAD=0|MFHIP_CELL_PRELOAD=2" REPS=2 bash tools/gpurun_ab.sh
