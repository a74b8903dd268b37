#!/bin/bash
# Round-3: full GPU suite on the current tree, then the placement A/B on the YAHOO shape (k=256).
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
CFG=YAHOO STEPS=2 AB="MFHIP_SYS_PLACE=0|MFHIP_SYS_PLACE=1" REPS=1 bash tools/gpurun_ab.sh
