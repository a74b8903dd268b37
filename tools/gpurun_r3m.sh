#!/bin/bash
# Round-3: systolic wave placement (heaviest waves on the least crowded CUs) -- systolic equality
# tests, A/B on NFLX and ML20M, and a wave trace with the placement on.
set -o pipefail
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py -m gpu -x -q --timeout 300 --timeout-method thread -k "systolic or fast or schedule or plan or ring" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB="MFHIP_SYS_PLACE=0|MFHIP_SYS_PLACE=1" REPS=2 bash tools/gpurun_ab.sh
CFG=ML20M AB="MFHIP_SYS_PLACE=0|MFHIP_SYS_PLACE=1" REPS=2 bash tools/gpurun_ab.sh
MFHIP_WAVE_TRACE=$O/wt_NFLX.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/trace.log 2>&1 || { echo "trace failed"; tail -3 $O/trace.log; exit 1; }
python tools/sys_trace.py $O/wt_NFLX.txt > $O/trace_NFLX.txt 2>&1 || true
grep -A2 "superstep [0-3]:" $O/trace_NFLX.txt
