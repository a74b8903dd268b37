#!/bin/bash
# Round-3: placement modes (1: heaviest on the least crowded CU slots; 2: per-CU wave counts chosen
# against a crowding factor, empty blocks as padding) -- systolic tests under mode 2, A/B.
set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
MFHIP_SYS_PLACE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_rank.py -m gpu -x -q --timeout 300 --timeout-method thread -k "systolic or fast or schedule or rank or ring" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB="MFHIP_SYS_PLACE=1|MFHIP_SYS_PLACE=2" REPS=2 bash tools/gpurun_ab.sh
CFG=ML20M AB="MFHIP_SYS_PLACE=1|MFHIP_SYS_PLACE=2" REPS=2 bash tools/gpurun_ab.sh
MFHIP_SYS_PLACE=2 MFHIP_WAVE_TRACE=$O/wt_NFLX.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/trace.log 2>&1 || { echo "trace failed"; tail -3 $O/trace.log; exit 1; }
python tools/sys_trace.py $O/wt_NFLX.txt > $O/trace_NFLX.txt 2>&1 || true
grep -A2 "superstep [0-2]:" $O/trace_NFLX.txt
