set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not YAHOO-1" > gpurun_out/r3b/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3b/pytest.log; exit 1; }
tail -1 gpurun_out/r3b/pytest.log
AB="MFHIP_CELL_PRELOAD=0|MFHIP_CELL_PRELOAD=1" bash tools/gpurun_ab.sh
CFG=ML20M AB="MFHIP_CELL_PRELOAD=0|MFHIP_CELL_PRELOAD=1" bash tools/gpurun_ab.sh
AB="MFHIP_HOT_PRIO=1|MFHIP_HOT_PRIO=2" REPS=1 bash tools/gpurun_ab.sh
CFGS="NFLX ML20M" NO_INTERF=1 bash tools/gpurun_diag.sh
