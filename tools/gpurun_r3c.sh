set -o pipefail
mkdir -p gpurun_out/r3c
hipcc -O3 --offload-arch=gfx950 -o gpurun_out/r3c/valu_lat tools/micro/valu_lat.hip > gpurun_out/r3c/build.log 2>&1 || { echo "micro build failed"; tail -5 gpurun_out/r3c/build.log; exit 1; }
timeout -k 10 60 gpurun_out/r3c/valu_lat > gpurun_out/r3c/valu_lat.txt 2>&1 || { echo "micro failed"; tail -5 gpurun_out/r3c/valu_lat.txt; exit 1; }
cat gpurun_out/r3c/valu_lat.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py -m gpu -x -q --timeout 300 --timeout-method thread -k "systolic or substep or schedule or plan" > gpurun_out/r3c/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3c/pytest.log; exit 1; }
tail -1 gpurun_out/r3c/pytest.log
AB="MFHIP_CELL_PRELOAD=0|MFHIP_CELL_PRELOAD=1" bash tools/gpurun_ab.sh
CFG=ML20M AB="MFHIP_CELL_PRELOAD=0|MFHIP_CELL_PRELOAD=1" bash tools/gpurun_ab.sh
