set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log; tail -15 gpurun_out/pytest_gpu.log
for kern in persistent substep; do
for w in -32 -64 -128 0; do
  MFHIP_FAST_KERNEL=$kern timeout -k 10 120 python bench.py --scale 0.1 --steps 2 --warmup 1 --no-cpu-baseline --fast-waves $w > gpurun_out/sw_${kern}_$w.log 2>&1 || { echo "FAIL $kern $w"; tail -3 gpurun_out/sw_${kern}_$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw_${kern}_$w.log').read().strip().splitlines()[-1]); print('$kern', $w, round(d['value']/1e6,1), d['ms_per_step'], d['roofline']['avg_launch_us'], d['config']['groups'], d['rmse'])"
done; done
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/full.log 2>&1 || exit 1
tail -1 gpurun_out/full.log
