set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_online.py -m gpu -x -q --timeout 300 --timeout-method thread -k "deterministic or det or block_update or golden or bit_exact or multi_shard" > gpurun_out/r3e/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3e/pytest.log; exit 1; }
tail -1 gpurun_out/r3e/pytest.log
for v in 1 2; do
  MFHIP_DET_SWEEP=$v timeout -k 10 300 python tools/det_chain_bench.py 128 30000 0 > gpurun_out/r3e/det_$v.log 2>&1 || { echo "det chain failed"; tail -5 gpurun_out/r3e/det_$v.log; exit 1; }
  echo "DET_SWEEP=$v: $(tail -1 gpurun_out/r3e/det_$v.log)"
done
for v in 1 2 1 2; do
  MFHIP_DET_SWEEP=$v timeout -k 10 300 python bench.py --mode det --steps 2 --warmup 1 --no-cpu-baseline --no-profile --online-batches 0 > gpurun_out/r3e/bench_det_$v.json 2> gpurun_out/r3e/bench_det_$v.err || { echo "det bench failed"; tail -5 gpurun_out/r3e/bench_det_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r3e/bench_det_$v.json').read().strip().splitlines()[-1]); print('DET_SWEEP=$v', d['ms_per_step'], 'ms', round(d['value']/1e6,1), 'Mups rmse', d['rmse'])"
done
# wait-cycle probe (experiment build): the trace's 9th column = shader cycles spent waiting for prefetched rows
export MFHIP_LIB=$PWD/large-scale-recommendation_amd/lib_probe/libmfhip.so
MFHIP_WAVE_TRACE=gpurun_out/r3e/wt_probe.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > gpurun_out/r3e/probe.log 2>&1 || { echo "probe bench failed"; tail -3 gpurun_out/r3e/probe.log; exit 1; }
python tools/sys_trace.py gpurun_out/r3e/wt_probe.txt | grep -A1 "superstep [0-3]" | grep busiest
MFHIP_WAVE_TRACE=gpurun_out/r3e/wt_probe_chain.txt timeout -k 10 300 python tools/chain_bench.py 128 100000 chain > gpurun_out/r3e/probe_chain.log 2>&1 || { echo "probe chain failed"; exit 1; }
python tools/sys_trace.py gpurun_out/r3e/wt_probe_chain.txt | grep "busiest wave:"
