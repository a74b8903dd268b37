# Deterministic leg A/B (NFLX, 2 epochs f64): LIBS="lib lib_exp ..." plus the det GPU tests on lib
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dsgd.py -k "det or golden" > gpurun_out/det_tests.log 2>&1 || { tail -30 gpurun_out/det_tests.log; exit 1; }
tail -2 gpurun_out/det_tests.log
for L in ${LIBS:-lib}; do
  MFHIP_LIB=large-scale-recommendation_amd/$L/libmfhip.so timeout -k 10 300 python bench.py --mode det --steps 2 --warmup 1 --no-cpu-baseline --no-profile --online-batches 0 > gpurun_out/det_$L.log 2> gpurun_out/det_$L.err || { echo FAIL $L; tail -5 gpurun_out/det_$L.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/det_$L.log').read().strip().splitlines()[-1]); print('$L', d['value'], d['ms_per_step'], d.get('rmse'))"
done
