# A/B the NFLX bench across library builds: LIBS="lib lib_exp ..." (dirs under the package)
mkdir -p gpurun_out
for L in ${LIBS:-lib}; do
  MFHIP_LIB=large-scale-recommendation_amd/$L/libmfhip.so timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-profile ${ARGS:-} > gpurun_out/cmp_$L.log 2>&1 || { echo FAIL $L; tail -3 gpurun_out/cmp_$L.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cmp_$L.log').read().strip().splitlines()[-1]); print('$L', round(d['value']/1e6), d['ms_per_step'], d['rmse'])"
done
