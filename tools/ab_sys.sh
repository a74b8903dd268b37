set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS FAILED; tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=large-scale-recommendation_amd/lib_base/libmfhip.so; else L=large-scale-recommendation_amd/lib/libmfhip.so; fi
    MFHIP_LIB=$L timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --online-batches 0 --det-epochs 0 --block-update-reps 0 --no-profile > $O/b_${lib}_$rep.json 2> $O/b_${lib}_$rep.err || { echo bench failed; tail -5 $O/b_${lib}_$rep.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/b_${lib}_$rep.json').read().strip().splitlines()[-1])
print('$lib', d['ms_per_step'], d['ml20m']['ms_per_step'], d.get('rmse_rel'), d['ml20m'].get('rmse_rel'))"
  done
done
