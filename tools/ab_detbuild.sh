#!/bin/bash
# Det sweep input built on the device (MFHIP_TEST=det_build=device) against the host build (default):
# the bit-exact GPU tests, then the NFLX det leg of bench.py in both modes with MFHIP_TIMING host waits.
set -o pipefail
O=gpurun_out/${1:?out dir}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dsgd.py tests/test_gpu_rank.py tests/test_gpu_online.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS FAILED; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for mode in host device; do
    if [ $mode = host ]; then unset MFHIP_TEST; else export MFHIP_TEST=det_build=device; fi
    MFHIP_TIMING=1 timeout -k 10 400 python bench.py --steps 1 --no-cpu-baseline --ml20m-epochs 0 --block-update-reps 0 --online-batches 0 --no-profile > $O/b_${mode}_$rep.json 2> $O/b_${mode}_$rep.err || { echo bench failed; tail -5 $O/b_${mode}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${mode}_$rep.json').read().strip().splitlines()[-1]); de=d['deterministic']
print('$mode', round(de['value']/1e6,1), 'Mups', de['ms_per_step'], 'ms/epoch, launch', de['avg_launch_us'], 'cold', round(de['cold_value']/1e6,1), 'rmse_eq', de['rmse_equal_to_ref'])"
    grep "det_run: 80" $O/b_${mode}_$rep.err | tail -1
  done
done
