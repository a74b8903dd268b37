#!/bin/bash
# Round-3: the det run's speculative next-run builds -- the whole GPU suite (det bitwise goldens,
# staged runs, rank rehearsal, online after det), then the det leg at 1 / 2 / 4 timed epochs.
set -o pipefail
O=gpurun_out/r3ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for E in 1 2 4; do
  timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs $E > $O/det_$E.json 2> $O/det_$E.err || { echo "det $E failed"; tail -3 $O/det_$E.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/det_$E.json').read().strip().splitlines()[-1])['deterministic']; print('$E epochs', d['ms_per_step'], 'ms/epoch', d['value'], 'kernel us', d['avg_launch_us'], 'rmse equal', d['rmse_equal_to_ref'])"
done
