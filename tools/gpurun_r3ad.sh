#!/bin/bash
# Round-3: det leg repeatability with the speculative builds (2 timed epochs = the bench default).
set -o pipefail
O=gpurun_out/r3ad
mkdir -p $O
for E in 2 2 1 2 4; do
  timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs $E > $O/det_$E.json 2> $O/det_$E.err || { echo "det $E failed"; tail -3 $O/det_$E.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/det_$E.json').read().strip().splitlines()[-1])['deterministic']; print('$E epochs', d['ms_per_step'], 'ms/epoch', d['value'], 'kernel us', d['avg_launch_us'], 'rmse equal', d['rmse_equal_to_ref'])"
done
