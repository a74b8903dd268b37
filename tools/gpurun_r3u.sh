#!/bin/bash
# Round-3: ML20M with more rotation groups -- does a larger G lose on step cost (CU crowding) or on
# waits (systolic coupling)?  Wave traces at the default model and at cheaper modelled cells.
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
for M in "6000,300,186" "3000,300,186" "1500,300,186"; do
  t=${M%%,*}
  MFHIP_SYS_MODEL=$M MFHIP_WAVE_TRACE=$O/wt_$t.txt timeout -k 10 300 python bench.py --config ML20M --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/bench_$t.log 2>&1 || { echo "trace $M failed"; tail -3 $O/bench_$t.log; exit 1; }
  echo "== model $M"; python tools/crowd_trace.py $O/wt_$t.txt 2>&1 | tee $O/crowd_$t.txt
done
for M in "6000,300,186" "3000,300,186" "1500,300,186"; do
  MFHIP_SYS_MODEL=$M timeout -k 10 300 python bench.py --config ML20M --steps 5 --warmup 1 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/b.json 2> $O/b.err || { echo "bench $M failed"; tail -3 $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$M', d['ms_per_step'], 'ms')"
done
