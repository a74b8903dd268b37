#!/bin/bash
# Round-3: speculative det builds no longer joined by sync -- GPU suite, then the driver's default
# bench command twice (det leg inside the full line).
set -o pipefail
O=gpurun_out/r3ae
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 600 python bench.py > $O/bench_$rep.json 2> $O/bench_$rep.err || { echo "bench failed"; tail -3 $O/bench_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$rep.json').read().strip().splitlines()[-1]); t=d['deterministic']; print('fast', d['ms_per_step'], d['value'], 'det', t['ms_per_step'], t['value'], t['rmse_equal_to_ref'], 'online', {p: v['value'] for p, v in d['online'].items()})"
done
