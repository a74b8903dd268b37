#!/bin/bash
# Round-3 closing run: the whole GPU suite, smoke(), and the systolic wave-trace summaries (placement on,
# the default build) of NFLX and ML20M.  Traces are summarised on the box and deleted (size).
set -o pipefail
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for cfg in NFLX ML20M; do
  MFHIP_WAVE_TRACE=/tmp/wt_$cfg.txt timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/trace_bench_$cfg.log 2>&1 || { echo "trace $cfg failed"; tail -3 $O/trace_bench_$cfg.log; exit 1; }
  { python tools/sys_trace.py /tmp/wt_$cfg.txt && python tools/crowd_trace.py /tmp/wt_$cfg.txt; } > $O/wave_trace_$cfg.txt 2>&1 || { echo "trace summary $cfg failed"; tail -3 $O/wave_trace_$cfg.txt; exit 1; }
  rm -f /tmp/wt_$cfg.txt
  echo "== $cfg"; grep -E "^kind|sum of superstep|busiest wave:" $O/wave_trace_$cfg.txt | head -8
done
