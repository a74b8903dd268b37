#!/bin/bash
# Round-3 diagnosis of the in-situ slowdown of the hot single-run chain: where every systolic wave
# runs (trace column 10: XCC / SE / CU / SIMD), the critical-wave priority A/B, the isolated and
# loaded deterministic f64 chain, and the PMC counter list.  Output under gpurun_out/r3g/.
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
MFHIP_WAVE_TRACE=$O/wt.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/trace_bench.log 2>&1 || { echo "trace bench failed"; tail -3 $O/trace_bench.log; exit 1; }
python tools/sys_trace.py $O/wt.txt > $O/trace.txt 2>&1 || { echo "sys_trace failed"; tail -3 $O/trace.txt; exit 1; }
grep -A2 "superstep [0-7]:" $O/trace.txt
for v in 1 2; do
  timeout -k 10 300 python tools/det_chain_bench.py 128 30000 0 > $O/det_chain_iso.log 2>&1 || { echo "det chain failed"; tail -3 $O/det_chain_iso.log; exit 1; }
done
tail -1 $O/det_chain_iso.log
timeout -k 10 300 python tools/det_chain_bench.py 128 30000 2000000 > $O/det_chain_bg.log 2>&1 || { echo "det chain bg failed"; tail -3 $O/det_chain_bg.log; exit 1; }
tail -1 $O/det_chain_bg.log
AB="MFHIP_HOT_PRIO=0|MFHIP_HOT_PRIO=2" REPS=2 bash tools/gpurun_ab.sh
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT[A-Z_]*" $O/counters.txt | sort -u | head -40
