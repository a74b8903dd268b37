# SQ wave-state counters of the fast sweep (one --pmc pass, 8 SQ counters), NFLX k=128, 1 epoch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM -d $R/gpurun_out/rocprof_sq -o sq --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile ${BENCH_ARGS:-} > $R/gpurun_out/prof_sq.log 2>&1 || { echo "sq failed"; tail -5 $R/gpurun_out/prof_sq.log; exit 1; }
cd $R && python3 tools/sq_summary.py gpurun_out/rocprof_sq/sq_counter_collection.csv
