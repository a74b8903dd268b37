# Round profile of the NFLX bench: full bench line (with the CPU baseline), rocprofv3 kernel
# trace + stats, and two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: TCC budget) summarised
# into a per-launch HBM traffic record (tools/pmc_summary.py).  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS=${BENCH_ARGS:-}
timeout -k 10 600 python bench.py $ARGS > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rocprof_kt -o kt --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile $ARGS > $R/gpurun_out/prof_kt.log 2>&1 || { echo "kt failed"; tail -5 $R/gpurun_out/prof_kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/rocprof_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile $ARGS > $R/gpurun_out/prof_fetch.log 2>&1 || { echo "fetch failed"; tail -5 $R/gpurun_out/prof_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/rocprof_write -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile $ARGS > $R/gpurun_out/prof_write.log 2>&1 || { echo "write failed"; tail -5 $R/gpurun_out/prof_write.log; exit 1; }
cd $R
head -4 gpurun_out/rocprof_kt/kt_kernel_stats.csv | cut -c1-160
