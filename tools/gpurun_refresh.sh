# Round record refresh for one config (CFG=NFLX|ML20M, K = its rank): rocprofv3 kernel trace +
# stats, two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: TCC budget) summarised on the box
# into gpurun_out/traffic_$CFG.json, then the full bench line (CPU baseline included) reading
# that traffic record.  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${CFG:-NFLX}
K=${K:-128}
G=${G:-0}
B="--config $CFG --no-cpu-baseline --no-profile"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_$CFG -o kt --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 $B > $R/gpurun_out/prof_kt_$CFG.log 2>&1 || { echo "kt failed"; tail -5 $R/gpurun_out/prof_kt_$CFG.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/fetch_$CFG -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > $R/gpurun_out/prof_fetch_$CFG.log 2>&1 || { echo "fetch failed"; tail -5 $R/gpurun_out/prof_fetch_$CFG.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/write_$CFG -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > $R/gpurun_out/prof_write_$CFG.log 2>&1 || { echo "write failed"; tail -5 $R/gpurun_out/prof_write_$CFG.log; exit 1; }
cd $R
python3 tools/pmc_summary.py --stats gpurun_out/kt_$CFG/kt_kernel_stats.csv \
  --fetch gpurun_out/fetch_$CFG/fetch_counter_collection.csv --write gpurun_out/write_$CFG/write_counter_collection.csv \
  --kernel k_sweep_pair_sys --config $CFG --mode fast --rank $K --groups $G --out gpurun_out/traffic_$CFG.json || exit 1
timeout -k 10 600 python bench.py --config $CFG --traffic-json gpurun_out/traffic_$CFG.json > gpurun_out/bench_full_$CFG.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_full_$CFG.log; exit 1; }
tail -1 gpurun_out/bench_full_$CFG.log
head -3 gpurun_out/kt_$CFG/kt_kernel_stats.csv | cut -c1-200
