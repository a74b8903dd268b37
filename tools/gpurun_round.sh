#!/bin/bash
# Round measurements on one MI355X: the default bench line (NFLX, with the CPU baseline, ONLINE
# and deterministic legs), the ML20M line, the rocprofv3 kernel trace + stats of the NFLX bench,
# and two separate --pmc passes (FETCH_SIZE, WRITE_SIZE: the TCC counter budget), summarised
# per launch by tools/pmc_summary.py.  Everything lands in gpurun_out/round/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py > $O/bench_NFLX.json 2> $O/bench_NFLX.err || { echo "bench NFLX failed"; tail -5 $O/bench_NFLX.err; exit 1; }
echo "NFLX: $(tail -c 300 $O/bench_NFLX.json)"
timeout -k 10 600 python bench.py --config ML20M > $O/bench_ML20M.json 2> $O/bench_ML20M.err || { echo "bench ML20M failed"; tail -5 $O/bench_ML20M.err; exit 1; }
echo "ML20M done"
LEAN="--no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0"
cd /tmp
for cfg in NFLX ML20M; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$cfg -o kt --output-format csv -- python3 $R/bench.py --config $cfg --steps 2 --warmup 1 $LEAN > $O/prof_kt_$cfg.log 2>&1 || { echo "kt $cfg failed"; tail -5 $O/prof_kt_$cfg.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$cfg -o fetch --output-format csv -- python3 $R/bench.py --config $cfg --steps 1 --warmup 0 $LEAN > $O/prof_fetch_$cfg.log 2>&1 || { echo "fetch $cfg failed"; tail -5 $O/prof_fetch_$cfg.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$cfg -o write --output-format csv -- python3 $R/bench.py --config $cfg --steps 1 --warmup 0 $LEAN > $O/prof_write_$cfg.log 2>&1 || { echo "write $cfg failed"; tail -5 $O/prof_write_$cfg.log; exit 1; }
  K=$([ $cfg = NFLX ] && echo 128 || echo 64)
  python3 $R/tools/pmc_summary.py --stats $(ls $O/kt_$cfg/*kernel_stats.csv | head -1) \
    --fetch $(ls $O/fetch_$cfg/*counter_collection.csv | head -1) --write $(ls $O/write_$cfg/*counter_collection.csv | head -1) \
    --kernel k_sweep_pair_sys --config $cfg --mode fast --rank $K --out $O/traffic_$cfg.json > /dev/null || { echo "summary $cfg failed"; exit 1; }
  echo "$cfg traffic: $(cat $O/traffic_$cfg.json | tr -d '\n' | cut -c1-300)"
done
