#!/bin/bash
# Round-3 profiles of the two kernels without committed rocprof evidence (k_det_sweep2: the
# deterministic f64 sweep, k_online_sweep: online micro-batches), the VALU / f64 latency
# microbenchmark, and the wait-cycle probe of the systolic pair sweep (experiment build
# lib_probe, MFHIP_WAITPROBE: the trace's clock column = shader cycles spent in the ring waits).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
cd $R
hipcc -O3 --offload-arch=gfx950 -o $O/valu_lat tools/micro/valu_lat.hip > $O/build.log 2>&1 || { echo "micro build failed"; tail -5 $O/build.log; exit 1; }
timeout -k 10 60 $O/valu_lat > $O/valu_lat.txt 2>&1 || { echo "micro failed"; tail -5 $O/valu_lat.txt; exit 1; }
cat $O/valu_lat.txt
# wait-cycle probe: busiest wave of the first supersteps, and the isolated one-wave chain
MFHIP_LIB=$R/large-scale-recommendation_amd/lib_probe/libmfhip.so MFHIP_WAVE_TRACE=$O/wt_probe.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 0 --det-epochs 0 > $O/probe.log 2>&1 || { echo "probe bench failed"; tail -3 $O/probe.log; exit 1; }
python tools/sys_trace.py $O/wt_probe.txt > $O/probe_trace.txt 2>&1 || { echo "sys_trace failed"; exit 1; }
grep -A1 "superstep [0-3]" $O/probe_trace.txt || true
MFHIP_LIB=$R/large-scale-recommendation_amd/lib_probe/libmfhip.so MFHIP_WAVE_TRACE=$O/wt_probe_chain.txt timeout -k 10 300 python tools/chain_bench.py 128 100000 chain > $O/probe_chain.log 2>&1 || { echo "probe chain failed"; tail -3 $O/probe_chain.log; exit 1; }
python tools/sys_trace.py $O/wt_probe_chain.txt > $O/probe_chain_trace.txt 2>&1 || true
grep "busiest wave:" $O/probe_chain_trace.txt || true
cd /tmp
DET="--mode det --steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 5 --det-epochs 0"
FAST="--steps 1 --warmup 0 --no-cpu-baseline --no-profile --online-batches 5 --det-epochs 0"
for leg in det fast; do
  ARGS=$([ $leg = det ] && echo "$DET" || echo "$FAST")
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$leg -o kt --output-format csv -- python3 $R/bench.py $ARGS > $O/prof_kt_$leg.log 2>&1 || { echo "kt $leg failed"; tail -5 $O/prof_kt_$leg.log; exit 1; }
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$leg -o fetch --output-format csv -- python3 $R/bench.py $ARGS > $O/prof_fetch_$leg.log 2>&1 || { echo "fetch $leg failed"; tail -5 $O/prof_fetch_$leg.log; exit 1; }
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/write_$leg -o write --output-format csv -- python3 $R/bench.py $ARGS > $O/prof_write_$leg.log 2>&1 || { echo "write $leg failed"; tail -5 $O/prof_write_$leg.log; exit 1; }
  echo "== $leg"; head -6 $(ls $O/kt_$leg/*kernel_stats.csv | head -1) | cut -c1-200
done
