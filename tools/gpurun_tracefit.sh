# one traced NFLX epoch set; per-kind startup / per-step fit and launch gaps (tools/trace_fit.py)
mkdir -p gpurun_out
MFHIP_WAVE_TRACE=gpurun_out/wt.txt timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile ${ARGS:-} > gpurun_out/b.log 2>&1 || { echo FAIL; tail -3 gpurun_out/b.log; exit 1; }
tail -c 300 gpurun_out/b.log; echo
python tools/trace_fit.py gpurun_out/wt.txt
