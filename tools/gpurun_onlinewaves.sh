mkdir -p gpurun_out
for W in 1024 4096 16384 4096; do
  MFHIP_ONLINE_WAVES=$W timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --det-epochs 0 > gpurun_out/w_$W.log 2>/dev/null || { echo FAIL $W; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/w_$W.log').read().strip().splitlines()[-1]); print('$W', round(d['online']['value']/1e6,1))"
done
