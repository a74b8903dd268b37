set -o pipefail
mkdir -p gpurun_out/r3d
for U in 0 2000; do
  if [ $U -gt 0 ]; then export CHAIN_USERS=$U; fi
  timeout -k 10 300 python tools/chain_bench.py 128 100000 chain > gpurun_out/r3d/chain_$U.log 2>&1 || { echo "chain failed"; tail -5 gpurun_out/r3d/chain_$U.log; exit 1; }
  echo "users=$U: $(grep substep gpurun_out/r3d/chain_$U.log)"
  timeout -k 10 300 python tools/det_chain_bench.py 128 30000 0 > gpurun_out/r3d/det_$U.log 2>&1 || { echo "det failed"; tail -5 gpurun_out/r3d/det_$U.log; exit 1; }
  echo "users=$U: $(tail -1 gpurun_out/r3d/det_$U.log)"
done
