# Rank-mode (RCCL ring) rehearsal on a one-GPU box: ranks share device 0 and claim distinct
# RCCL host ids (MFHIP_FAKE_HOSTS), so send/recv goes over loopback sockets.  Checks det
# bit-exactness against a single-process context, fast mode bitwise against in-process virtual
# shards (uniform G; with BLOCKS = 2 * WORLD the ring overlap path runs), then a small bench.
mkdir -p gpurun_out
export NCCL_DEBUG=WARN MFHIP_FAKE_HOSTS=1
W=${WORLD:-2}
export MFHIP_DEVICE_SHARERS=$W
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29511 tools/rank_check.py --mode det --blocks ${BLOCKS:-4} > gpurun_out/rank_det.log 2>&1 || { echo "det failed"; tail -20 gpurun_out/rank_det.log; exit 1; }
grep -E "world=|RANK_CHECK" gpurun_out/rank_det.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29512 tools/rank_check.py --mode fast --blocks ${BLOCKS:-4} --fast-waves -8 > gpurun_out/rank_fast.log 2>&1 || { echo "fast failed"; tail -20 gpurun_out/rank_fast.log; exit 1; }
grep -E "world=|RANK_CHECK" gpurun_out/rank_fast.log
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $W --steps 2 --warmup 1 --scale ${SCALE:-0.1} > gpurun_out/rank_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/rank_bench.log; exit 1; }
tail -1 gpurun_out/rank_bench.log
