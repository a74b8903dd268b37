mkdir -p gpurun_out
export NCCL_DEBUG=WARN
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rank_check.py --mode det > gpurun_out/rank_det.log 2>&1; echo "det rc=$?"; tail -5 gpurun_out/rank_det.log
