set -o pipefail
mkdir -p gpurun_out/r4scale
for n in 2 8; do
  MFHIP_FAKE_HOSTS=1 MFHIP_DEVICE_SHARERS=$n NCCL_DEBUG=ERROR timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29800+n)) bench.py --gpus $n --steps 3 --warmup 1 > gpurun_out/r4scale/n$n.json 2> gpurun_out/r4scale/n$n.err || { echo "n=$n failed"; tail -5 gpurun_out/r4scale/n$n.err; exit 1; }
  tail -1 gpurun_out/r4scale/n$n.json | cut -c1-400
done
