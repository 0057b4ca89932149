#!/bin/bash
# Round 5: the driver's multi-rank command form, rehearsed on the one-GPU box
# with both ranks on the card over gloo (RCCL refuses two ranks per device):
# torch.distributed.run --nproc-per-node 2 ... bench.py --gpus 2 --steps 20.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export DRONERL_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/r05_n2_gloo.log 2>&1
rc=$?; grep '^{' gpurun_out/r05_n2_gloo.log | tail -1 > gpurun_out/r05_n2_gloo.json; tail -3 gpurun_out/r05_n2_gloo.log | cut -c1-300; exit $rc
