#!/bin/bash
# bench.py's multi-rank path rehearsed on one GPU: 2 ranks over gloo sharing
# the card (RCCL refuses two ranks per GPU), the driver's --steps 20 form
ulimit -c 0
mkdir -p gpurun_out
DRONERL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 \
  --steps 20 --warmup 5 > gpurun_out/x_n2.log 2>&1; rc=$?
grep '^{' gpurun_out/x_n2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['ms_per_step'], d['ppo']['updates_per_s'], d['ppo']['config'].get('grad_allreduce'))"
tail -3 gpurun_out/x_n2.log; exit $rc
