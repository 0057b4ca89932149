#!/bin/bash
# configs[2] PPO (65,536 envs, 2x256, T=32, 10 epochs x 32 minibatches) at
# the curriculum level the configs[0] CPU anchor ends at (eps 4.8,
# tests/golden/c1_anchor.json): every env starts at eps 4.8 (drone.py:68-73's
# per-env bump keeps running on top; ~1,300 episodes per env in this run,
# so it never fires).  JSON lines every 10 updates.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
EPS=${1:-4.8}; STEPS=${2:-2.1e9}; SEED=${3:-0}
timeout -k 10 900 python -u -m drone_rl_amd.train --initial-eps $EPS --total-steps $STEPS \
  --log-every 10 --seed $SEED --checkpoint /tmp/c3_eps${EPS}_s$SEED.pt > gpurun_out/c3_eps${EPS}_s$SEED.jsonl 2> gpurun_out/c3_eps${EPS}_s$SEED.err
