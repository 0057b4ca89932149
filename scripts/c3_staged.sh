#!/bin/bash
# configs[2] PPO on the GYM variant (65,536 envs, 2x256, T=32, 10 epochs x 32
# minibatches) with a staged curriculum: eps 0 (target (0,0,1)) until update
# 300, then +0.05 every 20 updates up to eps 1.0 at update 680, held to 800
# (drone.py:68-73's per-env bump keeps running on top; it never fires at
# ~300 episodes per env).  JSON lines every 10 updates, one log per seed.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SCHED=$(python3 -c "print(','.join(f'{300 + 20 * i}:{0.05 * (i + 1):.2f}' for i in range(20)))")
for SEED in ${SEEDS:-0 1 2}; do
  timeout -k 10 400 python -u -m drone_rl_amd.train --eps-schedule "$SCHED" \
    --total-steps ${STEPS:-1.678e9} --log-every 10 --seed $SEED \
    --checkpoint /tmp/c3_staged_s$SEED.pt > gpurun_out/r03_ppo_c3_staged_s$SEED.jsonl \
    2> gpurun_out/r03_ppo_c3_staged_s$SEED.err || exit $?
  tail -1 gpurun_out/r03_ppo_c3_staged_s$SEED.jsonl
done
