#!/bin/bash
# configs[2] PPO on the GYM variant (65,536 envs, 2x256, T=32, minibatches of
# 65,536) with a staged curriculum: eps 0 (target (0,0,1)) until update
# START, then +INC every EVERY updates for STAGES stages (default 0.05 x 20:
# up to eps 1.0), then held (drone.py:
# 68-73's per-env bump keeps running on top; it never fires at a few hundred
# episodes per env).  JSON lines every 10 updates, one log per seed.
#   START EVERY INC STAGES UPDATES EPOCHS ENT EVAL_EPS TAG SEEDS: environment
#   overrides
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
START=${START:-300}; EVERY=${EVERY:-20}; UPDATES=${UPDATES:-800}; EPOCHS=${EPOCHS:-10}
ENT=${ENT:-0.0}; INC=${INC:-0.05}; STAGES=${STAGES:-20}
TAG=${TAG:-r03_ppo_c3_staged}
SCHED=$(python3 -c "print(','.join(f'{$START + $EVERY * i}:{$INC * (i + 1):.2f}' for i in range($STAGES)))")
STEPS=$((UPDATES * 2097152))
for SEED in ${SEEDS:-0 1 2}; do
  timeout -k 10 600 python -u -m drone_rl_amd.train --eps-schedule "$SCHED" \
    --total-steps $STEPS --epochs $EPOCHS --ent-coef $ENT --log-every 10 --seed $SEED \
    --checkpoint /tmp/${TAG}_s$SEED.pt > gpurun_out/${TAG}_s$SEED.jsonl \
    2> gpurun_out/${TAG}_s$SEED.err || exit $?
  tail -1 gpurun_out/${TAG}_s$SEED.jsonl
  # the trained policy at eps 1.0, deterministic (test.py's predict) and sampled
  timeout -k 10 300 python scripts/eval_policy.py /tmp/${TAG}_s$SEED.pt --eps ${EVAL_EPS:-1.0} \
    > gpurun_out/${TAG}_s${SEED}_eval.json || exit $?
  cat gpurun_out/${TAG}_s${SEED}_eval.json
done
