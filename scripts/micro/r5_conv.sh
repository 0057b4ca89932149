#!/bin/bash
# Round 5: the eps-0 hover run of round 2 (profiles/r02_ppo_c3_eps0_x6_s0.jsonl)
# repeated on the round-5 kernels (fused first-layer backward, direct
# finishes, fused operand images), seed 0, 1.6e9 env-steps.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m drone_rl_amd.train --initial-eps 0 --total-steps 1.6e9 \
  --log-every 10 --seed 0 --checkpoint /tmp/c3_r5.pt > gpurun_out/r05_c3_eps0_s0.jsonl 2> gpurun_out/r05_c3_eps0_s0.err
rc=$?; tail -2 gpurun_out/r05_c3_eps0_s0.jsonl; exit $rc
