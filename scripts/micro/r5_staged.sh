#!/bin/bash
# Round 5: the staged-curriculum run of round 3 (ent_coef 0.01, eps 0 -> 1.0)
# on the round-5 kernels, seeds 0 and 1, with the deterministic / sampled
# evaluation at eps 1.0.
cd "$(dirname "$0")/../.."
ENT=0.01 TAG=r05_ppo_c3_staged_ent01 SEEDS="0 1" bash scripts/c3_staged.sh
