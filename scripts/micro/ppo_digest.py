"""Digest of the policy parameters after two PPO updates (configs[2], seed
0) and the update rate over five more, for same-box A/B of library builds
run in separate processes (DRONERL_LIB=...): equal digests mean the builds
train bitwise the same."""
import hashlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402

tr = PPOTrainer(PPOConfig(seed=0))
tr.learn_step()
tr.learn_step()
torch.cuda.synchronize()
dig = hashlib.sha256(tr.policy.flat.detach().cpu().numpy().tobytes()).hexdigest()[:16]
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    tr.learn_step()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
ts.sort()
print(json.dumps({"lib": os.environ.get("DRONERL_LIB", "in-tree"), "params_digest": dig,
                  "updates_per_s_median": round(1 / ts[2], 4)}), flush=True)
