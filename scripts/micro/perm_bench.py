"""Time dr_permutation at configs[2]'s 2,097,152 rollout rows on the library
DRONERL_LIB names, per kernel by events around the whole call (REPS calls),
with a digest of the permutation (variants must agree bitwise).

  DRONERL_LIB=scripts/micro/build/lib_x.so python scripts/micro/perm_bench.py
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import ppo_kernels as K  # noqa: E402

REPS = int(os.environ.get("REPS", "50"))
n = 1 << 21
p = K.Permuter(n, "cuda")
for c in range(3):
    p(seed=7, counter=c)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for c in range(REPS):
    p(seed=7, counter=c)
e1.record()
torch.cuda.synchronize()
out = p(seed=7, counter=12345).cpu().numpy()
print(json.dumps({"lib": os.environ.get("DRONERL_LIB", "in-tree"),
                  "perm_us": round(e0.elapsed_time(e1) * 1e3 / REPS, 2),
                  "digest": hashlib.sha256(out.tobytes()).hexdigest()[:16]}), flush=True)
