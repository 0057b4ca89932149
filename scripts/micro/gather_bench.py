"""dr_gather_records at the trainer's shape (65,536 random rows of a
2,097,152-row record buffer, 15-d obs, advantage partials on): time per
launch (median of 7 event-timed batches) and the SHA-256 of every output,
for an A/B of library builds run in separate processes (DRONERL_LIB=...).

  python scripts/micro/gather_bench.py [--reps 200]
"""
import argparse
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402
from drone_rl_amd import ppo_kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=200)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
N, M, D = 32 * 65536, 65536, 15
obs = torch.randn(N, D, generator=g).to(dev)
act = torch.randn(N, 4, generator=g).to(dev)
lp, adv, ret = (torch.randn(N, generator=g).to(dev) for _ in range(3))
rec = torch.empty(N, K.RECORD_FLOATS, device=dev)
K.pack_rollout_records(obs, act, lp, adv, ret, rec)
idx = torch.randperm(N, generator=g)[:M].to(torch.int32).to(dev)
o, ac, ax = torch.empty(M, D, device=dev), torch.empty(M, 4, device=dev), torch.empty(M, 3, device=dev)
part = torch.empty(3 * ((M + 255) // 256), device=dev)


def call():
    K.gather_records(idx, rec, D, o, ac, ax, part)


call()
torch.cuda.synchronize()
h = hashlib.sha256()
for t in (o, ac, ax, part):
    h.update(t.cpu().numpy().tobytes())
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(7):
    st.record()
    for _ in range(a.reps):
        call()
    en.record()
    torch.cuda.synchronize()
    ts.append(st.elapsed_time(en) * 1e3 / a.reps)
ts.sort()
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "us": round(ts[3], 2),
                  "us_min": round(ts[0], 2), "sha": h.hexdigest()[:16]}))
