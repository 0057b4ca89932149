"""Time dr_ppo_head_loss_backward (both heads + PPO loss + backward through
the heads and the top tanh) on one 65,536-row minibatch of pre-activations,
actions / aux rows contiguous as the trainer's record gather leaves them
(ROWS=1: read through a permutation of a 2,097,152-row rollout buffer
instead, the rounds-3-5 form), deferred finish (defer=2), on the library DRONERL_LIB names;
digest of gz_pi / gz_vf and the per-block rows so variants that change
results show it.

  DRONERL_LIB=scripts/micro/build/lib_x.so python scripts/micro/head_bench.py
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import ppo_kernels as K  # noqa: E402

REPS = int(os.environ.get("REPS", "50"))
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
M, HD, NBUF = 65536, 256, 32 * 65536
z_pi = torch.randn(M, HD, generator=g).to(dev)
z_vf = torch.randn(M, HD, generator=g).to(dev)
w_act = (torch.randn(4, HD, generator=g) * 0.01).to(dev)
b_act = torch.zeros(4, device=dev)
w_val = (torch.randn(1, HD, generator=g) * 0.06).to(dev)
b_val = torch.zeros(1, device=dev)
log_std = torch.zeros(4, device=dev)
ROWS = os.environ.get("ROWS", "0") == "1"
NA = NBUF if ROWS else M
actions = (torch.randn(NA, 4, generator=g) * 0.5).to(dev)
aux = torch.randn(NA, 3, generator=g).to(dev)
aux[:, 0] = -4.0
rows = torch.randperm(NBUF, generator=g)[:M].to(torch.int32).to(dev) if ROWS else None
gz_pi, gz_vf = torch.empty_like(z_pi), torch.empty_like(z_vf)
gw_act, gb_act = torch.empty_like(w_act), torch.empty(4, device=dev)
gw_val, gb_val = torch.empty_like(w_val), torch.empty(1, device=dev)
gb_pi, gb_vf, g_ls = (torch.empty(HD, device=dev), torch.empty(HD, device=dev),
                      torch.empty(4, device=dev))
head = K.HeadLossBackward(M, HD, dev)


def run(adv_ready=True):
    # adv_ready: the advantage partials already in the workspace (written by
    # the first, adv_ready=False call), as the trainer's gather leaves them
    head(z_pi, z_vf, w_act, b_act, w_val, b_val, log_std, actions, aux, gz_pi, gz_vf, gw_act,
         gb_act, gw_val, gb_val, gb_pi, gb_vf, g_ls, rows=rows, preact=True, defer=2,
         adv_ready=adv_ready)


run(False)


def timed(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / REPS, 2)


out = {"lib": os.environ.get("DRONERL_LIB", "in-tree"), "head_us": timed(run)}
torch.cuda.synchronize()
hsh = hashlib.sha256()
for t in (gz_pi, gz_vf, head.ws):
    hsh.update(t.cpu().numpy().tobytes())
out["digest"] = hsh.hexdigest()[:16]
print(json.dumps(out), flush=True)
