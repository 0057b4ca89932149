"""dr_linear_tanh2 at the trainer's shape (65,536 gathered rows of a
2,097,152-row rollout buffer, obs_dim 15, 256 wide, both nets): time per
launch (median of 5 event-timed batches) and the SHA-256 of both outputs,
for an A/B of library builds run in separate processes (DRONERL_LIB=...).

  python scripts/micro/lt_ab.py [--m 65536] [--total 2097152] [--reps 50]
"""
import argparse
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402
from drone_rl_amd._lib import check, ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=65536)
ap.add_argument("--total", type=int, default=2097152)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
L = _lib.lib()
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
K, N = 15, 256
x = torch.randn(a.total, K, generator=g).to(dev)
rows = torch.randperm(a.total, generator=g)[:a.m].to(torch.int32).to(dev)
w = [(torch.randn(N, K, generator=g) * 0.3).to(dev) for _ in range(2)]
b = [(torch.randn(N, generator=g) * 0.1).to(dev) for _ in range(2)]
h = [torch.empty(a.m, N, device=dev) for _ in range(2)]
s = torch.cuda.current_stream().cuda_stream


xg = x[rows.long()].contiguous()       # the trainer's form: a gathered minibatch
out = {"lib": os.path.basename(os.path.dirname(_lib.LIB_PATH)) + "/" +
       os.path.basename(_lib.LIB_PATH)}
w256 = (torch.randn(2, 256, 256, generator=g) * 0.06).to(dev)
img = torch.empty(2 * L.dr_gemm_x6_weights_bytes(2), dtype=torch.uint8, device=dev)
ximg = torch.empty(L.dr_gemm_x6_x_bytes(a.m), dtype=torch.uint8, device=dev)
for mode, xx, rr in (("rows", x, ptr(rows)), ("dense", xg, None), ("x6", xg, None)):
    def call():
        if mode == "x6":   # the trainer's form: + both weight images and the obs image
            check(L.dr_linear_tanh2_x6(a.m, K, N, ptr(xx), rr, ptr(w[0]), ptr(b[0]), ptr(h[0]),
                                       ptr(w[1]), ptr(b[1]), ptr(h[1]), ptr(w256), ptr(img),
                                       ptr(ximg), s))
        else:
            check(L.dr_linear_tanh2(a.m, K, N, ptr(xx), rr, ptr(w[0]), ptr(b[0]), ptr(h[0]),
                                    ptr(w[1]), ptr(b[1]), ptr(h[1]), s))
    call()
    torch.cuda.synchronize()
    sha = hashlib.sha256(h[0].cpu().numpy().tobytes() + h[1].cpu().numpy().tobytes() +
                         (img.cpu().numpy().tobytes() + ximg.cpu().numpy().tobytes()
                          if mode == "x6" else b"")).hexdigest()[:16]
    ref = torch.tanh(xg.double() @ w[0].double().T + b[0].double())
    err = (h[0].double() - ref).abs().max().item()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        st.record()
        for _ in range(a.reps):
            call()
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en) * 1e3 / a.reps)
    ts.sort()
    byt = a.m * (K * 4 + 2 * N * 4)
    out[mode] = {"us": round(ts[2], 2), "us_min": round(ts[0], 2),
                 "frac": round(byt / ts[2] / 8e6, 3), "sha": sha, "abs_err": err}
print(json.dumps(out))
