"""dr_gemm_x6_wgrad at the trainer's shape (2 nets, 65,536 rows, 64 chunks):
time per launch (median of 5 event-timed batches) and the SHA-256 of the
partials, for an A/B of library builds run in separate processes
(DRONERL_LIB=...).

  python scripts/micro/wgrad_ab.py [--m 65536] [--chunks 64] [--reps 50]
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
ap.add_argument("--chunks", type=int, default=64)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
L = _lib.lib()
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
M, C = a.m, a.chunks
H = torch.tanh(torch.randn(2, M, 256, generator=g)).to(dev)
G = (torch.randn(2, M, 256, generator=g) * 1e-3).to(dev)
ws = torch.empty(2, C, 256, 256, device=dev)
s = torch.cuda.current_stream().cuda_stream
check(L.dr_gemm_x6_wgrad(2, M, C, ptr(G), ptr(H), ptr(ws), s))
torch.cuda.synchronize()
sha = hashlib.sha256(ws.cpu().numpy().tobytes()).hexdigest()[:16]
rows = M // C
ref = torch.bmm(G[:, :rows].transpose(1, 2).double(), H[:, :rows].double())
den = torch.bmm(G[:, :rows].transpose(1, 2).abs().double(), H[:, :rows].abs().double())
err = ((ws[:, 0].double() - ref).abs() / den).max().item()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(5):
    st.record()
    for _ in range(a.reps):
        check(L.dr_gemm_x6_wgrad(2, M, C, ptr(G), ptr(H), ptr(ws), s))
    en.record()
    torch.cuda.synchronize()
    ts.append(st.elapsed_time(en) * 1e3 / a.reps)
ts.sort()
print(json.dumps({"lib": os.path.basename(os.path.dirname(_lib.LIB_PATH)) + "/" +
                  os.path.basename(_lib.LIB_PATH), "us": round(ts[2], 2),
                  "us_min": round(ts[0], 2), "sha": sha, "rel_err": err}))
