"""dr_gemm_x6 (forward image) at the trainer's shape (2 nets, 65,536 rows):
time per launch (median of 5 event-timed batches, cold-ish: A is 128 MB) and
the SHA-256 of C, for an A/B of library builds run in separate processes
(DRONERL_LIB=...).

  python scripts/micro/x6_fwd_ab.py [--m 65536] [--reps 50]
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
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
L = _lib.lib()
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
M = a.m
A = torch.tanh(torch.randn(2, M, 256, generator=g)).to(dev)
W = (torch.randn(2, 256, 256, generator=g) * (2 / 256) ** 0.5).to(dev)
img = torch.empty(L.dr_gemm_x6_weights_bytes(2), dtype=torch.uint8, device=dev)
C = torch.empty(2, M, 256, device=dev)
s = torch.cuda.current_stream().cuda_stream
check(L.dr_gemm_x6_split_weights(2, ptr(W), 0, ptr(img), s))
check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
torch.cuda.synchronize()
sha = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
n = min(M, 4096)
ref = torch.bmm(A[:, :n].double(), W.transpose(1, 2).double())
den = torch.bmm(A[:, :n].abs().double(), W.transpose(1, 2).abs().double())
err = ((C[:, :n].double() - ref).abs() / den).max().item()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(5):
    st.record()
    for _ in range(a.reps):
        check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    en.record()
    torch.cuda.synchronize()
    ts.append(st.elapsed_time(en) * 1e3 / a.reps)
ts.sort()
print(json.dumps({"lib": os.path.basename(os.path.dirname(_lib.LIB_PATH)) + "/" +
                  os.path.basename(_lib.LIB_PATH), "us": round(ts[2], 2),
                  "us_min": round(ts[0], 2), "sha": sha, "rel_err": err}))
