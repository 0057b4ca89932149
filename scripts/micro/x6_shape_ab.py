"""Same-box A/B of the x6 forward GEMM's MFMA shape (round 6): run once per
library build (DRONERL_LIB=scripts/micro/build/lib_m16.so / lib_m32.so), in
alternating processes.  Random tanh activations and random weights at the
trainer's shape (2 nets, 65,536 rows); ~2 s of back-to-back launches first so
the clock has settled (MI355X_MICROARCH.md, DVFS give-back), then the median
of 7 event-timed batches.  Reports the relative error against an f64 GEMM for
both weight images (transpose 0 / 1).

  DRONERL_LIB=... python scripts/micro/x6_shape_ab.py [--m 65536] [--warm-s 2]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402
from drone_rl_amd._lib import check, ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=65536)
ap.add_argument("--reps", type=int, default=200)
ap.add_argument("--warm-s", type=float, default=2.0)
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
out = {"lib": os.path.basename(_lib.LIB_PATH), "m": M}
n = min(M, 4096)
for tr in (1, 0):
    check(L.dr_gemm_x6_split_weights(2, ptr(W), tr, ptr(img), s))
    check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    torch.cuda.synchronize()
    Wt = W if tr else W.transpose(1, 2)
    ref = torch.bmm(A[:, :n].double(), Wt.double())
    den = torch.bmm(A[:, :n].abs().double(), Wt.abs().double())
    out[f"rel_err_t{tr}"] = ((C[:, :n].double() - ref).abs() / den).max().item()
    # the full-size output against the f32 bmm (a layout slip shows as O(1))
    out[f"max_abs_vs_f32_t{tr}"] = (C - torch.bmm(A, Wt)).abs().max().item()
    out[f"sha_t{tr}"] = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
t_end = time.perf_counter() + a.warm_s
while time.perf_counter() < t_end:
    for _ in range(100):
        check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(7):
    st.record()
    for _ in range(a.reps):
        check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    en.record()
    torch.cuda.synchronize()
    ts.append(st.elapsed_time(en) * 1e3 / a.reps)
ts.sort()
fl = 6 * 2 * 2 * M * 256 * 256
out.update(us=round(ts[3], 2), us_min=round(ts[0], 2), us_max=round(ts[-1], 2),
           bf16_tflops=round(fl / ts[3] / 1e6, 1))
print(json.dumps(out))
