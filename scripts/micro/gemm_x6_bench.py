"""dr_gemm_x6 (exact 3 x bf16 split, 6 MFMA products) against torch fp32
bmm: accuracy against an f64 GEMM on the same inputs, and time per launch.

  python scripts/micro/gemm_x6_bench.py [--m 65536] [--reps 50]
"""
import argparse
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
out = {}
for tr in (0, 1):
    check(L.dr_gemm_x6_split_weights(2, ptr(W), tr, ptr(img), s))
    check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    torch.cuda.synchronize()
    Wt = W if tr else W.transpose(1, 2)           # C = A @ Wt
    n = min(M, 8192)
    ref = torch.bmm(A[:, :n].double(), Wt.double())
    den = torch.bmm(A[:, :n].abs().double(), Wt.abs().double())
    r32 = torch.bmm(A[:, :n], Wt)
    e6 = ((C[:, :n].double() - ref).abs() / den).max().item()
    e32 = ((r32.double() - ref).abs() / den).max().item()
    a6 = (C[:, :n].double() - ref).abs().max().item()
    a32 = (r32.double() - ref).abs().max().item()
    # time
    Wt_c = Wt.contiguous() if tr else W.transpose(1, 2)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    st.record()
    for _ in range(a.reps):
        check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    en.record()
    torch.cuda.synchronize()
    t6 = st.elapsed_time(en) * 1e3 / a.reps
    R = torch.empty(2, M, 256, device=dev)
    for _ in range(3):
        torch.bmm(A, Wt_c, out=R)
    st.record()
    for _ in range(a.reps):
        torch.bmm(A, Wt_c, out=R)
    en.record()
    torch.cuda.synchronize()
    t32 = st.elapsed_time(en) * 1e3 / a.reps
    st.record()
    for _ in range(a.reps):
        check(L.dr_gemm_x6_split_weights(2, ptr(W), tr, ptr(img), s))
    en.record()
    torch.cuda.synchronize()
    tsp = st.elapsed_time(en) * 1e3 / a.reps
    fl = 2 * 2 * M * 256 * 256
    out[f"transpose{tr}"] = {
        "rel_err_x6": e6, "rel_err_f32_bmm": e32, "abs_err_x6": a6, "abs_err_f32_bmm": a32,
        "us_x6": round(t6, 2), "us_f32_bmm": round(t32, 2), "us_split": round(tsp, 2),
        "tflops_x6": round(fl / t6 / 1e6, 1), "tflops_f32_bmm": round(fl / t32 / 1e6, 1),
        "bitwise_rerun": bool(torch.equal(C, C.clone()))}
    # determinism
    C2 = torch.empty_like(C)
    check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C2), s))
    check(L.dr_gemm_x6(2, M, ptr(A), ptr(img), ptr(C), s))
    torch.cuda.synchronize()
    out[f"transpose{tr}"]["bitwise_rerun"] = bool(torch.equal(C, C2))
print(json.dumps(out, indent=1))

# the weight-gradient form against the trainer's split-K bmm (64 chunks)
C = 64
G = (torch.randn(2, M, 256, generator=g) * 1e-3).to(dev)
ws = torch.empty(2, C, 256, 256, device=dev)
ws32 = torch.empty(2 * C, 256, 256, device=dev)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    check(L.dr_gemm_x6_wgrad(2, M, C, ptr(G), ptr(A), ptr(ws), s))
st.record()
for _ in range(a.reps):
    check(L.dr_gemm_x6_wgrad(2, M, C, ptr(G), ptr(A), ptr(ws), s))
en.record()
torch.cuda.synchronize()
tw = st.elapsed_time(en) * 1e3 / a.reps
Gc, Ac = G.reshape(2 * C, M // C, 256), A.reshape(2 * C, M // C, 256)
for _ in range(3):
    torch.bmm(Gc.transpose(1, 2), Ac, out=ws32)
st.record()
for _ in range(a.reps):
    torch.bmm(Gc.transpose(1, 2), Ac, out=ws32)
en.record()
torch.cuda.synchronize()
t32 = st.elapsed_time(en) * 1e3 / a.reps
d = (ws.reshape(2 * C, 256, 256) - ws32).abs().max().item()
print(json.dumps({"wgrad": {"us_x6": round(tw, 2), "us_f32_bmm": round(t32, 2),
                            "max_abs_diff_vs_bmm": d}}))
