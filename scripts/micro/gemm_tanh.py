"""Diagnostic: dr_linear_tanh_mfma vs addmm + tanh_ at M = 65,536, 256x256."""
import sys

import torch

sys.path.insert(0, ".")
from drone_rl_amd import ppo_kernels as K  # noqa: E402

M, H = 65536, 256
x = torch.randn(M, H, device="cuda")
w = torch.randn(H, H, device="cuda") * 0.06
b = torch.randn(H, device="cuda") * 0.1
out = torch.empty(M, H, device="cuda")
ref = torch.empty(M, H, device="cuda")


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def torch_path():
    torch.addmm(b, x, w.t(), out=ref)
    torch.tanh_(ref)


def mfma_path():
    K.linear_tanh_mfma(x, w, b, out)


tt, tm = t(torch_path), t(mfma_path)
torch_path()
mfma_path()
torch.cuda.synchronize()
print(f"addmm+tanh {tt:.1f} us   mfma fused {tm:.1f} us   max|diff| {(out - ref).abs().max().item():.2e}"
      f"   ({2 * M * H * H / tm / 1e6:.1f} TFLOP/s)")
