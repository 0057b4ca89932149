"""A/B of the 256x256 hidden-layer forward GEMM of both MLPs at M = 65,536:
two addmm (bias in the GEMM) vs one batched bmm without bias (bias added by
the consumer).  TunableOp tuning on (writes gpurun_out/tune_fwd/*.csv)."""
import os
import sys

import torch
import torch.cuda.tunable as tun

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tune_fwd"
os.makedirs(out, exist_ok=True)
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(os.path.join(out, "tunableop.csv"))
M, N = 65536, 256
x = torch.randn(2, M, N, device="cuda")
w = torch.randn(2, N, N, device="cuda") * 0.05
b = torch.randn(2, N, device="cuda")
y = torch.empty(2, M, N, device="cuda")


def two_addmm():
    for j in range(2):
        torch.addmm(b[j], x[j], w[j].t(), out=y[j])


def one_bmm():
    torch.bmm(x, w.transpose(1, 2), out=y)


def one_bmm_nt():
    torch.bmm(x, w, out=y)        # weights stored transposed (K, N)


for name, f in (("two_addmm", two_addmm), ("one_bmm", one_bmm), ("one_bmm_nt", one_bmm_nt)):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{name}: {us:.1f} us  ({2 * 2 * M * N * N / us / 1e6:.1f} TFLOP/s)", flush=True)
tun.write_file()
