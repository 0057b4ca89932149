"""Split-K weight-gradient GEMM of both MLPs' 256x256 layer at M = 65,536:
batched bmm over 2C row chunks + the chunk sum, for C in (8, 16, 32, 64),
TunableOp tuning on (each shape tuned over hipBLASLt + rocBLAS)."""
import os
import sys

import torch
import torch.cuda.tunable as tun

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tune_wgrad"
os.makedirs(out, exist_ok=True)
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(os.path.join(out, "tunableop.csv"))
M, N, K = 65536, 256, 256
gz = torch.randn(2, M, N, device="cuda")
x = torch.randn(2, M, K, device="cuda")
res = torch.empty(2, N, K, device="cuda")
ref = torch.bmm(gz.transpose(1, 2).double(), x.double())


def timed(f, it=50):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for C in (8, 16, 32, 64):
    ws = torch.empty(2 * C, N, K, device="cuda")

    def gemm():
        torch.bmm(gz.reshape(2 * C, M // C, N).transpose(1, 2), x.reshape(2 * C, M // C, K),
                  out=ws)

    def both():
        gemm()
        torch.sum(ws.view(2, C, N, K), dim=1, out=res)

    tg, tb = timed(gemm), timed(both)
    err = (res.double() - ref).abs().max().item() / ref.abs().max().item()
    print(f"C={C}: gemm {tg:.1f} us, gemm+sum {tb:.1f} us, rel err {err:.2e}", flush=True)
tun.write_file()
