"""Diagnostic: two per-net GEMMs vs one batched (2-net) GEMM for the
256x256 layer at M = 65,536 (fwd addmm, grad-input mm, split-K weight grad)."""
import torch

M, H = 65536, 256
dev = "cuda"
x = torch.randn(2, M, H, device=dev)
w = torch.randn(2, H, H, device=dev)
b = torch.randn(2, 1, H, device=dev)
out = torch.empty(2, M, H, device=dev)


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


def fwd2():
    for k in range(2):
        torch.addmm(b[k, 0], x[k], w[k].t(), out=out[k])


def fwdb():
    torch.baddbmm(b, x, w.transpose(1, 2), out=out)


def gi2():
    for k in range(2):
        torch.mm(x[k], w[k], out=out[k])


def gib():
    torch.bmm(x, w, out=out)


for C in (32, 64, 128):
    ws = torch.empty(2 * C, H, H, device=dev)
    gw = torch.empty(2, H, H, device=dev)

    def wg2():
        for k in range(2):
            torch.bmm(x[k].reshape(C, M // C, H).transpose(1, 2), x[k].reshape(C, M // C, H),
                      out=ws[k * C:(k + 1) * C])
            torch.sum(ws[k * C:(k + 1) * C], dim=0, out=gw[k])

    def wgb():
        torch.bmm(x.reshape(2 * C, M // C, H).transpose(1, 2), x.reshape(2 * C, M // C, H), out=ws)
        torch.sum(ws.view(2, C, H, H), dim=1, out=gw)
    print(f"wgrad C={C}: two {t(wg2):.1f} us  batched {t(wgb):.1f} us")
print(f"fwd addmm: two {t(fwd2):.1f} us  batched baddbmm {t(fwdb):.1f} us")
print(f"grad-input mm: two {t(gi2):.1f} us  batched bmm {t(gib):.1f} us")
