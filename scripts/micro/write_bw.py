"""Write-only and copy HBM bandwidth of simple torch kernels (128 MB
buffers, the size of the PPO first-layer activations)."""
import torch

n = 32 * 1024 * 1024          # 128 MB of f32
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")


def t(f, it=50):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e-3


s = t(lambda: a.fill_(1.0))
print(f"fill 128 MB: {s * 1e6:.1f} us = {4 * n / s / 1e12:.2f} TB/s", flush=True)
s = t(lambda: b.copy_(a))
print(f"copy 128 MB: {s * 1e6:.1f} us = {8 * n / s / 1e12:.2f} TB/s (r+w)", flush=True)
s = t(lambda: a.sum())
print(f"sum 128 MB: {s * 1e6:.1f} us = {4 * n / s / 1e12:.2f} TB/s", flush=True)
