"""Diagnostic: weight-gradient GEMM dW = g^T x over M=65536 rows (fp32),
torch default vs explicit split-K (bmm over C row chunks + sum)."""
import torch, time
torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"
M = 65536
def t(f, n=50):
    for _ in range(5): f()
    torch.cuda.synchronize(); a = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter() - a) / n * 1e6
for (N, K) in ((256, 256), (256, 15), (4, 256), (1, 256)):
    g = torch.randn(M, N, device=dev); x = torch.randn(M, K, device=dev)
    ref = g.t() @ x
    res = {"default": t(lambda: g.t() @ x)}
    for C in (16, 32, 64, 128, 256):
        f = lambda C=C: torch.bmm(g.view(C, M // C, N).transpose(1, 2), x.view(C, M // C, K)).sum(0)
        out = f()
        err = (out - ref).abs().max().item() / ref.abs().max().item()
        res[f"C{C}"] = round(t(f), 1)
        res[f"C{C}_err"] = f"{err:.1e}"
    # grad bias
    res["bias_sum"] = round(t(lambda: g.sum(0)), 1)
    res["bias_splitk"] = round(t(lambda: g.view(64, M // 64, N).sum(1).sum(0)), 1)
    print(N, K, {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}, flush=True)
# forward / input-grad GEMMs for reference
W = torch.randn(256, 256, device=dev); h = torch.randn(M, 256, device=dev); b = torch.randn(256, device=dev)
print("fwd addmm 65536x256x256", round(t(lambda: torch.addmm(b, h, W.t())), 1))
print("gx 65536x256x256", round(t(lambda: h @ W), 1))
print("tanh", round(t(lambda: torch.tanh(h)), 1))
