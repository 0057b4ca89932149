"""Time dr_gemm_x6 (C = A W), dr_gemm_x6_split_x and dr_gemm_x6_bwd_first at
65,536 rows x 2 nets on the library DRONERL_LIB names (kernel variants built
by scripts/micro/build_variant.sh), with a digest of the first-layer
workspace so variants that change results show it.

  DRONERL_LIB=scripts/micro/build/lib_x.so python scripts/micro/fl_bench.py
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402
from drone_rl_amd._lib import check, ptr  # noqa: E402

REPS = int(os.environ.get("REPS", "50"))
L = _lib.lib()
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
M = 65536
gz = (torch.randn(2, M, 256, generator=g) * 1e-3).to(dev)
W = (torch.randn(2, 256, 256, generator=g) * 0.06).to(dev)
h = torch.tanh(torch.randn(2, M, 256, generator=g)).to(dev)
x = torch.randn(M, 15, generator=g).to(dev)
s = torch.cuda.current_stream().cuda_stream
img = torch.empty(L.dr_gemm_x6_weights_bytes(2), dtype=torch.uint8, device=dev)
check(L.dr_gemm_x6_split_weights(2, ptr(W), 1, ptr(img), s))
ximg = torch.empty(L.dr_gemm_x6_x_bytes(M), dtype=torch.uint8, device=dev)
wsb = L.dr_first_layer_backward2_workspace_bytes(M, 15, 256)
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
C = torch.empty(2, M, 256, device=dev)


def timed(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / REPS, 2)


out = {"lib": os.environ.get("DRONERL_LIB", "in-tree")}
out["gemm_x6_us"] = timed(lambda: check(L.dr_gemm_x6(2, M, ptr(gz), ptr(img), ptr(C), s)))
out["split_x_us"] = timed(lambda: check(L.dr_gemm_x6_split_x(M, 15, ptr(x), ptr(ximg), s)))
out["bwd_first_us"] = timed(lambda: check(L.dr_gemm_x6_bwd_first(
    2, M, 15, ptr(gz), ptr(img), ptr(h), ptr(ximg), ptr(ws), wsb, 0, s)))
torch.cuda.synchronize()
out["ws_digest"] = hashlib.sha256(ws.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps(out), flush=True)
