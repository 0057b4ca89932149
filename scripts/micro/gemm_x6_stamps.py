"""Per-stage timeline of gemm_x6_kernel from a DR_X6_STAMPS=1 build
(s_memtime, shader clock): for blocks 0-7, every wave, stages 0-63:
  a = MFMA step 0 issued (from stage start), b = wait + barrier,
  c = step-1 fragment reads issued + MFMA step 1 issued.
Usage: python scripts/micro/gemm_x6_stamps.py path/to/lib.so [pp]
pp: the ping-pong kernel's stamps (per k16 step u: 0 = start, 1 = first
interval's work done, 2 = after its barrier, 3 = second interval's work
done; group A = waves 0-3 prep then MFMA, group B = waves 4-7 MFMA then prep)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402

L = ctypes.CDLL(sys.argv[1])
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(L, name, None)
    if f is not None:
        f.restype, f.argtypes = res, args
L.dr_x6_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
M = 65536
g = torch.Generator().manual_seed(0)
A = torch.tanh(torch.randn(2, M, 256, generator=g)).cuda()
W = (torch.randn(2, 256, 256, generator=g) * 0.06).cuda()
img = torch.empty(L.dr_gemm_x6_weights_bytes(2), dtype=torch.uint8, device="cuda")
C = torch.empty(2, M, 256, device="cuda")
s = torch.cuda.current_stream().cuda_stream
assert L.dr_gemm_x6_split_weights(2, A.data_ptr() * 0 + W.data_ptr(), 0, img.data_ptr(), s) == 0
for _ in range(5):
    assert L.dr_gemm_x6(2, M, A.data_ptr(), img.data_ptr(), C.data_ptr(), s) == 0
torch.cuda.synchronize()
buf = np.zeros(8 * 8 * 64 * 4, np.uint64)
assert L.dr_x6_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(8, 8, 64, 4).astype(np.int64)
if len(sys.argv) > 2 and sys.argv[2] == "pp":
    U = 64
    w1 = st[..., 1] - st[..., 0]            # first interval's work
    b1 = st[..., 2] - st[..., 1]            # first barrier wait
    w2 = st[..., 3] - st[..., 2]            # second interval's work
    b2 = st[:, :, 1:, 0] - st[:, :, :-1, 3]  # second barrier wait (to the next step)
    for name, sl in (("A (prep | MFMA)", slice(0, 4)), ("B (MFMA | prep)", slice(4, 8))):
        print(f"group {name}: work1 {np.median(w1[:, sl, 2:]):.0f}  bar1 {np.median(b1[:, sl, 2:]):.0f}  "
              f"work2 {np.median(w2[:, sl, 2:]):.0f}  bar2 {np.median(b2[:, sl, 2:]):.0f}  "
              f"(p90 work1 {np.percentile(w1[:, sl, 2:], 90):.0f}, work2 {np.percentile(w2[:, sl, 2:], 90):.0f})")
    step = st[:, :, 1:, 0] - st[:, :, :-1, 0]
    print(f"cycles per k16 step (median): {np.median(step):.0f}; MFMA-only per SIMD per step: 1536")
    sys.exit(0)
G = 32
st = st[:, :, :G]
a = st[..., 1] - st[..., 0]
b = st[..., 2] - st[..., 1]
c = st[..., 3] - st[..., 2]
nxt = st[:, :, 1:, 0] - st[:, :, :-1, 3]
tot = st[:, :, -1, 3] - st[:, :, 0, 0]
print(f"cycles per stage (median over blocks 0-7, waves, stages): step0 {np.median(a):.0f}  "
      f"wait+barrier {np.median(b):.0f}  step1 {np.median(c):.0f}  stage->stage gap {np.median(nxt):.0f}")
print(f"p90: step0 {np.percentile(a, 90):.0f}  wait {np.percentile(b, 90):.0f}  step1 {np.percentile(c, 90):.0f}")
print(f"whole block (32 stages): median {np.median(tot):.0f} cycles; per stage {np.median(tot) / G:.0f}; "
      f"MFMA-only per stage per SIMD (2 waves x 48 x 32): 3072")
print("stage-0..3 wait per wave (block 0):", b[0, :, :4].tolist())
