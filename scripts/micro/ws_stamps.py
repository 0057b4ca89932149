"""Row-step timeline of gemm_x6_ws_kernel from a DR_WS_STAMPS=1 build
(s_memtime = shader clock), blocks 0-7, waves 0-3, row steps 0-15:
  wait   = loop top -> staging of step k + 1 landed (vmcnt)
  mfma1  = phase 0 (column tile 0: 96 MFMAs, tile 1 stores, 4 split half-units)
  mfma2  = phase 1 (column tile 1: 96 MFMAs, tile 0 stores, 4 split half-units)
  epi    = epilogue (hi + lo, 32 stores)
  bar    = lgkmcnt(0) + barrier
Usage: python scripts/micro/ws_stamps.py path/to/lib.so"""
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
assert L.dr_gemm_x6_split_weights(2, W.data_ptr(), 0, img.data_ptr(), s) == 0
for _ in range(20):
    assert L.dr_gemm_x6(2, M, A.data_ptr(), img.data_ptr(), C.data_ptr(), s) == 0
torch.cuda.synchronize()
buf = np.zeros(8 * 4 * 24 * 8, np.uint64)
assert L.dr_x6_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(8, 4, 24, 8).astype(np.int64)
R = 16
pro = st[:, :, 23, 1] - st[:, :, 23, 0]
d = {"wait": st[:, :, :R, 1] - st[:, :, :R, 0], "mfma1": st[:, :, :R, 2] - st[:, :, :R, 1],
     "mfma2": st[:, :, :R, 3] - st[:, :, :R, 2], "epi": st[:, :, :R, 4] - st[:, :, :R, 3],
     "bar": st[:, :, :R, 5] - st[:, :, :R, 4]}
step = st[:, :, 1:R, 0] - st[:, :, :R - 1, 0]
tot = st[:, :, R - 1, 5] - st[:, :, 23, 0]
print(f"prologue (weights + rows 0,1 + split 0 + barrier): median {np.median(pro):.0f} cycles")
for k, v in d.items():
    print(f"{k:6s} median {np.median(v):6.0f}  p10 {np.percentile(v, 10):6.0f}  p90 {np.percentile(v, 90):6.0f}"
          f"   per step k (wave-median): {[int(x) for x in np.median(v.reshape(32, R), 0)]}")
print(f"row step (loop top -> next loop top) median {np.median(step):.0f}; MFMA-only 192 x 32 = 6144")
print(f"whole wave (kernel start -> last barrier) median {np.median(tot):.0f}")
# with the realtime stamps (23, 2) / (23, 3) (s_memrealtime, 100 MHz) and
# (23, 4) (s_memtime after the last row step): the shader clock and the
# waves' start / end spread in microseconds
rt0, rt1 = st[:, :, 23, 2], st[:, :, 23, 3]
if rt0.min() > 0 and rt1.min() > 0:
    loop = st[:, :, 23, 4] - st[:, :, 23, 0]
    us = (rt1 - rt0) / 100.0
    print(f"wave lifetime {np.median(us):.2f} us median (s_memrealtime); shader clock "
          f"{np.median(loop / us) / 1e3:.3f} GHz; prologue {np.median(pro) / np.median(loop / us):.2f} us")
    print(f"wave starts spread {(rt0.max() - rt0.min()) / 100.0:.2f} us, ends spread "
          f"{(rt1.max() - rt1.min()) / 100.0:.2f} us (blocks 0-7)")
