"""Stage timeline of gemm_x6_wgrad_kernel from a DR_WG_STAMPS=1 build
(s_memtime = shader clock), blocks 0-7, waves 0-7, stages 0-23:
  reads  = loop top -> the second k16 step's 24 transposed reads issued
  mfma0  = k16 step 0's 24 MFMAs (and the wait for their fragments)
  split  = the next stage's split + plane writes
  bar    = lgkmcnt(0) + barrier + the next stage's first-step reads issued
  mfma1  = k16 step 1's 24 MFMAs + the loads of stage g + 2
Usage: python scripts/micro/wg_stamps.py path/to/lib.so"""
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
L.dr_x6_diag_wg_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
M, C = 65536, 64
g = torch.Generator().manual_seed(0)
H = torch.tanh(torch.randn(2, M, 256, generator=g)).cuda()
G = (torch.randn(2, M, 256, generator=g) * 1e-3).cuda()
ws = torch.empty(2, C, 256, 256, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(20):
    assert L.dr_gemm_x6_wgrad(2, M, C, G.data_ptr(), H.data_ptr(), ws.data_ptr(), s) == 0
torch.cuda.synchronize()
buf = np.zeros(8 * 8 * 24 * 8, np.uint64)
assert L.dr_x6_diag_wg_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(8, 8, 24, 8).astype(np.int64)
R = 24
d = {"reads": st[..., 1] - st[..., 0], "mfma0": st[..., 2] - st[..., 1],
     "split": st[..., 3] - st[..., 2], "bar": st[..., 4] - st[..., 3],
     "mfma1": st[..., 5] - st[..., 4]}
for k, v in d.items():
    v = v[:, :, 1:R]
    print(f"{k:6s} median {np.median(v):6.0f}  p10 {np.percentile(v, 10):6.0f}  "
          f"p90 {np.percentile(v, 90):6.0f}  waves 0-3 {np.median(v[:, :4]):6.0f}  "
          f"waves 4-7 {np.median(v[:, 4:]):6.0f}")
step = st[:, :, 2:R, 0] - st[:, :, 1:R - 1, 0]
print(f"stage (loop top -> next loop top) median {np.median(step):.0f}; "
      f"MFMA per SIMD 96 x 32 = 3072")
