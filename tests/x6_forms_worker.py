"""Subprocess body of
tests/test_gemm_x6_gpu.py::test_x6_outputs_are_the_same_bytes_in_two_processes:
dr_gemm_x6 (both transposes) and dr_gemm_x6_wgrad on fixed seeded inputs;
prints the SHA-256 of the raw output bytes.  argv: m chunks."""
import hashlib
import sys

import torch

from drone_rl_amd import _lib
from drone_rl_amd._lib import check, ptr


def main():
    m, chunks = int(sys.argv[1]), int(sys.argv[2])
    L = _lib.lib()
    g = torch.Generator().manual_seed(123)
    A = torch.tanh(torch.randn(2, m, 256, generator=g)).cuda()
    W = (torch.randn(2, 256, 256, generator=g) * 0.06).cuda()
    Gr = (torch.randn(2, m, 256, generator=g) * 1e-3).cuda()
    img = torch.empty(L.dr_gemm_x6_weights_bytes(2), dtype=torch.uint8, device="cuda")
    C = torch.empty(2, m, 256, device="cuda")
    ws = torch.empty(2, chunks, 256, 256, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    h = hashlib.sha256()
    for tr in (0, 1):
        check(L.dr_gemm_x6_split_weights(2, ptr(W), tr, ptr(img), s))
        check(L.dr_gemm_x6(2, m, ptr(A), ptr(img), ptr(C), s))
        torch.cuda.synchronize()
        h.update(C.cpu().numpy().tobytes())
    check(L.dr_gemm_x6_wgrad(2, m, chunks, ptr(Gr), ptr(A), ptr(ws), s))
    torch.cuda.synchronize()
    h.update(ws.cpu().numpy().tobytes())
    print("sha", h.hexdigest())


if __name__ == "__main__":
    main()
