"""dr_gemm_x6: the 256 x 256 layer GEMM on the bf16 matrix cores with an exact
three-plane split of every f32 operand (csrc/gemm_x6.hip).

The reference computes this layer with torch fp32 (SB3 MlpExtractor,
/root/reference/train.py:36-43).  The bar here is accuracy against an f64
GEMM of the same f32 inputs: the x6 result must be at least as close to it
as torch's own fp32 GEMM (relative to sum_k |a_k b_k|, the scale every fp32
dot product's rounding error is bounded by), for both operand forms the
trainer uses (z = h W^T and grad_h = grad_z W), at the trainer's 65,536-row
minibatch and at the smallest legal size.  It is also deterministic."""
import pytest
import torch

from drone_rl_amd import _lib
from drone_rl_amd._lib import check, ptr

pytestmark = pytest.mark.gpu


def _run(A, W, transpose):
    L = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    img = torch.empty(L.dr_gemm_x6_weights_bytes(W.shape[0]), dtype=torch.uint8, device="cuda")
    C = torch.empty(A.shape[0], A.shape[1], 256, device="cuda")
    check(L.dr_gemm_x6_split_weights(W.shape[0], ptr(W), transpose, ptr(img), s))
    check(L.dr_gemm_x6(A.shape[0], A.shape[1], ptr(A), ptr(img), ptr(C), s))
    return C


def _errors(C, A, Wt, rows):
    ref = torch.bmm(A[:, :rows].double(), Wt.double())
    den = torch.bmm(A[:, :rows].abs().double(), Wt.abs().double()).clamp_min(1e-30)
    r32 = torch.bmm(A[:, :rows], Wt)
    e6 = ((C[:, :rows].double() - ref).abs() / den).max().item()
    e32 = ((r32.double() - ref).abs() / den).max().item()
    return e6, e32


@pytest.mark.parametrize("m", [128, 65536])
@pytest.mark.parametrize("transpose", [0, 1])
def test_gemm_x6_as_accurate_as_fp32(m, transpose):
    g = torch.Generator().manual_seed(m + transpose)
    A = torch.tanh(torch.randn(2, m, 256, generator=g)).cuda()
    W = (torch.randn(2, 256, 256, generator=g) * (2 / 256) ** 0.5).cuda()
    C = _run(A, W, transpose)
    Wt = W if transpose else W.transpose(1, 2)
    e6, e32 = _errors(C, A, Wt, min(m, 4096))
    assert e6 <= e32, (e6, e32)
    assert e6 < 4e-7
    # the tail rows too (the last tile of the second net)
    e6t, _ = _errors(C[:, -128:], A[:, -128:], Wt, 128)
    assert e6t < 4e-7


def test_gemm_x6_small_gradients_and_determinism():
    """grad_z-like operands (|x| ~ 1e-6 .. 1e-3, many exact zeros): the
    split keeps them exact (no bf16 underflow at these scales)."""
    g = torch.Generator().manual_seed(7)
    m = 8192
    A = torch.randn(2, m, 256, generator=g) * 10 ** (-3 - 3 * torch.rand(2, m, 256, generator=g))
    A[:, ::3] = 0.0
    A = A.cuda()
    W = (torch.randn(2, 256, 256, generator=g) * 0.06).cuda()
    C1 = _run(A, W, 1)
    C2 = _run(A, W, 1)
    assert torch.equal(C1, C2)
    e6, e32 = _errors(C1, A, W, 2048)
    assert e6 <= e32, (e6, e32)
    assert torch.all(C1[:, ::3] == 0)


def test_gemm_x6_one_net_and_bad_arguments():
    L = _lib.lib()
    g = torch.Generator().manual_seed(3)
    A = torch.randn(1, 256, 256, generator=g).cuda()
    W = torch.randn(1, 256, 256, generator=g).cuda()
    C = _run(A, W, 0)
    e6, e32 = _errors(C, A, W.transpose(1, 2), 256)
    assert e6 <= e32
    s = torch.cuda.current_stream().cuda_stream
    assert L.dr_gemm_x6(2, 100, ptr(A), ptr(W), ptr(C), s) == _lib.DR_ERR_INVALID
    assert L.dr_gemm_x6(3, 128, ptr(A), ptr(W), ptr(C), s) == _lib.DR_ERR_INVALID


@pytest.mark.parametrize("m,chunks", [(65536, 64), (3072, 4), (64, 2)])
def test_gemm_x6_wgrad_as_accurate_as_fp32(m, chunks):
    """The weight-gradient form: ws[b][c] = G[b, chunk c]^T H[b, chunk c]
    (torch's split-K bmm layout), against f64, relative to sum|g h|."""
    L = _lib.lib()
    g = torch.Generator().manual_seed(m)
    G = (torch.randn(2, m, 256, generator=g) * 1e-3).cuda()
    H = torch.tanh(torch.randn(2, m, 256, generator=g)).cuda()
    ws = torch.empty(2, chunks, 256, 256, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    check(L.dr_gemm_x6_wgrad(2, m, chunks, ptr(G), ptr(H), ptr(ws), s))
    rows = m // chunks
    for c in (0, chunks - 1):
        Gc, Hc = G[:, c * rows:(c + 1) * rows], H[:, c * rows:(c + 1) * rows]
        ref = torch.bmm(Gc.transpose(1, 2).double(), Hc.double())
        den = torch.bmm(Gc.transpose(1, 2).abs().double(), Hc.abs().double())
        r32 = torch.bmm(Gc.transpose(1, 2), Hc)
        e6 = ((ws[:, c].double() - ref).abs() / den).max().item()
        e32 = ((r32.double() - ref).abs() / den).max().item()
        assert e6 <= e32, (c, e6, e32)
        assert e6 < 4e-7
    ws2 = torch.empty_like(ws)
    check(L.dr_gemm_x6_wgrad(2, m, chunks, ptr(G), ptr(H), ptr(ws2), s))
    assert torch.equal(ws, ws2)
    assert L.dr_gemm_x6_wgrad(2, m, 3 * chunks + 1, ptr(G), ptr(H), ptr(ws), s) == \
        _lib.DR_ERR_INVALID


# SHA-256 of tests/x6_forms_worker.py's output bytes for its fixed seeds
X6_DIGESTS = {
    (384, 1): "325fc35bc39af98b2ba6429ed94eb0379783bd37ac24d8a2d19e96231638e9f3",
    (65536, 64): "3a877cae05c659cc815a03337c72a07e77df92d53b25ef4d0da837b55a57f1d1",
}


@pytest.mark.parametrize("m,chunks", [(128 * 3, 1), (65536, 64)])
def test_x6_outputs_are_the_same_bytes_in_two_processes(m, chunks):
    """dr_gemm_x6 (both image forms) and dr_gemm_x6_wgrad on fixed seeded
    inputs give the same bytes in two fresh processes (deterministic: fixed
    block -> row and chunk assignment, no atomics)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    digests = []
    for _ in range(2):
        env = dict(os.environ, PYTHONPATH=root)
        r = subprocess.run([sys.executable, os.path.join(root, "tests", "x6_forms_worker.py"),
                            str(m), str(chunks)], env=env, capture_output=True, text=True,
                           timeout=100)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        digests.append([l for l in r.stdout.splitlines() if l.startswith("sha")][0])
    assert digests[0] == digests[1], digests
    # pinned bytes (advisor r04): any edit claiming "bitwise the same" is
    # checked against these (re-pinned in round 6 for the 16x16x32 kernels,
    # after the accuracy and flagship parity tests passed on them:
    # gpurun_out r6e)
    assert digests[0] == "sha " + X6_DIGESTS[(m, chunks)], digests[0]
