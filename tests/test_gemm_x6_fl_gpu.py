"""dr_gemm_x6_bwd_first (round 5): the 256 x 256 layer's input gradient with
the first layer's backward fused into its epilogue (csrc/gemm_x6.hip
gemm_x6_fl16_kernel).  Checked against an f64 reference of the same math --
grad_z1 = (grad_z2 W1) (1 - h1^2), dW0 = grad_z1^T x, db0 = sum grad_z1 --
within the fp32 reduction-order bound the flagship PPO parity test uses
(Higham gamma_n sum |terms|), next to the unfused path (dr_gemm_x6 +
dr_first_layer_backward2) held to the same bound; and the X-planes image
is checked to be an exact three-plane split."""
import numpy as np
import pytest
import torch

from drone_rl_amd import _lib
from drone_rl_amd._lib import check, ptr

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


def _align(x):
    return (x + 255) & ~255


def _level1_total(ws, m, nets=2, k=15, n=256):
    """Sum over the ng level-1 groups the first-layer workspace holds (the
    dr_first_layer_backward2(defer = 1) layout) -> (dW (nets, n, k), db
    (nets, n)) in f64."""
    nb = min(-(-m // 16), 256)
    P = nets * (k + 1) * n
    gsize = -(-nb // 16)
    ng = -(-nb // gsize)
    off = _align(4 * nb * P) // 4
    part2 = ws.view(torch.float32)[off:off + ng * P].double().cpu().view(ng, nets, k + 1, n)
    tot = part2.sum(0)
    return tot[:, :k, :].transpose(1, 2).numpy(), tot[:, k, :].numpy()


def _bf16_to_f64(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


@pytest.mark.parametrize("m", [128, 384, 65536])
def test_split_x_is_an_exact_three_plane_split(m):
    """The observation image of the fused kernel (x6_split.h split_x_item):
    per 32-row step three planes of 64 lanes x 8 bf16, lane f + 16 q holding
    feature f (15: the constant 1) of rows 4 q + e (e < 4) and 16 + 4 q + e - 4
    (e >= 4); the planes sum exactly to x."""
    L = _lib.lib()
    g = torch.Generator().manual_seed(m)
    x = (torch.randn(m, 15, generator=g) * torch.exp(torch.randn(m, 15, generator=g) * 3)).cuda()
    img = torch.empty(L.dr_gemm_x6_x_bytes(m), dtype=torch.uint8, device="cuda")
    check(L.dr_gemm_x6_split_x(m, 15, ptr(x), ptr(img), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    rec = img.cpu().numpy().reshape(m // 32, -1)
    assert rec.shape[1] == 3072
    planes = rec.view(np.uint16).reshape(m // 32, 3, 4, 16, 8)       # p, q, f, e
    val = sum(_bf16_to_f64(planes[:, p]) for p in range(3))           # (g, q, f, e)
    e = np.arange(8)
    rows = np.where(e[None, :] < 4, 4 * np.arange(4)[:, None] + e[None, :],
                    16 + 4 * np.arange(4)[:, None] + e[None, :] - 4)  # (q, e)
    xs = x.double().cpu().numpy().reshape(m // 32, 32, 15)
    ref = np.ones((m // 32, 4, 16, 8))
    for f in range(15):
        ref[:, :, f, :] = xs[:, rows, f]
    assert np.array_equal(val, ref)


@pytest.mark.parametrize("m", [128, 3072, 65536])
def test_bwd_first_matches_f64_within_fp32_bound(m):
    L = _lib.lib()
    g = torch.Generator().manual_seed(7 + m)
    gz = (torch.randn(2, m, 256, generator=g) * 1e-3).cuda()
    W = (torch.randn(2, 256, 256, generator=g) * 0.06).cuda()
    h = torch.tanh(torch.randn(2, m, 256, generator=g) * 1.5).cuda()
    x = (torch.randn(m, 15, generator=g) * 2).cuda()
    s = torch.cuda.current_stream().cuda_stream
    nb = L.dr_gemm_x6_weights_bytes(2)
    img = torch.empty(nb, dtype=torch.uint8, device="cuda")
    check(L.dr_gemm_x6_split_weights(2, ptr(W), 1, ptr(img), s))       # C = A W
    ximg = torch.empty(L.dr_gemm_x6_x_bytes(m), dtype=torch.uint8, device="cuda")
    check(L.dr_gemm_x6_split_x(m, 15, ptr(x), ptr(ximg), s))
    wsb = L.dr_first_layer_backward2_workspace_bytes(m, 15, 256)
    ws_f = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    check(L.dr_gemm_x6_bwd_first(2, m, 15, ptr(gz), ptr(img), ptr(h), ptr(ximg), ptr(ws_f), wsb,
                                 0, s))
    # the unfused path into a second workspace
    gh = torch.empty(2, m, 256, device="cuda")
    check(L.dr_gemm_x6(2, m, ptr(gz), ptr(img), ptr(gh), s))
    ws_u = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    dw = torch.zeros(2, 256, 15, device="cuda")
    db = torch.zeros(2, 256, device="cuda")
    check(L.dr_first_layer_backward2(m, 15, 256, ptr(x), None, ptr(gh[0]), ptr(h[0]), ptr(dw[0]),
                                     ptr(db[0]), ptr(gh[1]), ptr(h[1]), ptr(dw[1]), ptr(db[1]),
                                     1, ptr(ws_u), wsb, s))
    torch.cuda.synchronize()
    # f64 reference and the envelope sum |terms|
    gz64, W64, h64, x64 = (t.double().cpu() for t in (gz, W, h, x))
    gh64 = torch.bmm(gz64, W64)
    d64 = 1 - h64 * h64
    gz1 = gh64 * d64
    ref_w = torch.einsum("bmn,mk->bnk", gz1, x64).numpy()
    ref_b = gz1.sum(1).numpy()
    env1 = torch.bmm(gz64.abs(), W64.abs()) * d64.abs()
    env_w = torch.einsum("bmn,mk->bnk", env1, x64.abs()).numpy()
    env_b = env1.sum(1).numpy()
    n_chain = 256 + 3 + 1024 + 64      # dot product, elementwise, row sum, groups (generous)
    gam = n_chain * U / (1 - n_chain * U)
    # direct: the per-block rows at the workspace start
    ws_d = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    check(L.dr_gemm_x6_bwd_first(2, m, 15, ptr(gz), ptr(img), ptr(h), ptr(ximg), ptr(ws_d), wsb,
                                 1, s))
    torch.cuda.synchronize()
    rows = L.dr_gemm_x6_bwd_first_rows(m)
    assert 1 <= rows <= min(-(-m // 16), 256)
    P = 2 * 16 * 256
    drows = ws_d.view(torch.float32)[:rows * P].double().cpu().view(rows, 2, 16, 256).sum(0)
    direct = (drows[:, :15, :].transpose(1, 2).numpy(), drows[:, 15, :].numpy())
    for name, ws in (("fused", ws_f), ("unfused", ws_u), ("direct", None)):
        w_, b_ = _level1_total(ws, m) if ws is not None else direct
        ew = np.abs(w_ - ref_w) / np.maximum(env_w, 1e-30)
        eb = np.abs(b_ - ref_b) / np.maximum(env_b, 1e-30)
        assert ew.max() <= gam and eb.max() <= gam, (name, ew.max(), eb.max(), gam)
    # deterministic: a second run gives the same bytes
    ws_2 = torch.zeros_like(ws_f)
    check(L.dr_gemm_x6_bwd_first(2, m, 15, ptr(gz), ptr(img), ptr(h), ptr(ximg), ptr(ws_2), wsb,
                                 0, s))
    torch.cuda.synchronize()
    assert torch.equal(ws_f, ws_2)


def test_bwd_first_argument_errors():
    L = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    a = torch.zeros(2, 128, 256, device="cuda")
    ws = torch.zeros(L.dr_first_layer_backward2_workspace_bytes(128, 15, 256), dtype=torch.uint8,
                     device="cuda")
    img = torch.zeros(L.dr_gemm_x6_weights_bytes(2), dtype=torch.uint8, device="cuda")
    xi = torch.zeros(L.dr_gemm_x6_x_bytes(128), dtype=torch.uint8, device="cuda")
    assert L.dr_gemm_x6_bwd_first(2, 100, 15, ptr(a), ptr(img), ptr(a), ptr(xi), ptr(ws),
                                  ws.numel(), 0, s) == _lib.DR_ERR_INVALID
    assert L.dr_gemm_x6_bwd_first(2, 128, 15, ptr(a), ptr(img), ptr(a), ptr(xi), ptr(ws), 16,
                                  0, s) == _lib.DR_ERR_INVALID
    assert L.dr_gemm_x6_bwd_first_rows(100) == 0 and L.dr_gemm_x6_bwd_first_rows(128) >= 1
    assert L.dr_gemm_x6_split_x(128, 16, ptr(a), ptr(xi), s) == _lib.DR_ERR_INVALID


def test_trainer_step_fused_equals_unfused_within_bound(monkeypatch):
    """One FusedTrainStep on the deferred-finish path with the fused kernel
    (its rows summed by the finish directly, and through the grouping launch)
    and without it (DRONERL_X6_FL=0): the first-layer gradients agree, every
    other gradient entry is bitwise the same."""
    from drone_rl_amd import ppo_kernels as K
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    m = 8192
    grads = []
    for fl, direct in (("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("DRONERL_X6_FL", fl)
        monkeypatch.setenv("DRONERL_X6_FL_DIRECT", direct)
        pol = ActorCritic(15, 4, (256, 256), seed=3, device="cuda")
        fs = FusedTrainStep(pol, m)
        g = torch.Generator().manual_seed(11)
        obs = torch.randn(m, 15, generator=g).cuda()
        act = (torch.rand(m, 4, generator=g) * 7.0).cuda()
        aux = torch.randn(m, 3, generator=g).cuda()
        head = K.HeadLossBackward(m, 256, "cuda", 0.2, 0.0, 0.5, True)
        grad, stats = fs.step(obs, act, aux, head, defer_finish=True)
        opt = K.ClipAdam(pol.flat.detach(), lr=0.0, max_grad_norm=1e30)   # no clip
        opt.step_finish(grad, fs.finish)
        torch.cuda.synchronize()
        grads.append((grad.clone(), {k: fs.gview(k).clone() for k in
                                      ("pi0.w", "pi0.b", "vf0.w", "vf0.b")}))
    gu, first_u = grads[-1]
    lo = pol.offsets["pi1.w"][0]                 # the first layer's entries come first
    for gf, first_f in grads[:-1]:
        assert torch.equal(gf[lo:], gu[lo:])
        for k in first_f:
            a, b = first_f[k].double(), first_u[k].double()
            scale = b.abs().max().item() + 1e-30
            assert (a - b).abs().max().item() <= 1e-4 * scale, k


@pytest.mark.parametrize("m,with_rows", [(128, False), (65536, False), (4096, True)])
def test_linear_tanh2_x6_builds_the_same_images(m, with_rows):
    """dr_linear_tanh2_x6: h0 / h1 bitwise dr_linear_tanh2's, the weight
    images bitwise dr_gemm_x6_split_weights(transpose 2)'s and the
    observation image bitwise dr_gemm_x6_split_x's (of x[rows] with rows)."""
    L = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(m + int(with_rows))
    total = 3 * m if with_rows else m
    x = torch.randn(total, 15, generator=g).cuda()
    rows = (torch.randperm(total, generator=g)[:m].to(torch.int32).cuda() if with_rows
            else None)
    w0, w1 = (torch.randn(256, 15, generator=g).cuda() * 0.3 for _ in range(2))
    b0, b1 = (torch.randn(256, generator=g).cuda() * 0.1 for _ in range(2))
    w256 = (torch.randn(2, 256, 256, generator=g) * 0.06).cuda()
    h = [torch.empty(m, 256, device="cuda") for _ in range(4)]
    nb = L.dr_gemm_x6_weights_bytes(2)
    img_a = torch.zeros(2 * nb, dtype=torch.uint8, device="cuda")
    img_b = torch.zeros(2 * nb, dtype=torch.uint8, device="cuda")
    xi_a = torch.zeros(L.dr_gemm_x6_x_bytes(m), dtype=torch.uint8, device="cuda")
    xi_b = torch.zeros_like(xi_a)
    rp = ptr(rows)
    check(L.dr_linear_tanh2(m, 15, 256, ptr(x), rp, ptr(w0), ptr(b0), ptr(h[0]), ptr(w1),
                            ptr(b1), ptr(h[1]), s))
    check(L.dr_gemm_x6_split_weights(2, ptr(w256), 2, ptr(img_a), s))
    xg = x[rows.long()].contiguous() if with_rows else x
    check(L.dr_gemm_x6_split_x(m, 15, ptr(xg), ptr(xi_a), s))
    check(L.dr_linear_tanh2_x6(m, 15, 256, ptr(x), rp, ptr(w0), ptr(b0), ptr(h[2]), ptr(w1),
                               ptr(b1), ptr(h[3]), ptr(w256), ptr(img_b), ptr(xi_b), s))
    torch.cuda.synchronize()
    assert torch.equal(h[0], h[2]) and torch.equal(h[1], h[3])
    assert torch.equal(img_a, img_b)
    assert torch.equal(xi_a, xi_b)
    # without the observation image: the weight images alone
    img_c = torch.zeros_like(img_a)
    check(L.dr_linear_tanh2_x6(m, 15, 256, ptr(x), rp, ptr(w0), ptr(b0), ptr(h[2]), ptr(w1),
                               ptr(b1), ptr(h[3]), ptr(w256), ptr(img_c), None, s))
    torch.cuda.synchronize()
    assert torch.equal(img_a, img_c) and torch.equal(h[0], h[2])
    assert L.dr_linear_tanh2_x6(m, 16, 256, ptr(x), rp, ptr(w0), ptr(b0), ptr(h[2]), ptr(w1),
                                ptr(b1), ptr(h[3]), ptr(w256), ptr(img_c), None,
                                s) == _lib.DR_ERR_INVALID
