"""GPU checks of the PPO HIP kernels against the CPU restatement of SB3's
PPO arithmetic (oracle/ppo_ref.py, oracle/ppo_ref.c).  SB3 itself is not
available, so these are "parity unpinned" w.r.t. the reference; they pin the
kernels to the restatement: GAE bit-exact, Philox-derived streams bit-exact,
float loss/gradients within 1e-5 (f32 reduction-order differences)."""
import numpy as np
import pytest
import torch

from oracle import cref, ppo_ref

pytestmark = pytest.mark.gpu


def test_gae_bitexact_vs_oracle():
    from drone_rl_amd import ppo_kernels as K
    rng = np.random.default_rng(0)
    T, N = 32, 50_000
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    st = (rng.random((T, N)) < 0.05).astype(np.uint8)
    lv = rng.normal(size=N).astype(np.float32)
    ld = (rng.random(N) < 0.05).astype(np.uint8)
    cu = lambda x: torch.from_numpy(x).cuda()  # noqa: E731
    adv, ret = K.gae(cu(r), cu(v), cu(st), cu(lv), cu(ld), 0.99, 0.95)
    ra, rr = cref.gae(r, v, st, lv, ld, 0.99, 0.95)
    np.testing.assert_array_equal(adv.cpu().numpy(), ra)
    np.testing.assert_array_equal(ret.cpu().numpy(), rr)


def test_policy_sample_distribution_and_logp():
    from drone_rl_amd import ppo_kernels as K
    n = 1 << 20
    mean = torch.randn(n, 4, device="cuda")
    log_std = torch.tensor([0.0, -0.5, 0.3, -1.0], device="cuda")
    raw = torch.empty_like(mean)
    clip = torch.empty_like(mean)
    logp = torch.empty(n, device="cuda")
    K.policy_sample(mean, log_std, seed=5, counter=17, lo=0.0, hi=7.3575,
                    actions_raw=raw, actions_clipped=clip, logp=logp)
    z = (raw - mean) / log_std.exp()
    assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 1) < 5e-3
    assert abs(((z.abs() < 1).float().mean() - 0.6827).item()) < 3e-3
    d = torch.distributions.Normal(mean, log_std.exp())
    ref = d.log_prob(raw).sum(1)
    assert torch.allclose(logp, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(clip, raw.clamp(0.0, 7.3575))
    # same (seed, counter) -> same draws; different counter -> different
    raw2 = torch.empty_like(mean)
    K.policy_sample(mean, log_std, 5, 17, 0.0, 7.3575, actions_raw=raw2)
    assert torch.equal(raw, raw2)
    K.policy_sample(mean, log_std, 5, 18, 0.0, 7.3575, actions_raw=raw2)
    assert not torch.equal(raw, raw2)


def test_permutation_valid_and_matches_philox_sort():
    from drone_rl_amd import ppo_kernels as K
    n = 5000
    perm = K.Permuter(n, "cuda")(seed=9, counter=3).cpu().numpy()
    assert np.array_equal(np.sort(perm), np.arange(n))
    keys = np.zeros(n, np.uint64)
    for i in range(n):
        r = cref.philox([i, 0, 3, 0x50000000], [9, 0])
        keys[i] = (np.uint64(r[0]) << np.uint64(32)) | np.uint64(r[1])
    np.testing.assert_array_equal(perm, np.argsort(keys, kind="stable"))
    big = K.Permuter(1 << 21, "cuda")(seed=1, counter=0)
    assert torch.equal(torch.sort(big.long()).values,
                       torch.arange(1 << 21, device="cuda"))


@pytest.mark.parametrize("n", [1, 2, 1000, 1025, 4097, 70001, 1 << 21])
def test_permutation_is_the_stable_key_argsort(n):
    """Bucket pass + per-bucket bitonic sorts == the stable argsort of the
    64-bit Philox keys (oracle/cref.permutation_np), at ragged sizes and at
    configs[2]'s 32 x 65,536 rollout rows; bitwise deterministic."""
    from drone_rl_amd import ppo_kernels as K
    p = K.Permuter(n, "cuda")
    got = p(seed=0x1234567890, counter=(7 << 32) + 5).cpu().numpy()
    np.testing.assert_array_equal(got, cref.permutation_np(n, 0x1234567890, (7 << 32) + 5))
    again = p(seed=0x1234567890, counter=(7 << 32) + 5, out=torch.empty_like(p.out))
    assert np.array_equal(again.cpu().numpy(), got)


def test_permutation_global_scratch_path(monkeypatch):
    """Buckets above the LDS capacity sort in global scratch (forced here by
    DRONERL_PERM_LDS_CAP; unreachable in practice at a mean of <= 1024)."""
    from drone_rl_amd import ppo_kernels as K
    for cap in ("0", "700"):
        monkeypatch.setenv("DRONERL_PERM_LDS_CAP", cap)
        n = 9000
        got = K.Permuter(n, "cuda")(seed=3, counter=11).cpu().numpy()
        np.testing.assert_array_equal(got, cref.permutation_np(n, 3, 11))


def test_permutation_graph_replays_are_fresh():
    """The permutation captured into a hipGraph (counter base on the device)
    replays to the eager permutation of each new counter, at configs[2]'s
    2,097,152 rows and 10 epochs per graph (rocPRIM's radix sort faulted on
    the second replay of such a graph; the bucket sort keeps no state)."""
    from drone_rl_amd import ppo_kernels as K
    n, E = 1 << 21, 10
    p = K.Permuter(n, "cuda")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    outs = torch.zeros(E, n, dtype=torch.int32, device="cuda")

    def body():
        for e in range(E):
            p.dev(seed=7, counter_base=ctr, counter_offset=e, out=outs[e])
    body()
    torch.cuda.synchronize()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cs), torch.cuda.graph(g, stream=cs):
        body()
    torch.cuda.current_stream().wait_stream(cs)
    for it in range(3):
        ctr.fill_(it * E)
        g.replay()
        torch.cuda.synchronize()
        for e in (0, E - 1):
            ref = p(seed=7, counter=it * E + e, out=torch.empty_like(p.out))
            assert torch.equal(ref, outs[e]), (it, e)


def test_gather_rows_exact():
    from drone_rl_amd import ppo_kernels as K
    src = torch.randn(100_000, 15, device="cuda")
    idx = torch.randint(0, 100_000, (4096,), device="cuda", dtype=torch.int32)
    assert torch.equal(K.gather_rows(idx, src), src[idx.long()])


@pytest.mark.parametrize("normalize", [True, False])
def test_ppo_loss_vs_torch_autograd(normalize):
    from drone_rl_amd import ppo_kernels as K
    rng = np.random.default_rng(1)
    m = 65536
    mean = rng.normal(2.0, 1.0, (m, 4)).astype(np.float32)
    log_std = np.array([0.1, -0.3, 0.0, 0.2], np.float32)
    actions = (mean + np.exp(log_std) * rng.normal(size=(m, 4))).astype(np.float32)
    old_logp = (rng.normal(-5.0, 1.0, m)).astype(np.float32)
    # make the ratio land on both sides of the clip interval
    d = torch.distributions.Normal(torch.from_numpy(mean), torch.from_numpy(np.exp(log_std)))
    lp = d.log_prob(torch.from_numpy(actions)).sum(1).numpy()
    old_logp = (lp - rng.normal(0, 0.2, m)).astype(np.float32)
    adv = rng.normal(0.3, 2.0, m).astype(np.float32)
    returns = rng.normal(size=m).astype(np.float32)
    values = rng.normal(size=m).astype(np.float32)
    stats, gm, gls, gv = ppo_ref.ppo_loss_torch(mean, log_std, values, actions, old_logp,
                                                adv, returns, 0.2, 0.01, 0.5, normalize)
    L = K.PPOLoss(m, "cuda", 0.2, 0.01, 0.5, normalize)
    cu = lambda x: torch.from_numpy(x).cuda()  # noqa: E731
    g_mean, g_ls, g_v, st = L(cu(mean), cu(log_std), cu(values), cu(actions), cu(old_logp),
                              cu(adv), cu(returns))
    st = st.cpu().numpy()
    names = ["loss", "policy_loss", "value_loss", "entropy_loss", "clip_fraction", "approx_kl"]
    for k, name in enumerate(names):
        assert abs(st[k] - stats[name]) <= 1e-5 * max(1.0, abs(stats[name])), name
    assert 0.05 < stats["clip_fraction"] < 0.95
    scale = np.abs(gm).max()
    np.testing.assert_allclose(g_mean.cpu().numpy(), gm, rtol=0, atol=1e-4 * scale)
    np.testing.assert_allclose(g_v.cpu().numpy(), gv, rtol=0, atol=1e-6)
    np.testing.assert_allclose(g_ls.cpu().numpy(), gls, rtol=1e-4, atol=1e-5)
    # the interleaved (m,3) aux form (the trainer's gathered rollout rows)
    # reads the same numbers: identical outputs
    keep = [t.clone() for t in (g_mean, g_ls, g_v, L.stats)]
    aux = cu(np.stack([old_logp, adv, returns], 1).copy())
    out = L(cu(mean), cu(log_std), cu(values), cu(actions), aux=aux)
    for a, b in zip(keep, out):
        assert torch.equal(a, b)


def test_clip_adam_vs_torch():
    from drone_rl_amd import ppo_kernels as K
    rng = np.random.default_rng(2)
    n = 141_065
    p = rng.normal(size=n).astype(np.float32)
    for gscale, step in ((10.0, 1), (1e-4, 7)):   # clipped, and not clipped
        g = (rng.normal(size=n) * gscale / np.sqrt(n)).astype(np.float32)
        m = (rng.normal(size=n) * 1e-3).astype(np.float32)
        v = (rng.random(n) * 1e-6).astype(np.float32)
        rp, rm, rv, rg, rnorm = ppo_ref.clip_adam_torch(p, g, m, v, step)
        opt = K.ClipAdam(torch.from_numpy(p.copy()).cuda())
        opt.m.copy_(torch.from_numpy(m))
        opt.v.copy_(torch.from_numpy(v))
        opt.t = step - 1
        gd = torch.from_numpy(g.copy()).cuda()
        norm = opt.step(gd).item()
        assert abs(norm - rnorm) <= 1e-5 * rnorm
        # f32 norms summed in a different order -> clip coefficients agree to
        # ~1e-6 relative; element tolerances are relative to each array's scale
        def close(a, b, rel):
            np.testing.assert_allclose(a, b, rtol=rel, atol=rel * np.abs(b).max())
        close(gd.cpu().numpy(), rg, 1e-5)
        close(opt.m.cpu().numpy(), rm, 1e-5)
        close(opt.v.cpu().numpy(), rv, 1e-5)
        close(opt.p.cpu().numpy() - p, rp - p, 1e-4)   # the update itself
        np.testing.assert_allclose(opt.p.cpu().numpy(), rp, rtol=1e-6, atol=1e-7)


def test_tanh_backward_fused_bias_grad():
    from drone_rl_amd import ppo_kernels as K
    for m, n in ((65536, 256), (1000, 64), (777, 12)):
        h = torch.tanh(torch.randn(m, n, device="cuda"))
        g = torch.randn(m, n, device="cuda")
        gz = torch.empty_like(h)
        gb = torch.empty(n, device="cuda")
        ws = torch.empty(K.tanh_backward_workspace_bytes(m, n) // 4 + 1, device="cuda")
        K.tanh_backward(g, h, gz, gb, ws)
        ref = g * (1 - h * h)
        assert torch.allclose(gz, ref, rtol=0, atol=0)
        assert torch.allclose(gb, ref.sum(0), rtol=1e-4, atol=1e-3)


def test_fused_train_step_matches_autograd():
    """The hand-written backward (fused tanh/bias kernel, split-K weight
    gradients) equals torch autograd through the same MLP."""
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    torch.manual_seed(0)
    pol = ActorCritic(15, 4, (256, 256), device="cuda", seed=3)
    m = 65536
    obs = torch.randn(m, 15, device="cuda")
    g_mean = torch.randn(m, 4, device="cuda") * 1e-3
    g_v = torch.randn(m, device="cuda") * 1e-3
    g_ls = torch.randn(4, device="cuda")
    fs = FusedTrainStep(pol, m)
    mean, value, cache = fs.forward(obs)
    grad = fs.backward(obs, cache, g_mean, g_v, g_ls).clone()
    pol.flat.grad = None
    mean2, value2 = pol(obs)
    assert torch.allclose(mean, mean2, atol=1e-5) and torch.allclose(value, value2, atol=1e-5)
    torch.autograd.backward([mean2, value2], [g_mean, g_v])
    ref = pol.flat.grad.clone()
    a, b, _ = pol.offsets["log_std"]
    ref[a:b] = g_ls
    for name, _, _ in pol.layout:
        lo, hi, _ = pol.offsets[name]
        scale = ref[lo:hi].abs().max().item() + 1e-12
        assert (grad[lo:hi] - ref[lo:hi]).abs().max().item() <= 1e-4 * scale, name


@pytest.mark.parametrize("k,n", [(15, 256), (12, 64), (18, 128)])
def test_linear_tanh_matches_torch(k, n):
    from drone_rl_amd import ppo_kernels as K
    m = 5001
    x = torch.randn(m, k, device="cuda")
    w = torch.randn(n, k, device="cuda") * 0.4
    b = torch.randn(n, device="cuda") * 0.1
    h = torch.empty(m, n, device="cuda")
    K.linear_tanh(x, w, b, h)
    ref = torch.tanh(torch.addmm(b, x, w.t()))
    assert (h - ref).abs().max().item() <= 2e-6


def test_policy_heads_match_torch():
    from drone_rl_amd import ppo_kernels as K
    m, hd = 3001, 256
    hp = torch.tanh(torch.randn(m, hd, device="cuda"))
    hv = torch.tanh(torch.randn(m, hd, device="cuda"))
    wa, ba = torch.randn(4, hd, device="cuda") * 0.1, torch.randn(4, device="cuda")
    wv, bv = torch.randn(1, hd, device="cuda") * 0.1, torch.randn(1, device="cuda")
    mean = torch.empty(m, 4, device="cuda")
    value = torch.empty(m, device="cuda")
    K.policy_heads(hp, hv, wa, ba, wv, bv, mean, value)
    assert (mean - torch.addmm(ba, hp, wa.t())).abs().max().item() <= 1e-5
    assert (value - torch.addmm(bv, hv, wv.t()).squeeze(1)).abs().max().item() <= 1e-5
    # pre-activation inputs: the layer's tanh is applied on load
    z = torch.randn(m, hd, device="cuda") * 2
    K.policy_heads(z, z, wa, ba, wv, bv, mean, value, preact=True)
    t = torch.tanh(z)
    assert (mean - torch.addmm(ba, t, wa.t())).abs().max().item() <= 1e-5
    assert (value - torch.addmm(bv, t, wv.t()).squeeze(1)).abs().max().item() <= 1e-5
    # top-layer biases added on load (the batched top GEMM leaves them out)
    zp, zv = torch.randn(hd, device="cuda"), torch.randn(hd, device="cuda")
    K.policy_heads(z, z, wa, ba, wv, bv, mean, value, preact=True, zb_pi=zp, zb_vf=zv)
    tp, tv = torch.tanh(z + zp), torch.tanh(z + zv)
    assert (mean - torch.addmm(ba, tp, wa.t())).abs().max().item() <= 1e-5
    assert (value - torch.addmm(bv, tv, wv.t()).squeeze(1)).abs().max().item() <= 1e-5


@pytest.mark.parametrize("arch,m", [((256, 256), 65536), ((64, 64), 64), ((64, 128), 1000)])
def test_fused_step_matches_unfused_path(arch, m):
    """FusedTrainStep.step (first-layer linear+tanh kernel, heads + loss +
    head backward kernel) == forward -> dr_ppo_loss -> hand backward, to f32
    summation-order noise; two runs are bitwise identical."""
    from drone_rl_amd import ppo_kernels as K
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    torch.manual_seed(1)
    pol = ActorCritic(15, 4, arch, device="cuda", seed=4)
    with torch.no_grad():
        pol.flat.mul_(3.0)              # non-trivial heads / log_std
    obs = torch.randn(m, 15, device="cuda")
    fs = FusedTrainStep(pol, m)
    with torch.no_grad():
        mean, value, cache = fs.forward(obs)
        d = torch.distributions.Normal(mean, pol.log_std.exp())
        act = d.sample()
        aux = torch.stack([d.log_prob(act).sum(1) + 0.1 * torch.randn(m, device="cuda"),
                           torch.randn(m, device="cuda"), torch.randn(m, device="cuda")], 1)
    L = K.PPOLoss(m, "cuda", 0.2, 0.01, 0.5, True)
    g_mean, g_ls, g_v, st = L(mean, pol.log_std.detach(), value, act, aux=aux)
    ref = fs.backward(obs, cache, g_mean, g_v, g_ls).clone()
    st_ref = st.clone()
    head = K.HeadLossBackward(m, arch[-1], "cuda", 0.2, 0.01, 0.5, True)
    grad, st2 = fs.step(obs, act, aux, head)
    grad = grad.clone()
    for name, _, _ in pol.layout:
        lo, hi, _ = pol.offsets[name]
        scale = ref[lo:hi].abs().max().item() + 1e-12
        # + an absolute floor for sums that cancel (e.g. the value bias: 65k
        # terms of ~3e-5 summing to ~2e-5 in a different order)
        assert (grad[lo:hi] - ref[lo:hi]).abs().max().item() <= 2e-4 * scale + 1e-7, name
    assert torch.allclose(st2, st_ref, rtol=1e-4, atol=1e-6)
    grad2, _ = fs.step(obs, act, aux, head)
    assert torch.equal(grad, grad2)


@pytest.mark.parametrize("k,n,m", [(15, 256, 65536), (12, 64, 1001), (18, 128, 77)])
def test_first_layer_backward_matches_torch(k, n, m):
    from drone_rl_amd import ppo_kernels as K
    x = torch.randn(m, k, device="cuda")
    h = torch.tanh(torch.randn(m, n, device="cuda"))
    g = torch.randn(m, n, device="cuda")
    gw = torch.empty(n, k, device="cuda")
    gb = torch.empty(n, device="cuda")
    K.FirstLayerBackward(m, k, n, "cuda")(g, h, x, gw, gb)
    gz = (g.double() * (1 - h.double() ** 2))
    ref_w = gz.t() @ x.double()
    ref_b = gz.sum(0)
    tol = 1e-5 * (gz.abs().t() @ x.double().abs()).max().item()
    assert (gw.double() - ref_w).abs().max().item() <= tol
    assert (gb.double() - ref_b).abs().max().item() <= 1e-5 * gz.abs().sum(0).max().item()


def test_fused_step_rows_in_place_equals_gathered():
    """Reading the minibatch through the permutation (rows=) inside the
    kernels is bitwise the same as gathering it first."""
    from drone_rl_amd import ppo_kernels as K
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    torch.manual_seed(2)
    pol = ActorCritic(15, 4, (256, 256), device="cuda", seed=5)
    total, m = 3 * 4096, 4096
    obs = torch.randn(total, 15, device="cuda")
    act = torch.rand(total, 4, device="cuda") * 7.3575
    aux = torch.randn(total, 3, device="cuda")
    rows = torch.randperm(total, device="cuda")[:m].to(torch.int32)
    fs = FusedTrainStep(pol, m)
    head = K.HeadLossBackward(m, 256, "cuda")
    g1, s1 = fs.step(obs, act, aux, head, rows=rows)
    g1, s1 = g1.clone(), s1.clone()
    r = rows.long()
    g2, s2 = fs.step(obs[r].contiguous(), act[r].contiguous(), aux[r].contiguous(), head)
    assert torch.equal(g1, g2) and torch.equal(s1, s2)


@pytest.mark.parametrize("k,n,m", [(15, 256, 65536), (18, 128, 1001), (12, 64, 77)])
def test_paired_first_layer_kernels_equal_single(k, n, m):
    """dr_linear_tanh2 / dr_first_layer_backward2 (both MLPs in one launch)
    are bitwise the single-net kernels, with and without rows=."""
    from drone_rl_amd import ppo_kernels as K
    g = torch.Generator(device="cuda").manual_seed(k * n + m)
    total = m + 13
    x = torch.randn(total, k, device="cuda", generator=g)
    rows = torch.randperm(total, device="cuda", generator=g)[:m].to(torch.int32)
    w = [torch.randn(n, k, device="cuda", generator=g) * 0.4 for _ in range(2)]
    b = [torch.randn(n, device="cuda", generator=g) * 0.1 for _ in range(2)]
    gh = [torch.randn(m, n, device="cuda", generator=g) for _ in range(2)]
    for r in (None, rows):
        xs = x[:m] if r is None else x
        h1 = [torch.empty(m, n, device="cuda") for _ in range(2)]
        for j in range(2):
            K.linear_tanh(xs, w[j], b[j], h1[j], r)
        h2 = [torch.empty(m, n, device="cuda") for _ in range(2)]
        K.linear_tanh2(xs, w[0], b[0], h2[0], w[1], b[1], h2[1], r)
        assert torch.equal(h1[0], h2[0]) and torch.equal(h1[1], h2[1])
        single = K.FirstLayerBackward(m, k, n, "cuda")
        ref = []
        for j in range(2):
            gw, gb = torch.empty(n, k, device="cuda"), torch.empty(n, device="cuda")
            single(gh[j], h1[j], xs, gw, gb, r)
            ref += [gw, gb]
        out = [torch.full((n, k), float("nan"), device="cuda"),
               torch.full((n,), float("nan"), device="cuda")] * 2
        out = [t.clone() for t in out]
        K.FirstLayerBackward2(m, k, n, "cuda")(xs, gh[0], h1[0], out[0], out[1],
                                               gh[1], h1[1], out[2], out[3], r)
        for a, c in zip(ref, out):
            assert torch.equal(a, c)


@pytest.mark.parametrize("m,d", [(65536, 15), (1000, 18), (300, 12)])
def test_gather_minibatch_equals_gathers_and_adv_pass(m, d):
    """dr_gather_minibatch == three dr_gather_rows, and the head step fed
    its advantage partials (normalize_advantage = 2) is bitwise the head
    step that computes them itself."""
    from drone_rl_amd import ppo_kernels as K
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    g = torch.Generator(device="cuda").manual_seed(m + d)
    total = 2 * m + 5
    obs = torch.randn(total, d, device="cuda", generator=g)
    act = torch.rand(total, 4, device="cuda", generator=g) * 7.3575
    aux = torch.randn(total, 3, device="cuda", generator=g)
    idx = torch.randperm(total, device="cuda", generator=g)[:m].to(torch.int32)
    o, a, x = (torch.empty(m, w, device="cuda") for w in (d, 4, 3))
    head = K.HeadLossBackward(m, 256, "cuda", 0.2, 0.0, 0.5, True)
    K.gather_minibatch(idx, obs, act, aux, o, a, x, adv_part=head.adv_part)
    r = idx.long()
    assert torch.equal(o, obs[r]) and torch.equal(a, act[r]) and torch.equal(x, aux[r])
    pol = ActorCritic(d, 4, (256, 256), device="cuda", seed=6)
    fs = FusedTrainStep(pol, m)
    st_out = torch.empty(8, device="cuda")
    g1, s1 = fs.step(o, a, x, head, adv_ready=True, stats_out=st_out)
    assert s1.data_ptr() == st_out.data_ptr()
    g1, s1 = g1.clone(), s1.clone()
    g2, s2 = fs.step(o, a, x, head)          # the head's own advantage pass
    assert torch.equal(g1, g2) and torch.equal(s1, s2)


@pytest.mark.parametrize("m,d", [(1, 7), (1025, 5), (4099, 15), (70001, 12)])
def test_gather_minibatch_ragged_and_runtime_widths(m, d):
    """dr_gather_minibatch at ragged row counts (partial last block of every
    section) and at obs widths without a compiled-in constant (the runtime
    divisor path): the rows of obs / actions / aux exactly."""
    from drone_rl_amd import ppo_kernels as K
    g = torch.Generator(device="cuda").manual_seed(m * 31 + d)
    total = 3 * m + 2
    obs = torch.randn(total, d, device="cuda", generator=g)
    act = torch.randn(total, 4, device="cuda", generator=g)
    aux = torch.randn(total, 3, device="cuda", generator=g)
    idx = torch.randperm(total, device="cuda", generator=g)[:m].to(torch.int32)
    o, a, x = (torch.full((m, w), float("nan"), device="cuda") for w in (d, 4, 3))
    K.gather_minibatch(idx, obs, act, aux, o, a, x)
    r = idx.long()
    assert torch.equal(o, obs[r]) and torch.equal(a, act[r]) and torch.equal(x, aux[r])


@pytest.mark.parametrize("m,d", [(65536, 15), (1, 15), (1025, 12), (4099, 5), (70001, 18),
                                 (300, 24)])
def test_gather_records_is_gather_minibatch(m, d):
    """The one-line record path (round 6): dr_pack_rollout_records once, then
    dr_gather_records writes exactly dr_gather_minibatch's bytes -- obs,
    action and aux rows and the advantage (count, mean, M2) partials -- at
    full size, ragged row counts and other obs widths; the records hold
    each row's values at their documented offsets."""
    from drone_rl_amd import ppo_kernels as K
    g = torch.Generator(device="cuda").manual_seed(m * 7 + d)
    total = 2 * m + 3
    obs = torch.randn(total, d, device="cuda", generator=g)
    act = torch.rand(total, 4, device="cuda", generator=g) * 7.3575
    lp, adv, ret = (torch.randn(total, device="cuda", generator=g) for _ in range(3))
    aux = torch.stack([lp, adv, ret], dim=1)
    rec = torch.full((total, K.RECORD_FLOATS), float("nan"), device="cuda")
    K.pack_rollout_records(obs, act, lp, adv, ret, rec)
    ao = 4 * ((d + 3) // 4)
    assert torch.equal(rec[:, :d], obs) and torch.equal(rec[:, ao:ao + 4], act)
    assert torch.equal(rec[:, ao + 4:ao + 7], aux)
    assert (rec[:, d:ao] == 0).all() and (rec[:, ao + 7:] == 0).all()
    idx = torch.randperm(total, device="cuda", generator=g)[:m].to(torch.int32)
    nb = (m + 255) // 256
    outs = []
    for use_rec in (False, True):
        o, a, x = (torch.full((m, w), float("nan"), device="cuda") for w in (d, 4, 3))
        part = torch.full((3 * nb,), float("nan"), device="cuda")
        if use_rec:
            K.gather_records(idx, rec, d, o, a, x, adv_part=part)
        else:
            K.gather_minibatch(idx, obs, act, aux, o, a, x, adv_part=part)
        outs.append((o, a, x, part))
    for u, v in zip(*outs):
        assert torch.equal(u, v)
    r = idx.long()
    assert torch.equal(outs[1][0], obs[r]) and torch.equal(outs[1][2], aux[r])


@pytest.mark.parametrize("arch,m", [((256, 256), 65536), ((64, 64), 1000), ((64, 128), 4096)])
def test_deferred_finish_equals_separate_finishes(arch, m):
    """FusedTrainStep.step(defer_finish=True) + ClipAdam.step_finish (the
    head / first-layer / split-K reductions and the norm in one launch) ==
    the separate finish launches + ClipAdam.step: stats bitwise, clipped
    gradient and updated parameters to f32 summation-order noise; reruns
    bitwise."""
    from drone_rl_amd import ppo_kernels as K
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    g = torch.Generator(device="cuda").manual_seed(m)
    obs = torch.randn(m, 15, device="cuda", generator=g)
    act = torch.rand(m, 4, device="cuda", generator=g) * 7.3575
    aux = torch.randn(m, 3, device="cuda", generator=g)

    def run(defer):
        pol = ActorCritic(15, 4, arch, device="cuda", seed=9)
        with torch.no_grad():
            pol.flat.mul_(2.0)
        fs = FusedTrainStep(pol, m)
        head = K.HeadLossBackward(m, arch[-1], "cuda", 0.2, 0.01, 0.5, True)
        opt = K.ClipAdam(pol.flat.data, 3e-4, eps=1e-5, max_grad_norm=0.5)
        st = torch.full((8,), float("nan"), device="cuda")
        outs = []
        for _ in range(2):                     # two optimizer steps
            grad, s = fs.step(obs, act, aux, head, stats_out=st, defer_finish=defer)
            if defer:
                norm = opt.step_finish(grad, fs.finish)
            else:
                norm = opt.step(grad)
            outs.append((grad.clone(), s.clone(), norm.clone()))
        torch.cuda.synchronize()
        return outs, pol.flat.detach().clone()

    (a, pa), (b, pb), (c, pc) = run(False), run(True), run(True)
    for (ga, sa, na), (gb, sb, nb) in zip(a, b):
        assert torch.equal(sa, sb)
        assert abs(na.item() - nb.item()) <= 1e-5 * na.item()
        scale = ga.abs().max().item()
        assert (ga - gb).abs().max().item() <= 1e-5 * scale
    assert (pa - pb).abs().max().item() <= 1e-5
    assert torch.equal(pb, pc) and all(torch.equal(x[0], y[0]) for x, y in zip(b, c))
