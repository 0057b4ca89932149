"""Host-side checks of the actor-critic layout and SB3-style init (CPU)."""
import numpy as np
import torch

from drone_rl_amd.policy import ActorCritic
from drone_rl_amd.ppo import PPOConfig


def test_param_count_and_names():
    p = ActorCritic(15, 4, (256, 256))
    assert p.num_params == 141_065            # 2x256 actor-critic
    sd = p.state_dict()
    assert sd["mlp_extractor.policy_net.0.weight"].shape == (256, 15)
    assert sd["mlp_extractor.value_net.2.weight"].shape == (256, 256)
    assert sd["action_net.weight"].shape == (4, 256)
    assert sd["value_net.weight"].shape == (1, 256)
    assert torch.equal(sd["log_std"], torch.zeros(4))
    small = ActorCritic(15, 4, (64, 64))
    assert small.num_params == 2 * (15 * 64 + 64 + 64 * 64 + 64) + 4 * 64 + 4 + 64 + 1 + 4


def test_orthogonal_init_gains_and_zero_bias():
    p = ActorCritic(15, 4, (256, 256), seed=3)
    for name, gain in (("pi1.w", np.sqrt(2)), ("vf0.w", np.sqrt(2))):
        w = p.p(name).detach().double()
        r = min(w.shape)
        s = torch.linalg.svdvals(w)
        assert torch.allclose(s[:r], torch.full((r,), gain, dtype=torch.float64), atol=1e-4)
    sv = torch.linalg.svdvals(p.p("action.w").detach().double())
    assert torch.allclose(sv, torch.full_like(sv, 0.01), atol=1e-6)
    for b in ("pi0.b", "pi1.b", "action.b", "vf0.b", "value.b"):
        assert torch.count_nonzero(p.p(b)) == 0


def test_flat_views_share_storage_and_grad():
    p = ActorCritic(15, 4, (32, 32))
    x = torch.randn(7, 15)
    mean, value = p(x)
    assert mean.shape == (7, 4) and value.shape == (7,)
    (mean.sum() + value.sum()).backward()
    g = p.flat.grad
    a, b, _ = p.offsets["log_std"]
    assert g.shape == (p.num_params,) and torch.count_nonzero(g[a:b]) == 0
    assert torch.count_nonzero(g[: a]) > 0


def test_state_dict_roundtrip():
    p = ActorCritic(15, 4, (64, 64), seed=1)
    q = ActorCritic(15, 4, (64, 64), seed=2)
    q.load_state_dict(p.state_dict())
    assert torch.equal(p.flat.detach(), q.flat.detach())


def test_config_defaults():
    c = PPOConfig.sb3_defaults()
    assert (c.n_steps, c.batch_size, c.n_epochs, c.net_arch) == (2048, 64, 10, (64, 64))
    assert c.gamma == 0.99 and c.gae_lambda == 0.95 and c.clip_range == 0.2
    assert c.ent_coef == 0.0 and c.vf_coef == 0.5 and c.max_grad_norm == 0.5


def test_splitk_linear_matches_autograd():
    from drone_rl_amd.policy import _SplitKLinear
    torch.manual_seed(0)
    x = torch.randn(8192, 33, requires_grad=True)
    w = torch.randn(17, 33, requires_grad=True)
    b = torch.randn(17, requires_grad=True)
    g = torch.randn(8192, 17)
    y = _SplitKLinear.apply(x, w, b, 64)
    y.backward(g)
    x2, w2, b2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_(), \
        b.detach().clone().requires_grad_()
    torch.nn.functional.linear(x2, w2, b2).backward(g)
    assert torch.allclose(y, torch.nn.functional.linear(x2, w2, b2), atol=1e-5)
    for a, r in ((x.grad, x2.grad), (w.grad, w2.grad), (b.grad, b2.grad)):
        assert torch.allclose(a, r, rtol=1e-4, atol=1e-3)


def test_tuned_gemm_table_covers_the_trainer_shapes():
    """The committed TunableOp table (policy.use_tuned_gemms) is well formed,
    validated for this image's stack, and holds the three batched GEMM shapes
    of a 65,536-row 2x256 minibatch."""
    import csv

    from drone_rl_amd.policy import TUNED_GEMMS_CSV
    rows = list(csv.reader(open(TUNED_GEMMS_CSV)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    assert val["PT_VERSION"] == torch.__version__.split("+")[0]
    sols = {r[1]: (r[2], float(r[3])) for r in rows if r[0] != "Validator"}
    for shape in ("tn_256_65536_256_B_2", "nn_256_65536_256_B_2", "nt_256_256_1024_B_128"):
        key = next(k for k in sols if k.startswith(shape))
        name, ms = sols[key]
        assert name.startswith(("Gemm_Rocblas_", "Gemm_Hipblaslt_")) and 0.05 < ms < 0.5
