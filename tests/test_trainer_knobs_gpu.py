"""Every selectable form of the trainer's optimizer step against the default
(verdict r05, what's weak #1 / next item 3; advisor r05): one FusedTrainStep
on a 2x256 minibatch, the env knob set before the policy and the step are
built (they read it there).

  * forms whose outputs are independent of the choice must give the same
    BYTES: the x6 operand images built by their own launches
    (DRONERL_X6_FUSED_IMAGES=0), the head's per-block rows summed through
    the grouping launch (DRONERL_HEAD_DIRECT=0), the fused first-layer GEMM
    after the weight gradient instead of before it (DRONERL_FL_FIRST=0);
  * forms that change the arithmetic are held to the flagship bound of a
    gradient entry against the default: the library fp32 GEMMs for the 256 x
    256 layer (DRONERL_GEMM_X6=0) and the non-deferred step (per-kernel
    finishes, PPOTrainer's DRONERL_DEFER_FINISH=0 path).
Reference computation: SB3 PPO.train's minibatch gradient
(/root/reference/train.py:36-43, 63-68)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

M = 8192
KNOBS = ("DRONERL_X6_FUSED_IMAGES", "DRONERL_HEAD_DIRECT", "DRONERL_FL_FIRST",
         "DRONERL_GEMM_X6", "DRONERL_X6_FL", "DRONERL_X6_FL_DIRECT")


def _step(monkeypatch, env, defer=True):
    from drone_rl_amd import ppo_kernels as K
    from drone_rl_amd.policy import ActorCritic, FusedTrainStep
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pol = ActorCritic(15, 4, (256, 256), seed=5, device="cuda")
    fs = FusedTrainStep(pol, M)
    g = torch.Generator().manual_seed(21)
    obs = torch.randn(M, 15, generator=g).cuda()
    act = (torch.rand(M, 4, generator=g) * 7.0).cuda()
    aux = torch.randn(M, 3, generator=g).cuda()
    head = K.HeadLossBackward(M, 256, "cuda", 0.2, 0.0, 0.5, True)
    grad, stats = fs.step(obs, act, aux, head, defer_finish=defer)
    if defer:
        opt = K.ClipAdam(pol.flat.detach(), lr=0.0, max_grad_norm=1e30)
        opt.step_finish(grad, fs.finish)
    torch.cuda.synchronize()
    return pol, grad.clone(), stats.clone()


@pytest.mark.parametrize("knob", ["DRONERL_X6_FUSED_IMAGES", "DRONERL_HEAD_DIRECT",
                                  "DRONERL_FL_FIRST"])
def test_knob_off_is_the_same_bytes(monkeypatch, knob):
    _, g1, s1 = _step(monkeypatch, {knob: "1"})
    _, g0, s0 = _step(monkeypatch, {knob: "0"})
    assert torch.equal(g0, g1), knob
    assert torch.equal(s0, s1), knob


def _per_tensor_close(pol, ga, gb, rel):
    for name in pol.offsets:
        a, b, _ = pol.offsets[name]
        x, y = ga[a:b].double(), gb[a:b].double()
        scale = y.abs().max().item() + 1e-30
        err = (x - y).abs().max().item()
        assert err <= rel * scale, (name, err, scale)


def test_library_gemms_within_bound(monkeypatch):
    """DRONERL_GEMM_X6=0: the 256 x 256 layer on the library's fp32 GEMMs.
    Both forms are fp32-accurate (the x6 product error is below one fp32
    rounding, tests/test_gemm_x6_gpu.py), so every gradient tensor agrees
    to 1e-4 of its largest entry (the bound of the flagship parity test's
    first-layer comparison)."""
    pol, g1, s1 = _step(monkeypatch, {})
    _, g0, s0 = _step(monkeypatch, {"DRONERL_GEMM_X6": "0"})
    _per_tensor_close(pol, g0, g1, 1e-4)
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-6)


def test_non_deferred_step_within_bound(monkeypatch):
    """The step with its reductions run by per-kernel finishes (what
    PPOTrainer runs with DRONERL_DEFER_FINISH=0) against the deferred
    default: the same products, the sums in a different grouping."""
    pol, g1, s1 = _step(monkeypatch, {})
    _, g0, s0 = _step(monkeypatch, {}, defer=False)
    _per_tensor_close(pol, g0, g1, 1e-4)
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-6)


def test_defer_finish_knob_selects_the_path(monkeypatch):
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=1024, n_steps=8, batch_size=2048, n_epochs=1, seed=1)
    for v, want in (("1", True), ("0", False)):
        monkeypatch.setenv("DRONERL_DEFER_FINISH", v)
        tr = PPOTrainer(cfg, device="cuda")
        assert tr.defer_finish is want
        st = tr.learn_step()
        assert torch.isfinite(st).all()
        tr.close()
