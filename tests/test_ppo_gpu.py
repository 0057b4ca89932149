"""End-to-end GPU PPO checks against the CPU restatement of SB3 PPO
(oracle/ppo_ref.py).  "Parity unpinned" w.r.t. the reference (SB3 is not
available); pinned to the restatement: rollout log-probs / values / GAE
recomputed on CPU, and a full PPO.train() (2 epochs x 4 minibatches, clip +
Adam) matched parameter-for-parameter."""
import numpy as np
import pytest
import torch

from oracle import ppo_ref

pytestmark = pytest.mark.gpu


def _trainer(net_arch=(64, 64), **kw):
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=2048, n_steps=8, batch_size=4096, n_epochs=2,
                    net_arch=net_arch, seed=5, **kw)
    return PPOTrainer(cfg)


def test_rollout_consistent_with_cpu():
    tr = _trainer()
    tr.collect_rollouts()
    T, N = tr.cfg.n_steps, tr.cfg.num_envs
    sd = tr.policy.state_dict()
    pi, vf, act, val, log_std = ppo_ref.sb3_policy_modules(sd, tr.cfg.net_arch)
    obs = tr.obs[:T].reshape(T * N, -1).cpu()
    with torch.no_grad():
        mean = act(pi(obs))
        values = val(vf(obs)).flatten()
        d = torch.distributions.Normal(mean, torch.ones_like(mean) * log_std.exp())
        logp = d.log_prob(tr.actions.reshape(T * N, 4).cpu()).sum(1)
    np.testing.assert_allclose(tr.values.reshape(-1).cpu(), values, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(tr.logp.reshape(-1).cpu(), logp, rtol=1e-4, atol=1e-4)
    # env saw the clipped action; buffer keeps the unclipped one (SB3)
    assert (tr.actions.min() < 0).item() or (tr.actions.max() > 7.3575).item()
    # GAE on the recorded rollout
    dn = tr.dones.cpu().numpy().astype(np.float32)
    adv, ret = ppo_ref.gae_numpy(tr.rewards.cpu().numpy(), tr.values.cpu().numpy(),
                                 dn[:T], tr.policy(tr.obs[T])[1].detach().cpu().numpy(),
                                 dn[T].astype(bool), 0.99, 0.95)
    np.testing.assert_allclose(tr.adv.cpu().numpy(), adv, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(tr.ret.cpu().numpy(), ret, rtol=1e-4, atol=1e-4)
    tr.close()


def test_train_matches_sb3_restatement():
    from drone_rl_amd import ppo_kernels as K
    tr = _trainer()
    tr.collect_rollouts()
    T, N, cfg = tr.cfg.n_steps, tr.cfg.num_envs, tr.cfg
    sd0 = tr.policy.state_dict()
    obs = tr.obs[:T].reshape(T * N, -1).cpu().clone()
    acts = tr.actions.reshape(T * N, 4).cpu().clone()
    aux = tr.aux.cpu().clone()
    perms = [K.Permuter(T * N, "cuda")(seed=cfg.seed * 104729, counter=e).cpu().numpy().copy()
             for e in range(cfg.n_epochs)]
    st = tr.train()
    assert torch.isfinite(st).all()
    got = tr.policy.state_dict()
    ref = ppo_ref.sb3_train(sd0, cfg.net_arch, obs, acts, aux[:, 0].contiguous(),
                            aux[:, 1].contiguous(), aux[:, 2].contiguous(), perms,
                            cfg.batch_size)
    for k, v in ref.items():
        delta_ref = (v - sd0[k]).numpy()
        delta_got = (got[k] - sd0[k]).numpy()
        scale = np.abs(delta_ref).max() + 1e-12
        # Adam steps are ~lr in size; f32 GEMM/reduction order differences
        # must stay a small fraction of the update itself
        assert np.abs(delta_got - delta_ref).max() <= 0.02 * scale, k
    tr.close()


def test_learning_loop_runs_finite():
    tr = _trainer()
    for _ in range(3):
        st = tr.learn_step()
        assert torch.isfinite(st).all()
    es = tr.episode_stats()
    assert es["episodes"] > 0 and np.isfinite(es["ep_rew_mean"])
    assert torch.isfinite(tr.policy.flat).all()
    tr.close()


def test_checkpoint_resume_is_bitexact(tmp_path):
    """Save after one iteration, resume in a fresh trainer: the next
    iteration reproduces the uninterrupted run bit for bit (every random
    stream is keyed by counters that the checkpoint carries; the env
    curriculum is saved too, unlike the reference's SB3 .zip)."""
    a = _trainer()
    a.learn_step()
    path = tmp_path / "ck.pt"
    a.save(path)
    a.learn_step()
    b = _trainer()
    b.load(path)
    b.learn_step()
    assert torch.equal(a.policy.flat.detach(), b.policy.flat.detach())
    assert torch.equal(a.env.get("pos"), b.env.get("pos"))
    assert torch.equal(a.env.get("ep_num"), b.env.get("ep_num"))
    assert a.num_timesteps == b.num_timesteps
    a.close()
    b.close()


def test_sb3_zip_roundtrip_on_gpu(tmp_path):
    """save_sb3 -> load_sb3 restores parameters, Adam state and the per-env
    curriculum, and training continues (SB3 itself: parity unpinned)."""
    a = _trainer()
    a.learn_step()
    a.env.set("eps", np.full(a.env.num_envs, 0.3))
    path = tmp_path / "dd.zip"
    a.save_sb3(path)
    b = _trainer()
    b.load_sb3(path)
    assert torch.equal(a.policy.flat.detach(), b.policy.flat.detach())
    assert torch.equal(a.opt.m, b.opt.m) and torch.equal(a.opt.v, b.opt.v)
    assert b.opt.t == a.opt.t and b.num_timesteps == a.num_timesteps
    assert (b.env.get("eps").cpu().numpy() == 0.3).all()
    assert torch.isfinite(b.learn_step()).all()
    a.close()
    b.close()


def test_sb3_zip_resume_continues_streams_and_schedule(tmp_path):
    """load_sb3 restores the iteration count from SB3's _n_updates: the
    resumed run continues the policy-noise / permutation streams and does not
    re-fire eps_schedule entries that already ran (which would overwrite the
    curriculum the sidecar restored)."""
    sched = ((0, 0.05), (2, 0.2))
    a = _trainer(eps_schedule=sched)
    a.learn_step()
    a.learn_step()          # update 0 set eps 0.05; the next fires at update 2
    a.env.set("eps", np.full(a.env.num_envs, 0.1))
    path = tmp_path / "dd.zip"
    a.save_sb3(path)
    b = _trainer(eps_schedule=sched)
    b.load_sb3(path)
    assert b.num_updates == a.num_updates == 2
    b.learn_step()          # update 2: noise counter base = 2 * T
    assert b._ctr.item() == 2 * b.cfg.n_steps and b.num_updates == 3
    assert (b.env.get("eps").cpu().numpy() >= 0.2).all()     # update-2 entry fired once
    c = _trainer(eps_schedule=((0, 0.05),))
    c.load_sb3(path)
    c.learn_step()           # the update-0 entry must not fire again
    assert (c.env.get("eps").cpu().numpy() >= 0.1).all()
    for t in (a, b, c):
        t.close()


@pytest.mark.parametrize("arch", [(64, 64), (256, 256)])
def test_overlapped_gather_is_bitwise_the_serial_loop(arch):
    """DRONERL_PPO_OVERLAP=1 (minibatch j + 1 gathered on a side stream
    beside step j, two buffer slots) trains bitwise as the serial loop,
    eager and graph-captured, across an epoch boundary (4 minibatches per
    epoch, 2 epochs)."""
    a, b, c = _trainer(net_arch=arch), _trainer(net_arch=arch), _trainer(net_arch=arch)
    b.overlap_gather = c.overlap_gather = True
    c.rollout_graph = c.train_graph = False
    for it in range(3):
        sa, sb, sc = a.learn_step(), b.learn_step(), c.learn_step()
        assert torch.equal(sa, sb) and torch.equal(sa, sc), it
        for t in (b, c):
            assert torch.equal(a.policy.flat.detach(), t.policy.flat.detach()), it
            assert torch.equal(a.opt.m, t.opt.m) and torch.equal(a.opt.v, t.opt.v), it
    assert b._tgraph is not None and b._slots is not None and c._tgraph is None
    assert b.head.ws.data_ptr() == b._slots[0][3].data_ptr()
    for t in (a, b, c):
        t.close()


def test_graphs_follow_host_scalar_changes():
    """A seed, learning-rate or loss-coefficient change after the rollout /
    training graphs were captured takes effect on the graph path exactly as
    on the eager path (the graphs are re-captured when a baked-in host value
    changes)."""
    a, b = _trainer(), _trainer()
    a.rollout_graph = a.train_graph = False
    b.rollout_graph = b.train_graph = True
    for it in range(5):
        if it == 3:
            for t in (a, b):
                t.env.seed(1234)
                t.opt.lr = 1e-4
                t.head.clip = 0.1
        sa, sb = a.learn_step(), b.learn_step()
        assert torch.equal(sa, sb), it
        assert torch.equal(a.policy.flat.detach(), b.policy.flat.detach()), it
        assert torch.equal(a.env.get("pos"), b.env.get("pos")), it
    assert b._rgraph is not None and b._tgraph is not None
    a.close()
    b.close()


def test_tuned_gemms_load_and_are_deterministic():
    """The committed TunableOp solutions (policy.use_tuned_gemms) load on the
    box, give a bitwise-reproducible minibatch gradient at the bench shape
    (65,536 rows, 2x256) and agree with the library-heuristic GEMMs to fp32
    reassociation error."""
    import torch.cuda.tunable as tun

    from drone_rl_amd.ppo import PPOConfig, PPOTrainer

    cfg = PPOConfig(num_envs=65536, n_steps=2, batch_size=65536, n_epochs=1, seed=3)
    tr = PPOTrainer(cfg)
    assert tr.tuned_gemms and tun.is_enabled(), "tuned GEMM table not loaded"
    tr.collect_rollouts()
    M = cfg.batch_size
    obs = tr.obs[:1].reshape(M, -1)
    act = tr.actions[:1].reshape(M, 4)
    aux = tr.aux[:M]

    def grad():
        g, st = tr.fused.step(obs, act, aux, tr.head)
        torch.cuda.synchronize()
        return g.clone(), st.clone()

    g1, s1 = grad()
    keys = " ".join(str(r) for r in tun.get_results())
    for shape in ("nt_256_256_1024_B_128", "nn_256_65536_256_B_2", "tn_256_65536_256_B_2"):
        assert shape in keys, shape
    g2, s2 = grad()
    assert torch.equal(g1, g2) and torch.equal(s1, s2)
    tun.enable(False)
    try:
        g3, s3 = grad()
    finally:
        tun.enable(True)
    scale = g3.abs().max().item()
    assert (g1 - g3).abs().max().item() <= 1e-4 * scale
    np.testing.assert_allclose(s1.cpu(), s3.cpu(), rtol=1e-4, atol=1e-6)
    tr.close()


@pytest.mark.parametrize("cfg", ["small", "sb3_1env", "configs2"])
def test_rollout_graph_is_bitwise_eager(cfg):
    """The rollout loop and PPO.train's minibatch loop captured into
    hipGraphs (after one eager warm-up iteration; the policy-noise and
    permutation counter bases and Adam's bias-correction schedule live on the
    device) replay to bitwise the eager rollouts and updates over several
    PPO iterations -- including configs[2] itself (65,536 envs, 2x256,
    65,536-row minibatches x 32 x 10 epochs per graph), where round 1's
    rocPRIM-sorted permutation faulted on the second replay."""
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer

    def make(graph):
        if cfg == "small":
            tr = _trainer()
        elif cfg == "configs2":
            tr = PPOTrainer(PPOConfig(seed=3))
        else:
            tr = PPOTrainer(PPOConfig.sb3_defaults(n_steps=128, seed=3))
        tr.rollout_graph = tr.train_graph = graph
        return tr

    a, b = make(False), make(True)
    for _ in range(4):
        sa = a.learn_step()
        sb = b.learn_step()
        assert torch.equal(sa, sb)
        for name in ("obs", "actions", "logp", "values", "rewards", "dones", "adv"):
            assert torch.equal(getattr(a, name), getattr(b, name)), name
        assert torch.equal(a.opt.m, b.opt.m) and a.opt.t == b.opt.t
    assert b._rgraph is not None and b._tgraph is not None
    assert torch.equal(a.policy.flat.detach(), b.policy.flat.detach())
    assert torch.equal(a.env.get("ep_num"), b.env.get("ep_num"))
    a.close()
    b.close()


@pytest.mark.parametrize("num_envs", [1000, 1024])
def test_rollout_and_first_epoch_share_one_gemm_path(num_envs):
    """advisor r02: the 256x256 layer's GEMM path is chosen once per trainer
    (dr_gemm_x6 only when the rollout's N rows AND the minibatch's M rows are
    multiples of 128), so the first epoch's ratio is exactly 1: with one
    epoch of one minibatch, approx_kl and clip_fraction are exactly 0."""
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=num_envs, n_steps=32, batch_size=num_envs * 32, n_epochs=1,
                    seed=6)
    tr = PPOTrainer(cfg)
    assert tr.policy.gemm_x6 == (num_envs % 128 == 0)
    tr.collect_rollouts()
    st = dict(zip(("loss", "policy_loss", "value_loss", "entropy_loss", "clip_fraction",
                   "approx_kl"), tr.train().tolist()))
    assert st["approx_kl"] == 0.0 and st["clip_fraction"] == 0.0, st
    tr.close()
