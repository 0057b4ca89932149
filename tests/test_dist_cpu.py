"""Data-parallel path on CPU with gloo, world_size 2.

Checks the product's DP plumbing (drone_rl_amd/dist.py, used by
PPOTrainer): parameter broadcast, env-id sharding, and that the all-reduced
(mean) gradient of two ranks' minibatch halves equals the single-process
gradient over the union minibatch (fp32 tolerance).  Advantage
normalisation is off here: SB3 normalises per minibatch, so with it on the
DP gradient is (by design) the mean of per-rank-normalised gradients.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drone_rl_amd import dist as D
from drone_rl_amd.policy import ActorCritic
from oracle import ppo_ref


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grad_of(policy, obs, act, old_logp, adv, ret):
    """flat.grad of the PPO minibatch loss, the way PPOTrainer.train forms it
    (loss head gradients from the restated SB3 loss, autograd through the
    MLP, log_std gradient added to its slice)."""
    policy.flat.grad = None
    mean, value = policy(obs)
    _, gm, gls, gv = ppo_ref.ppo_loss_torch(mean.detach().numpy(), policy.log_std.detach().numpy(),
                                           value.detach().numpy(), act, old_logp, adv, ret,
                                           0.2, 0.0, 0.5, normalize=False)
    torch.autograd.backward([mean, value], [torch.from_numpy(gm), torch.from_numpy(gv)])
    a, b, _ = policy.offsets["log_std"]
    policy.flat.grad[a:b] += torch.from_numpy(gls)
    return policy.flat.grad.clone()


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    # 1. broadcast: ranks start from different seeds, end equal to rank 0
    pol = ActorCritic(15, 4, (32, 32), seed=100 + rank)
    D.broadcast_params_(pol.flat.data)
    ref0 = ActorCritic(15, 4, (32, 32), seed=100)
    assert torch.equal(pol.flat.detach(), ref0.flat.detach())
    # 2. gradient all-reduce == union-minibatch gradient
    rng = np.random.default_rng(7)
    m = 256
    obs = rng.normal(size=(world * m, 15)).astype(np.float32)
    act = rng.normal(2.0, 1.0, (world * m, 4)).astype(np.float32)
    old_logp = rng.normal(-6.0, 0.5, world * m).astype(np.float32)
    adv = rng.normal(size=world * m).astype(np.float32)
    ret = rng.normal(size=world * m).astype(np.float32)
    sl = slice(rank * m, (rank + 1) * m)
    g_local = _grad_of(pol, torch.from_numpy(obs[sl]), act[sl], old_logp[sl], adv[sl], ret[sl])
    g = D.allreduce_mean_(g_local.clone(), world)
    g_union = _grad_of(pol, torch.from_numpy(obs), act, old_logp, adv, ret)
    scale = g_union.abs().max().item()
    assert (g - g_union).abs().max().item() <= 1e-5 * scale
    # all ranks hold the identical reduced gradient
    g_max = D.allreduce_max_(g.clone(), world)
    assert torch.equal(g_max, g)
    # 2b. the bucketed form (a middle bucket started early, the gaps at the
    # end) gives exactly the single all-reduce's result
    bar = D.BucketedAllReduce(g_local.clone(), world)
    bar.start(1000, g_local.numel() - 500)
    gb = bar.finish()
    assert torch.equal(gb, g)
    # 3. env shards are disjoint and cover [0, world*N)
    lo, hi = D.env_shard(rank, 65536)
    r = torch.tensor([lo, hi], dtype=torch.int64)
    allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allr, r)
    spans = sorted(tuple(x.tolist()) for x in allr)
    assert spans[0][0] == 0 and all(spans[k][1] == spans[k + 1][0] for k in range(world - 1))
    assert spans[-1][1] == world * 65536
    # 4. episode statistics: sums over ranks
    s = torch.tensor([1.0 + rank, 2.0, 3.0])
    D.allreduce_sum_(s, world)
    assert torch.equal(s, torch.tensor([3.0, 4.0, 6.0]))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_gloo_world2():
    mp.spawn(_worker, args=(2, _free_port()), nprocs=2, join=True)


def test_resume_finds_the_legacy_per_rank_checkpoint(tmp_path):
    """advisor r02: per-rank checkpoints are '<root>.rank<r><ext>'; a file
    under the earlier '<checkpoint>.rank<r>' name is still resumed from
    (with a warning) instead of silently starting over."""
    import warnings

    from drone_rl_amd.train import checkpoint_path, resume_path
    ck = str(tmp_path / "dd.pt")
    assert checkpoint_path(ck, 1, 2) == str(tmp_path / "dd.rank1.pt")
    assert resume_path(ck, 1, 2) is None
    legacy = tmp_path / "dd.pt.rank1"
    legacy.write_bytes(b"x")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert resume_path(ck, 1, 2) == str(legacy)
    assert any("legacy" in str(x.message) for x in w)
    (tmp_path / "dd.rank1.pt").write_bytes(b"y")
    assert resume_path(ck, 1, 2) == str(tmp_path / "dd.rank1.pt")
    assert resume_path(ck, 0, 1) is None
