"""One rank of the 2-rank data-parallel gradient check on the fused GPU
kernels (launched by tests/test_vecenv_dp_gpu.py): the flagship 2x256 net,
8,192 envs per rank.  Each rank forms its minibatch gradient with the fused
path (dr_linear_tanh2, batched GEMMs, dr_ppo_head_loss_backward,
dr_first_layer_backward2), the gradient is mean-all-reduced in one bucket
and in two buckets (bitwise equal), and rank 0 checks it against the
gradient of the UNION minibatch computed by one fused step over both ranks'
rows -- and the clip+Adam update that follows.

Tolerance: both sides sum the same per-row terms in fp32, in different
orders (split-K chunks of M/64 vs 2M/64 rows, the head's per-block partials,
one cross-rank add): each gradient entry is a sum of <= 65,536 terms, so the
reassociation error is bounded by ~ n * eps_f32 * sum|terms| and in practice
~1e-6 of the largest entry; 2e-5 of max|g| is the bar.  Advantage
normalisation is off: SB3 normalises per minibatch, so with it on the DP
gradient is by design the mean of per-rank-normalised gradients (the CPU
gloo test covers the same property for the autograd path).  Both ranks share
the test box's one GPU, so the group is gloo; RCCL runs the same call sites
on a multi-GPU node."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from drone_rl_amd import dist as D  # noqa: E402
from drone_rl_amd import ppo_kernels as K  # noqa: E402
from drone_rl_amd.policy import FusedTrainStep  # noqa: E402
from drone_rl_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    M = 16384
    cfg = PPOConfig(num_envs=8192, n_steps=4, batch_size=M, n_epochs=1, net_arch=(256, 256),
                    normalize_advantage=False, seed=5)
    tr = PPOTrainer(cfg, device=dev, rank=rank, world_size=world)
    tr.collect_rollouts()
    T, N = cfg.n_steps, cfg.num_envs
    idx = tr.perm(seed=17, counter=rank)[:M]
    K.gather_minibatch(idx, tr.obs[:T].reshape(T * N, -1), tr.actions.reshape(T * N, 4),
                       tr.aux, tr.mb_obs, tr.mb_act, tr.mb_aux, adv_part=tr.head.adv_part)
    grads = {}
    for buckets in (1, 2):
        bar = D.BucketedAllReduce(tr.fused.grad, world)
        g, _ = tr.fused.step(tr.mb_obs, tr.mb_act, tr.mb_aux, tr.head, adv_ready=True,
                             on_ready=bar.start if buckets == 2 else None)
        grads[buckets] = bar.finish().clone()
    assert torch.equal(grads[1], grads[2]), "bucketing changed the reduced gradient"
    g_dp = grads[1]
    rows = [torch.cat([t.cpu() for t in (tr.mb_obs, tr.mb_act, tr.mb_aux)], 1)]
    allr = [torch.zeros_like(rows[0]) for _ in range(world)]
    dist.all_gather(allr, rows[0])
    if rank == 0:
        u = torch.cat(allr, 0).to(dev)
        od = tr.mb_obs.shape[1]
        u_obs, u_act = u[:, :od].contiguous(), u[:, od:od + 4].contiguous()
        u_aux = u[:, od + 4:].contiguous()
        fu = FusedTrainStep(tr.policy, world * M)
        hu = K.HeadLossBackward(world * M, 256, dev, cfg.clip_range, cfg.ent_coef,
                                cfg.vf_coef, normalize_advantage=False)
        g_u, _ = fu.step(u_obs, u_act, u_aux, hu)
        scale = g_u.abs().max().item()
        err = (g_dp - g_u).abs().max().item()
        assert err <= 2e-5 * scale, f"DP gradient vs union: {err:.3e} (scale {scale:.3e})"
        # the optimizer step that follows agrees too
        p0 = tr.policy.flat.detach().clone()
        outs = []
        for g in (g_dp, g_u):
            tr.policy.flat.data.copy_(p0)
            opt = K.ClipAdam(tr.policy.flat.data, cfg.learning_rate, eps=1e-5,
                             max_grad_norm=cfg.max_grad_norm)
            opt.step(g.clone())
            outs.append(tr.policy.flat.detach().clone() - p0)
        du = outs[1].abs().max().item()
        assert (outs[0] - outs[1]).abs().max().item() <= 1e-3 * du
        print(f"union check: err {err:.3e} of {scale:.3e}", flush=True)
    tr.close()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()
