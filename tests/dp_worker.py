"""One rank of the 2-rank PPO data-parallel GPU check (launched by
tests/test_vecenv_dp_gpu.py).  Both ranks share the single GPU of the test
box, so the process group is gloo (RCCL refuses two ranks on one device);
the collective call sites are the ones RCCL uses on a multi-GPU node."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from drone_rl_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    cfg = PPOConfig(num_envs=1024, n_steps=16, batch_size=4096, n_epochs=2, net_arch=(64, 64),
                    seed=3 + 11 * rank)     # different seeds: broadcast must equalise
    tr = PPOTrainer(cfg, device="cuda:0", rank=rank, world_size=world)
    for _ in range(2):          # 32 steps: free-fall episodes end near step 22
        st = tr.learn_step()
        assert torch.isfinite(st).all()
    # parameters identical on every rank after synchronous DP updates
    p = tr.policy.flat.detach().clone()
    mx, mn = p.clone(), p.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    assert torch.equal(mx, mn), "ranks diverged"
    # envs are disjoint shards: global ids differ, so episodes differ
    es = tr.episode_stats()
    assert es["episodes"] > 0
    ep = tr.env.get("pos")[:4].cpu()
    other = [torch.zeros_like(ep) for _ in range(world)]
    dist.all_gather(other, ep)
    assert not torch.equal(other[0], other[1])
    tr.close()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok")


if __name__ == "__main__":
    main()
