"""One eager configs[2] PPO iteration (65,536 envs, T = 32, 2x256, 10 epochs x
32 minibatches of 65,536): the workload whose gather_minibatch_kernel
dispatches scripts/micro/r5_gather.sh counts with rocprofv3 --pmc."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from drone_rl_amd.ppo import PPOConfig, PPOTrainer  # noqa: E402

cfg = PPOConfig(num_envs=65536, n_steps=32, batch_size=65536, n_epochs=int(sys.argv[1]) if
                len(sys.argv) > 1 else 2, seed=0)
tr = PPOTrainer(cfg, device=torch.device("cuda", 0))
tr.learn_step()
torch.cuda.synchronize()
tr.close()
print("ok")
