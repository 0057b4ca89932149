"""Subprocess body of tests/test_rollout_gpu.py::test_rollout_forms_outside_their_default:
dr_rollout's kernel form is chosen once per process (DRONERL_ROLLOUT_WS, read
at the first launch), so each forced form runs in its own process.  K steps
of dr_rollout against K dr_step launches, bitwise, every output and the final
state.  argv: variant n K."""
import sys

import torch

from drone_rl_amd import DroneBatch, random_actions


def main():
    variant, n, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    a = DroneBatch(n, variant, dtype=torch.float64, seed=99, env_id_offset=5)
    b = DroneBatch(n, variant, dtype=torch.float64, seed=99, env_id_offset=5)
    for x in (a, b):
        x.reset()
        ep = x.get("ep_num").cpu()
        ep[::11] = 1999                     # the curriculum bump inside the launch
        x.set("ep_num", ep)
    acts = torch.empty(K, n, 4, device="cuda")
    for t in range(K):
        random_actions(n, seed=3, step=t, env_id_offset=5, out=acts[t])
    obs, rew, done = a.rollout(K, acts)
    for t in range(K):
        so, sr, sd = b.step(acts[t])
        assert torch.equal(obs[t], so) and torch.equal(rew[t], sr) and torch.equal(done[t], sd), t
    for k in ("pos", "vel", "euler", "omega", "target", "current_step", "ep_num", "eps"):
        assert torch.equal(a.get(k), b.get(k)), k
    assert int(done.sum()) > n // 8
    print("ok", variant, n, K)


if __name__ == "__main__":
    main()
