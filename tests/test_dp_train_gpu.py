"""configs[3] at its per-rank size through the real data-parallel trainer
(BASELINE.json configs[3]: 8 x 65,536 envs, PPO with one gradient
all-reduce per optimizer step; reference learn loop
/root/reference/train.py:63-68).  Two ranks on the box's one GPU over gloo;
tests/dp_train_worker.py holds the checks.  Also: the data-parallel step
structure at world 1 (force_dp_path) is bitwise the single-GPU step, and
its captured graph replays bitwise its eager form."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_configs3_per_rank_size_through_dp_train():
    port = str(_free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u",
                                       os.path.join(ROOT, "tests", "dp_train_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=600)
        outs.append(out.decode())
    print(outs[0][-2000:])
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, out[-3000:]
        assert f"rank {r} ok" in out
    assert "phase A ok" in outs[0] and "phase B ok" in outs[0]


def _run(force_dp, graph, iters=2):
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=8192, n_steps=8, batch_size=16384, n_epochs=2, seed=9,
                    force_dp_path=force_dp)
    tr = PPOTrainer(cfg)
    tr.train_graph = graph
    if iters < 0:                     # the initial parameters
        p = tr.policy.flat.detach().clone()
        tr.close()
        return p
    out = []
    for _ in range(iters + 1):        # + the eager warm-up iteration of the graph path
        st = tr.learn_step()
        out.append((st.clone(), tr.policy.flat.detach().clone(), tr.opt.m.clone(),
                    tr.opt.v.clone()))
    assert tr.dp_step == force_dp
    tr.close()
    return out


def test_dp_step_at_world1_graph_is_bitwise_eager_and_matches_single_gpu_step():
    """The data-parallel step (dr_grad_finish_run, then dr_clip_adam_sched at
    grad_scale 1) replayed from the captured training graph is bitwise its
    eager form.  Against the single-GPU fused step (dr_grad_finish_clip_adam_
    sched) it differs only in the summation order of the gradient norm (the
    fused launch sums its own blocks' squares; the DP step must norm the
    all-reduced gradient, so it runs a separate pass): one update agrees to
    fp32 rounding."""
    assert not torch.distributed.is_initialized()
    eager = _run(True, False)
    graph = _run(True, True)
    for a, b in zip(eager, graph):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    single = _run(False, True, iters=0)
    _, p_dp, m_dp, v_dp = eager[0]
    _, p_1, m_1, v_1 = single[0]
    p0 = _run(False, True, iters=-1)
    du = (p_1 - p0).abs().max().item()
    assert du > 0
    assert (p_dp - p_1).abs().max().item() <= 1e-3 * du
    assert torch.allclose(m_dp, m_1, rtol=1e-4, atol=1e-9)
    assert torch.allclose(v_dp, v_1, rtol=1e-4, atol=1e-12)
