"""GPU checks of the SB3 VecEnv / gymnasium facades (against the
reference's DummyVecEnv-style golden trajectory) and of the 2-rank PPO
data-parallel loop."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_sb3_vecenv_matches_reference_trajectory(golden):
    """DummyVecEnv + VecMonitor semantics through BatchedDroneVecEnv:
    obs, f32 rewards, dones, infos["terminal_observation"] /
    ["TimeLimit.truncated"] / ["episode"], for the reference's 16-env
    trajectory (host-uniform resets, state re-synchronised each step)."""
    from drone_rl_amd.vec_env import BatchedDroneVecEnv
    g = golden("gym_traj.npz")
    T, n, _ = g["actions"].shape
    venv = BatchedDroneVecEnv(n, rng="host", seed=0)
    venv.batch.set_reset_uniforms(g["reset_u"])
    obs = venv.reset()
    assert obs.shape == (n, 15) and obs.dtype == np.float32
    np.testing.assert_array_equal(obs, g["obs0"])
    assert venv.get_attr("ep_num") == [2] * n
    ep_ret = np.zeros(n, np.float32)
    ep_len = np.zeros(n, np.int64)
    for t in range(T):
        for k in ("pos", "vel", "euler", "omega", "target"):
            venv.batch.set(k, g["pre_" + k][t])
        venv.batch.set("current_step", g["pre_step"][t])
        venv.batch.set_reset_uniforms(np.nan_to_num(g["reset_uniforms"][t], nan=0.5))
        # traj_tb.py:34 reads get_attr('pos')[0] every step
        np.testing.assert_allclose(venv.get_attr("pos")[0], g["pre_pos"][t][0], rtol=1e-12)
        obs, rew, done, infos = venv.step(g["actions"][t])
        assert rew.dtype == np.float32 and done.dtype == bool and len(infos) == n
        np.testing.assert_array_equal(done, g["done"][t])
        np.testing.assert_allclose(obs, g["obs"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(rew, g["reward"][t].astype(np.float32), atol=1e-6)
        ep_ret += rew
        ep_len += 1
        for i in range(n):
            assert infos[i]["TimeLimit.truncated"] is False
            if done[i]:
                np.testing.assert_allclose(infos[i]["terminal_observation"],
                                           g["term_obs"][t][i], rtol=1e-6, atol=1e-6)
                ep = infos[i]["episode"]
                assert ep["l"] == ep_len[i]
                np.testing.assert_allclose(ep["r"], ep_ret[i], rtol=1e-5, atol=1e-6)
                ep_ret[i] = 0
                ep_len[i] = 0
            else:
                assert "terminal_observation" not in infos[i] and "episode" not in infos[i]
    venv.close()


def test_sb3_vecenv_api_surface():
    from drone_rl_amd.vec_env import BatchedDroneVecEnv
    venv = BatchedDroneVecEnv(8, seed=1)
    assert venv.num_envs == 8
    assert venv.observation_space.shape == (15,) and venv.action_space.shape == (4,)
    np.testing.assert_allclose(venv.action_space.high, 7.3575)
    venv.reset()
    assert venv.get_attr("mass") == [1.0] * 8 and venv.get_attr("g", [0, 3]) == [9.81] * 2
    venv.set_attr("pos", np.array([0.0, 0.0, 5.0]), indices=[2])
    assert np.array_equal(venv.get_attr("pos", 2)[0], [0.0, 0.0, 5.0])
    o = venv.env_method("reset", indices=[2])
    assert len(o) == 1 and o[0].shape == (15,) and o[0][2] == 1.0
    assert venv.env_is_wrapped(object) == [False] * 8
    assert len(venv.seed(5)) == 8
    with pytest.raises(AttributeError):
        venv.get_attr("no_such_attr")
    for _ in range(50):
        venv.step(np.random.uniform(0, 7.3575, (8, 4)).astype(np.float32))
    venv.close()


def test_gymnasium_facade():
    from drone_rl_amd.vec_env import DroneVectorEnv
    env = DroneVectorEnv(256, seed=2, split_time_limit=True)
    obs, info = env.reset(seed=4)
    assert obs.shape == (256, 15) and info == {}
    seen_done = False
    for _ in range(60):
        obs, rew, term, trunc, infos = env.step(
            np.random.uniform(0, 7.3575, (256, 4)).astype(np.float32))
        assert term.dtype == bool and trunc.dtype == bool and not (term & trunc).any()
        if term.any() or trunc.any():
            seen_done = True
            m = infos["_final_obs"]
            assert np.array_equal(m, term | trunc)
            assert infos["final_obs"][m].shape[1] == 15
            assert (infos["episode"]["l"][m] > 0).all()
    assert seen_done
    env.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("worker", ["dp_worker.py", "dp_grad_worker.py"])
def test_ppo_data_parallel_two_ranks(worker):
    """dp_worker: two DP PPO iterations keep the ranks' parameters identical
    on disjoint env shards; dp_grad_worker: the fused-kernel 2x256 gradient
    all-reduced over 2 ranks x 16,384 rows (1 and 2 buckets) equals the
    union-minibatch gradient."""
    port = str(_free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", worker)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=300)
        outs.append(out.decode())
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, out[-3000:]
        assert f"rank {r} ok" in out
