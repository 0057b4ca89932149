"""GIF recording of the single-env facade (the reference's DroneEnv
start_record / render / stop_record, drone.py:189-248, driven by test.py:9-21).

CPU: the drawing helpers -- the rotation (drone.py:161-174) against the
reference's column-2 use in the physics (R[:, 2] is the thrust direction the
golden step vectors were generated with), the motor layout, and a GIF of N
grabbed frames.  GPU: test.py end to end (an SB3 .zip from the GPU trainer,
deterministic predict, render per step, reset on done)."""
import numpy as np
import pytest

from drone_rl_amd.render import DroneRecorder, motor_positions, rotation_matrix


def test_rotation_matrix_is_the_reference_zyx_rotation():
    rng = np.random.default_rng(0)
    for _ in range(200):
        e = rng.uniform(-4, 4, 3)
        R = rotation_matrix(e)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert abs(np.linalg.det(R) - 1) < 1e-12
        phi, th, psi = e
        Rz = np.array([[np.cos(psi), -np.sin(psi), 0], [np.sin(psi), np.cos(psi), 0], [0, 0, 1]])
        Ry = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
        Rx = np.array([[1, 0, 0], [0, np.cos(phi), -np.sin(phi)], [0, np.sin(phi), np.cos(phi)]])
        np.testing.assert_allclose(R, Rz @ Ry @ Rx, atol=1e-12)


def test_motor_layout_at_rest():
    m = motor_positions([1.0, 2.0, 3.0], [0, 0, 0], 0.5)
    a = 0.5 / np.sqrt(2)
    np.testing.assert_allclose(m, [[1 + a, 2 + a, 3], [1 - a, 2 + a, 3], [1 - a, 2 - a, 3],
                                   [1 + a, 2 - a, 3]], atol=1e-15)


def test_recorder_writes_a_gif_with_one_frame_per_render(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    rec = DroneRecorder()
    out = tmp_path / "run.gif"
    rec.start_record(str(out), dpi=40, fps=20)
    for k in range(4):
        rec.render([0.1 * k, 0, 1 + 0.1 * k], [0.1 * k, -0.05 * k, 0.2], [0, 0, 1], 0.5)
    rec.stop_record()
    rec.close()
    im = PIL.open(out)
    assert im.format == "GIF" and getattr(im, "n_frames", 1) == 4


@pytest.mark.gpu
def test_eval_gif_like_reference_test_py(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    from drone_rl_amd.eval_gif import run
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    tr = PPOTrainer(PPOConfig(num_envs=256, n_steps=8, batch_size=512, n_epochs=1,
                              net_arch=(64, 64), seed=3))
    tr.learn_step()
    ck = tmp_path / "dd.zip"
    tr.save_sb3(ck)
    tr.close()
    out = tmp_path / "my_drone_run.gif"
    r = run(str(ck), str(out), steps=6, dpi=40, fps=20, seed=1)
    assert r["frames"] == 6 and np.isfinite(r["return"])
    im = PIL.open(out)
    assert im.format == "GIF" and im.n_frames == 6


@pytest.mark.gpu
def test_gym_render_keeps_the_reference_signature():
    """advisor r02: DroneGymEnv.render(mode="human", close=False) as the
    reference declares it (drone.py:273); callers passing a mode still draw."""
    import matplotlib
    matplotlib.use("Agg")
    from drone_rl_amd import DroneGymEnv
    env = DroneGymEnv()
    env.reset()
    for args, kw in (((), {}), (("human",), {}), (("rgb_array", False), {}),
                     ((), {"mode": "human", "close": False})):
        m = env.render(*args, **kw)
        assert np.asarray(m).shape == (4, 3)
    env.close()
