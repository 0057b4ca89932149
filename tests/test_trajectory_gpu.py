"""dr_gather_state and the trajectory recorder (traj_tb.py data path) on the
GPU, against a host-side replay of traj_tb.py's bookkeeping."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_gather_state_matches_get():
    from drone_rl_amd import DroneBatch, random_actions
    b = DroneBatch(1000, "moving", seed=3)
    b.reset()
    for t in range(30):
        b.step(random_actions(1000, seed=1, step=t))
    ids = torch.tensor([0, 999, 5, 5, 512], dtype=torch.int32, device="cuda")
    for f in ("pos", "omega", "target", "current_step", "ep_num", "eps", "motion"):
        assert torch.equal(b.gather(f, ids), b.get(f)[ids.long()]), f


def test_trajectory_recorder_replays_traj_tb():
    from drone_rl_amd import DroneBatch, random_actions
    from drone_rl_amd.trajectory import TrajectoryRecorder
    n, steps = 64, 400
    b = DroneBatch(n, "gym", seed=8)
    b.reset()
    blocks = []
    rec = TrajectoryRecorder(b, env_ids=(0, 7), record_interval=2, block_size=4, capacity=50,
                             on_block=lambda *a: blocks.append(a))
    # host replay of traj_tb.py:31-69 for env 0
    positions, count, buf, ref_blocks = [], 0, [], []
    for t in range(steps):
        _, _, d = b.step(random_actions(n, seed=2, step=t))
        rec.on_step(d)
        positions.append(b.get("pos")[0].cpu().numpy())
        if bool(d[0]):
            count += 1
            traj = np.array(positions[:-1])
            if count % 2 == 0:
                buf.append(traj)
            if count % 4 == 0 and buf:
                ref_blocks.append((count // 4, list(buf)))
                buf = []
            positions = []
    rec.flush()
    assert rec.episode_count == count > 8
    assert len(blocks) == len(ref_blocks)
    for (blk, s, e, trajs), (rblk, rtrajs) in zip(blocks, ref_blocks):
        assert blk == rblk and s == (blk - 1) * 4 + 1 and e == blk * 4
        assert len(trajs) == len(rtrajs)
        for x, y in zip(trajs, rtrajs):
            np.testing.assert_array_equal(x, y)
