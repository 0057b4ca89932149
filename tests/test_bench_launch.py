"""bench.py's launch forms: `python bench.py --gpus N`
starts N ranks itself; under torchrun WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--no-cpu-baseline"],
                       env=_env(WORLD_SIZE="2", RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr
    assert not r.stdout.strip()


def test_spawned_rank_failure_propagates_without_gpu():
    """With no GPU the spawned ranks fail at set_device: the launcher must
    return non-zero (not hang at a barrier, not print a line)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline",
                        "--ppo-updates", "0"],
                       env=_env(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES=""),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "exited with" in r.stderr
    assert not r.stdout.strip()


@pytest.mark.gpu
def test_direct_gpus2_starts_two_ranks():
    """The driver's BENCH form with --gpus 2, on the one-GPU box: both ranks
    share the card over gloo (RCCL refuses two ranks per device)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "20", "--warmup", "5",
                        "--ppo-updates", "1", "--no-companion", "--rollout-k", "0"],
                       env=_env(DRONERL_DIST_BACKEND="gloo"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["config"]["global_envs"] == 131072
    assert d["config"]["parallelism"].startswith("dp2")
    assert "cpu_baseline" not in d
    assert d["ppo"]["train_path"].startswith("data-parallel step")


def test_launcher_sigterm_takes_the_ranks_down():
    """A driver timeout that signals only the launcher's PID must not leave
    the ranks running (advisor r04): the launcher forwards SIGTERM and
    exits non-zero."""
    import signal
    import time

    import psutil
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline",
                          "--ppo-updates", "0"],
                         env=_env(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES=""),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    kids = []
    end = time.monotonic() + 60
    while time.monotonic() < end and len(kids) < 2:
        kids = psutil.Process(p.pid).children()
        time.sleep(0.02)
    assert len(kids) == 2
    p.send_signal(signal.SIGTERM)
    _, err = p.communicate(timeout=60)
    assert p.returncode != 0
    gone, alive = psutil.wait_procs(kids, timeout=30)
    assert not alive
