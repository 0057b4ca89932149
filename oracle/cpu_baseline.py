"""CPU baseline worker -- TEST / MEASUREMENT INFRASTRUCTURE ONLY.

The reference steps its env on the CPU, one DroneGymEnv per worker, through
SB3's VecEnv (/root/reference/train.py:33-35; SubprocVecEnv is the multi-core
form).  This module is the SubprocVecEnv-equivalent used by bench.py's
`cpu_baseline` leg: P worker processes, each owning E envs of the numpy port
(oracle/drone_np.GymDronePort, bit-exact with the reference), stepping them
serially with DummyVecEnv auto-reset semantics (terminal obs kept) on
pre-drawn U[0, 7.3575)^4 f32 actions, for a fixed wall-clock budget.  The
pipe IPC of a real SubprocVecEnv is NOT charged, so the figure is an upper
bound on the reference's CPU throughput.

Worker:   python -m oracle.cpu_baseline --envs E --seconds S --seed K
Pool:     run_pool(P, E, S) -> dict
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(n_envs: int, seconds: float, seed: int) -> dict:
    from oracle.drone_np import A_MAX, GymDronePort
    rng = np.random.default_rng(seed)
    envs = [GymDronePort(np.random.default_rng(seed * 100003 + i)) for i in range(n_envs)]
    obs = [e.reset() for e in envs]
    acts = rng.uniform(0, A_MAX, (64, n_envs, 4)).astype(np.float32)
    steps = 0
    t0 = time.perf_counter()
    k = 0
    while True:
        a = acts[k % 64]
        for i, e in enumerate(envs):
            o, r, d, info = e.step(a[i])
            if d:
                info["terminal_observation"] = o
                o = e.reset()
            obs[i] = o
        steps += n_envs
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return {"steps": steps, "elapsed": time.perf_counter() - t0}


def run_pool(procs: int, envs_per_proc: int, seconds: float) -> dict:
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1",
               MKL_NUM_THREADS="1", PYTHONPATH=ROOT)
    ps = [subprocess.Popen([sys.executable, "-m", "oracle.cpu_baseline", "--envs",
                            str(envs_per_proc), "--seconds", str(seconds), "--seed",
                            str(1000 + i)], stdout=subprocess.PIPE, env=env, cwd=ROOT)
          for i in range(procs)]
    res = []
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 10 + 120)
        if p.returncode != 0:
            raise RuntimeError("cpu baseline worker failed")
        res.append(json.loads(out.decode().strip().splitlines()[-1]))
    steps = sum(r["steps"] for r in res)
    elapsed = max(r["elapsed"] for r in res)
    return {"value": steps / elapsed, "steps": steps, "elapsed": elapsed,
            "procs": procs, "envs_per_proc": envs_per_proc}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    print(json.dumps(worker(a.envs, a.seconds, a.seed)))
