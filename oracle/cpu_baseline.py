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


def single_env(seconds: float) -> dict:
    """BASELINE.md CPU plan (i): one DroneGymEnv-equivalent, one process."""
    r = worker(1, seconds, 7)
    return {"value": round(r["steps"] / r["elapsed"], 1), "unit": "env-steps/s", "cores": 1,
            "sample": f"1 numpy-port env, DummyVecEnv auto-reset, {r['elapsed']:.2f} s"}


def numpy_batched(n: int, seconds: float) -> dict:
    """Plan (iii): VectorizedDroneEnv-style numpy-batched step of n envs in
    one process (oracle/drone_np.gym_step_batched; no resets)."""
    from oracle.drone_np import A_MAX, gym_step_batched
    rng = np.random.default_rng(3)
    s = {k: np.zeros((n, 3)) for k in ("pos", "vel", "euler", "omega", "target")}
    s["pos"][:, 2] = 1.0
    s["target"][:, 2] = 1.0
    s["step"] = np.zeros(n, np.int32)
    acts = rng.uniform(0, A_MAX, (8, n, 4)).astype(np.float32)
    steps, k = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        gym_step_batched(s, acts[k % 8])
        steps += n
        k += 1
    el = time.perf_counter() - t0
    return {"value": round(steps / el, 1), "unit": "env-steps/s", "cores": 1,
            "sample": f"{k} batched steps of {n} envs, {el:.2f} s"}


def c1_ppo(updates: int, threads: int) -> dict:
    """Plan (iv): configs[0] PPO (SB3 defaults, 1 env, 64x64) restated in
    torch-CPU (oracle/sb3_c1.py), `updates` iterations of 2048 steps."""
    import torch
    from oracle.sb3_c1 import run
    torch.set_num_threads(threads)
    r = run(steps=2048 * updates, seed=0, log_every=10 ** 9, log=lambda *_: None)
    return {"updates_per_s": round(updates / r["elapsed_s"], 4),
            "env_steps_per_s": round(2048 * updates / r["elapsed_s"], 1), "cores": threads,
            "sample": f"{updates} PPO iterations (2048 steps + 10 epochs x 32 minibatches of 64), "
                      f"{r['elapsed_s']:.1f} s, torch.set_num_threads({threads})"}


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
