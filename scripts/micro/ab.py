"""Interleaved A/B timing of libdronerl.so variants in ONE process (box-to-box
variance is larger than the effects being measured).  Each variant is a
separately built .so; its env_step is captured into a hipGraph of K steps
and the graphs are replayed alternately R times; medians are reported.
Usage: python scripts/micro/ab.py lib1.so lib2.so:ENV=VAL ... [--n N] [--dtype f64]
(ENV=VAL pairs are set while that library's handle is created)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)       # env-only diagnostic builds lack the PPO ABI
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--k", type=int, default=200)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--variant", type=int, default=0, help="0 gym, 2 moving")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, K = a.n, a.k
    acts = torch.rand(K, n, 4, device=dev) * 7.3575
    obs = torch.zeros(n, 18 if a.variant == 2 else 15, device=dev)
    rew = torch.zeros(n, device=dev)
    done = torch.zeros(n, dtype=torch.uint8, device=dev)
    runs = []
    for spec in a.libs:
        # "lib.so" or "lib.so:VAR=VAL,VAR=VAL" (env read by dr_create)
        path, _, envs = spec.partition(":")
        for kv in filter(None, envs.split(",")):
            k, _, val = kv.partition("=")
            os.environ[k] = val
        L = load(path)
        cfg = _lib.dr_config(num_envs=n, variant=a.variant, state_dtype=0 if a.dtype == "f64" else 1,
                             rng_mode=0, auto_reset=1, device=0, max_steps=0, seed=1,
                             env_id_offset=0, dt=0.0)
        h = ctypes.c_void_p()
        assert L.dr_create(ctypes.byref(cfg), ctypes.byref(h)) == 0
        st = torch.cuda.current_stream().cuda_stream
        L.dr_reset(h, obs.data_ptr(), st)
        for t in range(50):
            L.dr_step(h, acts[t % K].data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(), None, st)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                cs = torch.cuda.current_stream().cuda_stream
                for t in range(K):
                    L.dr_step(h, acts[t].data_ptr(), obs.data_ptr(), rew.data_ptr(),
                              done.data_ptr(), None, cs)
        torch.cuda.current_stream().wait_stream(s)
        runs.append((os.path.basename(path) + (":" + envs if envs else ""), L, h, g))
        for kv in filter(None, envs.split(",")):
            os.environ.pop(kv.partition("=")[0], None)
    torch.cuda.synchronize()
    times = {r[0]: [] for r in runs}
    for _ in range(a.reps):
        for name, L, h, g in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / K)
    print(json.dumps({k: {"median_us": round(float(np.median(v)), 3),
                          "min_us": round(float(np.min(v)), 3)} for k, v in times.items()}))


if __name__ == "__main__":
    main()
