"""Fixed cost of bench.py's timed region at small K (the driver runs
--steps 20): wall time of sync -> K-step graph replay -> sync against the
events' per-launch time, for the runtime's default wait mode and for
hipDeviceScheduleSpin / BlockingSync set before the device is initialised.
Usage: python scripts/micro/sync_overhead.py [default|spin|yield|blocking]"""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "default"
flags = {"default": None, "spin": 1, "yield": 2, "blocking": 4}[mode]
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
if flags is not None:
    assert hip.hipSetDeviceFlags(ctypes.c_uint(flags)) == 0
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

dev = torch.device("cuda", 0)
n = 65536
b = DroneBatch(n, "gym", dtype=torch.float64, device=dev, seed=2025, auto_reset=True)
b.reset()
out = {"mode": mode}
for K in (20, 200):
    acts = torch.empty(K, n, 4, device=dev)
    for t in range(K):
        random_actions(n, seed=7, step=t, out=acts[t])
    for t in range(K):
        b.step(acts[t])
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for t in range(K):
                b.step(acts[t])
    torch.cuda.current_stream(dev).wait_stream(st)
    for _ in range(3):
        g.replay()
    walls, evs = [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(40):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize(dev)
        walls.append((time.perf_counter() - t0) * 1e6)
        evs.append(e0.elapsed_time(e1) * 1e3)
    w, e = statistics.median(walls), statistics.median(evs)
    out[f"K{K}"] = {"wall_us": round(w, 1), "event_us": round(e, 1), "wall_per_step_us": round(w / K, 3),
                    "event_per_step_us": round(e / K, 3), "fixed_us": round(w - e, 1)}
print(json.dumps(out))
