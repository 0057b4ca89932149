"""Host wall of one dr_rollout launch + torch.cuda.synchronize under the
runtime's host-side settings the caller's environment selects (run once per
setting, each in a fresh process): the near-empty probe launch (64 envs, one
step) and the headline's 20-step launch at 65,536 envs, each with and without
the bench's event pair around the launch.  Median of 200 trials.

  HSA_ENABLE_INTERRUPT=0 python scripts/micro/host_wait.py [--spin]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

ap = argparse.ArgumentParser()
ap.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) first")
ap.add_argument("--trials", type=int, default=200)
a = ap.parse_args()
if a.spin:
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0

import torch  # noqa: E402

from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
res = {"env": {k: os.environ.get(k) for k in ("HSA_ENABLE_INTERRUPT", "AMD_DIRECT_DISPATCH",
                                             "HIP_FORCE_DEV_KERNARG")},
       "spin": a.spin}
E0, E1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
E0.record(st)
E1.record(st)
for n, k in ((64, 1), (65536, 20)):
    b = DroneBatch(n, "gym", dtype=torch.float64, device=dev, seed=2025, auto_reset=True)
    b.reset()
    acts = torch.empty(k, n, 4, device=dev)
    for t in range(k):
        random_actions(n, seed=7, step=t, out=acts[t])
    obs = torch.empty(k, n, 15, device=dev)
    rew = torch.empty(k, n, device=dev)
    done = torch.empty(k, n, dtype=torch.uint8, device=dev)
    args = (b.handle, k, acts.data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(),
            st.cuda_stream)
    fn = b.L.dr_rollout
    for ev in (False, True):
        walls, gpu = [], []
        for i in range(a.trials + 10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if ev:
                E0.record(st)
            fn(*args)
            if ev:
                E1.record(st)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if i >= 10:
                walls.append((t1 - t0) * 1e6)
                if ev:
                    gpu.append(E0.elapsed_time(E1) * 1e3)
        walls.sort()
        key = f"n{n}_k{k}_" + ("events" if ev else "plain")
        res[key] = {"wall_us_median": round(walls[len(walls) // 2], 2),
                    "wall_us_p10": round(walls[len(walls) // 10], 2)}
        if gpu:
            gpu.sort()
            res[key]["events_us_median"] = round(gpu[len(gpu) // 2], 2)
    if n == 65536:
        # bench.py's exact sequence before its one timed launch (two plain
        # repetitions, six dispatch-packet-timed ones), then the timed region
        # with torch.cuda.synchronize(device) or torch.cuda.synchronize()
        import gc

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__)))))
        import bench
        P0, P1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        P0.record(st)
        P1.record(st)
        for ext in (True, False):
            for dev_arg in (True, False):
                walls = []
                for rep in range(30):
                    for _ in range(2):
                        fn(*args)
                    if ext:
                        for _ in range(6):
                            b.L.dr_rollout_timed(*args, P0.cuda_event, P1.cuda_event)
                            torch.cuda.synchronize(dev)

                    def work():
                        E0.record(st)
                        fn(*args)
                        E1.record(st)
                    gc.disable()
                    sy = (lambda: torch.cuda.synchronize(dev)) if dev_arg else torch.cuda.synchronize
                    t0, t1 = bench.timed_region(work, sy, 1)
                    gc.enable()
                    walls.append((t1 - t0) / 1e3)
                first = walls[:3]
                walls = sorted(walls)
                res[f"bench_seq_ext{int(ext)}_devarg{int(dev_arg)}"] = {
                    "first_three_us": [round(w, 2) for w in first],
                    "wall_us_median": round(walls[len(walls) // 2], 2),
                    "wall_us_min": round(walls[0], 2), "wall_us_max": round(walls[-1], 2)}
    b.close()
print(json.dumps(res))
