"""Host wall of the headline's timed region (one 20-step dr_rollout launch
at 65,536 envs + torch.cuda.synchronize) with its event pair recorded three
ways: torch.cuda.Event.record, hipEventRecord through ctypes, and none
(plain launch).  Interleaved, median of TRIALS each.

  python scripts/micro/host_events.py
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

TRIALS = int(os.environ.get("TRIALS", "300"))
hip = ctypes.CDLL("libamdhip64.so")
hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipEventRecord.restype = ctypes.c_int
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
E0, E1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
E0.record(st)
E1.record(st)
n, k = 65536, 20
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
e0, e1, s = E0.cuda_event, E1.cuda_event, st.cuda_stream
rec = hip.hipEventRecord


def torch_ev():
    E0.record(st)
    fn(*args)
    E1.record(st)


def ctypes_ev():
    rec(e0, s)
    fn(*args)
    rec(e1, s)


def plain():
    fn(*args)


forms = {"torch_events": torch_ev, "ctypes_hipEventRecord": ctypes_ev, "plain": plain}
walls = {f: [] for f in forms}
gpu = {f: [] for f in forms}
for i in range(TRIALS + 10):
    for name, w in forms.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if i >= 10:
            walls[name].append((t1 - t0) * 1e6)
            if name != "plain":
                gpu[name].append(E0.elapsed_time(E1) * 1e3)
res = {}
for name in forms:
    w = sorted(walls[name])
    res[name] = {"wall_us_median": round(w[len(w) // 2], 2), "wall_us_p10": round(w[len(w) // 10], 2)}
    if gpu[name]:
        g = sorted(gpu[name])
        res[name]["events_us_median"] = round(g[len(g) // 2], 2)
print(json.dumps(res), flush=True)
b.close()
