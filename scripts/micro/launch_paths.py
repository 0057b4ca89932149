"""Host wall of ONE 20-step rollout-kernel launch at 65,536 envs (the driver's
bench.py --steps 20 form) by launch path: graph replay, DroneBatch.rollout,
and a raw ctypes call with prebuilt arguments.  Median of 200 trials, each
bracketed by synchronize like bench.py's timed region; "/none" without the
event pair, "timed/*" through dr_rollout_timed (the events bound to the
dispatch packet's timestamps)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from drone_rl_amd import DroneBatch, random_actions  # noqa: E402
from drone_rl_amd._lib import lib  # noqa: E402

N, K = 65536, 20
dev = torch.device("cuda", 0)
b = DroneBatch(N, "gym", dtype=torch.float64, device=dev, seed=2025, auto_reset=True)
b.reset()
acts = torch.empty(K, N, 4, device=dev)
for t in range(K):
    random_actions(N, seed=7, step=t, out=acts[t])
obs = torch.empty(K, N, 15, device=dev)
rew = torch.empty(K, N, device=dev)
done = torch.empty(K, N, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
L = lib()
fn = L.dr_rollout
args = (b.handle, K, acts.data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(), st.cuda_stream)


def py():
    b.rollout(K, acts, obs_out=obs, rew_out=rew, done_out=done)


def raw():
    fn(*args)


cs = torch.cuda.Stream(dev)
cs.wait_stream(st)
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(cs), torch.cuda.graph(g, stream=cs):
    py()
st.wait_stream(cs)
res = {}


def sync_dev():
    torch.cuda.synchronize()


def sync_ev_then_dev(e1):
    e1.synchronize()
    torch.cuda.synchronize()


E0, E1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
E0.record(st)
E1.record(st)
torch.cuda.synchronize()
ftimed = L.dr_rollout_timed
targs = args + (E0.cuda_event, E1.cuda_event)


def timed():
    ftimed(*targs)


def trial(f, how):
    torch.cuda.synchronize()
    e0, e1 = E0, E1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if f is timed:                  # the events ride on the dispatch packet
        f()
    elif how == "none":
        f()
    else:
        e0.record(st)
        f()
        e1.record(st)
    if how in ("dev", "none"):
        sync_dev()
    else:
        sync_ev_then_dev(e1)
    dt = time.perf_counter() - t0
    return dt, (0.0 if how == "none" and f is not timed else e0.elapsed_time(e1) * 1e3)


for name, f in (("graph", g.replay), ("python", py), ("raw_ctypes", raw), ("timed", timed)):
    for how in ("dev", "ev", "none"):
        if f is timed and how == "none":
            continue
        for _ in range(20):
            f()
        torch.cuda.synchronize()
        time.sleep(0.5)                 # idle, then one single-shot trial
        first = trial(f, how)
        w, e = [], []
        for _ in range(200):
            a, b_ = trial(f, how)
            w.append(a)
            e.append(b_)
        w.sort()
        e.sort()
        res[f"{name}/{how}"] = {"first": (round(first[0] * 1e6, 1), round(first[1], 1)),
                                "median": (round(w[100] * 1e6, 1), round(e[100], 1)),
                                "p10": round(w[20] * 1e6, 1), "p90": round(w[180] * 1e6, 1)}
for k, v in res.items():
    print(k, v)
