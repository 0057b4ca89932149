"""Host wall of ONE 20-step rollout launch at 65,536 envs (bench.py --steps 20
form: raw dr_rollout call bracketed by torch.cuda.synchronize), with HIP's
default device scheduling or hipDeviceScheduleSpin set before the context
exists.  argv[1]: spin | default.  Median / p10 / p90 of 300 trials."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
mode = sys.argv[1] if len(sys.argv) > 1 else "default"
if mode == "spin":
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))          # hipDeviceScheduleSpin
    print("hipSetDeviceFlags rc", rc)
import torch  # noqa: E402

from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

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
fn = b.L.dr_rollout
args = (b.handle, K, acts.data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(), st.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
e1.record(st)
torch.cuda.synchronize()
w, g = [], []
for i in range(320):
    fn(*args)
    fn(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(st)
    fn(*args)
    e1.record(st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if i >= 20:
        w.append(dt * 1e6)
        g.append(e0.elapsed_time(e1) * 1e3)
w.sort()
g.sort()
print(mode, {"wall_us": {"p10": round(w[30], 1), "median": round(w[150], 1), "p90": round(w[270], 1)},
             "events_us_median": round(g[150], 1)})
