"""Per-wave phase timeline of env_step_kernel from a DR_STAMPS=1 build.
Stamps (s_memrealtime, 100 MHz): 0 entry, 1 after the first sincos (euler
landed), 2 physics done, 3 reset branch done, 4 state stores issued,
5 obs stores issued; 6/7 s_memtime at entry/exit (shader clock)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import _lib  # noqa: E402

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 65536
L = ctypes.CDLL(path)
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(L, name)
    f.restype, f.argtypes = res, args
L.dr_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
dev = torch.device("cuda", 0)
acts = torch.rand(60, n, 4, device=dev) * 7.3575
obs = torch.zeros(n, 15, device=dev)
rew = torch.zeros(n, device=dev)
done = torch.zeros(n, dtype=torch.uint8, device=dev)
cfg = _lib.dr_config(num_envs=n, variant=0, state_dtype=0, rng_mode=0, auto_reset=1, device=0,
                     max_steps=0, seed=1, env_id_offset=0, dt=0.0)
h = ctypes.c_void_p()
assert L.dr_create(ctypes.byref(cfg), ctypes.byref(h)) == 0
st = torch.cuda.current_stream().cuda_stream
L.dr_reset(h, obs.data_ptr(), st)
res = []
mode = sys.argv[3] if len(sys.argv) > 3 else "sync"
graph = None
if mode == "graph":      # 20 back-to-back steps per replay; stamps = last step
    graph = torch.cuda.CUDAGraph()
    s2 = torch.cuda.Stream()
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s2):
        with torch.cuda.graph(graph, stream=s2):
            cs = torch.cuda.current_stream().cuda_stream
            for t in range(20):
                L.dr_step(h, acts[t].data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(),
                          None, cs)
    torch.cuda.current_stream().wait_stream(s2)
for t in range(60):
    if graph is not None:
        graph.replay()
    else:
        L.dr_step(h, acts[t].data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(), None, st)
    torch.cuda.synchronize()
    if t >= 40:
        nw = (n + 63) // 64
        buf = np.zeros(16384 * 8, np.uint64)
        assert L.dr_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
        s = buf[: nw * 8].reshape(nw, 8).astype(np.int64)
        t0 = s[:, 0].min()
        rel = (s[:, :6] - t0) * 10.0 / 1000.0   # us
        rs = (s[:, 6] >= s[:, 2]) & (s[:, 6] <= s[:, 3])   # reset this step
        rr = (s[rs] - t0) * 10.0 / 1000.0
        if len(rr) == 0:
            rr = np.full((1, 8), np.nan)
        res.append({"wave_start_p50_us": np.percentile(rel[:, 0], 50),
                    "wave_start_max_us": rel[:, 0].max(),
                    "first_data_p50_us": np.percentile(rel[:, 1] - rel[:, 0], 50),
                    "physics_p50_us": np.percentile(rel[:, 2] - rel[:, 1], 50),
                    "reset_p50_us": np.percentile(rel[:, 3] - rel[:, 2], 50),
                    "reset_p90_us": np.percentile(rel[:, 3] - rel[:, 2], 90),
                    "state_store_p50_us": np.percentile(rel[:, 4] - rel[:, 3], 50),
                    "obs_stage_p50_us": np.percentile(rel[:, 5] - rel[:, 4], 50),
                    "wave_life_p50_us": np.percentile(rel[:, 5] - rel[:, 0], 50),
                    "last_wave_end_us": rel[:, 5].max(),
                    "reset_uniforms_p50_us": np.percentile(rr[:, 6] - rr[:, 2], 50),
                    "reset_state_p50_us": np.percentile(rr[:, 7] - rr[:, 6], 50),
                    "reset_tail_p50_us": np.percentile(rr[:, 3] - rr[:, 7], 50)})
        buf[:] = 0
        L.dr_diag_stamps  # noqa: B018
print(json.dumps({k: round(float(np.median([r[k] for r in res])), 3) for k in res[0]}, indent=1))
