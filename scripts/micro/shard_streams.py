"""The 65,536-env random-policy step as S independent env shards (handles
with env_id_offset s*N/S, so the Philox reset draws and every output are
those of the single handle) on S HIP streams, K steps each, captured in one
hipGraph (fork / join by stream waits): per-step time of the whole batch.
  python scripts/micro/shard_streams.py [--n 65536] [--k 200] [--reps 9]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--k", type=int, default=200)
ap.add_argument("--reps", type=int, default=9)
ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4, 8])
a = ap.parse_args()
dev = torch.device("cuda", 0)
n, K = a.n, a.k
acts = torch.empty(K, n, 4, device=dev)
for t in range(K):
    random_actions(n, seed=7, step=t, out=acts[t])
graphs = {}
keep = []
for S in a.shards:
    m = n // S
    bs = [DroneBatch(m, "gym", dtype=torch.float64, device=dev, seed=2025, env_id_offset=s * m)
          for s in range(S)]
    for b in bs:
        b.reset()
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    main = torch.cuda.Stream(dev)
    main.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=main):
        for s in range(S):
            streams[s].wait_stream(main)
            with torch.cuda.stream(streams[s]):
                for t in range(K):
                    bs[s].step(acts[t, s * m:(s + 1) * m])
        for s in range(S):
            main.wait_stream(streams[s])
    torch.cuda.current_stream(dev).wait_stream(main)
    g.replay()
    torch.cuda.synchronize()
    graphs[S] = g
    keep.append((bs, streams, main))
times = {S: [] for S in a.shards}
for _ in range(a.reps):
    for S in a.shards:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graphs[S].replay()
        e1.record()
        torch.cuda.synchronize()
        times[S].append(e0.elapsed_time(e1) * 1e3 / K)
out = {f"shards{S}": {"us_per_step": round(statistics.median(v), 3),
                      "env_steps_per_s": round(n / statistics.median(v) * 1e6, 1),
                      "frac_305B": round(n * 305 / statistics.median(v) / 1e3 / 8000, 4)}
       for S, v in times.items()}
# the shards reproduce the single handle (same env ids, same actions)
ref = keep[0][0][0].get("pos") if a.shards[0] == 1 else None
if ref is not None:
    for (bs, _, _), S in zip(keep[1:], a.shards[1:]):
        pos = torch.cat([b.get("pos") for b in bs])
        out[f"shards{S}"]["pos_equal_to_single"] = bool(torch.equal(pos, ref))
print(json.dumps(out))
