"""Diagnostic: does splitting the 65,536-env step into S shards on S streams
(captured into one hipGraph with fork/join) overlap the per-kernel launch
boundary?  Compares per-step time of 1 handle vs S handles on S streams."""
import sys

import torch

sys.path.insert(0, ".")
from drone_rl_amd import DroneBatch, random_actions  # noqa: E402

N, K = 65536, 200
dev = torch.device("cuda", 0)
acts = torch.empty(K, N, 4, device=dev)
for t in range(K):
    random_actions(N, seed=7, step=t, out=acts[t])


def run(S, graph=True, reps=7):
    n = N // S
    bs = [DroneBatch(n, "gym", seed=2025, env_id_offset=j * n) for j in range(S)]
    for b in bs:
        b.reset()
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    main = torch.cuda.current_stream(dev)

    def body():
        for t in range(K):
            for j, b in enumerate(bs):
                with torch.cuda.stream(streams[j]):
                    b.step(acts[t, j * n:(j + 1) * n])

    def capture():
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g, stream=cs):
                cur = torch.cuda.current_stream(dev)
                for s in streams:
                    s.wait_stream(cur)
                body()
                for s in streams:
                    cur.wait_stream(s)
        main.wait_stream(cs)
        return g

    g = capture() if graph else None
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if graph:
            g.replay()
        else:
            for s in streams:
                s.wait_stream(main)
            body()
            for s in streams:
                main.wait_stream(s)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / K)
    ts.sort()
    return ts[len(ts) // 2]


for S in (1, 2, 4):
    print(f"S={S}: graph {run(S):.3f} us/step")
