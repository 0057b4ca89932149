"""Start skew of bench.timed_region across W gloo ranks on the CPU (max t0 -
min t0 of the ranks' CLOCK_MONOTONIC spans), with and without the common
start deadline (bench.start_deadline); 30 regions each, median and max.

  python scripts/micro/start_skew.py 8
"""
import json
import os
import socket
import sys
import time

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def worker(rank, world, port, q):
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    for align in (False, True):
        sk = []
        for _ in range(30):
            span = bench.timed_region(lambda: time.sleep(0.0002), lambda: None, world, align=align)
            spans = bench.gather_spans((*span, 0), world)
            sk.append(bench.node_timing(spans)["start_skew_us"])
        sk.sort()
        res["aligned" if align else "barrier_only"] = {"median_us": round(sk[len(sk) // 2], 1),
                                                       "max_us": round(sk[-1], 1)}
    dist.destroy_process_group()
    if rank == 0:
        q.put(res)


if __name__ == "__main__":
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, W, port, q)) for r in range(W)]
    for p in ps:
        p.start()
    out = q.get(timeout=300)
    for p in ps:
        p.join(60)
    print(json.dumps({"world": W, "backend": "gloo (CPU)", **out}))
