"""bench.py's timing rule (verdict r04 item 1): the
barrier and the device synchronize come before t0, no torch.distributed
call runs between t0 and t1, the ranks' CLOCK_MONOTONIC spans are exchanged
after the timer, and the whole-node wall is max(t1) - min(t0)."""
import os
import socket
import sys
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_node_timing_is_max_end_minus_min_start():
    spans = [(1_000, 5_000, 3_000_000), (2_000, 9_000, 2_000_000), (1_500, 4_000, 7_000_000)]
    t = bench.node_timing(spans)
    assert t["wall_s"] == (9_000 - 1_000) / 1e9
    assert t["max_rank_s"] == 7_000 / 1e9
    assert t["gpu_ms"] == 7.0
    assert t["ranks"] == 3
    assert t["start_skew_us"] == (2_000 - 1_000) / 1e3
    one = bench.node_timing([(10, 20, 1_000_000)])
    assert one["wall_s"] == one["max_rank_s"] == 10 / 1e9 and one["gpu_ms"] == 1.0
    with pytest.raises(ValueError):
        bench.node_timing([])
    with pytest.raises(ValueError):
        bench.node_timing([(5, 4, 0)])


def test_start_deadline_world1_is_the_ready_time():
    assert bench.start_deadline(12345, 1) == 12345


def test_timed_region_single_rank_orders_sync_and_clock():
    log = []
    clock = iter(range(100, 1000, 100))
    t0, t1 = bench.timed_region(lambda: log.append("work"), lambda: log.append("sync"), 1,
                                clock=lambda: (log.append("clock"), next(clock))[1])
    assert log == ["sync", "clock", "work", "sync", "clock"]
    assert (t0, t1) == (100, 200)


_COLLECTIVES = ("barrier", "all_reduce", "all_gather", "all_gather_object", "broadcast",
                "reduce", "gather", "scatter", "reduce_scatter", "all_to_all",
                "all_gather_into_tensor", "reduce_scatter_tensor", "send", "recv")


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    for name in _COLLECTIVES:
        fn = getattr(dist, name, None)
        if fn is None:
            continue

        def rec(*a, _fn=fn, _name=name, **k):
            t = time.monotonic_ns()
            r = _fn(*a, **k)
            calls.append((_name, t, time.monotonic_ns()))
            return r
        setattr(dist, name, rec)
    # rank 1 starts its work later: the node wall must cover both ranks
    work = (lambda: time.sleep(0.05 + 0.03 * rank))
    t0, t1 = bench.timed_region(work, lambda: None, world)
    spans = bench.gather_spans((t0, t1, 1_000_000 * (rank + 1)), world)
    tm = bench.node_timing(spans)
    dist.destroy_process_group()
    q.put((rank, t0, t1, calls, spans, tm))


def test_no_collective_inside_the_timed_region_gloo_world2():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    for rank, t0, t1, calls, spans, tm in res:
        names = [c[0] for c in calls]
        assert "barrier" in names and "all_gather" in names
        # every collective either finished before t0 or started after t1
        for name, a, b in calls:
            assert b <= t0 or a >= t1, (rank, name, a, b, t0, t1)
        # the barrier precedes the timer, the exchange follows it
        assert any(n == "barrier" and b <= t0 for n, a, b in calls)
        assert any(n == "all_gather" and a >= t1 for n, a, b in calls)
        assert spans == res[0][4]                       # both ranks see the same spans
        assert tm["wall_s"] == (max(s[1] for s in spans) - min(s[0] for s in spans)) / 1e9
        assert tm["gpu_ms"] == 2.0
        assert tm["wall_s"] >= tm["max_rank_s"] >= 0.08
        # the start deadline (one all_reduce MAX before t0) lines the ranks'
        # t0 up: the skew is scheduling jitter, far below the barrier's
        assert any(n == "all_reduce" and b <= t0 for n, a, b in calls)
        assert 0 <= tm["start_skew_us"] < 5_000, tm


def test_multi_node_spans_use_the_slowest_rank(monkeypatch):
    """Advisor r05: ranks on several nodes have unrelated CLOCK_MONOTONIC
    readings, so the node wall falls back to the slowest rank's own span and
    the start alignment is skipped."""
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert not bench.single_node(2)
    spans = [(1_000, 5_000, 1_000_000), (9_000_000_000, 9_000_007_000, 2_000_000)]
    t = bench.node_timing(spans)
    assert t["wall_s"] == t["max_rank_s"] == 7_000 / 1e9 and t["start_skew_us"] is None
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert bench.single_node(2)
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert bench.single_node(2) and bench.single_node(1)
