"""Benchmark: batched quadrotor env-steps/s on MI355X (BASELINE.json configs[1]).

Workload (N=1 GPU): 65,536 DroneGymEnv-equivalent envs per GPU, synthetic
random policy (actions i.i.d. U[0, 7.3575)^4 f32 from Philox, pre-generated
and resident in HBM before the timed region), DummyVecEnv auto-reset inside
the step, f64 state (the reference's precision), every step's obs / reward /
done written to HBM.  One "step" = one env step of the whole batch.  The
headline runs the steps through the K-step rollout kernel (dr_rollout: up to
32 steps per launch, the state in registers between steps; its outputs are
bitwise those of K single dr_step launches, tests/test_rollout_gpu.py); the
launches are captured in one hipGraph and replayed, bracketed by barrier +
synchronize on both sides; the max over ranks is taken.  `--headline step`
times one dr_step launch per step instead (the kernel PPO's rollout uses;
always reported as `single_step`).

Multi-GPU: one process per GPU, independent env shards (global env ids
rank*N+i), no data-path collective -> "scaling": "weak".  Two launch forms:
under torchrun (WORLD_SIZE set; it must equal --gpus), or directly as
`python bench.py --gpus N`, where this process starts the N ranks itself
(spawn_ranks; it never touches the GPU) and rank 0 prints the line.

The JSON line also carries
  roofline      the headline kernel: algorithmic bytes per launch (per env-
                step 81 B of actions / obs / reward / done, plus the f64 state
                read and written once per launch: 224 B / K)
                over its per-launch GPU time: for a direct launch (the
                driver's --steps 20) the dispatch-packet timestamps of the
                same launches repeated right before the timed region (the
                value's region holds the launches alone; an instrumented
                region with a HIP event pair around them is timed first and
                reported beside it), for a graph replay HIP events on the
                launch stream across the timed region;
  single_step   the same envs through one dr_step launch per step (305 B per
                env-step in f64), with its own roofline block;
  cpu_baseline  rank 0, N=1: the SubprocVecEnv-equivalent process pool over
                the fixture-pinned numpy port (oracle/cpu_baseline.py),
                run BEFORE the GPU is touched;
  ppo           PPO updates/s for configs[2] (65,536 envs, 2x256 tanh MLP,
                GAE lambda 0.95), when --ppo-updates > 0, with a roofline
                block: FLOP per update over the update time
                against the f32 matrix peak, and every kernel of one
                optimizer step timed by HIP events (MFMA fraction of the
                256x256 GEMMs, HBM fraction of the memory-bound kernels);
  rollout_kernel  K = 32 rollout-kernel launches with actions from HBM and
                with the random policy drawn in the kernel.
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BYTES_PER_ENV_STEP = {"f64": 305, "f32": 197}
# moving-target variant: + 9 f32 motion params read, + 3 f32 obs written
BYTES_PER_ENV_STEP_MOVING = {"f64": 353, "f32": 245}
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
# numbers read from committed profiles whose kernel sources differ from this
# tree's (committed_profile): reported in the line's committed_artefacts
# block, labelled stale, never inside a live block
ARTEFACTS = {}
# the headline's node timing at world > 1 (node_timing's rank figures),
# reported in the line beside the value
HEADLINE_NODE = {}
# the headline's walls with and without the HIP event pair (direct launches)
HEADLINE_WALLS = {}


def _atoi(v):
    """C atoi(): leading whitespace, an optional sign and the leading
    digits; 0 when there are none (how launch_rollout reads its env knobs)."""
    v = v.lstrip()
    i = 1 if v[:1] in "+-" else 0
    j = i
    while j < len(v) and v[j].isdigit():
        j += 1
    return int(v[:j]) if j > i else 0


def rollout_kernel_name(n_envs, n_cu, gen, variant="gym"):
    """The kernel dr_rollout launches for n_envs envs on a device with n_cu
    CUs -- the rule of launch_rollout (csrc/env_kernels.hip): the
    warp-specialised forms while the grid is at most one 256-env block per CU
    (DRONERL_ROLLOUT_WS=0/1 forces), of which the split-physics form for the
    gym variant with actions read from HBM; the one-role rollout kernel above
    that."""
    ws_env = os.environ.get("DRONERL_ROLLOUT_WS")
    ws = _atoi(ws_env) != 0 if ws_env is not None else n_envs <= 256 * n_cu
    if variant == "gym" and ws and not gen:
        return "env_rollout_ab_kernel"
    return "env_rollout_ws_kernel" if ws else "env_rollout_kernel"


PROVENANCE_JSON = os.path.join(ROOT, "profiles", "provenance.json")


def kernel_source_hash():
    """sha256 over the sources of libdronerl.so (csrc/*.hip, *.h, the
    Makefile and include/dronerl.h, in name order): what a committed
    profile was measured on.  Computed the same way here and on the GPU box
    (the sources travel with the tree)."""
    import hashlib
    csrc = os.path.join(ROOT, "drone_rl_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc)
                   if f.endswith((".hip", ".h")) or f == "Makefile")
    h = hashlib.sha256()
    for rel in [os.path.join("drone_rl_amd", "csrc", f) for f in files] + \
            [os.path.join("include", "dronerl.h")]:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def committed_profile(path, current_hash=None):
    """Provenance of a committed profile (profiles/provenance.json: the
    kernel_source_hash of the tree it was measured on): {"source": path
    relative to the repo, "matches_tree": bool, "measured_on": hash prefix}.
    Numbers read from a profile that does not match the current kernel
    sources are never mixed into the live blocks of the line (they go to
    the line's committed_artefacts block, labelled stale)."""
    rel = os.path.relpath(path, ROOT)
    try:
        prov = json.load(open(PROVENANCE_JSON))
    except (OSError, ValueError):
        prov = {}
    rec = prov.get(os.path.basename(path), {})
    h = rec.get("source_hash")
    cur = current_hash or kernel_source_hash()
    return {"source": rel, "matches_tree": bool(h) and h == cur,
            "measured_on": (h or "unknown")[:12]}


def committed_or_stale(key, path, value):
    """value (read from the committed profile at path) when that profile
    was measured on this tree's kernel sources, with its source; otherwise
    None here and the value filed under ARTEFACTS[key], labelled stale."""
    if value is None:
        return None
    prov = committed_profile(path)
    if prov["matches_tree"]:
        return dict(value, provenance=prov) if isinstance(value, dict) else \
            {"value": value, "provenance": prov}
    ARTEFACTS[key] = dict(prov, stale=True, values=value)
    return None


def pmc_rollout_valu_active(path):
    """SQ_ACTIVE_INST_VALU over the physics waves' share of SQ_WAVE_CYCLES of
    the K = 32 rollout kernel at 65,536 envs, per action source, from the
    committed PMC summary (scripts/pmc_summary.py output), or {} when absent."""
    try:
        d = json.load(open(path))
        return {k: d[k]["valu_active_frac_of_wave_cycles"]
                for k in ("actions_from_hbm", "random_policy_in_kernel") if k in d}
    except (OSError, ValueError, KeyError, TypeError):
        return {}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--state-dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph-warm-replays", type=int, default=1,
                    help="untimed replays of the captured step graph before the timed one")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-companion", action="store_true",
                    help="skip the 4,194,304-env companion measurement")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--ppo-updates", type=int, default=3,
                    help="timed PPO iterations for configs[2] (0 = skip)")
    ap.add_argument("--ppo-epochs", type=int, default=10)
    ap.add_argument("--grad-buckets", type=int, choices=[1, 2], default=1,
                    help="data-parallel gradient all-reduces per optimizer step")
    ap.add_argument("--ppo-steps", type=int, default=32, help="rollout length T")
    ap.add_argument("--extra", action="store_true",
                    help="also time the f32-state mode and the 4M-env size")
    ap.add_argument("--rollout-k", type=int, default=32,
                    help="steps per launch of the K-step rollout kernel line (0 = skip)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--kernel-stats",
                    default=os.path.join(ROOT, "profiles", "r06_kernel_stats.csv"),
                    help="rocprofv3 --stats csv whose kernel averages the ppo block reports")
    ap.add_argument("--rollout-grid-stats",
                    default=os.path.join(ROOT, "profiles", "r06_rollout_grid_stats.json"),
                    help="scripts/kernel_grid_stats.py output: the headline kernel's rocprof "
                         "durations at K = 32 on 65,536 envs")
    ap.add_argument("--pmc-rollout",
                    default=os.path.join(ROOT, "profiles", "r06_pmc_rollout.json"),
                    help="scripts/pmc_summary.py output of the K = 32 rollout kernel (its "
                         "VALU-active fractions are reported when it matches the tree)")
    ap.add_argument("--headline", choices=["rollout", "step"], default="rollout",
                    help="kernel of the headline value: the K-step rollout kernel or one "
                         "dr_step launch per step")
    ap.add_argument("--headline-k", type=int, default=32,
                    help="max steps per rollout-kernel launch in the headline")
    return ap.parse_args()


# Start alignment at world > 1: after the barrier and the device
# synchronize, the ranks agree on a common CLOCK_MONOTONIC deadline (the
# latest rank's ready time + this margin, one all_reduce MAX, still before
# t0) and spin until it, so that the barrier's release skew between the
# ranks' host threads does not enter the node wall max(t1) - min(t0).
START_MARGIN_NS = int(os.environ.get("DRONERL_START_MARGIN_NS", "2000000"))


def single_node(world):
    """Whether all `world` ranks share this node's CLOCK_MONOTONIC: torchrun's
    LOCAL_WORLD_SIZE equals WORLD_SIZE (spawn_ranks sets both; absent = one
    process).  Across nodes the monotonic clocks are unrelated, so the start
    alignment and the node wall max(t1) - min(t0) apply on one node only
    (advisor r05)."""
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return world <= 1 or lw is None or _atoi(lw) == world


def start_deadline(ready_ns, world, device=None, margin_ns=START_MARGIN_NS):
    """The common start time: max over ranks of ready_ns, plus margin_ns
    (one all_reduce MAX of an int64, on the device under RCCL)."""
    if world == 1:
        return ready_ns
    import torch
    import torch.distributed as dist
    dev = device if (device is not None and dist.get_backend() == "nccl") else "cpu"
    t = torch.tensor([ready_ns], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item()) + margin_ns


def timed_region(work, sync, world, clock=time.monotonic_ns, device=None, align=True):
    """The timing rule of every bench leg: a barrier
    and a device synchronize come BEFORE t0; at world > 1 the ranks then
    agree on a common start deadline and spin until it (start_deadline,
    also before t0); then t0, the work, a device synchronize and t1.  No
    torch.distributed call runs between t0 and t1 (at --steps 20 the timed
    region is one ~38 us launch, which an RCCL barrier across 8 GPUs would
    rival).  Returns (t0, t1) in ns of CLOCK_MONOTONIC, the clock every
    process of one node shares, so the ranks' spans can be compared after
    the timer (node_timing)."""
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    sync()
    if world > 1 and align and single_node(world):
        deadline = start_deadline(clock(), world, device)
        # bounded: a deadline far ahead means the clocks are not shared
        if deadline - clock() <= 100 * START_MARGIN_NS:
            while clock() < deadline:
                pass
    t0 = clock()
    work()
    sync()
    t1 = clock()
    return t0, t1


def gather_spans(span, world, device=None):
    """Every rank's (t0_ns, t1_ns, gpu_ns) of one timed region, exchanged
    AFTER the timer (one all_gather of 3 int64); [span] at world 1."""
    span = tuple(int(v) for v in span)
    if world == 1:
        return [span]
    import torch
    import torch.distributed as dist
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor(span, dtype=torch.int64, device=dev)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [tuple(int(v) for v in o.tolist()) for o in out]


def node_timing(spans):
    """Pure arithmetic over every rank's (t0_ns, t1_ns, gpu_ns): the whole
    node's wall of the timed region, max(t1) - min(t0) (CLOCK_MONOTONIC is
    shared by the node's processes; it covers the slowest rank and any skew
    between the ranks' starts), the slowest rank's own span, and the max
    over ranks of the GPU time.  Seconds / ms."""
    if not spans:
        raise ValueError("no spans")
    t0 = min(s[0] for s in spans)
    t1 = max(s[1] for s in spans)
    if any(s[1] < s[0] for s in spans):
        raise ValueError("a span ends before it starts")
    if not single_node(len(spans)):
        # ranks on several nodes: no shared clock, the slowest rank's span
        slow = max(s[1] - s[0] for s in spans) / 1e9
        return {"wall_s": slow, "max_rank_s": slow,
                "gpu_ms": max(s[2] for s in spans) / 1e6, "start_skew_us": None,
                "ranks": len(spans), "clock": "per-rank spans (multi-node)"}
    return {"wall_s": (t1 - t0) / 1e9,
            "max_rank_s": max(s[1] - s[0] for s in spans) / 1e9,
            "gpu_ms": max(s[2] for s in spans) / 1e6,
            "start_skew_us": (max(s[0] for s in spans) - t0) / 1e3,
            "ranks": len(spans)}


def cpu_share():
    """(P, affinity, why): the worker count for the CPU baseline.  P is the
    affinity count (P = len(os.sched_getaffinity(0))), lowered
    only to the CPU share this process is actually granted: a cgroup CPU
    quota, or the OMP_NUM_THREADS the GPU box sets to its per-GPU share
    (there the affinity mask shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    caps = {}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            caps["cgroup cpu.max quota"] = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        caps["OMP_NUM_THREADS"] = int(omp)
    p, why = aff, "sched_getaffinity"
    for k, v in caps.items():
        if v < p:
            p, why = v, k
    return p, aff, why


def cpu_baseline(seconds):
    from oracle.cpu_baseline import c1_ppo, cpu_model, numpy_batched, run_pool, single_env
    procs, aff, why = cpu_share()
    envs = 65536 // procs       # configs[1]'s 65,536 envs split across the workers
    r = run_pool(procs, envs, seconds)
    # BASELINE.md CPU plan (i), (iii), (iv) beside the headline (ii)
    plan = {"single_env": single_env(seconds),
            "numpy_batched_65536": numpy_batched(65536, seconds),
            "c1_ppo_sb3_defaults": c1_ppo(2, procs)}
    return {"value": round(r["value"], 1), "unit": "env-steps/s", "cores": procs,
            "affinity_cpus": aff, "cores_limited_by": why,
            "kind": "port",
            "sample": (f"{procs} worker processes x {envs} numpy-port envs (65,536 split "
                       f"across the workers; oracle/drone_np, "
                       f"bit-exact vs reference), random U[0,7.3575)^4 actions, DummyVecEnv "
                       f"auto-reset, {r['elapsed']:.2f} s wall each ({r['steps']} env-steps); "
                       f"SubprocVecEnv-equivalent without pipe IPC; CPU: {cpu_model()}"),
            "plan": plan}


def time_env(args, dtype_name, n_envs, rank, world, device, steps, warmup, variant="gym"):
    import torch

    from drone_rl_amd import DroneBatch, random_actions
    dtype = torch.float64 if dtype_name == "f64" else torch.float32
    b = DroneBatch(n_envs, variant, dtype=dtype, device=device, seed=2025,
                   env_id_offset=rank * n_envs, auto_reset=True)
    b.reset()
    total = warmup + steps
    # inputs resident in HBM before the timed region
    acts = torch.empty(total, n_envs, 4, dtype=torch.float32, device=device)
    for t in range(total):
        random_actions(n_envs, seed=7, step=t, env_id_offset=rank * n_envs, out=acts[t])
    for t in range(warmup):
        b.step(acts[t])
    stream = torch.cuda.current_stream(device)
    graph = None
    if not args.no_graph:
        s = torch.cuda.Stream(device)
        s.wait_stream(stream)
        with torch.cuda.stream(s):
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                for t in range(warmup, total):
                    b.step(acts[t])
        stream.wait_stream(s)
        # untimed replays of the captured graph: its first launch uploads
        # the graph to the device; the env simply runs K more warm-up steps
        # on the same pre-generated actions
        for _ in range(args.graph_warm_replays):
            graph.replay()
    torch.cuda.synchronize(device)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    for e in (ev0, ev1):
        e.record(stream)        # the events' lazy creation stays out of the timed region

    def work():
        ev0.record(stream)
        if graph is not None:
            graph.replay()
        else:
            for t in range(warmup, total):
                b.step(acts[t])
        ev1.record(stream)
    span = timed_region(work, torch.cuda.synchronize, world, device=device)
    tm = node_timing(gather_spans((*span, round(ev0.elapsed_time(ev1) * 1e6)), world, device))
    elapsed, gpu_ms = tm["wall_s"], tm["gpu_ms"]
    # sanity: the env is alive (episodes end and reset under a random policy)
    ep = b.get("ep_num").float().mean().item()
    b.close()
    del graph
    return elapsed, gpu_ms, ep


def time_headline(args, n_envs, rank, world, device, steps, warmup, kmax):
    """The headline: `warmup` untimed then `steps` timed env steps of the
    batch through dr_rollout, in launches of at most kmax steps (actions
    pre-generated in HBM, outputs of every step written).  The timed launches
    are one captured hipGraph when there are more than four of them
    (replayed once untimed first: its first launch uploads it; the env simply
    runs those steps again on the same actions), else direct C-ABI calls
    with prebuilt arguments (repeated three times untimed first).
    Returns (wall seconds, GPU ms over the timed launches, launches, mean ep_num)."""
    import torch

    from drone_rl_amd import DroneBatch, random_actions
    dtype = torch.float64 if args.state_dtype == "f64" else torch.float32
    b = DroneBatch(n_envs, "gym", dtype=dtype, device=device, seed=2025,
                   env_id_offset=rank * n_envs, auto_reset=True)
    b.reset()
    total = warmup + steps
    acts = torch.empty(total, n_envs, 4, dtype=torch.float32, device=device)
    for t in range(total):
        random_actions(n_envs, seed=7, step=t, env_id_offset=rank * n_envs, out=acts[t])
    k0 = min(kmax, max(steps, warmup, 1))
    obs = torch.empty(k0, n_envs, b.obs_dim, device=device)
    rew = torch.empty(k0, n_envs, device=device)
    done = torch.empty(k0, n_envs, dtype=torch.uint8, device=device)

    def run(t0, t1):
        n = 0
        while t0 < t1:
            k = min(k0, t1 - t0)
            b.rollout(k, acts[t0:t0 + k], obs_out=obs[:k], rew_out=rew[:k], done_out=done[:k])
            t0 += k
            n += 1
        return n
    run(0, warmup)
    stream = torch.cuda.current_stream(device)
    launches = -(-steps // k0)
    g = None
    if launches > 4 and not args.no_graph:
        # many launches: one graph replay instead of a host launch each
        cs = torch.cuda.Stream(device)
        cs.wait_stream(stream)
        with torch.cuda.stream(cs):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cs):
                run(warmup, total)
        stream.wait_stream(cs)
        g.replay()
        timed = g.replay
    else:
        # a few launches (the driver's --steps 20 is ONE): the C ABI called
        # directly with prebuilt arguments (scripts/micro/launch_paths.py:
        # 42.6 us host wall for one 20-step launch against 51.8 through a
        # graph replay), after untimed repetitions of the same launches (the
        # env simply runs those steps again on the same actions)
        calls = []
        t = warmup
        while t < total:
            k = min(k0, total - t)
            calls.append((b.handle, k, acts[t].data_ptr(), obs.data_ptr(), rew.data_ptr(),
                          done.data_ptr(), stream.cuda_stream))
            t += k
        fn = b.L.dr_rollout

        rcs = []

        def timed():
            for c in calls:
                rcs.append(fn(*c))
        for _ in range(2):
            timed()
    torch.cuda.synchronize(device)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    pk0 = torch.cuda.Event(enable_timing=True)
    pk1 = torch.cuda.Event(enable_timing=True)
    for e in (ev0, ev1, pk0, pk1):
        e.record(stream)        # the events' lazy creation stays out of the timed region
    packet_ms = None
    if g is None:
        # untimed repetitions right before the timed one, through
        # dr_rollout_timed: their events ride on the dispatch packets
        # (hipExtLaunchKernel), i.e. the kernels' own start / end timestamps,
        # the durations rocprofv3 reports (the timed launches below stay plain
        # dr_rollout calls: the extended launch costs ~3 us more host wall,
        # scripts/micro/launch_paths.py).  The first extended launch of a
        # process is a warm-up (BENCH_r03 read 95.9 us from a single one
        # against 28.6 us by events); the median of 5 after it is reported.
        reps = []
        for rep in range(6):
            for i, c in enumerate(calls):
                rcs.append(b.L.dr_rollout_timed(*c, pk0.cuda_event if i == 0 else None,
                                                pk1.cuda_event if i == len(calls) - 1 else None))
            torch.cuda.synchronize(device)
            if rep > 0:
                reps.append(pk0.elapsed_time(pk1))
        packet_ms = sorted(reps)[len(reps) // 2]
    def work_events():
        ev0.record(stream)
        timed()
        ev1.record(stream)
    if g is None:
        # one untimed rehearsal of the whole timed region (event records,
        # launch, synchronize; the env runs those steps again on the same
        # actions).  Round 5: the single timed launch read 41.3-42.3 us of
        # wall where repetitions of the identical sequence in one process
        # have a 37-39 us median (scripts/micro/host_wait.py); with this
        # rehearsal and the no-argument torch.cuda.synchronize (no device-
        # guard switch around it) it reads 38.1-39.2 us (3 runs, one box)
        timed_region(work_events, torch.cuda.synchronize, world, device=device)
    gc.disable()
    span_ev = timed_region(work_events, torch.cuda.synchronize, world, device=device)
    gc.enable()
    tm_ev = node_timing(gather_spans((*span_ev, round(ev0.elapsed_time(ev1) * 1e6)), world,
                                     device))
    HEADLINE_WALLS.clear()
    if g is None:
        # The value's own region (round 6, verdict r05 item 7): the launches
        # alone between t0 and t1 -- the HIP event pair above cost ~3 us of
        # queue time inside its region (profiles/r05_host_events.json).  The
        # GPU time of these launches is the packet-timestamped repetitions'
        # median measured right before (the same launches and arguments);
        # the instrumented region's wall and event time are reported beside.
        timed_region(timed, torch.cuda.synchronize, world, device=device)   # rehearsal
        gc.disable()
        span = timed_region(timed, torch.cuda.synchronize, world, device=device)
        gc.enable()
        tm = node_timing(gather_spans((*span, round(packet_ms * 1e6)), world, device))
        HEADLINE_WALLS.update({"wall_us": round(tm["wall_s"] * 1e6, 2),
                               "wall_us_with_event_pair": round(tm_ev["wall_s"] * 1e6, 2),
                               "event_pair_gpu_us": round(tm_ev["gpu_ms"] * 1e3, 3)})
    else:
        tm = tm_ev
    if g is None and any(rcs):
        from drone_rl_amd._lib import check
        check(next(r for r in rcs if r), b.handle)
    elapsed, gpu_ms = tm["wall_s"], tm["gpu_ms"]
    if world > 1:
        HEADLINE_NODE.update({"wall_us": round(tm["wall_s"] * 1e6, 2),
                              "slowest_rank_span_us": round(tm["max_rank_s"] * 1e6, 2),
                              "start_skew_us": (None if tm["start_skew_us"] is None
                                                else round(tm["start_skew_us"], 2)),
                              "start_alignment": "common CLOCK_MONOTONIC deadline agreed "
                                                 "before t0 (bench.start_deadline)"})
    ep =b.get("ep_num").float().mean().item()
    b.close()
    graphed = g is not None
    del g
    return elapsed, gpu_ms, launches, ep, packet_ms, graphed


def time_host_floor(device, reps=60):
    """The host side of one launch + synchronize on the headline's own path
    (a direct dr_rollout C-ABI call with prebuilt arguments, then
    torch.cuda.synchronize), measured on a launch whose kernel does almost no
    work: 64 envs, one step.  Returns median wall and median dispatch-packet
    duration (dr_rollout_timed) in us; their difference is the launch +
    completion cost that any single timed launch pays."""
    import torch

    from drone_rl_amd import DroneBatch, random_actions
    b = DroneBatch(64, "gym", dtype=torch.float64, device=device, seed=5, auto_reset=True)
    b.reset()
    acts = random_actions(64, seed=1, step=0).reshape(1, 64, 4).to(device)
    obs = torch.empty(1, 64, b.obs_dim, device=device)
    rew = torch.empty(1, 64, device=device)
    done = torch.empty(1, 64, dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device)
    c = (b.handle, 1, acts.data_ptr(), obs.data_ptr(), rew.data_ptr(), done.data_ptr(),
         stream.cuda_stream)
    fn = b.L.dr_rollout
    walls, pkts = [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for e in (e0, e1):
        e.record(stream)        # creates the events (torch creates them lazily)
    for r in range(reps):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        fn(*c)
        torch.cuda.synchronize(device)
        walls.append((time.perf_counter() - t0) * 1e6)
        b.L.dr_rollout_timed(*c, e0.cuda_event, e1.cuda_event)
        torch.cuda.synchronize(device)
        pkts.append(e0.elapsed_time(e1) * 1e3)
    b.close()
    walls, pkts = sorted(walls[5:]), sorted(pkts[5:])
    return walls[len(walls) // 2], pkts[len(pkts) // 2]


def time_rollout(args, n_envs, device, k, reps, gen, variant="gym", state_dtype=None):
    """The K-step rollout kernel (dr_rollout; dr_rollout_random when gen):
    `reps` launches of k steps each over the same 65,536 envs, captured in
    one hipGraph; returns the per-launch GPU time (HIP events on the launch
    stream) in seconds.  Reported beside the headline (the `rollout_kernel`
    block: fixed K, repeated launches, both action sources), never as `value`."""
    import torch

    from drone_rl_amd import DroneBatch, random_actions
    dtype = torch.float64 if (state_dtype or args.state_dtype) == "f64" else torch.float32
    b = DroneBatch(n_envs, variant, dtype=dtype, device=device, seed=2025, auto_reset=True)
    b.reset()
    obs = torch.empty(k, n_envs, b.obs_dim, device=device)
    rew = torch.empty(k, n_envs, device=device)
    done = torch.empty(k, n_envs, dtype=torch.uint8, device=device)
    acts = None
    if not gen:
        acts = torch.empty(reps, k, n_envs, 4, device=device)
        for r in range(reps):
            for t in range(k):
                random_actions(n_envs, seed=7, step=r * k + t, out=acts[r, t])

    def launch(r):
        if gen:
            b.rollout(k, None, seed=7, step0=r * k, obs_out=obs, rew_out=rew, done_out=done)
        else:
            b.rollout(k, acts[r], obs_out=obs, rew_out=rew, done_out=done)
    for r in range(2):
        launch(r)
    stream = torch.cuda.current_stream(device)
    s = torch.cuda.Stream(device)
    s.wait_stream(stream)
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for r in range(reps):
                launch(r)
    stream.wait_stream(s)
    g.replay()
    torch.cuda.synchronize(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    g.replay()
    e1.record(stream)
    torch.cuda.synchronize(device)
    per_launch = e0.elapsed_time(e1) / 1e3 / reps
    b.close()
    del g
    return per_launch


# PPO algorithmic work: forward FLOP per sample of the 2x256
# actor-critic (both MLPs' GEMMs and heads), training = 3 x forward per
# sample and epoch (forward, input gradient, weight gradient)
PPO_FWD_FLOP = 280064
F32_MATRIX_PEAK_TFLOPS = 157.3     # MI355X f32 MFMA = f32 vector peak (spec)
BF16_DENSE_PEAK_TFLOPS = 2500.0    # MI355X bf16 MFMA, dense (spec)


class _StopStep(Exception):
    """Raised by the timing hook to end a fused step after its j-th kernel."""
    pass


def ppo_kernel_times(tr, reps=20):
    """Every kernel of one configs[2] optimizer step (one 65,536-row
    minibatch: gather, the fused forward / loss / backward, the deferred
    finish + clip+Adam) timed in the trainer's own launch conditions: for
    j = 1 .. (number of kernels), `reps` repetitions of the step's first j kernels are captured
    into a hipGraph (FusedTrainStep.mark stops the step after its j-th
    kernel) and the replay is timed with HIP events on the stream; kernel j
    takes T_j - T_(j-1) per repetition (its launch gap included).  Runs after
    the timed region (it applies more optimizer steps)."""
    import torch

    cfg = tr.cfg
    M = cfg.batch_size
    idx = tr.perm(seed=99, counter=0)[:M]
    stream = torch.cuda.current_stream(tr.device)
    sched = tr.opt.schedule(tr.opt.t + 1, 1).to(tr.device)
    names = []

    def step_prefix(j, record=False):
        seen = [0]

        def mark(name):
            if record and name not in names:
                names.append(name)
            seen[0] += 1
            if seen[0] == j:
                raise _StopStep
        tr.fused.mark = mark
        try:
            tr.gather(idx, tr.mb_obs, tr.mb_act, tr.mb_aux, tr.head.adv_part)
            mark("gather_minibatch")
            grad, _ = tr.fused.step(tr.mb_obs, tr.mb_act, tr.mb_aux, tr.head, adv_ready=True,
                                    defer_finish=True)
            tr.opt.step_finish_sched(grad, tr.fused.finish, sched)
            mark("grad_finish_clip_adam")
        except _StopStep:
            pass
        finally:
            tr.fused.mark = None

    step_prefix(100, record=True)        # eager once: the kernel order, lazy init
    torch.cuda.synchronize(tr.device)

    def graph_us(fn):
        """fn() x reps captured in one hipGraph, replayed once untimed
        (upload) and once timed by HIP events on the stream: us per fn()."""
        cs = torch.cuda.Stream(tr.device)
        cs.wait_stream(stream)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cs), torch.cuda.graph(g, stream=cs):
            for _ in range(reps):
                fn()
        stream.wait_stream(cs)
        g.replay()                       # upload
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize(tr.device)
        del g
        return e0.elapsed_time(e1) * 1e3 / reps
    tj = [0.0]
    for j in range(1, len(names) + 1):
        tj.append(graph_us(lambda: step_prefix(j)))
    prefix = {n: tj[i + 1] - tj[i] for i, n in enumerate(names)}
    # the 256x256 layer's three GEMMs alone, each launch repeated back to back
    # on the trainer's buffers as the last step left them (the same kernels,
    # grids and operands; idempotent launches)
    from drone_rl_amd import _lib
    from drone_rl_amd.policy import gemm_x6, x6_weights
    f, pol = tr.fused, tr.policy
    iso = {}
    xw = x6_weights(pol, M)
    if xw is not None and getattr(f, "_acts2", None) is not None and f.C > 1:
        a0, a1, gz = f._acts2[0], f._acts2[1], f._gz2[1]
        g = f._g2.view(-1)[:2 * M * 256].view(2, M, 256)
        ws = f._ws2
        iso["gemm_x6_fwd"] = graph_us(lambda: gemm_x6(a0, xw.fwd, a1))
        if getattr(f, "_ximg", None) is not None:
            # the fused input-gradient GEMM + first-layer backward (its
            # level-1 partial sums included: the entry's two launches)
            iso["gemm_x6_bwd_first"] = graph_us(lambda: _lib.check(
                _lib.lib().dr_gemm_x6_bwd_first(
                    2, M, 15, gz.data_ptr(), xw.bwd.data_ptr(), a0.data_ptr(),
                    f._ximg.data_ptr(), f._first.ws.data_ptr(), f._first.ws.numel(),
                    int(pol.gemm_x6_fl_direct),
                    torch.cuda.current_stream(tr.device).cuda_stream)))
        else:
            iso["gemm_x6_bwd"] = graph_us(lambda: gemm_x6(gz, xw.bwd, g))
        # launched on the capturing stream (the current one inside graph_us)
        iso["gemm_x6_wgrad"] = graph_us(lambda: _lib.check(_lib.lib().dr_gemm_x6_wgrad(
            2, M, f.C, gz.data_ptr(), a0.data_ptr(), ws.data_ptr(),
            torch.cuda.current_stream(tr.device).cuda_stream)))
    return prefix, iso


# bench.py's PPO step names -> the kernel each launches (rocprofv3 names)
PPO_KERNEL_NAMES = {"gather_minibatch": "gather_records_kernel",
                    "linear_tanh": "linear_tanh_kernel", "ppo_head": "ppo_head_kernel",
                    "first_layer_bwd": "first_layer_bwd_kernel",
                    "gemm_x6_fwd": "gemm_x6_ws16_kernel", "gemm_x6_bwd": "gemm_x6_ws16_kernel",
                    "gemm_x6_wgrad": "gemm_x6_wgrad16_kernel",
                    "split_weights": "split_weights_kernel", "split_x": "split_x_kernel",
                    "gemm_x6_bwd_first": "gemm_x6_fl16_kernel"}


def rollout_rocprof_k32(path, n, state_dtype):
    """The split-physics rollout kernel's rocprofv3 durations at its largest
    grid (65,536 f64 envs, K = 32 launches only: scripts/micro/r4p3.sh's run,
    split by grid by scripts/kernel_grid_stats.py), with the HBM fraction of
    a K = 32 launch's algorithmic bytes; None when absent or for another
    configuration."""
    if n != 65536 or state_dtype != "f64":
        return None
    try:
        rows = [r for r in json.load(open(path)) if "env_rollout_ab_kernel<double" in r["kernel"]]
    except (OSError, ValueError, KeyError, TypeError):
        return None
    if not rows:
        return None
    r = max(rows, key=lambda r: r["grid"])
    byt = n * (32 * 81 + 224)
    return {"dispatches": r["dispatches"], "mean_us": r["mean_us"], "median_us": r["median_us"],
            "min_us": r["min_us"], "max_us": r["max_us"],
            "frac": round(byt / (r["mean_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "source": os.path.relpath(path, ROOT)}


def rocprof_averages(path):
    """{kernel name: average us} from a committed rocprofv3 --stats csv
    (profiles/r06_kernel_stats.csv: scripts/final_artifacts.sh's `kstats`
    run of this bench), or {} when absent."""
    import csv
    out = {}
    try:
        for r in csv.DictReader(open(path)):
            for k in set(PPO_KERNEL_NAMES.values()):
                if k + "(" in r["Name"] or k + "<" in r["Name"]:
                    out[k] = float(r["AverageNs"]) / 1e3
    except (OSError, KeyError, ValueError):
        return {}
    return out


def dominant_ppo_kernel(kern):
    """The optimizer step's kernel with the largest time per step (verdict
    r05 item 4): by rocprof_us when any entry carries it (the committed
    rocprofv3 summary matches the tree), else by the live prefix split.
    Only entries with a roofline bound compete."""
    key = "rocprof_us" if any("rocprof_us" in e for e in kern.values()) else "prefix_split_us"
    cands = {n: e[key] for n, e in kern.items() if key in e and "bound" in e}
    return max(cands, key=cands.get) if cands else None


def ppo_roofline(cfg, s_per_update, ktimes, rocprof=None, isolated=None, rocprof_source=None):
    """The ppo block's roofline.  Whole update: fp32-equivalent FLOP per
    second, reported against the f32 matrix peak only as
    `fp32_equiv_frac_of_f32_peak` (the 256x256 GEMMs run as 6 bf16 MFMA
    products per fp32 product, so that ratio may exceed 1 and is not a
    hardware utilisation).  Per kernel of one optimizer step: the prefix
    split's time (`prefix_split_us`, its method in kernel_timing) with the
    x6 GEMMs priced as bf16 MFMA work against the dense bf16 peak and the
    memory-bound kernels as algorithmic bytes (per 65,536-row minibatch,
    DESIGN.md 3) against HBM (`prefix_split_frac`); the GEMMs also timed
    alone (`isolated_us`, live); `rocprof_us` / `rocprof_frac` from a
    committed rocprofv3 summary that matches the current kernel sources
    (`rocprof_source`).  The dominant kernel is the one with the largest time
    per optimizer step (dominant_ppo_kernel)."""
    M, NT, E = cfg.batch_size, cfg.num_envs * cfg.n_steps, cfg.n_epochs
    flop_update = NT * PPO_FWD_FLOP * (1 + 3 * E)
    gemm_flop = 2 * 2 * M * 256 * 256            # both nets, one fp32 GEMM
    # the gather: 88 B of each row's record read (one 128-B line) + its 4-B
    # index, 88 B written
    rows = {"gather_minibatch": 2 * (15 + 4 + 3) * 4 + 4,
            "linear_tanh": 15 * 4 + 2 * 256 * 4,
            "ppo_head": 2 * 1024 + 2 * 1024 + 44,
            "first_layer_bwd": 2 * 2 * 1024 + 60,
            "split_x": 15 * 4 + 3136 // 32}            # x in, its three-plane record out
    if "gemm_x6_bwd_first" in ktimes and "split_x" not in ktimes:
        # dr_linear_tanh2_x6: the observation image (98 B per row) and the
        # weight images (2 MB per launch, 32 B per row at 65,536) as well
        rows["linear_tanh"] += 3136 // 32 + 32
    # the fused input-gradient GEMM also runs the first layer's weight
    # gradient (16 x 256 per net and row, features + bias) as x6 MFMA work
    fl_flop = gemm_flop + 2 * 2 * M * 16 * 256
    kern = {}
    rocprof = rocprof or {}
    isolated = isolated or {}

    def mfma_frac(us, flop=gemm_flop):
        return round(6 * flop / (us * 1e-6) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4)

    def hbm_frac(name, us):
        return round(rows[name] * M / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    for name, us in ktimes.items():
        e = {"prefix_split_us": round(us, 2)}
        rp = rocprof.get(PPO_KERNEL_NAMES.get(name, ""))
        if rp is not None:
            # the kernel's own average duration in whole training steps
            # (rocprofv3; the forward / input-gradient GEMM share one kernel)
            e["rocprof_us"] = round(rp, 2)
        if name.startswith("gemm_x6"):
            fl = fl_flop if name == "gemm_x6_bwd_first" else gemm_flop
            e.update({"bound": "mfma", "prefix_split_frac": mfma_frac(us, fl)})
            if name in isolated:
                e.update({"isolated_us": round(isolated[name], 2),
                          "isolated_frac": mfma_frac(isolated[name], fl)})
            if rp is not None:
                e["rocprof_frac"] = mfma_frac(rp, fl)
        elif name in rows:
            e.update({"bound": "hbm", "bytes": rows[name] * M,
                      "prefix_split_frac": hbm_frac(name, us)})
            if rp is not None:
                e["rocprof_frac"] = hbm_frac(name, rp)
        kern[name] = e
    ach = flop_update / s_per_update / 1e12
    out = {"unit": "TFLOP/s", "flop_per_update": flop_update,
           "fp32_equiv_tflops": round(ach, 2), "f32_matrix_peak": F32_MATRIX_PEAK_TFLOPS,
           "fp32_equiv_frac_of_f32_peak": round(ach / F32_MATRIX_PEAK_TFLOPS, 4),
           "basis": "fp32-equivalent FLOP per update (rollout forward 280,064 FLOP/sample + "
                    "3 x forward per sample and epoch, SURVEY.md 8d) / s_per_update; the "
                    "ratio to the f32 matrix peak is NOT a hardware utilisation (the 256x256 "
                    "GEMMs run as 6 bf16 MFMA products per fp32 product; their bf16-MFMA "
                    "fractions are in kernels_per_minibatch and dominant_kernel)",
           "rocprof_source": rocprof_source,
           "kernels_per_minibatch": kern}
    dom = dominant_ppo_kernel(kern)
    if dom is not None:
        e = kern[dom]
        basis = next(k for k in ("rocprof_us", "isolated_us", "prefix_split_us") if k in e)
        us = e[basis]
        if e["bound"] == "mfma":
            flop = 6 * (fl_flop if dom == "gemm_x6_bwd_first" else gemm_flop)
            ach, peak, unit = flop / (us * 1e-6) / 1e12, BF16_DENSE_PEAK_TFLOPS, "TFLOP/s"
        else:
            ach, peak, unit = rows[dom] * M / (us * 1e-6) / 1e9, HBM_PEAK_GBS, "GB/s"
        d = {"step": dom, "kernel": PPO_KERNEL_NAMES.get(dom, dom), "bound": e["bound"],
             "achieved": round(ach, 1), "peak": peak, "unit": unit,
             "frac": round(ach / peak, 4), "us": round(us, 2),
             "timing": {"rocprof_us": "the kernel's own rocprofv3 average in whole training "
                                      "steps (" + str(rocprof_source) + ")",
                        "isolated_us": "live: 20 back-to-back launches on the trainer's "
                                       "buffers in one hipGraph, HIP events",
                        "prefix_split_us": "live prefix split (kernel_timing)"}[basis],
             "selection": "the step's kernel with the largest time per optimizer step "
                          "(rocprof_us when the committed summary matches the tree, else "
                          "prefix_split_us)"}
        for k in ("isolated_us", "isolated_frac", "rocprof_us", "rocprof_frac"):
            if k in e and k != basis:
                d[k] = e[k]
        out["dominant_kernel"] = d
    return out


def time_ppo(args, rank, world, device, force_dp=False, dp_graph=False, profile=True,
             updates=None):
    """configs[2]/[3]: 65,536 envs per GPU + PPO (2x256 tanh MLP, GAE 0.95),
    one PPO iteration = T-step rollout + GAE + n_epochs x minibatches."""
    import torch
    import torch.distributed as dist

    from drone_rl_amd.policy import x6_weights
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=args.envs, n_steps=args.ppo_steps, batch_size=args.envs,
                    n_epochs=args.ppo_epochs, state_dtype=args.state_dtype, seed=0,
                    grad_buckets=args.grad_buckets, force_dp_path=force_dp, dp_graph=dp_graph)
    tr = PPOTrainer(cfg, device=device, rank=rank, world_size=world)
    # warm-up: the eager iteration, then the one that captures the rollout
    # and training graphs (replayed by every timed iteration)
    tr.learn_step()
    tr.learn_step()
    K = args.ppo_updates if updates is None else updates
    last = []

    def work():
        for _ in range(K):
            last[:] = [tr.learn_step()]
    span = timed_region(work, torch.cuda.synchronize, world, device=device)
    el = node_timing(gather_spans((*span, 0), world, device))["wall_s"]
    st = last[0]
    es =tr.episode_stats()
    stats = dict(zip(("loss", "policy_loss", "value_loss", "entropy_loss", "clip_fraction",
                      "approx_kl"), [round(x, 5) for x in st.tolist()[:6]]))
    coll = {"nccl": "RCCL"}.get(dist.get_backend(), dist.get_backend()) if world > 1 else (
        "RCCL" if tr.dp_collective else "no")
    path = ("data-parallel step (deferred finish -> " + coll + " all-reduce -> clip+Adam)"
            if tr.dp_step else "single-GPU fused step (deferred finish + clip+Adam)"
            if tr._train_fast() else "per-kernel finishes")
    res = {"updates_per_s": round(K / el, 4),
           "env_steps_per_s": round(K * cfg.n_steps * cfg.num_envs * world / el, 1),
           "s_per_update": round(el / K, 4),
           "train_path": path, "train_graph": tr._train_graphable(),
           "config": {"envs_per_gpu": cfg.num_envs, "n_steps": cfg.n_steps,
                      "minibatch": cfg.batch_size, "n_epochs": cfg.n_epochs,
                      "optimizer_steps_per_update": cfg.n_epochs * cfg.n_steps *
                      cfg.num_envs // cfg.batch_size,
                      "net_arch": list(cfg.net_arch), "mlp_dtype": "fp32",
                      "gemm": (("256x256 layer forward, input gradient and weight gradient: "
                                "dr_gemm_x6 / dr_gemm_x6_wgrad (fp32-accurate: exact 3-plane "
                                "bf16 split, 6 MFMA products, f32 accumulate)"
                                if x6_weights(tr.policy, cfg.batch_size) is not None else
                                "256x256 layer: " + ("hipBLASLt/rocBLAS, MI355X-tuned solutions "
                                                     "(TunableOp lookup)" if tr.tuned_gemms
                                                     else "hipBLASLt heuristic"))),
                      "grad_allreduce": ({"nccl": "rccl"}.get(dist.get_backend(),
                                                              dist.get_backend())
                                         + (" (2 buckets, the first overlapped with the "
                                            "first-layer backward)" if cfg.grad_buckets == 2
                                            else " (1 all-reduce of the flat gradient per "
                                                 "optimizer step)"))
                      if world > 1 or tr.dp_collective else "none"},
           "last_update_stats": stats, "episodes": es}
    if profile and world == 1 and tr._train_fast() and not tr.dp_step:
        prefix, iso = ppo_kernel_times(tr)
        rp = rocprof_averages(args.kernel_stats)
        prov = committed_profile(args.kernel_stats)
        if rp and not prov["matches_tree"]:
            ARTEFACTS["ppo_kernel_rocprof_us"] = dict(prov, stale=True, values=rp)
        live = prov["matches_tree"]
        res["roofline"] = ppo_roofline(cfg, el / K, prefix, rp if live else {}, iso,
                                       prov["source"] if live else None)
        res["roofline"]["kernel_timing"] = (
            "prefix_split_us: graph replays of the step's first j kernels x 20, timed by HIP "
            "events, kernel j = T_j - T_(j-1) (the step's tail and the next repetition's head "
            "shift with j, so cache effects land on neighbours: a per-kernel estimate, not a "
            "duration); isolated_us: the kernel alone, 20 launches in one graph; rocprof_us: "
            "the kernel's own duration in whole training steps (rocprofv3 --stats of this "
            "bench on the same kernel sources; HIP graphs on ROCm take no timed event nodes)")
    tr.close()
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`--gpus N` (N > 1) with no WORLD_SIZE in the environment: start N
    fresh child processes of this script, one per GPU (RANK = LOCAL_RANK = i,
    WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free MASTER_PORT), the same
    environment torchrun gives each rank.  This parent imports neither torch
    nor HIP: it only waits.  Rank 0 prints the JSON line itself (stdout is
    inherited); any rank failing ends the others (their exact PIDs) and the
    parent exits with that rank's status.  Returns the exit status."""
    import signal
    import subprocess
    env0 = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                DRONERL_BENCH_SPAWNED="1")
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)

    def stop(ps, grace=10.0):
        """SIGTERM the given ranks, then SIGKILL whatever is left after grace s."""
        for q in ps:
            if q.poll() is None:
                q.send_signal(signal.SIGTERM)
        end = time.monotonic() + grace
        for q in ps:
            try:
                q.wait(timeout=max(0.0, end - time.monotonic()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()

    def on_signal(signum, frame):
        # the launcher itself was told to stop (a driver timeout, ^C): take
        # the ranks down with it instead of leaving them on the GPUs
        sys.stderr.write(f"bench.py: launcher got signal {signum}; stopping the ranks\n")
        stop(procs)
        sys.exit(128 + signum)
    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    deadline = time.monotonic() + float(os.environ.get("DRONERL_BENCH_RANK_TIMEOUT", "3600"))
    try:
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with {r}; "
                                     f"stopping the other ranks\n")
                    stop(live)
            if live and time.monotonic() > deadline:
                # a rank stuck (e.g. in a collective whose peer died) must not
                # hold the launcher, or the GPUs, forever
                sys.stderr.write("bench.py: ranks exceeded DRONERL_BENCH_RANK_TIMEOUT; "
                                 "stopping them\n")
                stop(live)
                rc = rc or 124
            time.sleep(0.05)
    finally:
        for s_, h in old.items():
            signal.signal(s_, h)
    return rc


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    ws_env = os.environ.get("WORLD_SIZE")
    if ws_env is None and args.gpus > 1:
        # the direct form `python bench.py --gpus N`: this process becomes the
        # launcher of N ranks (the torchrun form sets WORLD_SIZE itself)
        sys.exit(spawn_ranks(args.gpus))
    world = int(ws_env or "1")
    if world != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch one rank "
                         f"per GPU with matching counts\n")
        sys.exit(2)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)      # before any GPU work

    import torch
    import torch.distributed as dist
    # one rank per GPU over RCCL.  DRONERL_DIST_BACKEND=gloo (with ranks
    # wrapping onto the available devices) only rehearses the multi-rank
    # path on a box with fewer GPUs than ranks (RCCL refuses 2 ranks/GPU).
    backend = os.environ.get("DRONERL_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    K, N = args.steps, args.envs
    n_cu = torch.cuda.get_device_properties(device).multi_processor_count
    sb = 8 if args.state_dtype == "f64" else 4
    state_b = (15 * sb + 4) + (12 * sb + 4)      # rollout kernel: state in + out per launch
    tj = {}
    try:
        tj = json.load(open(args.traffic_json))
    except (OSError, ValueError):
        pass
    if tj and not committed_profile(args.traffic_json)["matches_tree"]:
        # PMC traffic of other kernel sources: filed as stale, not reported live
        ARTEFACTS["traffic"] = dict(committed_profile(args.traffic_json), stale=True,
                                    values={k: v.get("hbm_bytes_per_launch")
                                            for k, v in tj.items() if isinstance(v, dict)})
        tj = {}

    def step_block(elapsed, gpu_ms, steps, n):
        pl = gpu_ms / 1e3 / steps
        bpe = BYTES_PER_ENV_STEP[args.state_dtype]
        ach = n * bpe / pl / 1e9
        tr = tj.get(f"{args.state_dtype}_{n}", {}).get("hbm_bytes_per_launch")
        return {"env_steps_per_s": round(n * world * steps / elapsed, 1),
                "ms_per_step": round(elapsed / steps * 1e3, 6),
                "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                             "traffic": tr,
                             "traffic_GBs": round(tr / pl / 1e9, 1) if tr else None,
                             "kernel": "env_step_kernel", "bytes_per_env_step": bpe,
                             "avg_launch_us": round(pl * 1e6, 3)}}

    el_s, gm_s, ep_s = time_env(args, args.state_dtype, N, rank, world, device, K, args.warmup)
    single = step_block(el_s, gm_s, K, N)
    if args.headline == "rollout":
        elapsed, gpu_ms, launches, ep, packet_ms, graphed = time_headline(
            args, N, rank, world, device, K, args.warmup, args.headline_k)
        per_launch_s = gpu_ms / 1e3 / launches
        bpe = 81 + state_b * launches / K
        achieved = N * K * bpe / (gpu_ms / 1e3) / 1e9
        kh = -(-K // launches)
        tr = tj.get(f"rollout_{args.state_dtype}_{N}_k{kh}", {}).get("hbm_bytes_per_launch")
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tr,
                "traffic_GBs": round(tr / per_launch_s / 1e9, 1) if tr else None,
                "kernel": rollout_kernel_name(N, n_cu, False), "steps_per_launch": kh,
                "launches": launches,
                "bytes_per_env_step": round(bpe, 2),
                "bytes_basis": "per env-step 16 action + 60 obs + 4 reward + 1 done; per "
                               "launch and env the f64 state read (124 B) and written (100 B) "
                               "once",
                "avg_launch_us": round(per_launch_s * 1e6, 3),
                "avg_launch_us_source": ("dispatch-packet timestamps (median of 5 "
                                         "repetitions of the timed launches, right before "
                                         "the timed region)" if packet_ms and not graphed
                                         else "HIP events on the launch stream across the "
                                              "timed region"),
                # the same algorithmic bytes over the timed region's host wall
                # (launch + synchronize included; the value's own clock)
                "frac_wall": round(N * K * bpe / elapsed / 1e9 / HBM_PEAK_GBS, 4),
                # the same kernel's own rocprofv3 durations, K = 32 launches
                # on 65,536 envs (the host-floor probe's 64-env launches of it
                # split off by grid)
                "rocprof_k32": committed_or_stale(
                    "rollout_rocprof_k32", args.rollout_grid_stats,
                    rollout_rocprof_k32(args.rollout_grid_stats, N, args.state_dtype)),
                # the same launches (median of 5 untimed repetitions right
                # before the timed one, after a warm-up) by their dispatch
                # packets' own timestamps: the kernel alone, without the
                # event records' queue time
                "avg_launch_us_packet": (round(packet_ms / launches * 1e3, 3)
                                         if packet_ms else None),
                # the instrumented region (HIP event pair around the launches):
                # its wall and the events' GPU time
                **({"walls": dict(HEADLINE_WALLS,
                                  frac_wall_with_event_pair=round(
                                      N * K * bpe / (HEADLINE_WALLS["wall_us_with_event_pair"]
                                                     * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                  avg_launch_us_events=round(
                                      HEADLINE_WALLS["event_pair_gpu_us"] / launches, 3))}
                   if HEADLINE_WALLS else {}),
                "limiter": "the f64 step, split by data over two waves per SIMD "
                           "(translation / rotation; memory waves stream the outputs beside "
                           "them; with no physics the stream alone takes ~30 us per 32 "
                           "steps, DESIGN.md section 3)"}
    else:
        elapsed, gpu_ms, ep = el_s, gm_s, ep_s
        roof = single["roofline"]
        graphed = not args.no_graph
    if args.headline == "rollout" and world == 1:
        # what one direct launch + synchronize costs on the host side (the
        # driver's --steps 20 is one launch): a near-empty launch on the same
        # path, wall against its dispatch packet
        # (a failure here is reported in the line, not fatal to it)
        try:
            fw, fp = time_host_floor(device)
            roof["host_floor_us"] = {"wall": round(fw, 2), "kernel_packet": round(fp, 2),
                                     "launch_and_sync": round(fw - fp, 2),
                                     "probe": "dr_rollout, 64 envs, 1 step, direct C-ABI call "
                                              "+ torch.cuda.synchronize, median of 55"}
        except Exception as ex:  # noqa: BLE001
            roof["host_floor_us"] = {"error": repr(ex)[:300]}
    value = N * world * K / elapsed
    out = {
        "metric": "env-steps/s (whole node) + PPO updates/s, 65 536 envs/GPU, 2x256 MLP",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.state_dtype,
        "data": "synthetic (random policy U[0,7.3575)^4 f32 actions, Philox, pre-generated in "
                "HBM; reset draws Philox)",
        "config": {"workload": "configs[1]: 65,536 batched DroneGymEnv envs per GPU, "
                               "random policy, dynamics-kernel throughput (auto-reset in step, "
                               "every step's obs / reward / done written)",
                   "envs_per_gpu": N, "global_envs": N * world,
                   "state_dtype": args.state_dtype, "hipgraph": graphed,
                   "kernel": ("dr_rollout (K-step rollout kernel, <= %d steps per launch)"
                              % args.headline_k if args.headline == "rollout"
                              else "dr_step (one launch per step)"),
                   "parallelism": f"dp{world} (independent env shards)"},
        "roofline": roof,
        "single_step": single,
        "mean_ep_num": round(ep, 2),
    }
    if HEADLINE_NODE:
        out["node_timing"] = dict(HEADLINE_NODE)
    if world == 1 and not args.no_companion:
        # cache-busting companion of the headline: the same
        # kernel at 4,194,304 envs, where the step is HBM-bound, not launch-
        # and latency-bound as at 65,536 (not the bench value)
        n4, k4 = 1 << 22, 200
        el4, gm4, _ = time_env(args, args.state_dtype, n4, 0, 1, device, k4, 20)
        pl4 = gm4 / 1e3 / k4
        ach4 = n4 * BYTES_PER_ENV_STEP[args.state_dtype] / pl4 / 1e9
        tr4 = tj.get(f"{args.state_dtype}_{n4}", {}).get("hbm_bytes_per_launch")
        out["companion"] = {"envs": n4, "steps": k4, "kernel": "env_step_kernel (dr_step)",
                            "env_steps_per_s": round(n4 * k4 / el4, 1),
                            "avg_launch_us": round(pl4 * 1e6, 3),
                            "roofline": {"bound": "hbm", "achieved": round(ach4, 1),
                                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                         "frac": round(ach4 / HBM_PEAK_GBS, 4),
                                         "traffic": tr4}}
        # the headline's own kernel past the 256-MB Infinity Cache: dr_rollout
        # at 4,194,304 envs, K = 32 steps per launch, actions read from HBM
        # (one launch writes ~11 GB of obs / reward / done)
        kr, reps = 32, 4
        plr = time_rollout(args, n4, device, kr, reps, False)
        bper = 81 + state_b / kr
        achr = n4 * kr * bper / plr / 1e9
        trr = tj.get(f"rollout_{args.state_dtype}_{n4}_k{kr}", {}).get("hbm_bytes_per_launch")
        out["companion_rollout"] = {
            "envs": n4, "steps_per_launch": kr, "launches": reps,
            "kernel": rollout_kernel_name(n4, n_cu, False),
            "env_steps_per_s": round(n4 * kr / plr, 1), "avg_launch_us": round(plr * 1e6, 3),
            "bytes_per_env_step": round(bper, 2),
            "roofline": {"bound": "hbm", "achieved": round(achr, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achr / HBM_PEAK_GBS, 4), "traffic": trr,
                         "traffic_GBs": round(trr / plr / 1e9, 1) if trr else None}}
    if world == 1 and args.rollout_k > 0:
        # SURVEY 7 "hard parts" (a): the K-step random-policy rollout kernel,
        # same envs and action stream, every step's obs / rew / done written
        # (bitwise the K single steps; tests/test_rollout_gpu.py)
        k, sb = args.rollout_k, (8 if args.state_dtype == "f64" else 4)
        state_b = (15 * sb + 4) + (12 * sb + 4)   # state in + out once per launch
        ro = {"k": k, "envs": N, "launches": 10}
        for gen in (False, True):
            pl = time_rollout(args, N, device, k, 10, gen)
            bpe = (65 if gen else 81) + state_b / k
            ach = N * k * bpe / pl / 1e9
            ro["random_policy_in_kernel" if gen else "actions_from_hbm"] = {
                # dr_rollout's default form per action source (env_kernels.hip
                # launch_rollout)
                "kernel": rollout_kernel_name(N, n_cu, gen),
                "env_steps_per_s": round(N * k / pl, 1),
                "avg_launch_us": round(pl * 1e6, 3), "us_per_step": round(pl * 1e6 / k, 3),
                "bytes_per_env_step": round(bpe, 2),
                "roofline": {"bound": "hbm", "achieved": round(ach, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 4)},
                "valu_active_frac_of_wave_cycles": committed_or_stale(
                    "rollout_valu_active_" + ("random_policy_in_kernel" if gen
                                              else "actions_from_hbm"), args.pmc_rollout,
                    pmc_rollout_valu_active(args.pmc_rollout).get(
                        "random_policy_in_kernel" if gen else "actions_from_hbm"))}
        out["rollout_kernel"] = ro
    if cpu is not None:
        out["cpu_baseline"] = cpu
    out["kernel_source_hash"] = kernel_source_hash()[:12]
    if args.ppo_updates > 0:
        out["ppo"] = time_ppo(args, rank, world, device)
    if args.extra and world == 1:
        ex = {}
        # the data-parallel optimizer step (PPOTrainer at world > 1: deferred
        # finish -> gradient all-reduce -> clip+Adam) timed on one GPU: with
        # no process group (all-reduce skipped), then on a one-rank RCCL
        # group with the all-reduce captured in the training graph
        if args.ppo_updates > 0:
            ex["ppo_dp_path_world1"] = time_ppo(args, 0, 1, device, force_dp=True,
                                                profile=False)
            try:
                import socket
                sk = socket.socket()
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
                sk.close()
                dist.init_process_group("nccl", rank=0, world_size=1, device_id=device,
                                        init_method=f"tcp://127.0.0.1:{port}")
                # the form N > 1 runs by default under RCCL (PPOConfig.dp_graph
                # off: the training loop eager, one all-reduce per step), then
                # the captured one
                for key, cap in (("ppo_dp_path_world1_rccl_eager", False),
                                 ("ppo_dp_path_world1_rccl_graph", True)):
                    ex[key] = time_ppo(args, 0, 1, device, force_dp=True, dp_graph=cap,
                                       profile=False)
            except Exception as e:      # report, keep the rest of the line
                ex["ppo_dp_path_world1_rccl_error"] = {"error": repr(e)[:300]}
            finally:
                if dist.is_initialized():
                    dist.destroy_process_group()
        for dn, n in (("f64", N), ("f32", N), ("f64", 1 << 22), ("f32", 1 << 22)):
            k = 200 if n > N else args.steps
            el, gm, _ = time_env(args, dn, n, 0, 1, device, k, 20)
            pl = gm / 1e3 / k
            ex[f"step_{dn}_{n}"] = {
                "env_steps_per_s": round(n * k / el, 1),
                "avg_launch_us": round(pl * 1e6, 3),
                "achieved_GBs": round(n * BYTES_PER_ENV_STEP[dn] / pl / 1e9, 1)}
        # configs[4]: the moving-target curriculum, 1M envs over 8 GPUs
        for dn, n in (("f64", 1 << 17), ("f64", 1 << 20)):
            k = 200 if n > N else args.steps
            el, gm, _ = time_env(args, dn, n, 0, 1, device, k, 20, variant="moving")
            pl = gm / 1e3 / k
            ex[f"moving_{dn}_{n}"] = {
                "env_steps_per_s": round(n * k / el, 1),
                "avg_launch_us": round(pl * 1e6, 3),
                "achieved_GBs": round(n * BYTES_PER_ENV_STEP_MOVING[dn] / pl / 1e9, 1)}
        # the K-step rollout kernel (in-kernel random policy, K = 32) at the
        # configs[4] sizes: per-GPU slice and whole 1M
        for gen in (False, True):         # f32 state through the rollout kernel
            pl = time_rollout(args, N, device, 32, 10, gen, state_dtype="f32")
            ex["rollout_f32_%d_%s" % (N, "random_policy_in_kernel" if gen else "actions_from_hbm")] = {
                "env_steps_per_s": round(N * 32 / pl, 1), "avg_launch_us": round(pl * 1e6, 3),
                "us_per_step": round(pl * 1e6 / 32, 3)}
        for n in (1 << 17, 1 << 20):
            pl = time_rollout(args, n, device, 32, 4, True, variant="moving")
            ex[f"rollout_moving_f64_{n}"] = {"env_steps_per_s": round(n * 32 / pl, 1),
                                             "avg_launch_us": round(pl * 1e6, 3),
                                             "us_per_step": round(pl * 1e6 / 32, 3)}
        out["extra"] = ex
    if ARTEFACTS:
        out["committed_artefacts"] = ARTEFACTS
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
