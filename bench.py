"""Benchmark: batched quadrotor env-steps/s on MI355X (BASELINE.json configs[1]).

Workload (N=1 GPU): 65,536 DroneGymEnv-equivalent envs per GPU, synthetic
random policy (actions i.i.d. U[0, 7.3575)^4 f32 from Philox, pre-generated
and resident in HBM before the timed region), DummyVecEnv auto-reset inside
the step, f64 state (the reference's precision).  One "step" = one
dr_step over the whole batch.  The K timed steps are captured in one
hipGraph and replayed (launch-bound loop), bracketed by barrier +
synchronize on both sides; the max over ranks is taken.

Multi-GPU: one process per GPU (torchrun), independent env shards (global
env ids rank*N+i), no data-path collective -> "scaling": "weak".

The JSON line also carries
  roofline      dominant kernel (env_step_kernel): algorithmic bytes per
                launch (N x 305 B in f64 mode, 197 B in f32) over
                its average per-launch GPU time from HIP events on the
                launch stream across the timed region;
  cpu_baseline  rank 0, N=1: the SubprocVecEnv-equivalent process pool over
                the fixture-pinned numpy port (oracle/cpu_baseline.py),
                run BEFORE the GPU is touched;
  ppo           PPO updates/s for configs[2] (65,536 envs, 2x256 tanh MLP,
                GAE lambda 0.95), when --ppo-updates > 0;
  rollout_kernel  the same envs and action stream through the K-step
                rollout kernel (dr_rollout: K steps per launch, state in
                registers, every step's outputs written), separately
                reported; `value` stays on the single-step kernel.
"""
import argparse
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
    return ap.parse_args()


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
    import torch.distributed as dist

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
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev0.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for t in range(warmup, total):
            b.step(acts[t])
    ev1.record(stream)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    if world > 1:
        t = torch.tensor([elapsed, gpu_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gpu_ms = float(t[0]), float(t[1])
    # sanity: the env is alive (episodes end and reset under a random policy)
    ep = b.get("ep_num").float().mean().item()
    b.close()
    del graph
    return elapsed, gpu_ms, ep


def time_rollout(args, n_envs, device, k, reps, gen, variant="gym", state_dtype=None):
    """The K-step rollout kernel (dr_rollout; dr_rollout_random when gen):
    `reps` launches of k steps each over the same 65,536 envs, captured in
    one hipGraph; returns the per-launch GPU time (HIP events on the launch
    stream) in seconds.  Reported beside the headline, never as `value`
    (the headline stays on the single-step kernel PPO uses)."""
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


def time_ppo(args, rank, world, device):
    """configs[2]/[3]: 65,536 envs per GPU + PPO (2x256 tanh MLP, GAE 0.95),
    one PPO iteration = T-step rollout + GAE + n_epochs x minibatches."""
    import torch
    import torch.distributed as dist

    from drone_rl_amd.policy import x6_weights
    from drone_rl_amd.ppo import PPOConfig, PPOTrainer
    cfg = PPOConfig(num_envs=args.envs, n_steps=args.ppo_steps, batch_size=args.envs,
                    n_epochs=args.ppo_epochs, state_dtype=args.state_dtype, seed=0,
                    grad_buckets=args.grad_buckets)
    tr = PPOTrainer(cfg, device=device, rank=rank, world_size=world)
    # warm-up: the eager iteration, then the one that captures the rollout
    # graph (replayed by every timed iteration)
    tr.learn_step()
    tr.learn_step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.ppo_updates):
        st = tr.learn_step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    es = tr.episode_stats()
    stats = dict(zip(("loss", "policy_loss", "value_loss", "entropy_loss", "clip_fraction",
                      "approx_kl"), [round(x, 5) for x in st.tolist()[:6]]))
    tr.close()
    K = args.ppo_updates
    return {"updates_per_s": round(K / el, 4),
            "env_steps_per_s": round(K * cfg.n_steps * cfg.num_envs * world / el, 1),
            "s_per_update": round(el / K, 4),
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
                                                  "optimizer step)")) if world > 1
                       else "none"},
            "last_update_stats": stats, "episodes": es}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
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

    elapsed, gpu_ms, ep = time_env(args, args.state_dtype, args.envs, rank, world, device,
                                   args.steps, args.warmup)
    K, N = args.steps, args.envs
    value = N * world * K / elapsed
    per_launch_s = gpu_ms / 1e3 / K
    bpe = BYTES_PER_ENV_STEP[args.state_dtype]
    achieved = N * bpe / per_launch_s / 1e9
    traffic = None
    try:
        tj = json.load(open(args.traffic_json))
        key = f"{args.state_dtype}_{N}"
        if key in tj:
            traffic = tj[key]["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
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
        "data": "synthetic (random policy U[0,7.3575)^4 f32 actions, Philox; "
                "reset draws Philox)",
        "config": {"workload": "configs[1]: 65,536 batched DroneGymEnv envs per GPU, "
                               "random policy, dynamics-kernel throughput (auto-reset in step)",
                   "envs_per_gpu": N, "global_envs": N * world,
                   "state_dtype": args.state_dtype, "hipgraph": not args.no_graph,
                   "parallelism": f"dp{world} (independent env shards)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_GBs": (round(traffic / per_launch_s / 1e9, 1)
                                     if traffic else None),
                     "kernel": "env_step_kernel", "bytes_per_env_step": bpe,
                     "avg_launch_us": round(per_launch_s * 1e6, 3)},
        "mean_ep_num": round(ep, 2),
    }
    if world == 1 and not args.no_companion:
        # cache-busting companion of the headline: the same
        # kernel at 4,194,304 envs, where the step is HBM-bound, not launch-
        # and latency-bound as at 65,536 (not the bench value)
        n4, k4 = 1 << 22, 200
        el4, gm4, _ = time_env(args, args.state_dtype, n4, 0, 1, device, k4, 20)
        pl4 = gm4 / 1e3 / k4
        ach4 = n4 * bpe / pl4 / 1e9
        tr4 = None
        try:
            tr4 = json.load(open(args.traffic_json))[f"{args.state_dtype}_{n4}"][
                "hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            pass
        out["companion"] = {"envs": n4, "steps": k4,
                            "env_steps_per_s": round(n4 * k4 / el4, 1),
                            "avg_launch_us": round(pl4 * 1e6, 3),
                            "roofline": {"bound": "hbm", "achieved": round(ach4, 1),
                                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                         "frac": round(ach4 / HBM_PEAK_GBS, 4),
                                         "traffic": tr4}}
    if world == 1 and args.rollout_k > 0:
        # SURVEY 7 "hard parts" (a): the K-step random-policy rollout kernel,
        # same envs and action stream, every step's obs / rew / done written
        # (bitwise the K single steps; tests/test_rollout_gpu.py)
        k, sb = args.rollout_k, (8 if args.state_dtype == "f64" else 4)
        state_b = (15 * sb + 4) + (12 * sb + 4)   # state in + out once per launch
        ro = {"kernel": "env_rollout_kernel", "k": k, "envs": N, "launches": 10}
        for gen in (False, True):
            pl = time_rollout(args, N, device, k, 10, gen)
            bpe = (65 if gen else 81) + state_b / k
            ach = N * k * bpe / pl / 1e9
            ro["random_policy_in_kernel" if gen else "actions_from_hbm"] = {
                "env_steps_per_s": round(N * k / pl, 1),
                "avg_launch_us": round(pl * 1e6, 3), "us_per_step": round(pl * 1e6 / k, 3),
                "bytes_per_env_step": round(bpe, 2),
                "roofline": {"bound": "valu (f64 issue; DESIGN.md 6)", "achieved": round(ach, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 4)}}
        out["rollout_kernel"] = ro
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if args.ppo_updates > 0:
        out["ppo"] = time_ppo(args, rank, world, device)
    if args.extra and world == 1:
        ex = {}
        saved = os.environ.get("DRONERL_STEP_KERNEL")
        for kern in ("quad", "lane"):
            os.environ["DRONERL_STEP_KERNEL"] = kern
            for dn, n in (("f64", N), ("f32", N), ("f64", 1 << 22), ("f32", 1 << 22)):
                k = 200 if n > N else args.steps
                el, gm, _ = time_env(args, dn, n, 0, 1, device, k, 20)
                pl = gm / 1e3 / k
                ex[f"{kern}_{dn}_{n}"] = {
                    "env_steps_per_s": round(n * k / el, 1),
                    "avg_launch_us": round(pl * 1e6, 3),
                    "achieved_GBs": round(n * BYTES_PER_ENV_STEP[dn] / pl / 1e9, 1)}
        os.environ["DRONERL_STEP_KERNEL"] = "lane"
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
        if saved is None:
            os.environ.pop("DRONERL_STEP_KERNEL", None)
        else:
            os.environ["DRONERL_STEP_KERNEL"] = saved
        out["extra"] = ex
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
