"""GPU-resident PPO over the batched quadrotor env (SB3 PPO semantics).

Replaces the reference's `PPO("MlpPolicy", env).learn(...)`
(/root/reference/train.py:36-43, 63-68; SB3 recalled in SURVEY.md Appendix C)
with a loop whose every byte stays in HBM:

  rollout (T steps):  policy fwd (torch GEMMs, MFMA)  ->  dr_policy_sample
                      (Gaussian action, log-prob, clip)  ->  dr_step_monitored
                      (env physics + auto-reset + VecMonitor stats)
  advantages:         dr_gae (reverse scan, one thread per env)
  update (epochs):    dr_permutation  ->  dr_gather_minibatch  ->  fused
                      MLP forward / loss / backward (policy.FusedTrainStep)
                      ->  one launch of the deferred reductions  ->  [RCCL
                      all-reduce of the flat grad when world > 1]  ->
                      clip_grad_norm_ + Adam (fused); the whole loop is one
                      hipGraph replay on one GPU

SB3-parity choices (documented deviations in DESIGN.md):
  * no value bootstrap at the 200-step limit by default (the reference's env
    is wrapped by shimmy's GymV21 compat, so SB3 sees terminated=True, not
    truncated); `bootstrap_timeouts=True` opts into SB3's TimeLimit handling
    (rewards[t] += gamma * V(terminal obs) where the episode hit the limit
    without crashing, OnPolicyAlgorithm.collect_rollouts);
  * advantages normalised per minibatch (mean, unbiased std + 1e-8);
  * the flat rollout index is t*N + n (SB3 uses n*T + t after
    swap_and_flatten; a uniformly random permutation makes the two
    statistically identical).
"""
from __future__ import annotations

import dataclasses
import os
import time

import torch

from . import dist as D
from . import ppo_kernels as K
from .env import MOTOR_MAX, DroneBatch
from .policy import ActorCritic, FusedTrainStep, PolicyInference, fusable, use_tuned_gemms


@dataclasses.dataclass
class PPOConfig:
    num_envs: int = 65536          # envs on this rank
    n_steps: int = 32              # rollout length T per env
    batch_size: int = 65536        # minibatch rows
    n_epochs: int = 10
    learning_rate: float = 3e-4
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_range: float = 0.2
    ent_coef: float = 0.0
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    normalize_advantage: bool = True
    net_arch: tuple = (256, 256)
    log_std_init: float = 0.0
    seed: int = 0
    state_dtype: str = "f64"       # env state precision ("f64" = reference)
    variant: str = "gym"
    # curriculum level every env starts at (drone.py:33 starts at 0.0 and
    # adds 0.1 per 2000 episodes of an env; with 65k envs per GPU that takes
    # ~4e9 steps, so large-batch runs of the moving target start higher)
    initial_eps: float = 0.0
    # staged curriculum for large batches: ((update, eps), ...) -- at the
    # start of that PPO iteration every env's eps is set to the value (the
    # per-env 2000-episode bump of drone.py:68-70 keeps running on top)
    eps_schedule: tuple = ()
    # look up the MI355X-tuned GEMM solutions (policy.use_tuned_gemms)
    tuned_gemms: bool = True
    # data parallel (world > 1): RCCL all-reduces of the flat gradient per
    # optimizer step.  1 = one all-reduce of the whole 564 KB buffer after
    # the backward; 2 = everything but the first layer
    # started asynchronously as soon as the fused backward finished it
    # (overlapping the first-layer backward), the first layer at the end
    grad_buckets: int = 1
    # the data-parallel optimizer step (deferred finish -> gradient
    # all-reduce -> clip+Adam from device scalars) even at world 1, where
    # the all-reduce is skipped unless a process group is initialised:
    # times the 8-GPU code path on one GPU (bench.py --extra, tests)
    force_dp_path: bool = False
    # capture the data-parallel training loop, RCCL all-reduces included,
    # into the training hipGraph (backend "nccl" only; DRONERL_DP_GRAPH=1).
    # Off by default: graph capture of RCCL collectives has only been run
    # on a one-rank group here (no multi-GPU box for the builder)
    dp_graph: bool = False
    # SB3's timeout bootstrap for envs that report TimeLimit truncation: at
    # the 200-step limit (drone.py:155-157, no crash) add gamma * V(terminal
    # obs) to that step's reward.  Off = the reference's semantics
    bootstrap_timeouts: bool = False

    @classmethod
    def sb3_defaults(cls, **kw):
        """The reference's train.py configuration: SB3 PPO defaults, one env,
        n_steps 2048, batch 64, 10 epochs, 64x64 tanh MLP."""
        base = dict(num_envs=1, n_steps=2048, batch_size=64, n_epochs=10,
                    net_arch=(64, 64))
        base.update(kw)
        return cls(**base)


class PPOTrainer:
    def __init__(self, cfg: PPOConfig, device=None, rank: int = 0, world_size: int = 1,
                 process_group=None):
        self.cfg = cfg
        self.rank, self.world = rank, world_size
        self.pg = process_group
        self.device = torch.device("cuda", torch.cuda.current_device()) \
            if device is None else torch.device(device)
        N, T = cfg.num_envs, cfg.n_steps
        if (N * T) % cfg.batch_size:
            raise ValueError("num_envs * n_steps must be a multiple of batch_size")
        if cfg.grad_buckets not in (1, 2):
            raise ValueError("grad_buckets must be 1 or 2")
        dev = self.device
        self.tuned_gemms = use_tuned_gemms() if cfg.tuned_gemms else False
        self.env = DroneBatch(N, cfg.variant, device=dev, seed=cfg.seed,
                              env_id_offset=D.env_shard(rank, N)[0], monitor=True,
                              keep_terminal_obs=cfg.bootstrap_timeouts,
                              dtype=torch.float64 if cfg.state_dtype == "f64" else torch.float32)
        if cfg.initial_eps:
            self.env.set("eps", torch.full((N,), float(cfg.initial_eps), dtype=torch.float64))
        od = self.env.obs_dim
        # every rank starts from the same parameters (the seed is shared);
        # with world > 1 rank 0's copy is also broadcast (sync_params)
        self.policy = ActorCritic(od, 4, cfg.net_arch, dev, cfg.log_std_init, cfg.seed)
        # one GEMM path for the rollout forward (N rows) AND the training
        # forward (M rows): dr_gemm_x6 needs a multiple of 128 rows, and if
        # only one of the two qualified the first epoch's ratio would no
        # longer be exactly 1 (PolicyInference's guarantee)
        if N % 128 or cfg.batch_size % 128:
            self.policy.gemm_x6 = False
        self.opt = K.ClipAdam(self.policy.flat.data, cfg.learning_rate, eps=1e-5,
                              max_grad_norm=cfg.max_grad_norm)
        f32 = dict(dtype=torch.float32, device=dev)
        self.obs = torch.zeros(T + 1, N, od, **f32)           # obs[t] -> action[t]
        self.dones = torch.ones(T + 1, N, dtype=torch.uint8, device=dev)
        self.actions = torch.zeros(T, N, 4, **f32)              # unclipped (SB3)
        self.act_env = torch.zeros(N, 4, **f32)                 # clipped, to the env
        self.logp = torch.zeros(T, N, **f32)
        self.values = torch.zeros(T, N, **f32)
        self.rewards = torch.zeros(T, N, **f32)
        self.ep_ret = torch.zeros(T, N, **f32)
        self.ep_len = torch.zeros(T, N, dtype=torch.int32, device=dev)
        self.adv = torch.zeros(T, N, **f32)
        self.ret = torch.zeros(T, N, **f32)
        self.aux = torch.zeros(T * N, 3, **f32)                 # (old logp, adv, return)
        # the fused path's minibatch source: every rollout row as one 128-B
        # record (obs, action, aux), packed once per iteration, so the
        # gather reads one cache line per row (dr_gather_records, round 6)
        self.rec = None
        # bootstrap_timeouts: per-step truncation flags (dr_step_monitored_trunc)
        self.trunc = torch.zeros(T, N, dtype=torch.uint8, device=dev) \
            if cfg.bootstrap_timeouts else None
        M = cfg.batch_size
        self.perm = K.Permuter(T * N, dev)
        self.mb_obs = torch.zeros(M, od, **f32)
        self.mb_act = torch.zeros(M, 4, **f32)
        self.mb_aux = torch.zeros(M, 3, **f32)
        self.loss = K.PPOLoss(M, dev, cfg.clip_range, cfg.ent_coef, cfg.vf_coef,
                              cfg.normalize_advantage)
        self.fused = FusedTrainStep(self.policy, M)
        # fused MLP path (first-layer linear+tanh, heads+loss+head backward)
        # when the architecture fits the kernels; else forward/loss/backward
        self.use_fused = fusable(self.policy)
        # single-GPU fused path: the step's last reductions + norm in one
        # launch before Adam (DRONERL_DEFER_FINISH=0: separate launches)
        self.defer_finish = (self.use_fused and self.fused.can_defer() and
                             os.environ.get("DRONERL_DEFER_FINISH", "1") != "0")
        # data-parallel optimizer step on the same kernels as the single-GPU
        # one: ONE finish launch of the deferred reductions, ONE all-reduce
        # of the flat gradient, ONE clip+Adam (grad_buckets 2 keeps the
        # older early-bucket step, whose finishes run per kernel)
        dp_want = world_size > 1 or cfg.force_dp_path
        self.dp_step = (dp_want and self.defer_finish and cfg.grad_buckets == 1)
        # the summing all-reduce runs when there are ranks to sum over, or
        # (force_dp_path) whenever a process group exists, so a one-rank
        # RCCL group exercises the collective and its graph capture
        self.dp_collective = self.dp_step and (
            world_size > 1 or (D.dist.is_available() and D.dist.is_initialized()))
        self.dp_graph = self.dp_step and (
            cfg.dp_graph or os.environ.get("DRONERL_DP_GRAPH", "0") == "1")
        if self.use_fused:
            self.head = K.HeadLossBackward(M, cfg.net_arch[-1], dev, cfg.clip_range,
                                           cfg.ent_coef, cfg.vf_coef, cfg.normalize_advantage)
            self.infer = PolicyInference(self.policy, N)
        self.num_updates = 0
        self.num_timesteps = 0
        self._rolled = False
        # rollout loop captured into a hipGraph after one eager warm-up
        # iteration (DRONERL_ROLLOUT_GRAPH=0: always eager)
        self.rollout_graph = os.environ.get("DRONERL_ROLLOUT_GRAPH", "1") != "0"
        self._rgraph, self._rwarm, self._rkey = None, False, None
        # likewise PPO.train's minibatch loop (single-GPU fused path): one
        # replay per iteration instead of ~15 launches per optimizer step from
        # Python (the reference's 64-row minibatches are launch-bound).  Every
        # kernel in it keeps no state across launches (the permutation is this
        # library's bucket sort: rocPRIM's onesweep radix sort, used in round
        # 1, faulted on the second replay of a captured graph at configs[2]
        # size).  DRONERL_TRAIN_GRAPH=0: always eager.
        self.train_graph = os.environ.get("DRONERL_TRAIN_GRAPH", "1") != "0"
        # the next minibatch's gather on a side stream, beside this
        # minibatch's step, into a second set of minibatch buffers
        # (DRONERL_PPO_OVERLAP=1; same kernels and inputs, bitwise the same)
        self.overlap_gather = os.environ.get("DRONERL_PPO_OVERLAP", "0") == "1"
        self._slots, self._side = None, None
        self._tgraph, self._twarm, self._tstats, self._tkey = None, False, None, None
        self._ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        # optional TrajectoryTensorboardCallback equivalent (trajectory.py)
        self.trajectory = None
        self.env.reset(self.obs[0])
        if self.world > 1:
            self.sync_params()

    # ------------------------------------------------------------ DP plumbing
    def sync_params(self):
        D.broadcast_params_(self.policy.flat.data, group=self.pg)

    def _allreduce_grad(self, g):
        D.allreduce_mean_(g, self.world, group=self.pg)

    # ---------------------------------------------------------------- phases
    @torch.no_grad()
    def collect_rollouts(self):
        cfg, T = self.cfg, self.cfg.n_steps
        if self._rolled:                              # continue where we stopped
            self.obs[0].copy_(self.obs[T])
        self.dones[0].copy_(self.dones[T])          # episode_starts of step 0
        self._rolled = True
        fwd = self.infer if self.use_fused else self.policy
        # noise counter of step t = num_updates * T + t, its base on the device
        self._ctr.fill_(self.num_updates * T)
        key = self._graph_key("rollout")
        if self._rgraph is not None and key != self._rkey:
            self._rgraph = None       # a host scalar baked into the graph changed
        self._rkey = key
        if not (self.rollout_graph and self.trajectory is None):
            self._rollout_steps(fwd)
        elif self._rgraph is not None:
            self._rgraph.replay()
        elif not self._rwarm:
            self._rollout_steps(fwd)     # eager once: lazy library init
            self._rwarm = True
        else:
            # the T-step loop (policy forward, sample, env step) captured once
            # and replayed every iteration: one launch instead of ~8T from
            # Python (matters at few envs: the reference's 1-env config)
            cur = torch.cuda.current_stream(self.device)
            cs = torch.cuda.Stream(self.device)
            cs.wait_stream(cur)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(cs), torch.cuda.graph(g, stream=cs):
                self._rollout_steps(fwd)
            cur.wait_stream(cs)
            g.replay()
            self._rgraph = g
        if self.trajectory is not None:
            self.trajectory.flush()
        _, last_values = fwd(self.obs[T])
        K.gae(self.rewards, self.values, self.dones[:T], last_values, self.dones[T],
              cfg.gamma, cfg.gae_lambda, advantages=self.adv, returns=self.ret)
        # (old log-prob, advantage, return) rows: the unfused path's minibatch
        # source, and what callers inspect after a rollout
        torch.stack([self.logp.reshape(-1), self.adv.reshape(-1), self.ret.reshape(-1)],
                    dim=1, out=self.aux)
        if self.use_fused:
            if self.rec is None:
                self.rec = torch.zeros(T * cfg.num_envs, K.RECORD_FLOATS, dtype=torch.float32,
                                       device=self.device)
            K.pack_rollout_records(self.obs[:T].reshape(T * cfg.num_envs, -1),
                                   self.actions.reshape(-1, 4), self.logp.reshape(-1),
                                   self.adv.reshape(-1), self.ret.reshape(-1), self.rec)
        self.num_timesteps += T * cfg.num_envs * self.world

    def _rollout_steps(self, fwd):
        T, ls = self.cfg.n_steps, self.policy.log_std
        for t in range(T):
            mean, value = fwd(self.obs[t])
            self.values[t].copy_(value)
            K.policy_sample_dev(mean, ls, seed=self.cfg.seed * 7919 + self.rank,
                                counter_base=self._ctr, counter_offset=t, lo=0.0,
                                hi=MOTOR_MAX, actions_raw=self.actions[t],
                                actions_clipped=self.act_env, logp=self.logp[t])
            # VecMonitor outputs land in this step's slice (done rows only)
            self.env.ep_ret = self.ep_ret[t]
            self.env.ep_len = self.ep_len[t]
            self.env.step(self.act_env, obs_out=self.obs[t + 1], rew_out=self.rewards[t],
                          done_out=self.dones[t + 1],
                          trunc_out=None if self.trunc is None else self.trunc[t])
            if self.trunc is not None:
                # SB3 collect_rollouts: rewards[idx] += gamma * V(terminal
                # obs) for envs whose episode was truncated at the limit
                _, v_term = fwd(self.env.term_obs)
                self.rewards[t].add_(torch.where(self.trunc[t].bool(),
                                                 v_term * self.cfg.gamma, 0.0))
            if self.trajectory is not None:
                self.trajectory.on_step(self.dones[t + 1])

    def _graph_key(self, kind: str):
        """Every host-side value a captured graph holds as a kernel argument
        (the rest -- noise / permutation counters, Adam's bias corrections --
        is read from device memory on each replay).  A graph whose key no
        longer matches is dropped and re-captured, so env.seed(), a config
        change or a new learning rate take effect on the graph path exactly
        as on the eager path."""
        c = self.cfg
        if kind == "rollout":
            return (self.env.seed_value, c.seed, self.rank, c.num_envs, c.n_steps)
        o = self.opt
        return (c.seed, self.rank, c.n_epochs, c.batch_size, c.clip_range, c.ent_coef,
                c.vf_coef, c.normalize_advantage, float(o.lr), o.b1, o.b2, o.eps,
                o.max_norm, float(self.head.clip), float(self.head.ent), float(self.head.vf),
                self.head.norm)

    def _train_fast(self) -> bool:
        """The deferred-finish step with device-side Adam scalars: the
        single-GPU step, or the data-parallel split step."""
        return self.use_fused and self.defer_finish and (self.world == 1 or self.dp_step)

    def _train_graphable(self) -> bool:
        if not (self.train_graph and self._train_fast()):
            return False
        if not self.dp_collective:
            return True
        # a collective inside the captured loop: RCCL only, and opt-in
        return self.dp_graph and D.dist.get_backend(self.pg) == "nccl"

    def _train_body(self, obs_flat, act_flat, nmb):
        """PPO.train's epochs x minibatches on the single-GPU fused path with
        every per-step scalar on the device (permutation counter base, Adam's
        bias-correction schedule): the same kernels and numerics as train(),
        capturable into one hipGraph."""
        cfg, M = self.cfg, self.cfg.batch_size
        if self.overlap_gather:
            return self._train_body_overlap(obs_flat, act_flat, nmb)
        j = 0
        for epoch in range(cfg.n_epochs):
            perm = self.perm.dev(seed=cfg.seed * 104729 + self.rank, counter_base=self._pctr,
                                 counter_offset=epoch)
            for k in range(nmb):
                idx = perm[k * M:(k + 1) * M]
                self.gather(idx, self.mb_obs, self.mb_act, self.mb_aux, self.head.adv_part)
                self._train_minibatch(j, self.mb_obs, self.mb_act, self.mb_aux)
                j += 1

    def gather(self, idx, obs_out, act_out, aux_out, adv_part):
        """The fused path's minibatch gather (RolloutBuffer.get's indexing)
        from this iteration's packed rollout records: one launch, one cache
        line per row, the same bytes as dr_gather_minibatch."""
        K.gather_records(idx, self.rec, self.env.obs_dim, obs_out, act_out, aux_out,
                         adv_part=adv_part)

    def _train_minibatch(self, j, mb_obs, mb_act, mb_aux):
        """Optimizer step j on one gathered minibatch (its advantage partials
        in self.head.adv_part)."""
        grad, _ = self.fused.step(mb_obs, mb_act, mb_aux, self.head, adv_ready=True,
                                  stats_out=self._tstats[j], defer_finish=True)
        if self.dp_step:
            # finish -> one all-reduce (sum) of the 564 KB flat gradient ->
            # clip+Adam on its mean
            self.fused.finish.run(self.device)
            if self.dp_collective:
                D.allreduce_flat_sum_(grad, group=self.pg)
            self.opt.step_sched(grad, self._sched[j], 1.0 / self.world)
        else:
            self.opt.step_finish_sched(grad, self.fused.finish, self._sched[j])

    def _train_body_overlap(self, obs_flat, act_flat, nmb):
        """_train_body with minibatch j + 1's gather on a side stream while
        step j runs on the current one.  Two slots of minibatch buffers (obs,
        actions, aux, the head workspace that holds the advantage partials):
        gather j + 1 waits for everything issued before step j (step j - 1
        read its slot), step j waits for gather j's event.  The permutation
        of the next epoch is formed on the current stream after its last
        gather was waited for."""
        cfg, M = self.cfg, self.cfg.batch_size
        S = cfg.n_epochs * nmb
        if self._slots is None:
            ws2 = torch.empty_like(self.head.ws)
            self._slots = [(self.mb_obs, self.mb_act, self.mb_aux, self.head.ws),
                           (torch.empty_like(self.mb_obs), torch.empty_like(self.mb_act),
                            torch.empty_like(self.mb_aux), ws2)]
            self._side = torch.cuda.Stream(self.device)
            self._gev = [torch.cuda.Event(), torch.cuda.Event()]
        cur = torch.cuda.current_stream(self.device)
        side, slots, ev = self._side, self._slots, self._gev
        perm = [None]

        def make_perm(epoch):
            perm[0] = self.perm.dev(seed=cfg.seed * 104729 + self.rank,
                                    counter_base=self._pctr, counter_offset=epoch)

        def gather(j):
            k = j % nmb
            o, a, x, ws = slots[j & 1]
            self.gather(perm[0][k * M:(k + 1) * M], o, a, x, ws)

        ws0 = self.head.ws
        try:
            make_perm(0)
            gather(0)
            for j in range(S):
                if j > 0:
                    cur.wait_event(ev[j & 1])
                if j + 1 < S:
                    if (j + 1) % nmb == 0:
                        make_perm((j + 1) // nmb)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        gather(j + 1)
                        ev[(j + 1) & 1].record(side)
                o, a, x, ws = slots[j & 1]
                self.head.ws = ws
                self._train_minibatch(j, o, a, x)
        finally:
            self.head.ws = ws0

    def _train_graphed(self):
        cfg = self.cfg
        T, N, M = cfg.n_steps, cfg.num_envs, cfg.batch_size
        nmb = T * N // M
        S = cfg.n_epochs * nmb
        if self._tstats is None:
            self._tstats = torch.zeros(S, 8, dtype=torch.float32, device=self.device)
            self._sched = torch.zeros(S, 2, dtype=torch.float32, device=self.device)
            self._pctr = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._pctr.fill_(self.num_updates * cfg.n_epochs)
        self.opt.schedule(self.opt.t + 1, S, out=self._sched)
        self.opt.t += S
        obs_flat = self.obs[:T].reshape(T * N, -1)
        act_flat = self.actions.reshape(T * N, 4)
        key = self._graph_key("train")
        if self._tgraph is not None and key != self._tkey:
            self._tgraph = None
        self._tkey = key
        if not self._train_graphable():
            self._train_body(obs_flat, act_flat, nmb)       # eager (e.g. DP over gloo)
        elif self._tgraph is not None:
            self._tgraph.replay()
        elif not self._twarm:
            self._train_body(obs_flat, act_flat, nmb)       # eager once: lazy init
            self._twarm = True
        else:
            cur = torch.cuda.current_stream(self.device)
            cs = torch.cuda.Stream(self.device)
            cs.wait_stream(cur)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(cs), torch.cuda.graph(g, stream=cs):
                self._train_body(obs_flat, act_flat, nmb)
            cur.wait_stream(cs)
            g.replay()
            self._tgraph = g
        self.num_updates += 1
        return self._tstats.mean(0)

    @torch.no_grad()
    def train(self):
        if self._train_fast():
            return self._train_graphed()
        cfg = self.cfg
        T, N, M = cfg.n_steps, cfg.num_envs, cfg.batch_size
        obs_flat = self.obs[:T].reshape(T * N, -1)
        act_flat = self.actions.reshape(T * N, 4)
        log_std = self.policy.log_std.detach()
        nmb = T * N // M
        stats = torch.zeros(cfg.n_epochs * nmb, 8, dtype=torch.float32, device=self.device)
        j = 0
        for epoch in range(cfg.n_epochs):
            perm = self.perm(seed=cfg.seed * 104729 + self.rank,
                             counter=self.num_updates * cfg.n_epochs + epoch)
            for k in range(nmb):
                idx = perm[k * M:(k + 1) * M]
                # gathered copies: the consumers then stream rows in order
                # (reading through `rows=idx` in the kernels measured 3 %
                # slower: 60-B random rows waste most of each cache line)
                if self.use_fused:
                    # one launch gathers obs, actions and aux rows and the
                    # advantage partials the head's normalisation needs
                    self.gather(idx, self.mb_obs, self.mb_act, self.mb_aux,
                                self.head.adv_part)
                    kw = dict(adv_ready=True, stats_out=stats[j])
                    if self.world > 1:
                        # DP: one all-reduce of the flat gradient, or (2
                        # buckets) the early bucket started while the
                        # first-layer backward still runs
                        bar = D.BucketedAllReduce(self.fused.grad, self.world, self.pg)
                        early = bar.start if self.cfg.grad_buckets == 2 else None
                        grad, st = self.fused.step(self.mb_obs, self.mb_act, self.mb_aux,
                                                   self.head, on_ready=early, **kw)
                        bar.finish()
                    elif self.defer_finish:
                        # single GPU: the head / first-layer / split-K
                        # reductions and the norm in one launch before Adam
                        grad, st = self.fused.step(self.mb_obs, self.mb_act, self.mb_aux,
                                                   self.head, defer_finish=True, **kw)
                        self.opt.step_finish(grad, self.fused.finish)
                        j += 1
                        continue
                    else:
                        grad, st = self.fused.step(self.mb_obs, self.mb_act, self.mb_aux,
                                                   self.head, **kw)
                else:
                    K.gather_rows(idx, obs_flat, out=self.mb_obs)
                    K.gather_rows(idx, act_flat, out=self.mb_act)
                    K.gather_rows(idx, self.aux, out=self.mb_aux)
                    mean, value, cache = self.fused.forward(self.mb_obs)
                    g_mean, g_ls, g_v, st = self.loss(mean, log_std, value, self.mb_act,
                                                      aux=self.mb_aux)
                    grad = self.fused.backward(self.mb_obs, cache, g_mean, g_v, g_ls)
                    self._allreduce_grad(grad)
                self.opt.step(grad)
                if st.data_ptr() != stats[j].data_ptr():
                    stats[j].copy_(st)
                j += 1
        self.num_updates += 1
        return stats.mean(0)

    def learn_step(self):
        """One PPO iteration: rollout + GAE + n_epochs of minibatch updates."""
        for upd, eps in self.cfg.eps_schedule:
            if int(upd) == self.num_updates:
                self.env.set("eps", torch.full((self.cfg.num_envs,), float(eps),
                                               dtype=torch.float64))
        self.collect_rollouts()
        return self.train()

    def episode_stats(self):
        """Mean return / length of the episodes that ended in the last rollout
        (VecMonitor's ep_info_buffer role; all-reduced over ranks)."""
        done = self.dones[1:].bool()
        s = torch.stack([torch.where(done, self.ep_ret, 0).sum(),
                         torch.where(done, self.ep_len, 0).sum().float(),
                         done.sum().float()])
        D.allreduce_sum_(s, self.world, group=self.pg)
        n = max(s[2].item(), 1.0)
        return {"ep_rew_mean": s[0].item() / n, "ep_len_mean": s[1].item() / n,
                "episodes": int(s[2].item())}

    def learn(self, total_timesteps: int, log_every: int = 1, logger=print):
        t0 = time.perf_counter()
        while self.num_timesteps < total_timesteps:
            st = self.learn_step()
            if logger and self.rank == 0 and self.num_updates % log_every == 0:
                es = self.episode_stats()
                s = st.tolist()
                logger({"update": self.num_updates, "timesteps": self.num_timesteps,
                        "fps": int(self.num_timesteps / (time.perf_counter() - t0)),
                        **es, "eps_mean": float(self.env.get("eps").mean()),
                        **dict(zip(K.PPOLoss.STATS, s))})
        return self

    # ------------------------------------------------------------ checkpoint
    _ENV_FIELDS = ("pos", "vel", "euler", "omega", "target", "current_step", "ep_num", "eps",
                   "ep_return", "ep_length")

    def _env_fields(self):
        return self._ENV_FIELDS + (("motion",) if self.cfg.variant == "moving" else ())

    def state_dict(self):
        """Everything needed to resume bit-for-bit on the same device count:
        parameters (SB3 names too), Adam moments and step, the env state
        including the per-env curriculum (ep_num, eps) that the reference's
        SB3 .zip does NOT save (drone.py:18,33), rollout continuation, and
        the counters that key every Philox stream."""
        T = self.cfg.n_steps
        return {
            "config": dataclasses.asdict(self.cfg),
            "flat": self.policy.flat.detach().cpu().clone(),
            "policy": self.policy.state_dict(),
            "adam": {"exp_avg": self.opt.m.cpu().clone(), "exp_avg_sq": self.opt.v.cpu().clone(),
                     "step": self.opt.t},
            "env": {k: self.env.get(k).cpu() for k in self._env_fields()},
            "last_obs": self.obs[T if self._rolled else 0].cpu().clone(),
            "last_dones": self.dones[T].cpu().clone(),
            "num_updates": self.num_updates, "num_timesteps": self.num_timesteps,
            "rank": self.rank, "world_size": self.world,
        }

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load_state_dict(self, sd):
        T = self.cfg.n_steps
        with torch.no_grad():
            self.policy.flat.copy_(sd["flat"].to(self.device))
            self.opt.m.copy_(sd["adam"]["exp_avg"].to(self.device))
            self.opt.v.copy_(sd["adam"]["exp_avg_sq"].to(self.device))
            self.opt.t = int(sd["adam"]["step"])
            for k, v in sd["env"].items():
                self.env.set(k, v)
            self.obs[0].copy_(sd["last_obs"].to(self.device))
            self.dones[T].copy_(sd["last_dones"].to(self.device))
        self._rolled = False
        self.num_updates = int(sd["num_updates"])
        self.num_timesteps = int(sd["num_timesteps"])

    def load(self, path):
        self.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))

    def save_sb3(self, path):
        """stable-baselines3 PPO .zip (train.py:70 ``model.save``); see sb3_zip."""
        from . import sb3_zip
        sb3_zip.save(self, path)

    def load_sb3(self, path):
        """Resume from an SB3 PPO .zip (train.py:10-31 ``PPO.load``): params,
        Adam state, timesteps (+ curriculum when written by save_sb3)."""
        from . import sb3_zip
        ck = sb3_zip.load_into(self, path)
        self._rolled = False
        self.dones[self.cfg.n_steps].fill_(1)
        with torch.no_grad():
            self.env.reset(self.obs[0])
        return ck

    def close(self):
        self.env.close()
