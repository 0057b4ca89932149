/*
 * dronerl.h -- C ABI of libdronerl.so, the MI355X (gfx950) batched
 * quadrotor environment and PPO kernels.
 *
 * Boundary.  The reference's env boundary is the gym.Env pair
 *   DroneGymEnv.reset() -> obs(15,) f32               /root/reference/drone.py:270-271 (-> 48-75)
 *   DroneGymEnv.step(a(4,) f32) -> (obs, r, done, {})  /root/reference/drone.py:266-268 (-> 81-159)
 * consumed through SB3 DummyVecEnv + VecMonitor (train.py:33-35), and the
 * batched variant VectorizedDroneEnv.reset/step (vectorized_drone.py:38-57,
 * 135-216).  This library replaces that whole layer (L0 physics + L1 env API
 * + L2 vectorisation) with one GPU-resident batch of N envs.
 *
 * Conventions
 *  - Every data pointer passed to a compute entry point is DEVICE memory
 *    (e.g. a torch tensor's data_ptr on the handle's device) or, for the
 *    per-step I/O of dr_reset / dr_step / dr_step_monitored, pinned host
 *    memory (hipHostMalloc): the kernel then reads the actions from and
 *    writes its outputs to host memory over PCIe (zero-copy), so a
 *    host-buffer step is one launch and one stream sync.  The caller owns
 *    all I/O buffers; the library owns the persistent env state (SoA).
 *  - `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *    Compute entry points only enqueue work: they are asynchronous with
 *    respect to the host and safe to capture into a hipGraph.
 *  - Return value: DR_OK (0) or a negative DR_ERR_* code.  A message for the
 *    last error on a handle is available from dr_last_error(handle);
 *    dr_last_error(NULL) reports errors that happened without a handle
 *    (dr_create).  No C++ exception crosses this ABI.
 *  - A handle is not thread-safe; use one handle per host thread.
 *  - Layouts: actions (N,4) f32 row-major; obs (N,15) f32 row-major for the
 *    "gym" variant, (N,12) for "vectorized"; rewards (N,) f32; dones (N,) u8.
 */
#ifndef DRONERL_H_
#define DRONERL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DR_ABI_VERSION 16

enum dr_status {
    DR_OK = 0,
    DR_ERR_INVALID = -1,   /* bad argument / shape / null handle          */
    DR_ERR_HIP = -2,       /* a HIP runtime call or kernel launch failed  */
    DR_ERR_NOMEM = -3,     /* device allocation failed                    */
    DR_ERR_UNSUPPORTED = -4
};

enum dr_variant {
    DR_VARIANT_GYM = 0,        /* DroneGymEnv, drone.py:13-274             */
    DR_VARIANT_VECTORIZED = 1, /* VectorizedDroneEnv, vectorized_drone.py  */
    /* Moving-target trajectory tracking (BASELINE.json configs[4]; an
       extension with no reference oracle, spec in DESIGN.md section 11):
       gym physics, reset and curriculum; the target moves per axis k as
       c_k + a_k sin(w_k t + ph_k) with per-episode (a, w, ph), a = eps * U,
       so eps = 0 reproduces DR_VARIANT_GYM exactly; obs (N,18) = gym obs +
       target velocity; reward = the gym reward against the moving target. */
    DR_VARIANT_MOVING = 2
};

enum dr_state_dtype {
    DR_STATE_F64 = 0,  /* reference precision (numpy float64 state)       */
    DR_STATE_F32 = 1   /* fp32 state: half the state bytes, unit-floor parity */
};

enum dr_rng_mode {
    /* reset uniforms from counter-based Philox4x32-10 keyed by seed with
       counter (episode number, global env id, tag|block): two blocks give
       the five draws as 32-bit uniforms w * 2^-32.  Reproducible and
       independent of how many other envs reset, or in which order.      */
    DR_RNG_PHILOX = 0,
    /* reset uniforms read from a caller-provided device buffer (N,5) f64,
       row i = the 5 draws env i's next reset consumes, in the reference's
       draw order (pos x, pos y, target x, y, z; drone.py:57,73).  This is
       how parity runs replay numpy's MT19937 stream.                     */
    DR_RNG_HOST_UNIFORMS = 1
};

enum dr_field {   /* dr_get_state / dr_set_state, all device buffers      */
    DR_FIELD_POS = 0,       /* (N,3) f64                                     */
    DR_FIELD_VEL = 1,       /* (N,3) f64                                     */
    DR_FIELD_EULER = 2,     /* (N,3) f64  roll, pitch, yaw (never wrapped)   */
    DR_FIELD_OMEGA = 3,     /* (N,3) f64                                     */
    DR_FIELD_TARGET = 4,    /* (N,3) f64                                     */
    DR_FIELD_STEP = 5,      /* (N,)  i32  current_step (drone.py:28,155)     */
    DR_FIELD_EP_NUM = 6,    /* (N,)  i32  ep_num (drone.py:18,61)            */
    DR_FIELD_EPS = 7,       /* (N,)  f64  curriculum eps (drone.py:33,70)    */
    DR_FIELD_EP_RETURN = 8, /* (N,)  f32  running episode return (monitor)   */
    DR_FIELD_EP_LENGTH = 9, /* (N,)  i32  running episode length (monitor)   */
    DR_FIELD_MOTION = 10    /* (N,9) f32  moving variant: a xyz, w xyz, ph xyz
                               (DR_FIELD_TARGET is then the motion centre)  */
};

typedef struct dr_config {
    int64_t num_envs;       /* N >= 1                                        */
    int32_t variant;        /* enum dr_variant                               */
    int32_t state_dtype;    /* enum dr_state_dtype                           */
    int32_t rng_mode;       /* enum dr_rng_mode                              */
    int32_t auto_reset;     /* 1: DummyVecEnv semantics (reset a done env in
                               the same step, obs_out = reset obs); 0: raw
                               env semantics (caller resets).  Ignored (0)
                               for the vectorized variant, which never
                               auto-resets (vectorized_drone.py:211-213).    */
    int32_t device;         /* HIP device ordinal                            */
    int32_t max_steps;      /* 0 = variant default (200 gym, 1000 vectorized) */
    uint64_t seed;          /* Philox key                                    */
    int64_t env_id_offset;  /* global id of env 0 (rank * N for DP shards)   */
    double dt;              /* 0 = reference default 0.02 (drone.py:14)      */
} dr_config;

typedef struct dr_handle dr_handle;

/* Library ABI version (DR_ABI_VERSION of the build). */
int dr_abi_version(void);

/* Create N envs on cfg->device.  Mirrors the reference constructor: every
   env performs one reset (drone.py:46), so ep_num starts at 1.  In
   DR_RNG_HOST_UNIFORMS mode no uniform buffer exists yet, so that first
   reset uses u = 0.5 for all five draws (pos (0,0,1); the target is
   (0,0,1) anyway while eps = 0).  Replaces DroneGymEnv.__init__
   (drone.py:255-264) and VectorizedDroneEnv.__init__ (vectorized_drone.py:13-36).
   Synchronous: returns after the state is initialised. */
int dr_create(const dr_config *cfg, dr_handle **out);
int dr_destroy(dr_handle *h);

int64_t dr_num_envs(const dr_handle *h);
int dr_obs_dim(const dr_handle *h);   /* 15 gym, 12 vectorized, 18 moving */

/* Reset every env and write (N,obs_dim) obs.  Replaces DroneEnv.reset
   (drone.py:48-75) called on each env by VecEnv.reset, and
   VectorizedDroneEnv.reset (vectorized_drone.py:38-57). */
int dr_reset(dr_handle *h, float *obs_out, void *stream);

/* Reset only envs with mask[i] != 0 ((N,) u8); obs_out rows of other envs are
   rewritten with their current obs.  (DummyVecEnv-free callers, test
   harnesses.)  Not available for the vectorized variant. */
int dr_reset_masked(dr_handle *h, const uint8_t *mask, float *obs_out,
                    void *stream);

/* One env step for all N envs.  Replaces DroneEnv.step (drone.py:81-159)
   looped by DummyVecEnv.step_wait, and VectorizedDroneEnv.step
   (vectorized_drone.py:135-216).
     actions        (N,4) f32, NOT clipped (the reference env does not clip)
     obs_out        (N,obs_dim) f32; with auto_reset, rows of done envs hold
                    the reset observation (DummyVecEnv semantics)
     rew_out        (N,) f32 (SB3 buffers rewards as f32)
     done_out       (N,) u8
     terminal_obs_out  nullable (N,obs_dim) f32: for done envs the obs
                    BEFORE the auto-reset ("terminal_observation"); rows of
                    envs that are not done are left untouched.            */
int dr_step(dr_handle *h, const float *actions, float *obs_out,
            float *rew_out, uint8_t *done_out, float *terminal_obs_out,
            void *stream);

/* dr_step plus VecMonitor bookkeeping (running f32 return, i32 length per
   env): for done envs the finished episode's return/length are written to
   ep_return_out / ep_length_out ((N,) each; other rows untouched) and the
   running counters restart.  SB3 VecMonitor.step_wait equivalent. */
int dr_step_monitored(dr_handle *h, const float *actions, float *obs_out,
                      float *rew_out, uint8_t *done_out,
                      float *terminal_obs_out, float *ep_return_out,
                      int32_t *ep_length_out, void *stream);

/* dr_step_monitored plus the gymnasium TimeLimit split: truncated_out (N) u8
   (non-null) gets 1 where the episode ended at the step limit without a
   crash (drone.py:155-157 vs 154), 0 elsewhere.  The reference's env reports
   both as terminated (SB3 sees it through shimmy's GymV21 compatibility), so
   only PPOConfig.bootstrap_timeouts uses it: SB3's rewards[i] += gamma *
   V(terminal_obs[i]) for truncated envs.  (ABI v12.) */
int dr_step_monitored_trunc(dr_handle *h, const float *actions, float *obs_out,
                            float *rew_out, uint8_t *done_out, float *terminal_obs_out,
                            float *ep_return_out, int32_t *ep_length_out,
                            uint8_t *truncated_out, void *stream);

/* Device-side state access (parity injection, checkpointing, get_attr). */
int dr_get_state(dr_handle *h, int field, void *out, void *stream);
/* dr_get_state for k selected envs: out row j = field of env env_ids[j]
   ((k,3) f64 for vector fields, (k,) for scalars, (k,9) f32 for MOTION).
   The per-step `get_attr('pos')` of TrajectoryTensorboardCallback
   (traj_tb.py:34) without copying the whole batch. */
int dr_gather_state(dr_handle *h, int field, const int32_t *env_ids, int64_t k,
                    void *out, void *stream);
int dr_set_state(dr_handle *h, int field, const void *in, void *stream);

/* DR_RNG_HOST_UNIFORMS: device pointer to (N,5) f64 ((N,14) for the moving
   variant: the 5 gym draws, then a xyz, w xyz, ph xyz) read by every later
   reset until replaced.  The buffer must stay alive while work using it is
   in flight. */
int dr_set_reset_uniforms(dr_handle *h, const double *u_dev);

/* Replace the Philox key used by later resets (VecEnv.seed).  Takes effect
   for work enqueued after the call. */
int dr_set_seed(dr_handle *h, uint64_t seed);

/* Synthetic random policy: out (n,4) f32 i.i.d. U[lo,hi) from Philox keyed
   by seed with counter (env_id_offset + i, step).  Not part of the
   reference; it generates the benchmark's action stream. */
int dr_random_actions(int64_t n, uint64_t seed, int64_t env_id_offset,
                      int64_t step, float lo, float hi, float *out,
                      void *stream);

/* K successive steps in ONE launch, the state held in registers between
   steps: outputs identical, bit for bit, to k calls of
   dr_step(h, actions + t*N*4, obs_out + t*N*obs_dim, rew_out + t*N,
   done_out + t*N, NULL) for t = 0..k-1 (auto-reset per the handle; no
   terminal obs, no VecMonitor counters).  The random-policy rollout loop
   `a = action_space.sample(); env.step(a)` over DroneEnv.step
   (drone.py:81-159) k times, without the per-step state round trip
   through HBM or the per-launch gap.
     actions   (k,N,4) f32, 16-byte aligned
     obs_out   (k,N,obs_dim) f32; rew_out (k,N) f32; done_out (k,N) u8
   k * N <= 2^31.  DR_RNG_HOST_UNIFORMS handles with auto-reset are
   DR_ERR_UNSUPPORTED (their reset draws are supplied per step).  (ABI v11.) */
int dr_rollout(dr_handle *h, int32_t k, const float *actions, float *obs_out,
               float *rew_out, uint8_t *done_out, void *stream);

/* dr_rollout with its kernel's start / end recorded into two hipEvent_t
   (either may be NULL) by hipExtLaunchKernel: the events take the dispatch
   packet's own timestamps, so timing a launch adds no packets to the
   stream (a benchmark's hipEventRecord pair costs several microseconds of
   host and queue time around a ~35 us launch).  Same outputs as
   dr_rollout.  (ABI v13.) */
int dr_rollout_timed(dr_handle *h, int32_t k, const float *actions, float *obs_out,
                     float *rew_out, uint8_t *done_out, void *stream,
                     void *start_event, void *stop_event);

/* dr_rollout on the synthetic random policy drawn in-kernel: step t's
   actions are exactly dr_random_actions(N, action_seed, env_id_offset of
   the handle, action_step0 + t, lo, hi).  actions_out nullable: (k,N,4) f32
   copy of the drawn actions.  (ABI v11.) */
int dr_rollout_random(dr_handle *h, int32_t k, uint64_t action_seed,
                      int64_t action_step0, float lo, float hi, float *actions_out,
                      float *obs_out, float *rew_out, uint8_t *done_out,
                      void *stream);

const char *dr_last_error(const dr_handle *h);

/* ---------------------------------------------------------------------------
 * PPO kernels (stable-baselines3 PPO arithmetic; the
 * reference calls it at train.py:36-43, 63-68).  All buffers are device
 * memory; layouts are time-major (T,N) so a fixed step is contiguous.
 * ------------------------------------------------------------------------- */

/* GAE reverse scan, RolloutBuffer.compute_returns_and_advantage:
   delta_t = r_t + g*V_{t+1}*(1-start_{t+1}) - V_t,
   A_t = delta_t + g*l*(1-start_{t+1})*A_{t+1}; the last step uses
   (1-last_dones) and last_values; R = A + V.  All arithmetic is f32 with
   numpy's NEP-50 rounding: gamma -> f32, gamma*lambda formed in f64 then
   rounded to f32 (SB3 multiplies two python floats first). */
int dr_gae(int64_t T, int64_t N, const float *rewards, const float *values,
           const uint8_t *episode_starts, const float *last_values,
           const uint8_t *last_dones, double gamma, double gae_lambda,
           float *advantages, float *returns, void *stream);

/* Diagonal-Gaussian action sampling for the rollout:
   a = mean + exp(log_std) * z, z ~ N(0,1) (Philox + Box-Muller keyed by
   (seed, counter, row)); logp = sum_j log N(a_j; mean_j, std_j);
   actions_clipped = clip(a, lo, hi) (what SB3 passes to env.step).
   actions_raw / logp / actions_clipped may each be NULL. */
int dr_policy_sample(int64_t n, const float *mean, const float *log_std,
                     uint64_t seed, uint64_t counter, float lo, float hi,
                     float *actions_raw, float *actions_clipped, float *logp,
                     void *stream);

/* dr_policy_sample with counter = *counter_base + counter_offset, the base
   read on the device (8-byte aligned u64): a rollout loop captured once
   into a hipGraph draws fresh noise on every replay when the caller
   advances the base between replays.  Bitwise dr_policy_sample for the same
   counter.  (ABI v8.) */
int dr_policy_sample_dev(int64_t n, const float *mean, const float *log_std,
                         uint64_t seed, const uint64_t *counter_base,
                         uint64_t counter_offset, float lo, float hi,
                         float *actions_raw, float *actions_clipped, float *logp,
                         void *stream);

/* Uniform random permutation of [0,n) (RolloutBuffer.get's
   np.random.permutation): the stable argsort of 64-bit Philox keys, by a
   bucket pass on the top key bits plus per-bucket bitonic sorts (no state
   kept across launches: graph-capturable).  dr_permutation_workspace_bytes
   gives the scratch size for n. */
size_t dr_permutation_workspace_bytes(int64_t n);
int dr_permutation(int64_t n, uint64_t seed, uint64_t counter, int32_t *out,
                   void *workspace, size_t workspace_bytes, void *stream);
/* dr_permutation with counter = *counter_base + counter_offset, the base a
   device u64 (8-byte aligned): graph-capturable epochs.  (ABI v9.) */
int dr_permutation_dev(int64_t n, uint64_t seed, const uint64_t *counter_base,
                       uint64_t counter_offset, int32_t *out, void *workspace,
                       size_t workspace_bytes, void *stream);

/* Gather a minibatch: dst[k,:] = src[idx[k],:] for row width `width`
   (floats), k < m.  Used to form minibatches from the flat rollout. */
int dr_gather_rows(int64_t m, int64_t width, const int32_t *idx,
                   const float *src, float *dst, void *stream);

/* A whole PPO.train minibatch in one launch (RolloutBuffer.get's
   `self.observations[batch_inds]` etc.): obs_out[r,:] = obs[idx[r],:]
   (obs_dim floats), actions_out[r,:] = actions[idx[r],:] (4 floats, rows
   16-byte aligned), aux_out[r,:] = aux[idx[r],:] (old_logp, advantage,
   return).  With adv_part non-null it also writes the per-256-row
   (count, mean, M2) partials of the gathered advantages that
   dr_ppo_head_loss_backward's normalisation consumes: pass the head's
   workspace and normalize_advantage = 2 there to skip its own pass. */
int dr_gather_minibatch(int64_t m, const int32_t *idx, int64_t obs_dim,
                        const float *obs, const float *actions,
                        const float *aux, float *obs_out, float *actions_out,
                        float *aux_out, float *adv_part, void *stream);

/* One-line rollout records (ABI v16, round 6): the PPO.train minibatch
   gather of RolloutBuffer.get (`self.observations[batch_inds]`,
   `self.actions[...]`, old log-probs / advantages / returns) reads one
   aligned 128-B line per row instead of three arrays' lines.
   dr_pack_rollout_records writes record r (DR_RECORD_FLOATS floats) from
   rollout row r once per iteration: floats 0 .. obs_dim-1 = obs[r,:], from
   a = 4 ceil(obs_dim / 4): a .. a+3 = actions[r,:], a+4 .. a+6 = (logp[r],
   adv[r], ret[r]), the rest 0 (obs_dim <= 24: 16 / 20 for the 15-d gym and
   18-d moving obs; actions and records 16-byte aligned; n rows).
   dr_gather_records then writes exactly dr_gather_minibatch's outputs
   (obs_out (m, obs_dim), actions_out (m, 4), aux_out (m, 3), the advantage
   partials when adv_part is non-null) from the records of rows idx[0..m). */
#define DR_RECORD_FLOATS 32
int dr_pack_rollout_records(int64_t n, int64_t obs_dim, const float *obs,
                            const float *actions, const float *logp, const float *adv,
                            const float *ret, float *records, void *stream);
int dr_gather_records(int64_t m, const int32_t *idx, int64_t obs_dim, const float *records,
                      float *obs_out, float *actions_out, float *aux_out, float *adv_part,
                      void *stream);

/* Tanh-layer backward fused with the bias gradient (the MLP backward of
   PPO.train): grad_z = grad_h * (1 - h^2) for an (m, n) activation h =
   tanh(z), and bias_grad[j] = sum_i grad_z[i, j].  n must be a multiple of
   4 and <= 1024.  `workspace` >= dr_tanh_backward_workspace_bytes(m, n). */
size_t dr_tanh_backward_workspace_bytes(int64_t m, int64_t n);
int dr_tanh_backward(int64_t m, int64_t n, const float *grad_h, const float *h,
                     float *grad_z, float *bias_grad, void *workspace,
                     size_t workspace_bytes, void *stream);

/* First MLP layer forward fused with its activation: h = tanh(x W^T + b)
   for x (m,k), W (n,k), b (n), h (m,n) (SB3 MlpExtractor's Linear + Tanh,
   the narrow-input layer).  k in {4,8,12,15,16,18,24,32}; n % 4 == 0,
   n <= 256; h 16-byte aligned.  Replaces an addmm plus a separate tanh pass
   over the (m,n) activation.  `rows` (nullable, m int32): input row r is
   x[rows[r]] -- a minibatch read in place from the rollout buffer through
   its permutation (RolloutBuffer.get without the gather copy). */
int dr_linear_tanh(int64_t m, int64_t k, int64_t n, const float *x,
                   const int32_t *rows, const float *w, const float *b, float *h,
                   void *stream);

/* dr_linear_tanh for both MLPs of the actor-critic (pi: w0/b0/h0, vf:
   w1/b1/h1) over the same input rows, in one launch. */
int dr_linear_tanh2(int64_t m, int64_t k, int64_t n, const float *x,
                    const int32_t *rows, const float *w0, const float *b0,
                    float *h0, const float *w1, const float *b1, float *h1,
                    void *stream);

/* Backward of the first layer h = tanh(x W^T + b), fused: for grad_h (m,n)
   = dLoss/dh, forms grad_z = grad_h * (1 - h^2) in registers (never stored)
   and writes grad_w (n,k) = grad_z^T x and grad_b (n) = sum_r grad_z
   (dr_tanh_backward + the weight-gradient GEMM in one pass; the input
   gradient of the first layer is not needed).  k as dr_linear_tanh; n % 4
   == 0, n <= 256; grad_h and h 16-byte aligned.  `rows` as dr_linear_tanh
   (x row r = x[rows[r]]).  Deterministic.
   `workspace` >= dr_first_layer_backward_workspace_bytes(m, k, n). */
size_t dr_first_layer_backward_workspace_bytes(int64_t m, int64_t k, int64_t n);
int dr_first_layer_backward(int64_t m, int64_t k, int64_t n, const float *grad_h,
                            const float *h, const float *x, const int32_t *rows,
                            float *grad_w, float *grad_b, void *workspace,
                            size_t workspace_bytes, void *stream);

/* dr_first_layer_backward for both MLPs (net 0: grad_h0/h0 -> grad_w0/
   grad_b0, net 1: grad_h1/h1 -> grad_w1/grad_b1) over the same input x in
   one launch (plus one column-sum and one finish launch for both).
   Bitwise the same results as two dr_first_layer_backward calls.  defer
   != 0 leaves the last reduction (and the grad_w / grad_b writes) to
   dr_grad_finish_clip_adam.
   `workspace` >= dr_first_layer_backward2_workspace_bytes(m, k, n). */
size_t dr_first_layer_backward2_workspace_bytes(int64_t m, int64_t k, int64_t n);
int dr_first_layer_backward2(int64_t m, int64_t k, int64_t n, const float *x,
                             const int32_t *rows, const float *grad_h0,
                             const float *h0, float *grad_w0, float *grad_b0,
                             const float *grad_h1, const float *h1,
                             float *grad_w1, float *grad_b1, int defer,
                             void *workspace, size_t workspace_bytes,
                             void *stream);

/* Policy heads for rollouts (ActorCriticPolicy.forward's action_net /
   value_net): mean (m,4) = h_pi W_act^T + b_act, value (m) = h_vf W_val^T +
   b_val, for the top hidden activations h_pi, h_vf (m,hd), hd % 4 == 0,
   hd <= 256.  With preact != 0 the inputs are the top layer's
   PRE-activations z and tanh(z + zb) is applied on load (the layer's
   separate tanh pass is then skipped); zb_pi / zb_vf (nullable, hd floats,
   16-byte aligned; only with preact) are the top layer's biases when its
   GEMM left them out.  Row buffers 16-byte aligned. */
int dr_policy_heads(int64_t m, int64_t hd, int preact, const float *h_pi,
                    const float *h_vf, const float *zb_pi, const float *zb_vf,
                    const float *w_act, const float *b_act, const float *w_val,
                    const float *b_val, float *mean, float *value, void *stream);

/* One PPO.train minibatch step from the top hidden layer down, fused:
   heads (as dr_policy_heads), the loss of dr_ppo_loss (aux = interleaved
   (m,3) rows of old_logp, advantage, return; with `rows` non-null, minibatch
   row r reads actions / aux row rows[r]), and the backward through the
   heads and the top tanh:
     gz_pi = (dL/dmean W_act) * (1 - h_pi^2),  gz_vf = (dL/dvalue W_val) *
     (1 - h_vf^2)   (m,hd) each, for the hidden-layer backward,
   plus the gradients of W_act (4,hd), b_act (4), W_val (1,hd), b_val (1),
   the top hidden biases b_pi, b_vf (hd) and log_std (4), and stats (8) as
   dr_ppo_loss.  Gradient outputs are written (not accumulated); they may be
   views into one flat gradient buffer.  Deterministic (fixed-order partial
   sums).  `preact`, zb_pi, zb_vf as dr_policy_heads (h_pi / h_vf
   pre-activations; grad_z uses tanh(z + zb)).  `workspace` >= dr_ppo_head_workspace_bytes(m, hd).
   normalize_advantage: 0 off, 1 on, 2 on with the advantage partials
   already written to the head of `workspace` by dr_gather_minibatch.
   defer != 0: the gradient / stats outputs are NOT written here; the
   reduced partials stay in `workspace` for dr_grad_finish_clip_adam (defer
   2: unreduced, for a finish with head_direct = 1; no grouping launch). */
size_t dr_ppo_head_workspace_bytes(int64_t m, int64_t hd);
int dr_ppo_head_loss_backward(int64_t m, int64_t hd, int preact, const float *h_pi,
                              const float *h_vf, const float *zb_pi,
                              const float *zb_vf, const float *w_act,
                              const float *b_act, const float *w_val,
                              const float *b_val, const float *log_std,
                              const float *actions, const float *aux,
                              const int32_t *rows, float clip_range,
                              float ent_coef, float vf_coef,
                              int normalize_advantage, float *gz_pi,
                              float *gz_vf, float *g_w_act, float *g_b_act,
                              float *g_w_val, float *g_b_val, float *g_b_pi,
                              float *g_b_vf, float *g_log_std, float *stats,
                              int defer, void *workspace, size_t workspace_bytes,
                              void *stream);

/* Fused PPO loss + gradient of the loss w.r.t. the policy head outputs
   (PPO.train: normalised advantage, ratio/clip surrogate, value MSE,
   entropy).  Inputs for a minibatch of m rows:
     mean (m,4), log_std (4), values (m), actions (m,4), old_logp (m),
     advantages (m), returns (m); old_logp / advantages / returns are read
     with element stride aux_stride (1: three arrays; 3: one interleaved
     (m,3) array of rows (old_logp, advantage, return), the rollout
     buffer's gathered minibatch, no repacking copies).
   Outputs:
     grad_mean (m,4), grad_values (m), grad_log_std (4): dLoss/d(.)
     stats (8) f32: [loss, policy_loss, value_loss, entropy_loss,
                     clip_fraction, approx_kl, adv_mean, adv_std]
   `workspace` >= dr_ppo_loss_workspace_bytes(m). */
size_t dr_ppo_loss_workspace_bytes(int64_t m);
int dr_ppo_loss(int64_t m, const float *mean, const float *log_std,
                const float *values, const float *actions,
                const float *old_logp, const float *advantages,
                const float *returns, int64_t aux_stride, float clip_range,
                float ent_coef,
                float vf_coef, int normalize_advantage, float *grad_mean,
                float *grad_values, float *grad_log_std, float *stats,
                void *workspace, size_t workspace_bytes, void *stream);

/* clip_grad_norm_(max_norm) + Adam step over one flat fp32 parameter
   buffer (torch.optim.Adam semantics, bias-corrected, eps outside sqrt).
   `step` is the 1-based Adam step count.  grad_norm_out (1) f32 nullable.
   lr / betas / eps are doubles because torch forms 1-beta, lr/bias_correction
   from Python floats before rounding them to f32 scalars.
   `workspace` >= dr_adam_workspace_bytes(n). */
size_t dr_adam_workspace_bytes(int64_t n);
int dr_clip_adam(int64_t n, float *params, float *grads, float *exp_avg,
                 float *exp_avg_sq, double lr, double beta1, double beta2,
                 double eps, float max_grad_norm, int64_t step,
                 float *grad_norm_out, void *workspace,
                 size_t workspace_bytes, void *stream);

/* The deferred reductions of one fused PPO.train minibatch step (the
   single-GPU path): the level-2 partial sums left by
   dr_ppo_head_loss_backward(..., defer = 1) and
   dr_first_layer_backward2(..., defer = 1), and the split-K chunk sum of
   the weight gradients above the first layer,
     chunk_dst[g*chunk_size + i] = sum_c chunks[(g*chunk_count + c)*chunk_size + i].
   Any of the three sources may be NULL (segment skipped); together they
   must write every entry of the flat gradient passed to
   dr_grad_finish_clip_adam, whose norm they also form. */
typedef struct dr_grad_finish {
    const void *head_workspace;      /* dr_ppo_head_loss_backward's */
    int64_t head_m, head_hd;
    const float *log_std;
    float ent_coef, vf_coef;
    float *g_w_act, *g_b_act, *g_w_val, *g_b_val, *g_b_pi, *g_b_vf, *g_log_std;
    float *stats;                    /* (8), as dr_ppo_head_loss_backward */
    const void *first_workspace;     /* dr_first_layer_backward2's */
    int64_t first_m, first_k, first_n;
    float *g_w0, *g_b0, *g_w1, *g_b1;
    const float *chunks;
    int64_t chunk_groups, chunk_count, chunk_size;
    float *chunk_dst;
    /* 0: first_workspace holds dr_first_layer_backward2's level-1 groups;
       > 0: that many per-block rows at its start, left by
       dr_gemm_x6_bwd_first(..., direct = 1) (= dr_gemm_x6_bwd_first_rows(m);
       summed by the finish, no grouping launch).  (ABI v15.) */
    int64_t first_rows;
    /* 0: head_workspace holds the level-1 groups; 1: the head kernel's
       per-block rows, left by dr_ppo_head_loss_backward(..., defer = 2)
       (summed by the finish in the grouped order: bitwise the same).
       (ABI v15.) */
    int64_t head_direct;
} dr_grad_finish;

/* dr_clip_adam fused with the deferred gradient finish: one launch reduces
   every deferred partial into `grads` (and the loss stats) and forms the
   norm partials, a second applies clip_grad_norm_ + Adam.  Two launches
   instead of six.  `workspace` >= dr_grad_finish_workspace_bytes(f). */
size_t dr_grad_finish_workspace_bytes(const dr_grad_finish *f);
int dr_grad_finish_clip_adam(const dr_grad_finish *f, int64_t n, float *params,
                             float *grads, float *exp_avg, float *exp_avg_sq,
                             double lr, double beta1, double beta2,
                             double eps, float max_grad_norm, int64_t step,
                             float *grad_norm_out, void *workspace,
                             size_t workspace_bytes, void *stream);

/* Host-only: torch.optim.Adam's step-dependent scalars for step >= 1, as
   dr_clip_adam / dr_grad_finish_clip_adam form them: out[0] = lr /
   (1 - beta1^step), out[1] = sqrt(1 - beta2^step), in double, then f32.
   (ABI v9.) */
int dr_adam_schedule(double lr, double beta1, double beta2, int64_t step, float *out);

/* dr_grad_finish_clip_adam with the step's two scalars read on the device
   from `sched` (2 floats, 8-byte aligned, filled from dr_adam_schedule):
   a training loop captured once into a hipGraph replays with the right
   bias corrections when the host rewrites the schedule between replays.
   Bitwise dr_grad_finish_clip_adam for the same step.  (ABI v9.) */
int dr_grad_finish_clip_adam_sched(const dr_grad_finish *f, int64_t n, float *params,
                                   float *grads, float *exp_avg, float *exp_avg_sq,
                                   double lr, double beta1, double beta2, double eps,
                                   float max_grad_norm, const float *sched,
                                   float *grad_norm_out, void *workspace,
                                   size_t workspace_bytes, void *stream);

/* The data-parallel split of dr_grad_finish_clip_adam_sched (SB3 PPO.train
   + the north_star's one gradient all-reduce per optimizer step over ranks,
   /root/reference/train.py:63-68): dr_grad_finish_run reduces every deferred
   partial of `f` into the flat gradient (and the loss stats) in ONE launch;
   the caller then sums the gradient over ranks (RCCL all-reduce) and
   dr_clip_adam_sched applies clip_grad_norm_ + Adam to grad_scale * grads
   (grad_scale = 1 / world: the mean) with the step's scalars read on the
   device from `sched` (dr_adam_schedule).  At grad_scale 1 the pair is
   bitwise dr_grad_finish_clip_adam_sched; both are graph-capturable.
   dr_grad_finish_run's `workspace` >= dr_grad_finish_workspace_bytes(f);
   dr_clip_adam_sched's >= dr_adam_workspace_bytes(n).  (ABI v12.) */
int dr_grad_finish_run(const dr_grad_finish *f, void *workspace, size_t workspace_bytes,
                   void *stream);
int dr_clip_adam_sched(int64_t n, float *params, float *grads, float *exp_avg,
                       float *exp_avg_sq, double beta1, double beta2, double eps,
                       float max_grad_norm, float grad_scale, const float *sched,
                       float *grad_norm_out, void *workspace, size_t workspace_bytes,
                       void *stream);

/* ---- fp32-accurate 256 x 256 layer GEMM on the bf16 matrix cores ---------
   Replaces the torch fp32 Linear of SB3's MlpExtractor 256 -> 256 layer
   (forward z = h W^T and the input gradient grad_h = grad_z W; reference
   policy net_arch at /root/reference/train.py:36-43).  Operands are split
   exactly into three bf16 planes and multiplied with six MFMA products per
   element pair (csrc/gemm_x6.hip); the error against an f64 GEMM is below
   the f32 MFMA GEMM's.  (ABI v10.) */

/* Bytes of the pre-split weight image of `batch` (1 or 2) 256 x 256 layers. */
size_t dr_gemm_x6_weights_bytes(int64_t batch);

/* Split `batch` row-major 256 x 256 f32 weights w (consecutive) into the
   image dr_gemm_x6 reads: transpose 0 for C = A W^T, 1 for C = A W, 2 for
   both in one launch (the transpose-0 image at img, the transpose-1 image
   right after it).  img 16-byte aligned, dr_gemm_x6_weights_bytes(batch)
   bytes (twice that for transpose 2). */
int dr_gemm_x6_split_weights(int64_t batch, const float *w, int transpose, void *img,
                             void *stream);

/* C[b] = A[b] . Bt[b]^T for b < batch: A (batch, m, 256) f32, C (batch, m,
   256) f32, Bt given by img.  m a positive multiple of 128; a, img and c
   16-byte aligned.  Deterministic. */
int dr_gemm_x6(int64_t batch, int64_t m, const float *a, const void *img, float *c,
               void *stream);

/* The layer's weight gradient on the same arithmetic, split over `chunks`
   row chunks: ws[b][c] (256 x 256) = G[b][rows of chunk c]^T H[b][rows of
   chunk c] for G (batch, m, 256) = grad_z and H (batch, m, 256) = the layer
   input (torch's split-K bmm layout; the caller sums the chunks).
   m / chunks a positive multiple of 32; pointers 16-byte aligned.
   Deterministic.  (ABI v10.) */
int dr_gemm_x6_wgrad(int64_t batch, int64_t m, int64_t chunks, const float *g, const float *h,
                     float *ws, void *stream);

/* The first-layer operand image of dr_gemm_x6_bwd_first: the minibatch
   observations x (m x k f32 row-major, k <= 15) with a constant 1 as the
   16th feature, split exactly into three bf16 planes in the MFMA fragment
   order (dr_gemm_x6_x_bytes(m) bytes, 16-byte aligned).  (ABI v15.) */
size_t dr_gemm_x6_x_bytes(int64_t m);
int dr_gemm_x6_split_x(int64_t m, int64_t k, const float *x, void *ximg, void *stream);

/* The 256 x 256 layer's input gradient with the first layer's backward
   fused into its epilogue (replaces dr_gemm_x6(2, m, grad_z, img W-form,
   grad_h) followed by dr_first_layer_backward2(..., defer = 1); PPO.train's
   backward through SB3's MlpExtractor, /root/reference/train.py:36-43):
   grad_h1 = grad_z W per net stays in registers, grad_z1 = grad_h1 (1 - h^2)
   with h (2, m, 256) the first layer's activations, and the first layer's
   weight and bias gradients accumulate on the matrix cores against ximg
   (dr_gemm_x6_split_x of the same minibatch's x, k = 15).  `workspace` is
   dr_first_layer_backward2's (>= dr_first_layer_backward2_workspace_bytes(m,
   15, 256)) and is left exactly as its defer = 1 form leaves it: the next
   dr_grad_finish / dr_grad_finish_clip_adam with first_workspace =
   workspace writes the gradients.  With direct != 0 the kernel's per-block
   rows are left at the workspace start instead (no grouping launch) for a
   finish with first_rows = dr_gemm_x6_bwd_first_rows(m).  batch 2, m a
   positive multiple of 128, pointers 16-byte aligned.  Deterministic.
   (ABI v15.) */
int dr_gemm_x6_bwd_first(int64_t batch, int64_t m, int64_t k, const float *grad_z,
                         const void *img, const float *h, const void *ximg, void *workspace,
                         size_t workspace_bytes, int direct, void *stream);
/* The number of per-block rows dr_gemm_x6_bwd_first(..., direct = 1) leaves
   at m rows on the current device (0 for an invalid m). */
int64_t dr_gemm_x6_bwd_first_rows(int64_t m);

/* dr_linear_tanh2 (k = 15, n = 256) with the x6 GEMMs' operand images built
   by extra blocks of the same launch: both weight forms of the 256 x 256
   layer into img (dr_gemm_x6_split_weights(2, w256, 2, img) -- w256 the
   (2, 256, 256) weights of both nets) and, with ximg non-null, the
   observation image of dr_gemm_x6_bwd_first (dr_gemm_x6_split_x of x, read
   through rows when given; m a multiple of 128).  The same bytes as the
   separate launches.  (ABI v15.) */
int dr_linear_tanh2_x6(int64_t m, int64_t k, int64_t n, const float *x, const int32_t *rows,
                       const float *w0, const float *b0, float *h0, const float *w1,
                       const float *b1, float *h1, const float *w256, void *img, void *ximg,
                       void *stream);

#ifdef __cplusplus
}
#endif
#endif /* DRONERL_H_ */
