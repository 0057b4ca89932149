"""CPU oracle for the drone_rl hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline.  The product
path (drone_rl_amd, libdronerl.so) never imports or links it.

  drone_ref.c / cref.py   C restatement of DroneEnv.step/reset and
                          VectorizedDroneEnv.step (op-for-op, f64)
  drone_np.py             numpy restatement: single-env DroneGymEnv port
                          (the CPU baseline's per-env loop) + batched form
  ppo_ref.c / ppo_ref.py  Philox, GAE and SB3 PPO loss/Adam restatements

Parity status: the env oracles are pinned to golden vectors produced by the
reference itself (tests/golden/make_golden.py); the PPO oracle is
"parity unpinned" (stable-baselines3 is neither vendored nor installed).
"""
