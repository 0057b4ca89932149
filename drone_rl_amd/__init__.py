"""drone_rl_amd -- MI355X-native batched quadrotor env + PPO (the hot path of
henryplas/drone_rl).

Product path: libdronerl.so (HIP, gfx950; C ABI in include/dronerl.h) driven
through ctypes.  There is no CPU fallback: constructing an env without the
library or without a HIP device raises.
"""
__version__ = "0.1.0"

from .env import (DT, G, MASS, MAX_STEPS, MOTOR_MAX, DroneBatch,  # noqa: F401
                  DroneGymEnv, random_actions)
