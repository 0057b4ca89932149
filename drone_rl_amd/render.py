"""3-D drone rendering and GIF recording from the GPU env's state: the
reference's DroneEnv.start_record / render / stop_record (drone.py:189-248),
used by test.py:9-21 to record a trained policy.

The state (pos, euler, target) is read from the device batch each frame
(one field read per quantity through pinned host memory); the drawing is
matplotlib's, as in the reference: a 3-D axes with the target (green), the
drone centre (red), the four motors (blue) on the two arms (purple), the
motors placed by the body->inertial rotation of the current Euler angles,
axes fixed to x, y in [-5, 5], z in [0, 5], frames grabbed by PillowWriter.
This is off the hot path (one env, host-side drawing)."""
from __future__ import annotations

import numpy as np


def rotation_matrix(euler) -> np.ndarray:
    """Body -> inertial rotation for ZYX Euler angles (roll, pitch, yaw), as
    DroneEnv._rotation_matrix (drone.py:161-174); host-side, for drawing."""
    phi, theta, psi = (float(x) for x in euler)
    cf, sf = np.cos(phi), np.sin(phi)
    ct, st = np.cos(theta), np.sin(theta)
    cp, sp = np.cos(psi), np.sin(psi)
    return np.array([
        [cp * ct, cp * st * sf - sp * cf, cp * st * cf + sp * sf],
        [sp * ct, sp * st * sf + cp * cf, sp * st * cf - cp * sf],
        [-st, ct * sf, ct * cf]])


def motor_positions(pos, euler, arm_length: float) -> np.ndarray:
    """(4, 3) motor centres: the X-configuration offsets (drone.py:220-225)
    rotated into the inertial frame and shifted by pos."""
    a = arm_length / np.sqrt(2)
    offsets = np.array([[a, a, 0.0], [-a, a, 0.0], [-a, -a, 0.0], [a, -a, 0.0]])
    return np.asarray(pos, np.float64) + (rotation_matrix(euler) @ offsets.T).T


class DroneRecorder:
    """Figure + PillowWriter state of one env (the reference keeps it on the
    env as _fig / _writer)."""

    def __init__(self):
        self._fig = None
        self._ax = None
        self._writer = None

    @staticmethod
    def _plt():
        import matplotlib
        if matplotlib.get_backend().lower() not in ("agg", "module://matplotlib_inline.backend_inline"):
            try:
                matplotlib.use("Agg")          # headless, as the reference (drone.py:4-5)
            except Exception:
                pass
        import matplotlib.pyplot as plt
        return plt

    def start_record(self, filename="drone_run.mp4", dpi=200, fps=20, bitrate=-1):
        """drone.py:189-198: a PillowWriter on the env's figure (the reference
        accepts `bitrate` and ignores it; so does this)."""
        plt = self._plt()
        from matplotlib.animation import PillowWriter
        if self._fig is None:
            self._fig = plt.figure()
        self._writer = PillowWriter(fps=fps)
        self._writer.setup(self._fig, filename, dpi)

    def stop_record(self):
        """drone.py:200-204: finish and save."""
        if self._writer is not None:
            self._writer.finish()
            self._writer = None

    def render(self, pos, euler, target, arm_length, ax=None):
        """drone.py:206-248 on the given state; grabs a frame when recording."""
        plt = self._plt()
        if ax is None:
            if self._fig is None:
                self._fig = plt.figure()
            if self._ax is None:
                self._ax = self._fig.add_subplot(111, projection="3d")
            ax = self._ax
        ax.clear()
        target = np.asarray(target, np.float64)
        pos = np.asarray(pos, np.float64)
        ax.scatter(target[0], target[1], target[2], color="green", s=50, label="Target")
        motors = motor_positions(pos, euler, arm_length)
        ax.plot([motors[0, 0], motors[2, 0]], [motors[0, 1], motors[2, 1]],
                [motors[0, 2], motors[2, 2]], color="purple", lw=2)
        ax.plot([motors[1, 0], motors[3, 0]], [motors[1, 1], motors[3, 1]],
                [motors[1, 2], motors[3, 2]], color="purple", lw=2)
        ax.scatter(pos[0], pos[1], pos[2], color="red", s=20, label="Center")
        ax.scatter(motors[:, 0], motors[:, 1], motors[:, 2], color="blue", s=20, label="Motors")
        ax.set_xlim(-5, 5)
        ax.set_ylim(-5, 5)
        ax.set_zlim(0, 5)
        ax.set_xlabel("X")
        ax.set_ylabel("Y")
        ax.set_zlabel("Z")
        plt.draw()
        if self._writer is not None:
            self._writer.grab_frame()
        else:
            plt.pause(0.001)
        return motors

    def close(self):
        self.stop_record()
        if self._fig is not None:
            self._plt().close(self._fig)
            self._fig = self._ax = None
