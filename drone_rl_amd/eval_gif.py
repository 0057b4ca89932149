"""Record a trained policy flying the GPU env to a GIF: the reference's
test.py (load dd.zip, 100 deterministic steps, env.render() per step, reset on
done, GIF via PillowWriter; /root/reference/test.py:1-26).

  python -m drone_rl_amd.eval_gif --checkpoint dd.zip --out my_drone_run.gif
"""
from __future__ import annotations

import argparse
import time


def run(checkpoint: str, out: str, steps: int = 100, dpi: int = 200, fps: int = 20,
        seed: int | None = None, device=None):
    from .env import DroneGymEnv
    from .sb3_zip import load_policy
    t0 = time.time()
    env = DroneGymEnv(seed=seed, device=device)
    model = load_policy(checkpoint, device=device)
    env.start_record(out, dpi=dpi, fps=fps)
    obs = env.reset()
    rewards = []
    for _ in range(steps):
        action, _ = model.predict(obs, deterministic=True)
        obs, reward, done, _ = env.step(action)
        rewards.append(reward)
        env.render()
        if done:
            obs = env.reset()
    env.stop_record()
    env.close()
    return {"frames": steps, "return": float(sum(rewards)), "seconds": time.time() - t0}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--checkpoint", default="./dd.zip")
    ap.add_argument("--out", default="my_drone_run.gif")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--dpi", type=int, default=200)
    ap.add_argument("--fps", type=int, default=20)
    ap.add_argument("--seed", type=int, default=None)
    a = ap.parse_args(argv)
    r = run(a.checkpoint, a.out, a.steps, a.dpi, a.fps, a.seed)
    print(r["seconds"])


if __name__ == "__main__":
    main()
