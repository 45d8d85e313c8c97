#!/usr/bin/env python3
"""Where does k_play's time go?  Times, with HIP events on the launch stream:
  reset        k_reset: the deal alone (Fisher-Yates + hand sort), all games
  play9        9 env-steps from a fresh deal (no auto-reset deal inside)
  play1+deal   the 10th env-step + the auto-reset deal
  episode      one full bench launch (10 env-steps incl. the deal)
for numpy-MT and Philox, with and without int8 obs.   usage: breakdown.py [B]
(back-to-back launches, so small kernels are not inflated by host latency)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import torch  # noqa: E402

from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402


def timed(fn, reps=20):
    """mean time of `reps` back-to-back calls (the queue stays full: kernel time, not host latency)"""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    res = {}
    for rng in ("numpy", "philox"):
        for obs in (True, False):
            env = VecSechsNimmtEnv(B, 4, seed=0, rng=rng)
            env.reset()
            out10 = env.rollout(10, want_obs=obs, want_actions=True)
            out9 = env.rollout(9, want_obs=obs, want_actions=True)
            out1 = env.rollout(1, want_obs=obs, want_actions=True)
            torch.cuda.synchronize()
            r = {}
            r["episode"] = timed(lambda: env.rollout(10, out=out10))
            r["reset"] = timed(lambda: env.reset())
            t_r9 = timed(lambda: (env.reset(), env.rollout(9, out=out9)))
            t_r91 = timed(lambda: (env.reset(), env.rollout(9, out=out9), env.rollout(1, out=out1)))
            r["play9"] = t_r9 - r["reset"]
            r["play1+deal"] = t_r91 - t_r9
            res[f"{rng}{'+obs' if obs else ''}"] = r
            print(rng, "obs" if obs else "no-obs", json.dumps({k: round(v, 1) for k, v in r.items()}), flush=True)
            env.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
