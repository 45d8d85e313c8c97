#!/usr/bin/env python3
"""Is the bench step host-bound?  Times the enqueue of K rollouts (no sync)
against the wall time to their completion, at the bench size and at a tiny
size (where the device work is negligible: pure per-call cost).
Usage: python tools/host_rate.py [numpy|philox] [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import torch  # noqa: E402

from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402


def run(B, rng, K, split=None):
    N, T = 4, 10
    env = VecSechsNimmtEnv(B, N, seed=0, rng=rng, device="cuda:0")
    if split is not None:
        env.set_option(play_split=split)
    env.reset()
    dev = env.device
    out = {
        "rewards": torch.empty((T, B, N), dtype=torch.int32, device=dev),
        "done": torch.empty((T, B), dtype=torch.uint8, device=dev),
        "actions": torch.empty((T, B, N), dtype=torch.uint8, device=dev),
        "obs": torch.empty((T, B, N, 48), dtype=torch.int8, device=dev),
    }
    for _ in range(5):
        env.rollout(T, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        env.rollout(T, out=out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    env.close()
    return {"B": B, "rng": rng, "split": split, "enqueue_us_per_call": (t1 - t0) / K * 1e6,
            "wall_us_per_call": (t2 - t0) / K * 1e6}


def main():
    rng = sys.argv[1] if len(sys.argv) > 1 else "numpy"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    res = [run(65536, rng, K), run(256, rng, K)]
    if rng == "numpy":
        res.append(run(65536, rng, K, split=3))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
