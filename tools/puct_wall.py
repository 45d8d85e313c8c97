#!/usr/bin/env python3
"""Config-4 (bench_puct's engine) wall-time split per decision: GPU time of
decide() by events vs host wall, and a cProfile of one timed game.
usage: python tools/puct_wall.py [games]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))
import torch  # noqa: E402


def main():
    from rl_6_nimmt.puct import BatchedPUCT, make_actor
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    games = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    env = VecSechsNimmtEnv(games, 4, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedPUCT(env, make_actor(), mc_per_card=10, mc_max=100, seed=4, net_dtype=torch.bfloat16, graph=True)
    env.reset()
    eng.play_episode()
    torch.cuda.synchronize()
    env.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(10):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        a.record()
        acts = eng.decide(10 - t)
        b.record()
        h1 = time.perf_counter()
        env.step(acts)
        torch.cuda.synchronize()
        h2 = time.perf_counter()
        print(f"n={10 - t}: decide GPU {a.elapsed_time(b):8.2f} ms, host enqueue {1e3 * (h1 - h0):7.2f} ms, "
              f"decide+step wall {1e3 * (h2 - h0):8.2f} ms", flush=True)
    print(f"episode wall {1e3 * (time.perf_counter() - t0):.1f} ms")
    env.reset()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    eng.play_episode()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(18)


if __name__ == "__main__":
    main()
