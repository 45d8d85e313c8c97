"""One config-4 game (8192 x 4-player games, every seat PUCT, mc_max 100)
with eager launches (no hipGraph): the target of PMC passes over the rollout
kernels (rocprofv3's counter collection does not survive graph replay here).
usage: python tools/puct_eager.py [games]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import torch  # noqa: E402


def main():
    from rl_6_nimmt.puct import BatchedPUCT, make_actor
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    games = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    env = VecSechsNimmtEnv(games, 4, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedPUCT(env, make_actor(), mc_per_card=10, mc_max=100, seed=4, net_dtype=torch.bfloat16, graph=False)
    env.reset()
    eng.play_episode()
    torch.cuda.synchronize()
    print("rows", eng.rows_evaluated)


if __name__ == "__main__":
    main()
