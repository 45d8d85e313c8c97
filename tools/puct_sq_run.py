"""A short eager config-4 workload for counter passes (rocprofv3 --pmc does
not survive hipGraph replays here): 2048 4-player games, every seat PUCT
(mc_max 100), bf16 MLP, the first three decisions."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))
from rl_6_nimmt.puct import BatchedPUCT, make_actor  # noqa: E402
from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

env = VecSechsNimmtEnv(2048, 4, seed=3, rng="philox")
torch.manual_seed(0)
eng = BatchedPUCT(env, make_actor(), mc_per_card=10, mc_max=100, seed=4, net_dtype=torch.bfloat16, graph=False)
env.reset()
for t in range(3):
    env.step(eng.decide(10 - t))
torch.cuda.synchronize()
print("rows", eng.rows_evaluated)
