"""PyTorch TunableOp over the config-4 policy-MLP GEMM shapes: plays the
bench_puct workload once with tuning on (every rollout hand size of 8192
4-player games), then writes the selected hipBLASLt / rocBLAS solutions to
the CSV that bench.py's PUCT leg loads (tuning off) when present.
  gpurun -- python tools/tune_puct.py <out.csv>"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))
sys.path.insert(0, ROOT)
out = sys.argv[1]
import torch.cuda.tunable as tun  # noqa: E402

tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(20)
tun.set_max_tuning_iterations(30)
tun.set_filename(out, insert_device_ordinal=False)
from rl_6_nimmt.puct import BatchedPUCT, make_actor  # noqa: E402
from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

env = VecSechsNimmtEnv(8192, 4, seed=3, rng="philox")
torch.manual_seed(0)
eng = BatchedPUCT(env, make_actor(), mc_per_card=10, mc_max=100, seed=4, net_dtype=torch.bfloat16, graph=False)
env.reset()
for t in range(10):  # one decision per hand size, a few rollouts each: every GEMM shape of the game
    n = 10 - t
    eng.mc_max = 2
    acts = eng.decide(n)
    env.step(acts)
torch.cuda.synchronize()

print("tuned", len(tun.get_results()), "->", out)
