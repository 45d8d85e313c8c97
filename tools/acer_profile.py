"""Where an ACER update's GPU time goes: BatchedACER at league-like size
(13 107 games x 4 seats = 52 428 deciders, minibatch 5), one learn() under
torch.profiler -- the top GPU kernels / ops with their input shapes.
usage: python tools/acer_profile.py [games]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import torch  # noqa: E402


def main():
    from rl_6_nimmt.acer import BatchedACER, make_actor_critic
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    games = int(sys.argv[1]) if len(sys.argv) > 1 else 13107
    env = VecSechsNimmtEnv(games, 4, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedACER(env, make_actor_critic().to(env.device), seed=4, net_dtype=torch.bfloat16, warmup=2,
                      minibatch=5, capacity=7)
    opt = torch.optim.Adam(eng.actor.parameters())
    for _ in range(7):
        eng.play_episode()
        eng.learn(opt)
    eng.play_episode()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    eng.learn(opt)
    ev1.record()
    torch.cuda.synchronize()
    print(f"learn(): {ev0.elapsed_time(ev1):.1f} ms, decider_chunk {eng.decider_chunk}, deciders {eng.D}")
    eng.play_episode()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        eng.learn(opt)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=25,
                                                              max_name_column_width=60, max_shapes_column_width=90))


if __name__ == "__main__":
    main()
