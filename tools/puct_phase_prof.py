#!/usr/bin/env python3
"""Phase split of k_puct_rollouts (config 4's whole-rollout kernel;
diagnostics).  Loads libsechs_prof.so (make -C rl-6-nimmt_amd
libsechs_prof.so: -DSECHS_PHASE_PROF), plays one config-4 game (8192 x
4-player games, every seat PUCT, mc_max 100, bf16 net, eager launches) and
prints the share of wave cycles per phase: the rollout-state copy-in, the
seat rows, the per-seat layer-1 MFMA, the candidate tiles, the step.
usage: python tools/puct_phase_prof.py [games]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SECHS_LIB", os.path.join(ROOT, "rl-6-nimmt_amd", "libsechs_prof.so"))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import torch  # noqa: E402

NAMES = ["copy_in", "seat_rows", "layer1_base", "tiles", "step", "step_t0"]


def main():
    from rl_6_nimmt import _native as nat
    from rl_6_nimmt.puct import BatchedPUCT, make_actor
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    games = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    env = VecSechsNimmtEnv(games, 4, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedPUCT(env, make_actor(), mc_per_card=10, mc_max=100, seed=4, net_dtype=torch.bfloat16, graph=False)
    env.reset()
    buf = (ctypes.c_uint64 * 8)()
    nat.check(nat.lib().sn_debug_puct_phases(buf, 8), "sn_debug_puct_phases")  # clear
    eng.play_episode()
    torch.cuda.synchronize()
    nat.check(nat.lib().sn_debug_puct_phases(buf, 8), "sn_debug_puct_phases")
    waves = max(int(buf[7]), 1)
    tot = sum(int(buf[k]) for k in range(len(NAMES)))
    res = {"games": games, "waves": waves, "cycles_per_wave": round(tot / waves, 1)}
    for k, nm in enumerate(NAMES):
        res[nm] = {"cycles_per_wave": round(int(buf[k]) / waves, 1), "frac": round(int(buf[k]) / max(tot, 1), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
