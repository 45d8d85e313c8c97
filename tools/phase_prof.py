#!/usr/bin/env python3
"""Phase split of k_play's step loop (diagnostics).

Loads the libsechs_prof.so variant (make -C rl-6-nimmt_amd libsechs_prof.so,
built with -DSECHS_PHASE_PROF), runs the bench workload (65 536 x 4-player
DrunkHamster self-play, numpy-MT, int8 obs + outputs) and prints the share of
wave cycles per phase.  Usage: python tools/phase_prof.py [games] [launches] [rng] [play_split]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SECHS_LIB", os.path.join(ROOT, "rl-6-nimmt_amd", "libsechs_prof.so"))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import ctypes  # noqa: E402

import torch  # noqa: E402

from rl_6_nimmt import _native as nat  # noqa: E402
from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

NAMES = ["prologue", "obs", "draw", "resolve", "store", "shuffle_targets", "epilogue", "hands", "shuffle_apply",
         "b1_wait", "b2_wait"]
PRODUCER = ["draws", "b1_wait", "shuffle_targets", "shuffle_apply", "hands", "draws2", "b2_wait", "store", "twist"]
NP = len(NAMES) + len(PRODUCER)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rng = sys.argv[3] if len(sys.argv) > 3 else "numpy"
    N, T = 4, 10
    env = VecSechsNimmtEnv(B, N, seed=0, rng=rng, device="cuda:0")
    if len(sys.argv) > 4:
        env.set_option(play_split=int(sys.argv[4]))
    env.reset()
    dev = env.device
    out = {
        "rewards": torch.empty((T, B, N), dtype=torch.int32, device=dev),
        "done": torch.empty((T, B), dtype=torch.uint8, device=dev),
        "actions": torch.empty((T, B, N), dtype=torch.uint8, device=dev),
        "obs": torch.empty((T, B, N, 48), dtype=torch.int8, device=dev),
    }
    for _ in range(3):
        env.rollout(T, out=out)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * (NP + 2))()
    nat.lib().sn_debug_phases(buf, NP + 2)  # clear
    for _ in range(launches):
        env.rollout(T, out=out)
    torch.cuda.synchronize()
    nat.check(nat.lib().sn_debug_phases(buf, NP + 2), "sn_debug_phases")
    waves = max(int(buf[NP]), 1)
    tot = sum(int(buf[k]) for k in range(len(NAMES)))
    res = {"games": B, "launches": launches, "rng": rng, "waves": waves,
           "cycles_per_wave_launch": round(tot / waves, 1)}
    for k, nm in enumerate(NAMES):
        res[nm] = {"cycles_per_wave": round(int(buf[k]) / waves, 1), "frac": round(int(buf[k]) / max(tot, 1), 4)}
    pw = int(buf[NP + 1])
    if pw:  # role-split kernel: the producer waves' own split
        o = len(NAMES)
        ptot = sum(int(buf[o + k]) for k in range(len(PRODUCER)))
        res["producer"] = {"waves": pw, "cycles_per_wave_launch": round(ptot / pw, 1)}
        for k, nm in enumerate(PRODUCER):
            res["producer"][nm] = {"cycles_per_wave": round(int(buf[o + k]) / pw, 1),
                                   "frac": round(int(buf[o + k]) / max(ptot, 1), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
