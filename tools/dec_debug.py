#!/usr/bin/env python3
"""Decode-ahead debugging (diagnostics): first divergence of the DEC rollout
from the oracle, with the game's decoder start position and its record."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from rl_6_nimmt import _native as nat  # noqa: E402
from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

B, N = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 4
for dec in (1, 0):
    env = VecSechsNimmtEnv(B, N, seed=12345, rng="numpy")
    env.set_option(pipe_dec=dec)
    env.reset()
    ref = O.VecOracle(B, N, 104, rng_mode=O.RNG_NUMPY_MT, seed=12345)
    ref.reset()
    out = env.rollout(10, want_actions=True)
    rr, rd, ra, ro = ref.rollout(10)
    got = out["actions"].cpu().numpy()
    bad = np.argwhere(got != ra)
    print("dec", dec, "mismatches", len(bad), "games", len(set(bad[:, 1].tolist())))
    if dec and len(bad):
        L = nat.lib()
        pos = np.zeros(B, dtype=np.uint32)
        for slot in range(9):
            nat.check(L.sn_debug_pipe_words(env._h, 0, slot, pos.ctypes.data_as(ctypes.c_void_p)), "pabsc")
            print("pabsc", slot, pos[:8])
        rec = np.zeros((6, B, 4), dtype=np.uint32)
        nat.check(L.sn_debug_pipe_words(env._h, 2, 0, rec.ctypes.data_as(ctypes.c_void_p)), "rec")
        games = sorted(set(bad[:, 1].tolist()))[:6]
        ok = [g for g in range(B) if g not in set(bad[:, 1].tolist())][:4]
        for g in games + ok:
            w = rec[:, g, :].reshape(-1)
            first = bad[bad[:, 1] == g][:1]
            print("game", g, "first bad (step, seat)", first[:, [0, 2]].tolist(), "start", hex(w[0]), "start&15", w[0] & 15,
                  "offs", [(int(w[1 + t // 2]) >> (16 * (t & 1))) & 0xFFFF for t in range(10)])
            print("   ours", got[:4, g].tolist(), "ref", ra[:4, g].tolist())
    env.close()
