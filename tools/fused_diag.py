#!/usr/bin/env python3
"""Timing diagnostics of the headline step under pipeline options (no parity:
SECHS_QUAD_DBG bits 3/4 skip the fused twist and overrun on purpose).
usage: python tools/fused_diag.py  (options from env: FD_QUAD, FD_FUSED,
FD_ROUND, FD_EVERY; SECHS_PIPE_SERIAL / SECHS_QUAD_DBG as the library reads them)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))
import bench  # noqa: E402
from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402


def main():
    e = lambda k, d: int(os.environ.get(k, d))  # noqa: E731
    env = VecSechsNimmtEnv(65536, 4, seed=0, rng="numpy")
    env.set_option(play_quad=e("FD_QUAD", 1), pipe_fused=e("FD_FUSED", 0), twist_round=e("FD_ROUND", 0),
                   twist_every=e("FD_EVERY", 1))
    env.reset()
    out = bench.make_out(env, 65536, True)
    wall, kern_ms, kt = bench.time_rollouts(env, out, 100, 10, 1)
    torch.cuda.synchronize()
    print(json.dumps({"cfg": {k: os.environ.get(k) for k in ("FD_QUAD", "FD_FUSED", "FD_ROUND", "FD_EVERY",
                                                               "SECHS_PIPE_SERIAL", "SECHS_QUAD_DBG")},
                      "ms_per_step": wall / 100 * 1e3, "launch_ms": kern_ms, "play_ms": kt["k_play"],
                      "ahead_ms": kt.get("k_mt_ahead"), "pipe_errors": env.pipe_errors()}))


if __name__ == "__main__":
    main()
