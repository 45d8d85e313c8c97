"""Phase split of k_reset1 (the one-game deal) from the libsechs_prof.so
variant: mean shader-clock cycles per call in import, decode, twist, state
out (store), shuffle apply, deal, results out."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SECHS_LIB", os.path.join(ROOT, "rl-6-nimmt_amd", "libsechs_prof.so"))
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))
from rl_6_nimmt import SechsNimmtEnv, _native as nat  # noqa: E402

NP = 20
buf = (ctypes.c_uint64 * (NP + 2))()
env = SechsNimmtEnv(4, verbose=False)
np.random.seed(0)
for _ in range(20):
    env.reset()
nat.lib().sn_debug_phases(buf, NP + 2)  # clear
n = 500
for _ in range(n):
    env.reset()
nat.check(nat.lib().sn_debug_phases(buf, NP + 2), "sn_debug_phases")
names = {11: "import", 13: "decode", 19: "twist", 18: "state_out", 14: "shuffle_apply", 15: "deal", 17: "results_out"}
calls = buf[NP + 1]
out = {v: buf[k] / max(1, calls) for k, v in names.items()}
out["calls"] = calls
print(json.dumps(out))
