"""A/B of SN_OPT_AHEAD_DELAY on the headline step (65 536 x 4p, numpy-MT,
int8 obs): ms per 10-step launch for several side-stream delays, interleaved
and repeated, plus the host's enqueue time per launch.  GPU box only."""
import json
import sys
import time

sys.path.insert(0, "rl-6-nimmt_amd")
import torch  # noqa: E402

from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

B, N, T, STEPS = 65536, 4, 10, 200
env = VecSechsNimmtEnv(B, N, seed=0, rng="numpy")
env.reset()
out = {"rewards": torch.empty((T, B, N), dtype=torch.int32, device=env.device),
       "done": torch.empty((T, B), dtype=torch.uint8, device=env.device),
       "actions": torch.empty((T, B, N), dtype=torch.uint8, device=env.device),
       "obs": torch.empty((T, B, N, 48), dtype=torch.int8, device=env.device)}
delays = [int(x) for x in (sys.argv[1:] or ["0", "3", "6", "10", "15"])]
res = {d: [] for d in delays}
for rep in range(3):
    for d in delays:
        env.set_option(ahead_delay=d)
        for _ in range(5):
            env.rollout(T, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(STEPS):
            env.rollout(T, out=out)
        enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        res[d].append((1e3 * wall / STEPS, 1e3 * enq / STEPS))
        print(json.dumps({"delay_us": d, "rep": rep, "ms_per_step": res[d][-1][0], "enqueue_ms": res[d][-1][1]}), flush=True)
assert env.pipe_errors() == 0
print(json.dumps({"best_ms": {d: min(x[0] for x in v) for d, v in res.items()}}))
