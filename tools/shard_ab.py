"""Headline step as K concurrent shard handles on one GPU (65 536 x 4p,
numpy-MT, int8 obs): handle k owns games [k B/K, (k+1) B/K) (game_offset), on
its own torch stream, so one handle's queue hand-off gap is filled by the
others' kernels.  (1) parity: K = 2 shards reproduce the K = 1 trajectories
bit for bit over 20 launches; (2) timing: ms per 10-step step of all 65 536
games for K = 1, 2, 4, interleaved, 3 reps x 200 steps.  GPU box only."""
import json
import sys
import time

sys.path.insert(0, "rl-6-nimmt_amd")
import torch  # noqa: E402

from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

B, N, T = 65536, 4, 10


def shards(K):
    hs = []
    for k in range(K):
        b = B // K
        env = VecSechsNimmtEnv(b, N, seed=0, game_offset=k * b, rng="numpy")
        env.reset()
        out = {"rewards": torch.empty((T, b, N), dtype=torch.int32, device=env.device),
               "done": torch.empty((T, b), dtype=torch.uint8, device=env.device),
               "actions": torch.empty((T, b, N), dtype=torch.uint8, device=env.device),
               "obs": torch.empty((T, b, N, 48), dtype=torch.int8, device=env.device)}
        st = torch.cuda.Stream() if K > 1 else torch.cuda.current_stream()
        hs.append((env, out, st))
    torch.cuda.synchronize()
    return hs


def step(hs):
    for env, out, st in hs:
        with torch.cuda.stream(st):
            env.rollout(T, out=out)


cfg = {K: shards(K) for K in (1, 2, 4)}
for i in range(20):
    step(cfg[1])
    step(cfg[2])
    torch.cuda.synchronize()
    for key in cfg[1][0][1]:
        cat = torch.cat([o[key] for _, o, _ in cfg[2]], dim=1)
        assert torch.equal(cat, cfg[1][0][1][key]), (i, key)
print(json.dumps({"parity": "K=2 shards == K=1 over 20 launches"}), flush=True)
res = {K: [] for K in cfg}
for rep in range(3):
    for K, hs in cfg.items():
        for _ in range(5):
            step(hs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            step(hs)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / 200
        res[K].append(ms)
        print(json.dumps({"shards": K, "rep": rep, "ms_per_step": ms, "G_env_steps_per_s": B * T / ms / 1e6}), flush=True)
for K, hs in cfg.items():
    for env, _, _ in hs:
        assert env.pipe_errors() == 0
print(json.dumps({"best_ms": {K: min(v) for K, v in res.items()}}))
