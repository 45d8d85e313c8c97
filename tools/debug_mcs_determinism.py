"""Debug helper: stratified MCS playouts, lane by lane, vs the oracle after
unrelated GPU work (the case that once returned a different sum)."""
import sys

sys.path.insert(0, "/root/repo")
sys.path.insert(0, "/root/repo/rl-6-nimmt_amd")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from rl_6_nimmt import _native as nat  # noqa: E402
from rl_6_nimmt.mcs import BatchedMCS  # noqa: E402
from rl_6_nimmt.vec_env import VecSechsNimmtEnv  # noqa: E402

warm = int(sys.argv[1]) if len(sys.argv) > 1 else 0
if warm:
    e2 = VecSechsNimmtEnv(65536, 4, seed=0, rng="numpy")
    e2.reset()
    e2.rollout(30, want_actions=True, want_obs=True)
    torch.cuda.synchronize()
    del e2
B, N, R, seed = 24, 4, 64, 0xC0FFEE
env = VecSechsNimmtEnv(B, N, seed=7, rng="philox", game_offset=5)
env.reset()
mcs = BatchedMCS(env, rollouts=R, seed=seed)
nat.check(nat.lib().sn_mcs_memorize(env._h, nat.ptr(mcs.avail), 104, env._stream()), "mem")
po = torch.zeros((B * N, 10, R), dtype=torch.int32, device=env.device)
for rep in range(3):
    nat.check(nat.lib().sn_mcs_rollouts_ex(env._h, nat.ptr(mcs.avail), R, seed, 0, nat.ptr(mcs.sums), nat.ptr(po),
                                           env._stream()), "rollouts")
    p = po.cpu().numpy()
    s = mcs.sums.cpu().numpy()
    board, hands = env.board().cpu().numpy(), env.hands().cpu().numpy()
    bad = []
    for d in range(B * N):
        g, q = divmod(d, N)
        G = O.Game(N)
        G.set_position([[c for c in row if c >= 0] for row in board[g]], [[c for c in h if c >= 0] for h in hands[g]])
        mem = O.mcs_memorize([], G, q)
        ref = O.mcs_stratified(G, q, mem, R, seed, 0, 5 + g)
        if not np.array_equal(ref, s[d]):
            bad.append((d, np.nonzero(ref != s[d])[0].tolist()))
    print("warm", warm, "rep", rep, "mismatching decisions:", bad, "lane sums (27,8):", int(p[27, 8].sum()), int(s[27, 8]))
    if bad and rep == 0:
        np.save("/root/repo/gpurun_out/playouts_bad.npy", p)
    if rep == 1:
        np.save("/root/repo/gpurun_out/playouts_good.npy", p)
