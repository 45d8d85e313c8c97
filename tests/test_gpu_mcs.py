"""GPU parity of the Monte-Carlo search engines.

* reference-exact: sn_mcs_play_exact and the drop-in MCSAgent replay the
  reference's seeded GameSession(MCSAgent, DrunkHamster, ...) games
  (tests/golden/mcs_games.json) move for move;
* stratified (config 3): sn_mcs_memorize / sn_mcs_rollouts / sn_mcs_choose
  match the oracle's restatement bit for bit.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_play_exact_replays_reference_mcs_games():
    from rl_6_nimmt.mcs import play_exact
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    for g in load("mcs_games.json")["games"]:
        n = len(g["seats"])
        env = VecSechsNimmtEnv(1, n, seed=g["seed"], rng="numpy")
        acts, rews, status = play_exact(env, g["seats"], g["mc_per_card"], g["mc_max"])
        if "error" in g:
            assert status[0].item() == 1, g
            continue
        assert status[0].item() == 0
        assert acts[:, 0].cpu().tolist() == g["actions"], (g["seats"], g["seed"])
        assert rews[:, 0].cpu().tolist() == g["rewards"]


def test_play_exact_batch_matches_oracle():
    """many games at once (one lane each), vs the oracle's reference-exact MCS"""
    from rl_6_nimmt.mcs import play_exact
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    B = 96
    env = VecSechsNimmtEnv(B, 4, seed=1000, rng="numpy")
    acts, rews, status = play_exact(env, "MRMR", 2, 12)
    acts, rews, status = acts.cpu().numpy(), rews.cpu().numpy(), status.cpu().numpy()
    for g in range(B):
        rc, a, r = O.mcs_game("MRMR", 2, 12, 1000 + g)
        if rc == -2:
            assert status[g] == 1
            continue
        assert status[g] == 0
        assert np.array_equal(acts[:, g], a) and np.array_equal(rews[:, g], r), g


def test_dropin_mcs_agent_in_game_session():
    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent

    for g in load("mcs_games.json")["games"]:
        if "error" in g or g["mc_max"] > 100:
            continue
        agents = [MCSAgent(mc_max=g["mc_max"], mc_per_card=g["mc_per_card"]) if c == "M" else DrunkHamster() for c in g["seats"]]
        np.random.seed(g["seed"])
        sess = GameSession(*agents)
        sess.play_game()
        assert sess.results[0].tolist() == g["results"], (g["seats"], g["seed"])


def _oracle_game(board, hands, n_players):
    G = O.Game(n_players)
    G.set_position([[c for c in row if c >= 0] for row in board], [[c for c in h if c >= 0] for h in hands])
    return G


@pytest.mark.parametrize("N", [4, 2, 5])
def test_stratified_engine_matches_oracle(N):
    from rl_6_nimmt.mcs import BatchedMCS
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    B, R, seed = 24, 64, 0xC0FFEE
    env = VecSechsNimmtEnv(B, N, seed=7, rng="philox", game_offset=5)
    env.reset()
    mcs = BatchedMCS(env, rollouts=R, seed=seed)
    mem = [[None] * N for _ in range(B)]
    for step in range(10):
        board, hands = env.board().cpu().numpy(), env.hands().cpu().numpy()
        acts = mcs.decide(step_id=step)
        sums = mcs.sums.cpu().numpy().reshape(B, N, 10)
        acts = acts.cpu().numpy()
        avail_dev = mcs.avail.cpu().numpy().view(np.uint32).T.reshape(B, N, 4)
        for g in range(B):
            G = _oracle_game(board[g], hands[g], N)
            for p in range(N):
                mem[g][p] = O.mcs_memorize(mem[g][p] or [], G, p)
                words = np.zeros(4, dtype=np.uint64)
                for c in mem[g][p]:
                    words[c >> 5] |= np.uint64(1) << np.uint64(c & 31)
                assert np.array_equal(avail_dev[g, p], words.astype(np.uint32)), (step, g, p)
                ref = O.mcs_stratified(G, p, mem[g][p], R, seed, step, 5 + g)
                assert np.array_equal(sums[g, p], ref), (step, g, p)
                n = len(G.hands[p])
                best = int(np.argmax(ref[:n])) if n > 1 else 0
                assert acts[g, p] == G.hands[p][best]
        rew, done, inv = env.step(torch.from_numpy(acts))
        assert (inv.cpu().numpy() == -1).all()


def test_stratified_engine_matches_oracle_at_bench_rollouts():
    """BASELINE config 3's search size -- 256 playouts per legal move -- on a
    256-game subset of the bench's batch (4 MCS seats, philox), every
    decision of every seat bit-exact against the oracle's stratified MCS
    (the oracle runs in parallel threads: its C calls release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    from rl_6_nimmt.mcs import BatchedMCS
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    B, N, R, seed = 256, 4, 256, 0xBEEF
    env = VecSechsNimmtEnv(B, N, seed=1, rng="philox")
    env.reset()
    mcs = BatchedMCS(env, rollouts=R, seed=seed)
    mem = [[[] for _ in range(N)] for _ in range(B)]
    pool = ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1))
    for step in range(10):
        board, hands = env.board().cpu().numpy(), env.hands().cpu().numpy()
        acts = mcs.decide(step_id=step).cpu().numpy()
        sums = mcs.sums.cpu().numpy().reshape(B, N, 10)
        games = [_oracle_game(board[g], hands[g], N) for g in range(B)]
        for g in range(B):
            for p in range(N):
                mem[g][p] = O.mcs_memorize(mem[g][p], games[g], p)

        def one(gp):
            g, p = gp
            return O.mcs_stratified(games[g], p, mem[g][p], R, seed, step, g)

        refs = list(pool.map(one, [(g, p) for g in range(B) for p in range(N)]))
        for i, ref in enumerate(refs):
            g, p = divmod(i, N)
            assert np.array_equal(sums[g, p], ref), (step, g, p)
            n = len(games[g].hands[p])
            best = int(np.argmax(ref[:n])) if n > 1 else 0
            assert acts[g, p] == games[g].hands[p][best], (step, g, p)
        rew, done, inv = env.step(torch.from_numpy(acts))
        assert (inv.cpu().numpy() == -1).all()
    pool.shutdown()
