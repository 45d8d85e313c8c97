"""GPU parity of the batched tournament (league.py, BASELINE config 5).

* slot g of a tournament handle replays the reference's
  `np.random.seed(seed + g); Tournament(min, max) over K DrunkHamster agents;
  play_game() x games` -- seat draws, results -- bit for bit (golden F11,
  tests/golden/tournament_games.json, recorded from the reference itself);
* at the bench's size (65 536 slots): records independent of the sharding
  (two half-size handles == one handle), per-game invariants of the scoring
  (relative positions of a game sum to k/2, one winner per game, Elo sum
  conserved), agent ids distinct per game.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _league(B, K, lo, hi, seed, game_offset=0, rng="numpy"):
    from rl_6_nimmt.league import BatchedTournament

    t = BatchedTournament(B, lo, hi, seed=seed, game_offset=game_offset, rng=rng)
    for i in range(K):
        t.add_player(f"a{i}")
    return t


def test_league_slots_replay_reference_tournaments():
    from rl_6_nimmt.league import decode_seats

    groups = {}
    for r in load("tournament_games.json")["league"]:
        groups.setdefault((r["num_agents"], r["min_players"], r["max_players"]), []).append(r)
    assert len(groups) == 3
    for (K, lo, hi), recs in groups.items():
        base = recs[0]["seed"]
        assert [r["seed"] for r in recs] == list(range(base, base + len(recs)))
        games = len(recs[0]["results"])
        t = _league(len(recs), K, lo, hi, seed=base)
        rec = t.play_games(games).cpu()
        k, ids = decode_seats(rec[..., 0], hi)
        for j, r in enumerate(recs):
            for e in range(games):
                seats, res = r["seats"][e], r["results"][e]
                assert int(k[e, j]) == len(seats), (K, lo, hi, j, e)
                assert ids[e, j, : len(seats)].tolist() == seats, (K, lo, hi, j, e)
                assert rec[e, j, 1: 1 + len(seats)].tolist() == res, (K, lo, hi, j, e)
                assert not rec[e, j, 1 + len(seats):].any()
        assert t.env.pipe_errors() == 0
        t.close()


@pytest.mark.parametrize("rng", ["numpy", "philox"])
def test_league_full_size_sharding_and_scoring_invariants(rng):
    from rl_6_nimmt.league import decode_seats, relative_positions, winners

    B, K, lo, hi, G = 65536, 5, 2, 4, 3
    t = _league(B, K, lo, hi, seed=7, rng=rng)
    rec = t.play_games(G)
    t2 = _league(B // 2, K, lo, hi, seed=7, game_offset=B // 2, rng=rng)
    rec2 = t2.play_games(G)
    assert torch.equal(rec[:, B // 2:], rec2)
    k, ids = decode_seats(rec[..., 0], hi)
    assert int(k.min()) >= lo and int(k.max()) <= hi
    counts = torch.bincount(k.reshape(-1), minlength=hi + 1)[lo:].cpu().numpy()
    assert counts.min() > 0.3 * counts.max()  # every player count occurs (uniform choice)
    valid = ids >= 0
    assert int(ids.max()) < K
    s = torch.sort(torch.where(valid, ids, 100 + torch.arange(hi, device=ids.device)), dim=-1).values
    assert not (s[..., 1:] == s[..., :-1]).any()  # distinct agents per game (replace=False)
    res = rec[..., 1:]
    pen = -res.sum(dim=-1)
    assert int(res.max()) <= 0 and int(pen.max()) <= 171
    assert not res[~valid].any()
    rel = relative_positions(res, k)
    assert torch.allclose(rel.sum(dim=-1), k.double() / 2)
    w = winners(res, k)
    assert bool((w < k).all())
    stats = t.agent_stats()
    assert int(stats[:, 0].sum()) == int(k.sum())
    assert int(stats[:, 3].sum()) == G * B
    elos = t.replay_elo()
    assert abs(elos.sum() - K * 1600.0) < 1e-6 * K * 1600.0  # pairwise Elo exchanges conserve the sum
    if rng == "numpy":
        assert t.env.pipe_errors() == 0 and t2.env.pipe_errors() == 0
    t.close()
    t2.close()
