"""Pin the CPU oracle against the reference's own outputs (tests/golden/).

These run on CPU only.  If they fail, every GPU parity claim that compares
against the oracle is void -- so they come first.
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# ------------------------------------------------------------------ F0 MT19937
def test_mt_seeding_matches_numpy_legacy():
    d = load("mt19937.json")
    for rec in d["seeds"]:
        r = O.Rng(O.RNG_NUMPY_MT, rec["seed"])
        key = r.key
        assert list(key[:8]) == rec["key_head"]
        assert list(key[-8:]) == rec["key_tail"]
        assert rec["pos"] == 624
        raw = [r.next() for _ in range(len(rec["raw_u32"]))]
        assert raw == rec["raw_u32"]  # crosses one twist boundary (700 > 624)


def test_shuffle_matches_np_random_shuffle():
    d = load("mt19937.json")
    for rec in d["shuffles"]:
        r = O.Rng(O.RNG_NUMPY_MT, rec["seed"])
        a = list(r.shuffle(np.arange(104))) + list(r.shuffle(np.arange(57)))
        assert a == rec["deck104_then_deck57"], rec["seed"]


def test_choice_matches_np_random_choice():
    d = load("mt19937.json")
    for rec in d["choices"]:
        r = O.Rng(O.RNG_NUMPY_MT, rec["seed"])
        for n, pick in rec["n_and_pick"]:
            arr = np.arange(n) * 3 + 1
            assert arr[r.interval(n - 1)] == pick


def test_philox_known_answer():
    # Random123 philox4x32-10 known-answer vectors (kat_vectors)
    assert list(O.philox([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(O.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == [
        0xD16CFE09,
        0x94FDCCEB,
        0x5001E420,
        0x24126EA1,
    ]


# ------------------------------------------------------------------ rules
def test_card_heads_table():
    heads = [O.card_heads(c) for c in range(104)]
    assert sum(heads) == 171
    assert heads[54] == 7 and heads[10] == 5 and heads[9] == 3 and heads[4] == 2 and heads[0] == 1


def test_notebook_games_replay():
    d = load("notebook_games.json")
    for g in d["games"]:
        n = len(g["names"])
        G = O.Game(n)
        G.set_position(g["board"], g["hands"])
        assert [list(G.obs(p)) for p in range(n)] == g["obs0"]
        for acts, rec in zip(g["actions"], g["steps"]):
            bad, rew = G.step(acts)
            assert bad == -1
            assert list(rew) == rec["rewards"]
            assert G.board == rec["board"]
            assert G.done() == rec["done"]
            assert [list(G.obs(p)) for p in range(n)] == rec["obs"]
        assert [-s for s in G.scores] == g["final_scores"]


def test_random_games_seeded():
    meta = load("random_games_meta.json")
    z = np.load(os.path.join(GOLDEN, "random_games.npz"))
    for cfg in meta["configs"]:
        k, n, c, summ = cfg["key"], cfg["num_players"], cfg["num_cards"], cfg["include_summaries"]
        for s in range(cfg["seeds"]):
            rng = O.Rng(O.RNG_NUMPY_MT, s)
            G = O.Game(n, c)
            G.reset(rng)
            assert [row[0] for row in G.board] == list(z[k + "_board0"][s])
            assert G.hands == z[k + "_hands0"][s].tolist()
            for t in range(10):
                assert np.array_equal(np.stack([G.obs(p, summ) for p in range(n)]), z[k + "_obs"][s, t])
                acts = [G.random_action(rng, p) for p in range(n)]
                assert acts == z[k + "_actions"][s, t].tolist()
                bad, rew = G.step(acts)
                assert bad == -1 and rew.tolist() == z[k + "_rewards"][s, t].tolist()
                assert G.done() == (t == 9)
            assert np.array_equal(np.stack([G.obs(p, summ) for p in range(n)]), z[k + "_obs"][s, 10])
            assert [-x for x in G.scores] == z[k + "_results"][s].tolist()


def test_random_sessions_stream_continuation():
    d = load("random_sessions.json")
    for rec in d["sessions"]:
        n = rec["num_players"]
        if "episodes" in rec:
            eps = rec["episodes"]
        else:
            eps = len(rec["results"])
        v = O.VecOracle(1, n, rng_mode=O.RNG_NUMPY_MT, seed=rec["seed"])
        v.reset()
        rew, done, _, _ = v.rollout(10 * eps)
        per_ep = rew[:, 0, :].reshape(eps, 10, n).sum(axis=1)
        if "episodes" in rec:
            assert per_ep[-1].tolist() == rec["results_last"]
            assert per_ep.sum(axis=0).tolist() == rec["results_sum"]
            assert (v.sum_results()[0]).tolist() == rec["results_sum"]
        else:
            assert per_ep.tolist() == rec["results"]
        assert done[:, 0].reshape(eps, 10)[:, -1].all() and not done[:, 0].reshape(eps, 10)[:, :-1].any()


def test_vec_oracle_game_offset_is_seed_offset():
    a = O.VecOracle(8, 4, rng_mode=O.RNG_NUMPY_MT, seed=100, game_offset=0)
    b = O.VecOracle(4, 4, rng_mode=O.RNG_NUMPY_MT, seed=100, game_offset=4)
    for v in (a, b):
        v.reset()
    ra = a.rollout(25)[0]
    rb = b.rollout(25)[0]
    assert np.array_equal(ra[:, 4:], rb)


def test_edge_cases():
    d = load("edge_cases.json")
    for case in d["cases"]:
        n = len(case["hands"])
        summ = case["include_summaries"]
        G = O.Game(n)
        G.set_position(case["board"], case["hands"])
        assert [list(G.obs(p, summ)) for p in range(n)] == case["obs0"], case["label"]
        if "error" in case:
            if case["error"]["type"] == "AssertionError":
                assert len(case["actions"]) != n
                continue
            bad, _ = G.step(case["actions"])
            assert bad >= 0
            msg = f"Player {bad + 1} tried to play card {case['actions'][bad] + 1}, but their hand is {case['hands'][bad]}"
            assert msg == case["error"]["message"], case["label"]
            continue
        bad, rew = G.step(case["actions"])
        e = case["expect"]
        assert bad == -1, case["label"]
        assert rew.tolist() == e["rewards"], case["label"]
        assert G.board == e["board"], case["label"]
        assert G.hands == e["hands"], case["label"]
        assert G.scores == e["scores"], case["label"]
        assert G.done() == e["done"]
        assert [list(G.obs(p, summ)) for p in range(n)] == e["obs"], case["label"]


# ------------------------------------------------------------------ F4 MCS
def test_mcs_games_reference_exact():
    d = load("mcs_games.json")
    for g in d["games"]:
        rc, a, r = O.mcs_game(g["seats"], g["mc_per_card"], g["mc_max"], g["seed"])
        if "error" in g:
            assert rc == -2, g
            continue
        assert rc == 0
        assert a.tolist() == g["actions"], (g["seats"], g["seed"])
        assert r.tolist() == g["rewards"]
        assert r.sum(axis=0).tolist() == g["results"]


def test_league_records_replay_reference_tournaments():
    """golden F11 "league": seeded reference Tournament(lo, hi) over K
    DrunkHamster agents -- oracle.league_records (the device's record format)
    reproduces every seat draw and result"""
    groups = {}
    for r in load("tournament_games.json")["league"]:
        groups.setdefault((r["num_agents"], r["min_players"], r["max_players"]), []).append(r)
    for (K, lo, hi), recs in groups.items():
        base, G = recs[0]["seed"], len(recs[0]["results"])
        out = O.league_records(K, lo, hi, seed=base, slots=len(recs), games=G)
        for j, r in enumerate(recs):
            for e in range(G):
                seats, res = r["seats"][e], r["results"][e]
                w = int(out[e, j, 0])
                assert w & 15 == len(seats)
                assert [(w >> (4 + 4 * p)) & 15 for p in range(len(seats))] == seats
                assert out[e, j, 1: 1 + len(seats)].tolist() == res


def test_mixed_league_restatement_replays_reference_tournaments():
    """the oracle's DrunkHamster + MCSAgent tournament streams
    (league_mixed_records) replay golden F11's "dropin" leagues -- seeded
    reference Tournament.play_game() sequences with MCS seats searching on the
    same global numpy stream (tournament.py:132-177, mcts.py:43-188): seat
    draws, results; no Q6 decision in them"""
    for lg in load("tournament_games.json")["dropin"]:
        G, hi = len(lg["games"]), lg["max_players"]
        rec, q6 = O.league_mixed_records(lg["kinds"], lg["min_players"], hi, lg["mc_per_card"], lg["mc_max"],
                                         seed=lg["seed"], slots=1, games=G)
        assert int(q6.sum()) == 0
        for e, g in enumerate(lg["games"]):
            k = len(g["names"])
            w = int(rec[e, 0, 0])
            assert w & 15 == k
            assert [lg["agents"][(w >> (4 + 4 * p)) & 15] for p in range(k)] == g["names"], (lg["kinds"], e)
            assert rec[e, 0, 1: 1 + k].tolist() == g["results"], (lg["kinds"], e)
    # an all-DrunkHamster roster is the DrunkHamster restatement
    r, _ = O.league_mixed_records("RRRRR", 2, 4, seed=5, slots=32, games=3)
    assert np.array_equal(r, O.league_records(5, 2, 4, seed=5, slots=32, games=3))
