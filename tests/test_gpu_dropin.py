"""The reference's own API on the MI355X engine: seeded scripts written for
the reference (np.random.seed + GameSession(...)) give the reference's results."""
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


def test_game_session_random_games_all_sizes():
    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import DrunkHamster

    meta = load("random_games_meta.json")
    z = np.load(os.path.join(GOLDEN, "random_games.npz"))
    for cfg in meta["configs"]:
        if cfg["num_cards"] != 104 or not cfg["include_summaries"]:
            continue
        n = cfg["num_players"]
        for s in range(min(cfg["seeds"], 6)):
            np.random.seed(s)
            sess = GameSession(*[DrunkHamster() for _ in range(n)])
            sess.play_game()
            assert sess.results[0].tolist() == z[cfg["key"] + "_results"][s].tolist(), (n, s)


def test_game_session_multi_episode_stream():
    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import DrunkHamster

    for r in load("random_sessions.json")["sessions"]:
        if "results" not in r or r["num_players"] > 4:
            continue
        np.random.seed(r["seed"])
        sess = GameSession(*[DrunkHamster() for _ in range(r["num_players"])])
        for _ in range(len(r["results"])):
            sess.play_game()
        assert [x.tolist() for x in sess.results] == r["results"]


@pytest.mark.parametrize("n", [2, 4, 10])
def test_scalar_reset_matches_numpy_shuffle(n):
    """sn_reset1 (the wave-parallel one-game deal) against numpy itself:
    env.py:99-112's np.random.shuffle of arange(104) from numpy states at
    every position class -- fresh, mid-block, a deal that crosses into the
    next 624-word block (numpy twists there), pos = 624 (twist first) -- the
    hands, rows and numpy's state afterwards."""
    from rl_6_nimmt import SechsNimmtEnv

    env = SechsNimmtEnv(n, verbose=False)
    for seed, skip in [(0, 0), (1, 1), (2, 300), (3, 480), (4, 560), (5, 600), (6, 623), (7, 624), (8, 1000)]:
        rs = np.random.RandomState(seed)
        rs.randint(0, 2**32, size=skip, dtype=np.uint64)
        st = rs.get_state()
        np.random.set_state(st)
        env.reset()
        deck = np.arange(104, dtype=np.int32)
        rs.shuffle(deck)
        cards = list(deck)
        hands = [sorted(int(c) for c in cards[10 * p:10 * p + 10]) for p in range(n)]
        rows = [int(cards[103 - r]) for r in range(4)]
        assert [[int(c) for c in h] for h in env._hands] == hands, (n, seed, skip)
        assert [[int(c) for c in r] for r in env._board] == [[c] for c in rows], (n, seed, skip)
        got, want = np.random.get_state(), rs.get_state()
        assert np.array_equal(got[1], want[1]) and got[2] == want[2], (n, seed, skip, got[2], want[2])


def test_env_dropin_trace_and_errors():
    from rl_6_nimmt import InvalidMoveException, SechsNimmtEnv

    meta = load("random_games_meta.json")
    z = np.load(os.path.join(GOLDEN, "random_games.npz"))
    cfg = [c for c in meta["configs"] if c["num_players"] == 3 and c["num_cards"] == 104][0]
    k = cfg["key"]
    np.random.seed(2)
    env = SechsNimmtEnv(3, verbose=False)
    states, legal = env.reset()
    assert all(s.dtype == np.int64 and s.shape == (47,) for s in states)
    assert np.array_equal(np.stack(states), z[k + "_obs"][2, 0])
    assert env.action_space.n == 104 and env.observation_space.shape == (47,)
    for t in range(10):
        acts = z[k + "_actions"][2, t].tolist()
        (states, legal), rew, done, info = env.step(acts)
        assert rew.dtype == np.int32 and rew.tolist() == z[k + "_rewards"][2, t].tolist()
        assert np.array_equal(np.stack(states), z[k + "_obs"][2, t + 1])
        assert done == (t == 9) and info == {}
    # errors: wrong arity and illegal cards keep the reference's types and messages
    env.reset_to([[10], [20], [30], [40]], [[5, 6], [7, 8], [50, 51]])
    with pytest.raises(AssertionError):
        env.step([5, 7])
    with pytest.raises(InvalidMoveException, match=r"Player 2 tried to play card 10, but their hand is \[7, 8\]"):
        env.step([5, 9, 50])
    # sn_step1's per-seat trace words are 0 after an illegal step (include/sechs.h), not the last step's
    assert not env._out[2 + 14 * 3: 2 + 15 * 3].any()
    (states, legal), rew, done, _ = env.step([5, 7, 51])  # state untouched by the failed step
    assert legal == [[6], [8], [50]]


def test_notebook_games_through_dropin_env():
    from rl_6_nimmt import SechsNimmtEnv

    for G in load("notebook_games.json")["games"]:
        env = SechsNimmtEnv(2, player_names=G["names"])
        states, legal = env.reset_to([list(r) for r in G["board"]], [list(h) for h in G["hands"]])
        assert [s.tolist() for s in states] == G["obs0"]
        for acts, rec in zip(G["actions"], G["steps"]):
            (states, legal), rew, done, _ = env.step(acts)
            assert rew.tolist() == rec["rewards"] and env._board == rec["board"] and done == rec["done"]
        env.render()
        assert (-env._scores).tolist() == G["final_scores"]


def test_notebook_debug_trace_through_dropin_env(caplog):
    """the drop-in env's verbose log is the reference's -- per
    step, cards ascending: "<name> (player p) plays card c" (env.py:128), on
    an undercut "  ...chooses to replace row r" (env.py:145), on a scored row
    "  ...and gains h Hornochsen" (env.py:165) -- line for line against the
    notebook's rendered DEBUG output (F1 `trace`)."""
    import logging

    from rl_6_nimmt import SechsNimmtEnv

    games = load("notebook_games.json")["games"]
    assert sum(any("chooses" in x for x in G["trace"]) for G in games) >= 3
    for G in games:
        env = SechsNimmtEnv(len(G["names"]), player_names=G["names"], verbose=True)
        env.reset_to([list(r) for r in G["board"]], [list(h) for h in G["hands"]])
        caplog.clear()
        with caplog.at_level(logging.DEBUG, logger="rl_6_nimmt.env"):
            for acts in G["actions"]:
                env.step(acts)
        got = [r.getMessage() for r in caplog.records if r.name == "rl_6_nimmt.env" and r.levelno == logging.DEBUG]
        assert got == G["trace"]


def test_tournament_dropin_plays_games():
    from rl_6_nimmt import Tournament
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent

    np.random.seed(11)
    t = Tournament(min_players=2, max_players=4)
    t.add_player("Random1", DrunkHamster())
    t.add_player("Random2", DrunkHamster())
    t.add_player("MCS", MCSAgent(mc_max=20, mc_per_card=2))
    t.add_player("Random3", DrunkHamster())
    for _ in range(6):
        t.play_game()
    assert t.total_games == 6
    assert sum(t.played_games.values()) >= 12
    for name in t.agents:
        assert all(s <= 0 for s in t.tournament_scores[name])
        assert all(0.0 <= p <= 1.0 for p in t.tournament_positions[name])
        assert len(t.elos[name]) == 1 + t.played_games[name]
    assert "Tournament after 6 games:" in str(t)


def test_tournament_dropin_replays_reference_leagues():
    """Golden F11 (a): seeded reference Tournament.play_game() sequences over
    DrunkHamster and MCSAgent seats -- seat draws (tournament.py:166-177),
    results, relative positions, winners and the per-agent tallies -- replayed
    through the drop-in Tournament on the GPU.  _compute_elos is a no-op on
    both sides (multi_elo is absent: Elo unpinned)."""
    from rl_6_nimmt import GameSession, Tournament
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent

    d = load("tournament_games.json")["dropin"]
    assert len(d) == 3
    for lg in d:
        np.random.seed(lg["seed"])
        specs = [(n, MCSAgent(mc_max=lg["mc_max"], mc_per_card=lg["mc_per_card"]) if k == "M" else DrunkHamster())
                 for n, k in zip(lg["agents"], lg["kinds"])]
        t = Tournament(min_players=lg["min_players"], max_players=lg["max_players"])
        for n, a in specs:
            t.add_player(n, a)
        t._compute_elos = lambda names, scores, t=t: [t.elos[n][-1] for n in names]
        for g in lg["games"]:
            names, agents = t._choose_players(None)
            assert list(names) == g["names"], lg["seed"]
            sess = GameSession(*agents)
            sess.play_game(render=False)
            scores = sess.results[0]
            t.score_game(names, scores)
            assert [int(x) for x in scores] == g["results"], lg["seed"]
            assert np.allclose(t._compute_relative_positions(scores), g["relative"])
            assert names[int(np.argmax(scores))] == g["winner"]
        assert t.total_games == lg["total_games"]
        for n, tl in lg["tallies"].items():
            assert t.played_games[n] == tl["played_games"]
            assert [int(x) for x in t.tournament_scores[n]] == tl["scores"]
            assert np.allclose(t.tournament_positions[n], tl["positions"])
            assert [float(x) for x in t.tournament_wins[n]] == tl["wins"]
