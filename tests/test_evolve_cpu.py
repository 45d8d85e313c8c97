"""Tournament.evolve / copy_player / remove_player / score_game pinned to
the reference itself (golden F13, tests/golden/evolve_games.json, recorded by
tools/gen_fixtures.py from seeded reference tournaments with evolve() between
blocks of games: every metric, copies / max_players / max_per_descendant
combinations, two or three evolves per tournament).

The recorded games (seat names, results) are fed to the drop-in Tournament's
score_game and to the batched tournament's tallies (as device-format
records), then evolve runs: the roster (dict order, active flags, families),
the tallies and the Elo must equal the reference's before and after every
evolve.  The ranking quirks come from the reference, not from a restatement:
'tournament_wins' / 'tournament_positions' sort ascending, ties keep the
roster order (stable sort), 'elo' ranks by the latest Elo, positions are
float32 means.  Elo values: the build's multi_elo restatement stood in for
the absent package in the generator (parity of the Elo arithmetic itself
stays unpinned; here it is the same function on both sides).
Reference: /root/reference/rl_6_nimmt/tournament.py:54-164."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

CASES = json.load(open(os.path.join(GOLDEN, "evolve_games.json")))["cases"]


def _ev(block):
    ev = dict(block["evolve"])
    ev["copies"] = tuple(ev["copies"])
    return ev


def _check_dropin(t, roster):
    assert list(t.agents.keys()) == [r["name"] for r in roster]
    for r in roster:
        n = r["name"]
        assert t.active[n] == r["active"] and t.descendants[n] == r["descendant"], n
        assert t.played_games[n] == r["played_games"], n
        assert [int(x) for x in t.tournament_scores[n]] == r["scores"], n
        assert [float(x) for x in t.tournament_positions[n]] == r["positions"], n
        assert t.tournament_wins[n] == r["wins"], n
        assert [float(x) for x in t.elos[n]] == r["elos"], n


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_dropin_evolve_replays_reference(ci):
    from rl_6_nimmt.agents import DrunkHamster
    from rl_6_nimmt.tournament import Tournament

    case = CASES[ci]
    t = Tournament(case["min_players"], case["max_players"])
    for i in range(case["num_agents"]):
        t.add_player(f"a{i}", DrunkHamster())
    evolves = 0
    for block in case["blocks"]:
        for g in block["games"]:
            t.score_game(g["names"], np.array(g["results"], dtype=np.int32))
        if "evolve" in block:
            _check_dropin(t, block["before"])
            t.evolve(**_ev(block))
            _check_dropin(t, block["after"])
            evolves += 1
    assert evolves >= 2 and t.total_games == case["total_games"]


def _records(games, active, hi):
    """the recorded games as one records block of a 1-slot tournament handle
    (seats word k | active index << (4 + 4p), results, 0 past k)"""
    rec = torch.zeros((len(games), 1, 1 + hi), dtype=torch.int32)
    for e, g in enumerate(games):
        w = len(g["names"])
        for p, n in enumerate(g["names"]):
            w |= active.index(n) << (4 + 4 * p)
        rec[e, 0, 0] = w
        rec[e, 0, 1: 1 + len(g["results"])] = torch.tensor(g["results"], dtype=torch.int32)
    return rec


def _check_batched(bt, roster):
    assert bt.names == [r["name"] for r in roster]
    st = bt.agent_stats().numpy()
    for i, r in enumerate(roster):
        n = r["name"]
        assert bt.active[n] == r["active"] and bt.descendants[n] == r["descendant"], n
        assert st[i, 0] == r["played_games"] and st[i, 1] == sum(r["scores"]), n
        assert st[i, 3] == sum(r["wins"]), n
        pos = np.concatenate(bt.positions[n]) if bt.positions[n] else np.zeros(0, np.float32)
        assert pos.dtype == np.float32 and [float(x) for x in pos] == r["positions"], n
        assert bt.elos[i] == r["elo"], n


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_batched_evolve_replays_reference(ci):
    from rl_6_nimmt.agents import DrunkHamster
    from rl_6_nimmt.league import BatchedTournament

    case = CASES[ci]
    hi = case["max_players"]
    bt = BatchedTournament(1, case["min_players"], hi, fused=False)
    for i in range(case["num_agents"]):
        bt.add_player(f"a{i}", DrunkHamster())
    for block in case["blocks"]:
        active = bt.active_agents()
        bt.records.append((_records(block["games"], active, hi), torch.tensor([bt.names.index(n) for n in active])))
        bt.record_names.append(tuple(active))
        bt.total_games += len(block["games"])
        if "evolve" in block:
            _check_batched(bt, block["before"])
            bt.evolve(**_ev(block))
            _check_batched(bt, block["after"])
    assert bt.total_games == case["total_games"]


def test_batched_winner_is_the_references_rule():
    """Tournament.winner (tournament.py:197-206) over the F13 rosters: the
    best float32 mean relative position over every agent, active or not"""
    from rl_6_nimmt.agents import DrunkHamster
    from rl_6_nimmt.league import BatchedTournament
    from rl_6_nimmt.tournament import Tournament

    for case in CASES:
        hi = case["max_players"]
        t = Tournament(case["min_players"], hi)
        bt = BatchedTournament(1, case["min_players"], hi, fused=False)
        for i in range(case["num_agents"]):
            t.add_player(f"a{i}", DrunkHamster())
            bt.add_player(f"a{i}", DrunkHamster())
        for block in case["blocks"]:
            active = bt.active_agents()
            for g in block["games"]:
                t.score_game(g["names"], np.array(g["results"], dtype=np.int32))
            bt.records.append((_records(block["games"], active, hi), torch.tensor([bt.names.index(n) for n in active])))
            bt.record_names.append(tuple(active))
            if "evolve" in block:
                t.evolve(**_ev(block))
                bt.evolve(**_ev(block))
            with np.errstate(all="ignore"):
                assert bt.winner().__name__ == t.winner().__name__
