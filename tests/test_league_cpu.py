"""Host logic of the batched tournament (league.py) that needs no GPU:
the roster evolution (Tournament.evolve / copy_player / remove_player,
tournament.py:54-130) against the drop-in Tournament on the same tallies,
and the agent -> engine classification."""
import numpy as np
import pytest
import torch


def _pair(names, scores, positions, wins, elos):
    from rl_6_nimmt.agents import DrunkHamster
    from rl_6_nimmt.league import BatchedTournament
    from rl_6_nimmt.tournament import Tournament

    ref = Tournament()
    bt = BatchedTournament(8, fused=False)
    for i, n in enumerate(names):
        ref.add_player(n, DrunkHamster())
        bt.add_player(n, DrunkHamster())
        ref.tournament_scores[n] = list(scores[i])
        ref.tournament_positions[n] = list(np.asarray(positions[i], dtype=np.float32))  # float32, as the reference's
        bt.positions[n] = [np.asarray(positions[i], dtype=np.float32)]
        ref.tournament_wins[n] = list(wins[i])
        ref.played_games[n] = len(scores[i])
        ref.elos[n] = [1600.0, elos[i]]
        bt.stats[i] = [len(scores[i]), sum(scores[i]), sum(positions[i]), sum(wins[i])]
        bt.elos[i] = elos[i]
    return ref, bt


@pytest.mark.parametrize("metric", ["elo", "tournament_scores", "tournament_positions", "tournament_wins"])
@pytest.mark.parametrize("copies,max_players,max_per", [((2,), None, 2), ((2,), 4, 2), ((3, 2), 5, 1), ((1,), 3, None)])
def test_batched_evolve_matches_reference_roster(metric, copies, max_players, max_per):
    rng = np.random.default_rng(hash((metric, copies, max_players, max_per)) & 0xFFFF)
    names = [f"ag{i}" for i in range(6)]
    scores = [list(rng.integers(-20, 0, size=rng.integers(1, 6))) for _ in names]
    positions = [list(rng.random(len(s)).round(3)) for s in scores]
    wins = [list(rng.integers(0, 2, size=len(s)).astype(float)) for s in scores]
    elos = list(1500 + rng.random(len(names)) * 200)
    ref, bt = _pair(names, scores, positions, wins, elos)
    for _ in range(2):  # twice: the second round ranks clones and their families
        ref.evolve(copies=copies, max_players=max_players, max_per_descendant=max_per, metric=metric)
        bt.evolve(copies=copies, max_players=max_players, max_per_descendant=max_per, metric=metric)
        assert list(ref.agents.keys()) == bt.names
        assert ref.active == bt.active
        assert ref.descendants == bt.descendants
        for i, n in enumerate(bt.names):
            assert bt.stats[i, 0] == len(ref.tournament_scores[n])
            assert np.isclose(bt.stats[i, 1], sum(ref.tournament_scores[n]))
            assert np.isclose(bt.elos[i], ref.elos[n][-1])


def test_agent_kinds():
    from rl_6_nimmt.agents import BatchedACERAgent, BatchedReinforceAgent, DrunkHamster, MCSAgent, PolicyMCSAgent
    from rl_6_nimmt.agents import PUCTAgent, PUCTCustomedAgent
    from rl_6_nimmt.league import agent_kind

    assert agent_kind(DrunkHamster()) == "random"
    assert agent_kind(MCSAgent()) == "mcs"
    assert agent_kind(PUCTAgent()) == "puct" and agent_kind(PolicyMCSAgent()) == "puct"
    assert agent_kind(PUCTCustomedAgent()) == "customed"
    assert agent_kind(BatchedACERAgent()) == "acer"
    assert agent_kind(BatchedReinforceAgent()) == "reinforce"
    from rl_6_nimmt.agents import AGENTS

    for name, cls in AGENTS.items():  # every registered agent the drop-in has takes a seat
        try:
            agent = cls()
        except TypeError:
            continue
        assert agent_kind(agent) in ("random", "mcs", "puct", "customed", "acer", "reinforce"), name
