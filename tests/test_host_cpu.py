"""Host-side logic that needs no GPU: tournament scoring (golden F7), the
multiplayer Elo stand-in, evolve bookkeeping, the agent registry."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_positions_match_reference():
    from rl_6_nimmt.tournament import Tournament

    for c in load("positions.json")["cases"]:
        s = np.array(c["scores"], dtype=np.int32)
        assert Tournament._compute_relative_positions(s).tolist() == c["relative"]
        assert Tournament._compute_absolute_positions(s).tolist() == c["absolute"]
        assert int(np.argmax(s)) == c["winner_index"]


def test_elo_properties():
    """parity unpinned (multi_elo absent): conservation and ordering properties"""
    from rl_6_nimmt.elo import EloPlayer, calc_elo

    rng = np.random.RandomState(0)
    for _ in range(50):
        n = rng.randint(2, 6)
        elos = rng.uniform(1400, 1800, n)
        places = rng.permutation(n) + 1.0
        new = calc_elo([EloPlayer(p, e) for p, e in zip(places, elos)], 32)
        assert abs(sum(new) - sum(elos)) < 1e-9  # zero-sum
        # equal ratings: the winner gains, the loser loses
    new = calc_elo([EloPlayer(1, 1600), EloPlayer(2, 1600)], 32)
    assert new == [1616.0, 1584.0]
    new = calc_elo([EloPlayer(1.5, 1600), EloPlayer(1.5, 1600)], 32)
    assert new == [1600.0, 1600.0]


class _Dummy:
    def __init__(self):
        self.w = 1


def test_tournament_bookkeeping_and_evolve():
    import torch

    from rl_6_nimmt.tournament import Tournament

    class A(torch.nn.Module):
        pass

    t = Tournament(min_players=2, max_players=3)
    for name in ["a", "b", "c", "d"]:
        t.add_player(name, A())
    assert len(t) == 4
    t.score_game(["a", "b", "c"], np.array([-3, -10, -3], dtype=np.int32))
    assert t.tournament_wins["a"] == [1.0] and t.tournament_wins["c"] == [0.0]
    assert t.tournament_positions["a"][0] == pytest.approx(0.75)
    assert t.played_games["b"] == 1 and t.total_games == 1
    assert t.elos["b"][-1] < 1600 < t.elos["a"][-1]
    table = str(t)
    assert "Tournament after 1 games:" in table and " Agent                | Games |" in table
    t.evolve(copies=(2,), max_players=None, max_per_descendant=2, metric="elo")
    names = t.active_agents()
    assert "a_0" in names and "a_1" in names and "a" not in t.agents  # best agent cloned twice
    assert t.agents["a_0"].__name__ == "a_0"


def test_registry_and_spaces():
    from rl_6_nimmt.agents import AGENTS, DrunkHamster, MCSAgent
    from rl_6_nimmt.agents.base import Agent

    assert AGENTS["random"] is DrunkHamster and AGENTS["mcts"] is MCSAgent
    a = MCSAgent(mc_max=50)
    assert isinstance(a, Agent) and a.num_actions == 104 and a.state_length == 47
    np.random.seed(3)
    legal = [4, 17, 88]
    picks = [int(DrunkHamster()(None, legal)[0]) for _ in range(20)]
    np.random.seed(3)
    ref = [int(np.random.choice(np.array(legal, dtype=np.int32), size=1)[0]) for _ in range(20)]
    assert picks == ref


def test_mcs_agent_memory_bookkeeping():
    """card memory semantics of mcts.py:62-89 (host side of the drop-in agent)"""
    import torch

    from rl_6_nimmt.agents import MCSAgent

    a = MCSAgent()
    state = torch.tensor([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 4, 1, 1, 1, 1, 50, 60, 70, 80, 3, 1, 1, 1]
                         + [50, -1, -1, -1, -1, -1, 60, -1, -1, -1, -1, -1, 70, -1, -1, -1, -1, -1, 80, -1, -1, -1, -1, -1],
                         dtype=torch.float)
    legal = list(range(1, 11))
    a._initialize_game(state)
    a._memorize_cards(state, legal)
    assert a.num_players == 4
    assert len(a.available_cards) == 104 - 10 - 4
    assert 50 not in a.available_cards and 0 in a.available_cards
    assert a._compute_n_mc(10) == 100 and a._compute_n_mc(3) == 60 and a._compute_n_mc(2) == 20


def test_normalization_golden():
    import torch

    from rl_6_nimmt.utils.preprocessing import SechsNimmtStateNormalization

    d = load("normalization.json")
    x = torch.tensor(d["x_with_action"], dtype=torch.float32)
    assert torch.equal(SechsNimmtStateNormalization(action=True)(x), torch.tensor(d["y_with_action"]))
    assert torch.equal(SechsNimmtStateNormalization(action=False)(x[:, 1:]), torch.tensor(d["y_without_action"]))


def test_policy_golden_with_reference_weights():
    """PUCTAgent._compute_policy with the reference's own initial weights
    (torch.manual_seed(0); PUCTAgent()) reproduces its probabilities"""
    import torch

    from rl_6_nimmt.agents import PUCTAgent

    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    a = PUCTAgent()
    sd = {k: torch.from_numpy(z[k]) for k in a.actor.state_dict()}
    a.actor.load_state_dict(sd)
    for p in range(4):
        legal = [int(c) for c in z["legal"][p] if c >= 0]
        with torch.no_grad():
            probs = a._compute_policy(legal, torch.tensor(z["states"][p]).float()).numpy()
        assert np.allclose(probs, z["probs"][p][: len(legal)], rtol=0, atol=1e-7)


def test_reference_init_matches():
    """same module layout and init order as the reference: torch.manual_seed(0); PUCTAgent() gives its weights"""
    import torch

    from rl_6_nimmt.agents import PUCTAgent

    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    torch.manual_seed(0)
    a = PUCTAgent()
    for k, v in a.actor.state_dict().items():
        assert np.array_equal(v.numpy(), z[k]), k


def test_puct_formulas_golden():
    from rl_6_nimmt.agents import PUCTAgent

    a = PUCTAgent()
    d = load("puct_math.json")
    for c in d["cases"]:
        legal = c["legal"]
        outcomes = {x: list(o) for x, o in zip(legal, c["outcomes"])}
        probs = np.array(c["probs"], dtype=np.float32)
        pucts = a._compute_pucts(legal, outcomes, probs)
        ref = [np.nan if v is None else v for v in c["pucts"]]
        assert np.array_equal(np.asarray(pucts), np.asarray(ref), equal_nan=True)
        assert [float(v) for v in a._normalize_q(outcomes)] == c["normalize_q"]


def test_customed_and_reinforce_seeded_init_match_reference():
    """Host-side agents (no GPU): seeded constructions give the reference's
    initial weights (golden F9/F10), so seeded scripts train the same nets."""
    import torch

    from rl_6_nimmt.agents import AGENTS, BatchedReinforceAgent, PUCTCustomedAgent

    assert AGENTS["reinforce"] is BatchedReinforceAgent
    W = np.load(os.path.join(GOLDEN, "customed_weights.npz"))
    spec = json.load(open(os.path.join(GOLDEN, "customed_games.json")))
    for si, sess in enumerate(spec["sessions"][:3]):
        torch.manual_seed(sess["seed"])
        agents = [PUCTCustomedAgent(mc_max=200) if c == "C" else None for c in sess["seats"]]
        for i, a in enumerate(agents):
            if a is None:
                continue
            for k, v in a.actor.state_dict().items():
                assert torch.equal(v, torch.from_numpy(W[f"s{si}_a{i}_init_{k}"])), (si, i, k)
            assert a.actor.head_nets[0][0].out_features == 2
    W = np.load(os.path.join(GOLDEN, "reinforce_weights.npz"))
    spec = json.load(open(os.path.join(GOLDEN, "reinforce_games.json")))
    sess = spec["sessions"][0]
    torch.manual_seed(sess["seed"])
    a = BatchedReinforceAgent(**sess["kwargs"])
    for k, v in a.actor.state_dict().items():
        assert torch.equal(v, torch.from_numpy(W[f"s0_a0_init_{k}"])), k


def test_discounted_returns_formula():
    """utils/various.py:41-50: G_t = r_t + gamma G_{t+1}"""
    from rl_6_nimmt.agents.policy import compute_discounted_returns

    r = [0.0, -3.0, 0.0, -5.0, -1.0]
    g = compute_discounted_returns(r, 0.9).numpy()
    want = np.zeros(5)
    acc = 0.0
    for t in range(4, -1, -1):
        acc = r[t] + 0.9 * acc
        want[t] = acc
    assert np.allclose(g, want, rtol=0, atol=1e-6)


def _random_league_records(rng, G, K, N):
    rec = np.zeros((G, 1 + N), dtype=np.int32)
    for i in range(G):
        k = int(rng.randint(2, N + 1))
        ids = rng.permutation(K)[:k]
        w = k
        for p, a in enumerate(ids):
            w |= int(a) << (4 + 4 * p)
        rec[i, 0] = w
        # few distinct values: many ties
        rec[i, 1: 1 + k] = -rng.randint(0, 6 if i % 2 else 40, size=k)
    return rec


def test_native_elo_replay_equals_python_replay():
    """sn_elo_replay (host C++ in libsechs.so, no GPU call) == the sequential
    Python replay of Tournament._compute_elos with elo.py, bit for bit."""
    from rl_6_nimmt import _native as nat  # noqa: F401  (loads libsechs.so)
    from rl_6_nimmt.elo import EloPlayer, calc_elo
    from rl_6_nimmt.league import replay_league_elo
    from rl_6_nimmt.tournament import Tournament
    import torch

    rng = np.random.RandomState(5)
    for K, N in ((5, 4), (6, 6), (3, 2)):
        rec = _random_league_records(rng, 3000, K, N)
        elos = np.full(K, 1600.0)
        for row in rec:
            k = row[0] & 15
            ids = [(int(row[0]) >> (4 + 4 * p)) & 15 for p in range(k)]
            places = Tournament._compute_absolute_positions(row[1: 1 + k])
            new = calc_elo([EloPlayer(pl, elos[a]) for pl, a in zip(places, ids)], 32)
            for a, e in zip(ids, new):
                elos[a] = e
        got = replay_league_elo(torch.from_numpy(rec), K, N, 1600.0, 32.0)
        assert np.array_equal(got, elos), (K, N)


def test_league_scoring_matches_reference_formulas():
    """league.relative_positions / winners (vectorised) == Tournament's
    per-game formulas on the golden F7 cases and random tied games."""
    import torch

    from rl_6_nimmt.league import relative_positions, winners
    from rl_6_nimmt.tournament import Tournament

    cases = [np.array(c["scores"], dtype=np.int64) for c in load("positions.json")["cases"]]
    rng = np.random.RandomState(2)
    cases += [-rng.randint(0, 4, size=rng.randint(2, 7)) for _ in range(300)]
    P = 6
    R = np.zeros((len(cases), P), dtype=np.int64)
    k = np.array([len(c) for c in cases])
    for i, c in enumerate(cases):
        R[i, : len(c)] = c
    rel = relative_positions(torch.from_numpy(R), torch.from_numpy(k)).numpy()
    win = winners(torch.from_numpy(R), torch.from_numpy(k)).numpy()
    for i, c in enumerate(cases):
        ref = Tournament._compute_relative_positions(c)
        assert np.allclose(rel[i, : len(c)], ref, atol=1e-6), c
        assert win[i] == int(np.argmax(c))
