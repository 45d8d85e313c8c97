"""GPU checks of the "Alpha0.5" PUCT engine (sechs_puct.hip + policy MLP).

Floating-point parity (PUCT rollouts sample from torch's RNG
in the reference, so bitwise replay is unpinned):
  * PUCT root formula kernel == the reference's numbers (golden F5), exactly;
  * candidate rows (fp32) == SechsNimmtStateNormalization of [card, obs], exactly;
  * root probabilities with the reference's weights == golden F8 within 1e-5 (fp32 net);
  * search statistics are self-consistent and PUCT beats random play.
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


def test_puct_score_kernel_matches_reference_formula():
    from rl_6_nimmt import _native as nat

    cases = load("puct_math.json")["cases"]
    D = len(cases)
    n = np.zeros(D, dtype=np.int32)
    stats = np.zeros((D, 24), dtype=np.int32)
    hist = np.zeros((D, 172), dtype=np.int32)
    probs = np.zeros((D, 10), dtype=np.float32)
    for d, c in enumerate(cases):
        n[d] = len(c["legal"])
        allo = []
        for k, outs in enumerate(c["outcomes"]):
            stats[d, k] = int(sum(outs))
            stats[d, 10 + k] = len(outs)
            allo += outs
        stats[d, 20] = len(allo)
        if allo:
            stats[d, 21], stats[d, 22] = int(min(allo)), int(max(allo))
        for o in allo:
            hist[d, int(o) + 171] += 1
        probs[d, : n[d]] = c["probs"]
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(a).to(dev)
    pu = torch.zeros((D, 10), dtype=torch.float64, device=dev)
    ch = torch.zeros((D,), dtype=torch.int32, device=dev)
    args = [t(n), t(stats), t(hist), t(probs)]
    nat.check(nat.lib().sn_puct_score(D, *[nat.ptr(a) for a in args], 2.0, nat.ptr(pu), nat.ptr(ch),
                                      nat.stream_handle()), "sn_puct_score")
    pu, ch = pu.cpu().numpy(), ch.cpu().numpy()
    for d, c in enumerate(cases):
        ref = np.array([np.nan if v is None else v for v in c["pucts"]])
        assert np.array_equal(pu[d, : n[d]], ref, equal_nan=True), d
        assert ch[d] == c["choice"], d


def _engine(B=64, N=4, mask=None, dtype=torch.float32, mc_max=8, mc_per_card=2, seed=5, weights=None):
    from rl_6_nimmt.puct import BatchedPUCT, make_actor
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(B, N, seed=seed, rng="philox")
    env.reset()
    torch.manual_seed(0)
    actor = make_actor()
    if weights is not None:
        actor.load_state_dict(weights)
    return env, BatchedPUCT(env, actor, mc_per_card=mc_per_card, mc_max=mc_max, seed=seed, seats_mask=mask,
                            net_dtype=dtype)


def test_root_rows_are_normalised_observations():
    from rl_6_nimmt import _native as nat
    from rl_6_nimmt.utils.preprocessing import SechsNimmtStateNormalization

    env, eng = _engine(B=50)
    n = 10
    q = eng._params(n)
    rows = torch.empty((eng.D * n, 48), dtype=torch.float32, device=env.device)
    import ctypes

    nat.check(nat.lib().sn_puct_root_rows(env._h, ctypes.byref(q), nat.ptr(rows), 0, env._stream()), "root_rows")
    obs = env.obs(torch.int64).float()  # [B, N, 47]
    hands = env.hands().long()          # [B, N, 10]
    cards = hands.reshape(-1, 10).float()
    ref_in = torch.cat((cards.reshape(-1, 1), obs.reshape(-1, 1, 47).expand(-1, 10, -1).reshape(-1, 47)), dim=1)
    ref = SechsNimmtStateNormalization(action=True)(ref_in.cpu())
    assert torch.equal(rows.cpu(), ref)


def test_root_probs_match_reference_policy():
    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    weights = {k: torch.from_numpy(z[k]) for k in z.files if "net" in k}
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env, eng = _engine(B=1, weights=weights)
    b = np.full((1, 4, 6), -1, dtype=np.int8)
    s = z["states"][0]
    for r in range(4):
        row = [c for c in s[23 + 6 * r: 29 + 6 * r] if c >= 0]
        b[0, r, : len(row)] = row
    h = np.stack([z["legal"][p] for p in range(4)])[None].astype(np.int8)
    env.reset_to(torch.from_numpy(b), torch.from_numpy(h))
    eng.decide(10)
    probs = eng.root_probs.cpu().numpy()
    for p in range(4):
        assert np.allclose(probs[p], z["probs"][p], atol=1e-5), p


def test_search_statistics_consistent():
    env, eng = _engine(B=32, mc_max=12, mc_per_card=2)
    for t in range(10):
        n = 10 - t
        acts = eng.decide(n)
        if n > 1:
            st, hist = eng.stats.cpu().numpy(), eng.hist.cpu().numpy()
            n_mc = eng.n_mc(n)
            assert (st[:, 10:10 + n].sum(axis=1) == n_mc).all()
            assert (st[:, 20] == n_mc).all() and (hist.sum(axis=1) == n_mc).all()
            vals = np.arange(172) - 171
            assert ((hist * vals).sum(axis=1) == st[:, :10].sum(axis=1)).all()
            best = eng.best_index.cpu().numpy()
            for d in range(eng.D):
                cnt = st[d, 10:10 + n]
                means = np.where(cnt > 0, st[d, :n] / np.maximum(cnt, 1), -np.inf)
                assert best[d] == int(np.argmax(means))
        rew, done, inv = env.step(acts)
        assert (inv.cpu().numpy() == -1).all()


def test_puct_beats_random_seats():
    torch.manual_seed(1)
    env, eng = _engine(B=512, mask=0b0001, dtype=torch.bfloat16, mc_max=100, mc_per_card=10, seed=9)
    total = eng.play_episode().float().mean(dim=0).cpu().numpy()
    assert total[0] > total[1:].mean() + 2.0, total


def test_dropin_puct_agent_session_and_learning():
    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import DrunkHamster, PUCTAgent

    torch.manual_seed(0)
    agent = PUCTAgent(mc_max=20, mc_per_card=2)
    agent.train()
    before = [p.detach().clone() for p in agent.actor.parameters()]
    np.random.seed(0)
    sess = GameSession(agent, DrunkHamster(), DrunkHamster())
    sess.play_game()
    assert len(sess.results) == 1 and (sess.results[0] <= 0).all()
    after = list(agent.actor.parameters())
    assert any(not torch.equal(a, b) for a, b in zip(after, before))  # one Adam step at episode end
