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


def test_root_probs_bf16_match_reference_policy():
    """The bench's net dtype: bf16 rows, weights and activations (8-bit
    mantissa, ~0.4 % relative per rounding) against the reference's fp32
    probabilities (golden F8).  Tolerance |dp| <= 3e-3 on these ~0.1
    probabilities: 3x the worst error of the same bf16 forward on the host
    CPU (1.05e-3)."""
    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    weights = {k: torch.from_numpy(z[k]) for k in z.files if "net" in k}
    env, eng = _engine(B=1, weights=weights, dtype=torch.bfloat16)
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
        assert np.allclose(probs[p], z["probs"][p], rtol=0, atol=3e-3), (p, np.abs(probs[p] - z["probs"][p]).max())
        assert abs(probs[p].sum() - 1.0) < 1e-5


def test_playout_sampling_follows_the_policy():
    """k_puct_step's Categorical(probs).sample() (mcts.py:209-217) with
    Philox uniforms: the same position in every game, the root move SAMPLED
    (puct_root=False), 64 playouts per decision -> 131 072 samples of the
    root policy; per-move frequencies within 5 standard errors of
    softmax(logits) computed on the host from the same fp32 net."""
    from rl_6_nimmt.utils.preprocessing import SechsNimmtStateNormalization
    from rl_6_nimmt.puct import BatchedPUCT, make_actor
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    B = 2048
    env = VecSechsNimmtEnv(B, 4, seed=21, rng="philox")
    env.reset()
    b = env.board()[:1].expand(B, -1, -1).contiguous()
    h = env.hands()[:1].expand(B, -1, -1).contiguous()
    env.reset_to(b, h)
    torch.manual_seed(3)
    actor = make_actor()
    with torch.no_grad():  # a peaked policy, so the check has teeth
        actor.head_nets[0][0].weight.mul_(40.0)
    eng = BatchedPUCT(env, actor, mc_per_card=10, mc_max=64, seed=5, seats_mask=0b0001, puct_root=False,
                      net_dtype=torch.float32)
    eng.decide(10)
    visits = eng.stats.cpu().numpy()[:, 10:20].sum(axis=0).astype(np.float64)
    total = visits.sum()
    assert total == B * 64
    obs = env.obs(torch.int64).float().cpu()[0, 0]
    hand = h[0, 0].long().cpu()
    x = torch.cat((hand.float()[:, None], obs[None, :].expand(10, -1)), dim=1)
    with torch.no_grad():
        (logits,) = actor(SechsNimmtStateNormalization(action=True)(x))
    probs = torch.softmax(logits.flatten().double(), 0).numpy()
    assert probs.max() > 3 * probs.min(), probs  # far from uniform
    assert np.allclose(eng.root_probs.cpu().numpy()[0], probs, atol=1e-5)
    freq = visits / total
    se = np.sqrt(probs * (1 - probs) / total)
    assert np.all(np.abs(freq - probs) <= 5 * se + 1e-7), (freq, probs)


def test_policy_loss_matches_reference_training_loss():
    """BatchedPUCT.policy_loss == PolicyMCSAgent._train (mcts.py:245-261):
    -sum over the episode's searched decisions of log pi(chosen root move),
    pi = softmax(actor(SechsNimmtStateNormalization([card, obs]))) with the
    reference's fp32 rows (mcts.py:219-228) -- value and gradient, although
    the search ran a bf16 net (training rows are recorded in fp32)."""
    from rl_6_nimmt.utils.preprocessing import SechsNimmtStateNormalization

    env, eng = _engine(B=32, dtype=torch.bfloat16, mc_max=8, mc_per_card=2, seed=13)
    env.reset()
    norm = SechsNimmtStateNormalization(action=True)
    seen = []
    for t in range(10):
        n = 10 - t
        obs = env.obs(torch.int64).float().cpu()
        hands = env.hands().long().cpu()
        acts = eng.decide(n, record=True)
        if n > 1:
            seen.append((obs, hands, n, eng.best_index.cpu().clone()))
        rew, done, inv = env.step(acts)
        assert (inv.cpu() == -1).all()
    assert len(eng.decisions) == 9
    loss = eng.policy_loss()
    grads = torch.autograd.grad(loss, list(eng.actor.parameters()))
    loss = loss.detach()
    ref = torch.zeros(())
    N = env.num_players
    for obs, hands, n, best in seen:
        for g in range(env.num_games):
            for p in range(N):
                x = torch.cat((hands[g, p, :n].float()[:, None], obs[g, p][None, :].expand(n, -1)), dim=1)
                (logits,) = eng.actor(norm(x))
                probs = torch.softmax(logits, dim=0).flatten()
                ref = ref - torch.log(probs[int(best[g * N + p])])
    rgrads = torch.autograd.grad(ref, list(eng.actor.parameters()))
    ref = ref.detach()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref)), (float(loss), float(ref))
    # one decider's term alone is the reference's per-episode loss (what a
    # BatchedTournament(updates_per_round="games") steps on), and the chunks
    # of any split sum to the whole
    with torch.no_grad():
        for d in (0, 5, eng.D - 1):
            g, p = divmod(d, N)
            one = torch.zeros(())
            for obs, hands, n, best in seen:
                x = torch.cat((hands[g, p, :n].float()[:, None], obs[g, p][None, :].expand(n, -1)), dim=1)
                (logits,) = eng.actor(norm(x))
                one = one - torch.log(torch.softmax(logits, dim=0).flatten()[int(best[d])])
            got = float(eng.policy_loss(d, d + 1))
            assert abs(got - float(one)) <= 1e-5 * max(1.0, abs(float(one))), (d, got, float(one))
        bounds = [0, 7, 40, 41, eng.D]
        parts = sum(float(eng.policy_loss(a, b)) for a, b in zip(bounds[:-1], bounds[1:]))
        assert abs(parts - float(loss)) <= 1e-5 * abs(float(loss)), (parts, float(loss))
    # (the head bias's gradient is a sum of softmax residuals that is 0 in
    # exact arithmetic: compare at an absolute floor of 1e-4)
    for a, r in zip(grads, rgrads):
        assert torch.allclose(a.cpu(), r, rtol=1e-4, atol=1e-4), (a, r)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_graph_replay_equals_eager_search(dtype):
    """graph=True (one captured hipGraph of a decision's rollout chain per
    hand size, the decision counter read from device memory) gives the same
    statistics, actions and root probabilities as launching eagerly, over a
    whole game (every hand size, each graph replayed 4 x 1 decisions, and
    captured once)."""
    res = []
    for graph in (False, True):
        env, eng = _engine(B=96, dtype=dtype, mc_max=12, mc_per_card=2, seed=17)
        eng.graph = graph
        out = []
        for t in range(10):
            n = 10 - t
            acts = eng.decide(n).clone()
            out.append((acts.cpu(), eng.stats.cpu().clone(), eng.hist.cpu().clone(), eng.root_probs.cpu().clone()))
            env.step(acts)
        res.append((out, eng.rows_evaluated))
    (a, ra), (b, rb) = res
    assert ra == rb
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert torch.equal(u, v)


def test_search_statistics_consistent_bf16_full_size():
    """Config 4's shape: 8192 games, every seat searching, bf16 net through
    the layer-1 split and the padded head's strided bf16 logits; one
    decision at n = 10 and n = 4 -- the playout counts, the outcome
    histogram and the chosen moves agree with each other."""
    env, eng = _engine(B=8192, dtype=torch.bfloat16, mc_max=12, mc_per_card=2, seed=31)
    eng.graph = True
    for t in range(10):
        n = 10 - t
        acts = eng.decide(n)
        if n in (10, 4):
            st, hist = eng.stats.cpu().numpy(), eng.hist.cpu().numpy()
            n_mc = eng.n_mc(n)
            assert (st[:, 10:10 + n].sum(axis=1) == n_mc).all()
            assert (st[:, 20] == n_mc).all() and (hist.sum(axis=1) == n_mc).all()
            vals = np.arange(172) - 171
            assert ((hist * vals).sum(axis=1) == st[:, :10].sum(axis=1)).all()
            cnt = st[:, 10:10 + n]
            means = np.where(cnt > 0, st[:, :n] / np.maximum(cnt, 1), -np.inf)
            assert (eng.best_index.cpu().numpy()[: eng.D] == np.argmax(means, axis=1)).all()
        rew, done, inv = env.step(acts)
        assert (inv.cpu().numpy() == -1).all()
    assert bool(done.all())


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


def test_dropin_puct_agent_copies_after_searching():
    """Tournament.copy_player deep-copies agents: a PUCTAgent that has
    searched (device engines, captured graphs) copies without them, and the
    copy searches with its own engine and the same weights."""
    import copy

    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import DrunkHamster, PUCTAgent

    torch.manual_seed(0)
    agent = PUCTAgent(mc_max=8, mc_per_card=2)
    agent.train()
    np.random.seed(1)
    GameSession(agent, DrunkHamster(), DrunkHamster()).play_game()
    clone = copy.deepcopy(agent)
    assert clone._engine is None and not getattr(clone, "_engines", None)
    for a, b in zip(agent.actor.parameters(), clone.actor.parameters()):
        assert torch.equal(a, b)
    np.random.seed(2)
    sess = GameSession(clone, DrunkHamster(), DrunkHamster(), DrunkHamster())
    sess.play_game()
    assert (sess.results[0] <= 0).all()


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


# ---------------------------------------------------------------------------
# PUCTCustomedAgent (mcts.py:325-451): golden F9
# ---------------------------------------------------------------------------
def test_dropin_customed_agent_replays_reference_training_sessions():
    """Seeded GameSessions of the drop-in PUCTCustomedAgent (training on,
    Adam at every episode end) against the reference's recorded sessions:
    seeded init weights, every move, log-prob, value outcome and loss, the
    final weights and the session results are identical (fp32 host net)."""
    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import DrunkHamster, PUCTCustomedAgent

    spec = load("customed_games.json")
    W = np.load(os.path.join(GOLDEN, "customed_weights.npz"))
    for si, sess in enumerate(spec["sessions"]):
        seats, seed = sess["seats"], sess["seed"]
        torch.manual_seed(seed)
        agents = [PUCTCustomedAgent(mc_max=200) if c == "C" else DrunkHamster() for c in seats]
        rec = {}
        for i, c in enumerate(seats):
            if c != "C":
                continue
            a = agents[i]
            a.train()
            for k, v in a.actor.state_dict().items():
                assert torch.equal(v, torch.from_numpy(W[f"s{si}_a{i}_init_{k}"])), (si, i, k)
            rec[i] = {"info": [], "loss": []}
            fwd, lrn = a.forward, a.learn

            def fwd_rec(state, legal_actions, *x, _f=fwd, _i=i, **k):
                act, info = _f(state, legal_actions, *x, **k)
                rec[_i]["info"].append([int(act), float(info["log_prob"]), float(info["outcome"])])
                return act, info

            def lrn_rec(*x, _l=lrn, _i=i, **k):
                loss = _l(*x, **k)
                if k.get("episode_end"):
                    rec[_i]["loss"].append(float(loss))
                return loss

            a.forward, a.learn = fwd_rec, lrn_rec
        np.random.seed(seed)
        s = GameSession(*agents)
        for _ in range(sess["games"]):
            s.play_game()
        assert [[int(x) for x in r] for r in s.results] == sess["results"], si
        for i in rec:
            got, want = np.array(rec[i]["info"]), np.array(sess["trace"][str(i)]["info"])
            assert np.array_equal(got[:, 0], want[:, 0]), (si, i)
            # fp32 host math: CPUs round differently (vector widths), so floats
            # are compared to 1e-4; the moves themselves must be identical
            assert np.allclose(got[:, 1:], want[:, 1:], rtol=0, atol=1e-4), (si, i)
            assert np.allclose(rec[i]["loss"], sess["trace"][str(i)]["loss"], rtol=1e-5, atol=1e-4), (si, i)
            for k, v in agents[i].actor.state_dict().items():
                got, want = v.numpy().copy(), W[f"s{si}_a{i}_final_{k}"].copy()
                if k == "head_nets.0.0.bias":
                    # the policy-logit bias shifts every candidate's logit
                    # equally: softmax ignores it, its exact gradient is 0 and
                    # Adam scales the rounding noise (which differs between
                    # host CPUs) to up to lr per step -- bounded, not compared
                    assert abs(got[0] - want[0]) <= 3e-3 * sess["games"], (si, i)
                    got, want = got[1:], want[1:]
                assert np.allclose(got, want, rtol=0, atol=1e-4), (si, i, k)


def _customed(B=256, N=4, mask=None, dtype=torch.float32, seed=3):
    from rl_6_nimmt.puct import BatchedPUCTCustomed, make_actor_value
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(B, N, seed=seed, rng="philox")
    torch.manual_seed(0)
    actor = make_actor_value()
    return env, BatchedPUCTCustomed(env, actor, seats_mask=mask, net_dtype=dtype, seed=seed)


@pytest.mark.parametrize("mask", [None, 0b0101])
def test_batched_customed_matches_host_agent_math(mask):
    """Every decision of the batched engine (sn_puct_root_rows -> fp32 MLP ->
    sn_pcv_choose) equals the drop-in agent's _compute_policy_and_value on the
    same observation: first argmax of the values, log pi and value within
    1e-5; the batched loss equals the per-game reference loss summed."""
    from rl_6_nimmt.utils.preprocessing import SechsNimmtStateNormalization

    env, eng = _customed(B=64, mask=mask)
    env.reset()
    norm = SechsNimmtStateNormalization(action=True)
    actor = eng.actor
    N = env.num_players
    seats = [p for p in range(N) if mask is None or (mask >> p) & 1]
    per_step = []
    for t in range(10):
        n = 10 - t
        obs = env.obs(torch.int64).float().cpu()  # [B, N, 47]
        hands = env.hands().long().cpu()           # [B, N, 10]
        acts = eng.decide(n, record=True)
        got_a, got_lp, got_v = acts.cpu().numpy(), eng.log_prob.cpu().numpy(), eng.value.cpu().numpy()
        for g in range(0, env.num_games, 7):
            for j, p in enumerate(seats):
                d = g * len(seats) + j
                cards = hands[g, p, :n].float()[:, None]
                x = torch.cat((cards, obs[g, p][None, :].expand(n, -1)), dim=1)
                with torch.no_grad():
                    (out,) = actor(norm(x))
                k = int(torch.argmax(out[:, 1]))
                assert got_a[g, p] == int(hands[g, p, k]), (t, g, p)
                assert abs(got_v[d] - float(out[k, 1])) < 1e-5
                assert abs(got_lp[d] - float(torch.log_softmax(out[:, 0], 0)[k])) < 1e-5
        if len(seats) < N:
            rnd = eng._random_moves()
            keep = torch.tensor([p in seats for p in range(N)], device=env.device)
            acts = torch.where(keep[None, :], acts, rnd)
        rew, done, inv = env.step(acts)
        assert (inv.cpu() == -1).all()
        per_step.append(rew)
    per_step = torch.stack(per_step)
    loss = eng.loss(per_step)
    # per-game reference form (mcts.py:431-451), on the recorded rows
    ref = 0.0
    for j, p in enumerate(seats):
        for g in range(env.num_games):
            d = g * len(seats) + j
            vals, lps = [], []
            for rows, n, best in eng.decisions:
                (out,) = actor(rows[d * n:(d + 1) * n].cpu())
                k = int(best[d])
                vals.append(out[k, 1])
                lps.append(torch.log_softmax(out[:, 0], 0)[k])
            target = float(per_step[:-1, g, p].sum())
            ref = ref + torch.nn.functional.mse_loss(torch.stack(vals), torch.full((10,), target)) \
                - torch.stack(lps).sum()
    assert abs(float(loss) - float(ref)) <= 1e-4 * abs(float(ref)), (float(loss), float(ref))


def test_batched_customed_learning_step_changes_weights():
    env, eng = _customed(B=128, dtype=torch.bfloat16)
    total, per_step = eng.play_episode(record=True)
    assert (total <= 0).all() and total.shape == (128, 4)
    opt = torch.optim.Adam(eng.actor.parameters())
    before = [p.detach().clone() for p in eng.actor.parameters()]
    loss = eng.loss()
    opt.zero_grad()
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)
    assert any(not torch.equal(a.cpu(), b.cpu()) for a, b in zip(eng.actor.parameters(), before))


@pytest.mark.parametrize("B,n", [(64, 7), (37, 10), (256, 4), (10000, 8)])
def test_fused_mlp_equals_module_forward(B, n):
    """sn_puct_mlp_seats (seat rows, layer 1's per-seat part on MFMA, the
    card column + ReLU, layer 2 + ReLU and the head in one kernel) gives
    every rollout candidate's policy logit: equal to the same factored
    arithmetic restated in PyTorch f32 from the same bf16 values (to f32
    summation order: a bf16 ulp of the seat base here and there), and to
    the module's own bf16 forward on the full rows.  Ragged row counts (a
    short last 64-row tile) included; B = 10 000 gives the persistent
    workgroups several 64-seat groups each."""
    env, eng = _engine(B=B, dtype=torch.bfloat16, mc_max=4, mc_per_card=2, seed=29)
    for t in range(10 - n):
        env.step(eng.decide(10 - t))
    _check_mlp_kernels(env, eng, n)


def _check_mlp_kernels(env, eng, n, live=None):
    """the rollout-logit kernel against its factored arithmetic restated in
    PyTorch and the module's forward at n_cur = n, 3, 1 (rows the decision
    list's rollouts would evaluate); live: bool [D * N] -- seats of the
    rollouts' games (a tournament game of k < N players has N - k absent
    seats, whose logits are never read), None = all"""
    import ctypes

    from rl_6_nimmt import _native as nat

    N = env.num_players
    net = eng.sync_net()
    w1c, w2p, head, w1s = net.fused()
    w1, b1 = net.layers[0]
    w2, b2 = net.layers[1]
    H = w1.shape[0]
    q = eng._params(n)
    L, h, st = nat.lib(), env._h, env._stream()
    eng.memorize()
    nat.check(L.sn_puct_deal(h, ctypes.byref(q), st), "deal")
    tol = 2 ** -6
    for m in (n, 3, 1):
        S, R = eng.D * N, eng.D * N * m
        sel = torch.ones((R,), dtype=torch.bool, device=env.device) if live is None else \
            live.to(env.device).repeat_interleave(m)
        rows = torch.empty((R, 48), dtype=torch.bfloat16, device=env.device)
        nat.check(L.sn_puct_rows(h, ctypes.byref(q), m, nat.ptr(rows), 1, st), "rows")
        lg2 = torch.full((R,), float("nan"), dtype=torch.float32, device=env.device)
        nat.check(L.sn_puct_mlp_seats(h, ctypes.byref(q), m, nat.ptr(w1s), nat.ptr(w1c), nat.ptr(w2p), nat.ptr(head),
                                      nat.ptr(lg2), st), "mlp_seats")
        torch.cuda.synchronize()
        # the factored arithmetic: base = bf16(W1 [0, obs] + b1) per seat, h1 = bf16(relu(base + card w1c)),
        # h2 = bf16(relu(W2 h1 + b2)), logit = wh . h2 + bh (f32 accumulation throughout)
        seat = rows.view(S, m, 48)[:, 0].float().clone()
        seat[:, 0] = 0.0
        base = (seat @ w1.float().t() + b1.float()).to(torch.bfloat16).float()
        h1 = torch.relu(base.repeat_interleave(m, dim=0) + rows[:, :1].float() * w1c[None, :H]).to(torch.bfloat16)
        x2 = torch.relu(h1.float() @ w2.float().t() + b2.float()).to(torch.bfloat16).float()
        ref = x2 @ net.head_w[:, 0].float() + net.head_b[0].float()
        assert not torch.isnan(lg2[sel]).any()
        assert torch.allclose(lg2[sel], ref[sel], rtol=2 * tol, atol=2 * tol), (lg2 - ref)[sel].abs().max()
        with torch.no_grad():
            (want,) = net.module(rows)
        want = want[:, 0].float()
        assert torch.allclose(lg2[sel], want[sel], rtol=4 * tol, atol=4 * tol), (lg2 - want)[sel].abs().max()


def test_fused_and_rows_rollouts_agree_in_law(monkeypatch):
    """a whole PUCT search with the one-kernel MLP (the default) and with the
    generic path (candidate rows + the module's PyTorch forward; same
    weights, same Philox streams): the two bf16 roundings of the factored
    layer 1 may flip a sample now and then, so the searches agree in law --
    mean root visit counts and chosen moves match closely over 2 048
    decisions"""
    from rl_6_nimmt.puct import FusedMLP

    res = {}
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(FusedMLP, "fused", lambda self: None)
        env, eng = _engine(B=512, dtype=torch.bfloat16, mc_max=20, mc_per_card=10, seed=41)
        acts = eng.decide(10)
        torch.cuda.synchronize()
        res[fused] = (acts.clone(), eng.stats.clone(), eng.rows_evaluated)
    a1, s1, r1 = res[True]
    a2, s2, r2 = res[False]
    assert r1 == r2
    assert torch.equal(s1[:, 10:20].sum(dim=1), s2[:, 10:20].sum(dim=1))  # every rollout backed up
    agree = float((a1 == a2).float().mean())
    assert agree > 0.6, agree
    m1, m2 = s1[:, :10].double().sum() / s1[:, 10:20].double().sum(), s2[:, :10].double().sum() / s2[:, 10:20].double().sum()
    assert abs(float(m1 - m2)) < 0.5, (float(m1), float(m2))


def test_seat_parallel_step_equals_one_lane_step(monkeypatch):
    """k_puct_step_seats (one lane per seat) and k_puct_step (one lane per
    decision) draw the same Philox uniforms and resolve the same cards: a
    whole PUCT search gives identical statistics and moves (a plain handle;
    the tournament branches: test_league_puct_kernels_on_tournament_decisions)"""
    res = {}
    for lanes in ("1", "0"):
        monkeypatch.setenv("SECHS_PUCT_STEP_SEATS", lanes)
        env, eng = _engine(B=300, dtype=torch.float32, mc_max=12, mc_per_card=3, seed=17)
        acts = [eng.decide(10).clone()]
        env.step(acts[-1])
        acts.append(eng.decide(9).clone())
        torch.cuda.synchronize()
        res[lanes] = (acts, eng.stats.clone(), eng.hist.clone())
    assert all(torch.equal(a, b) for a, b in zip(res["1"][0], res["0"][0]))
    assert torch.equal(res["1"][1], res["0"][1]) and torch.equal(res["1"][2], res["0"][2])


def test_league_puct_kernels_on_tournament_decisions(monkeypatch):
    """the tournament branches of the PUCT kernels (players_of,
    absent seats q >= k of 2- and 3-player games, the live/dead seat lanes)
    on a BatchedTournament decision list (a PUCT agent among DrunkHamsters,
    2..4 players): the whole-rollout kernel (sn_puct_rollouts),
    k_puct_step_seats and the one-lane k_puct_step give identical records
    over whole games (the same Philox uniforms, the same cards), and on the live seats of a fresh deal's decision list the
    rollout-logit kernel equals its factored arithmetic and the module's
    forward (_check_mlp_kernels)"""
    from rl_6_nimmt import _native as nat
    from rl_6_nimmt.agents import DrunkHamster, PUCTAgent
    from rl_6_nimmt.league import BatchedTournament

    def league():
        torch.manual_seed(0)
        t = BatchedTournament(192, 2, 4, seed=13)
        for name, a in [("P", PUCTAgent(mc_max=12, mc_per_card=3)), ("R0", DrunkHamster()), ("R1", DrunkHamster()),
                        ("R2", DrunkHamster())]:
            t.add_player(name, a)
        return t

    recs = {}
    # whole rollouts in one kernel (sn_puct_rollouts), the seat-lane step and the one-lane step
    for form, rollouts, lanes in (("fused", "1", "1"), ("seats", "0", "1"), ("lane", "0", "0")):
        monkeypatch.setenv("SECHS_PUCT_ROLLOUTS", rollouts)
        monkeypatch.setenv("SECHS_PUCT_STEP_SEATS", lanes)
        t = league()
        recs[form] = t.play_games(2).cpu()
        assert t.mode == "step"
        t.close()
    assert torch.equal(recs["fused"], recs["lane"]) and torch.equal(recs["seats"], recs["lane"])
    k = recs["lane"][..., 0] & 15
    assert int(k.min()) == 2 and int(k.max()) == 4  # absent seats on the lists
    monkeypatch.delenv("SECHS_PUCT_STEP_SEATS")
    monkeypatch.delenv("SECHS_PUCT_ROLLOUTS")
    t = league()
    t.play_games(1)
    env = t.env
    nat.check(nat.lib().sn_reset(env._h, None, env._stream()), "sn_reset")  # a fresh seat draw + deal
    t._use_decisions()
    eng = t.engines["P"]
    kk, _ = t.seats()
    N = env.num_players
    g = eng.dec.long() // N
    live = (torch.arange(N, device=env.device)[None, :] < kk.to(env.device).long()[g][:, None]).reshape(-1)
    assert eng.D > 0 and not bool(live.all())
    _check_mlp_kernels(env, eng, 10, live=live)
    t.close()


def test_batched_deal_equals_per_rollout_deals(monkeypatch):
    """sn_puct_deal_batch (rollouts dealt 16 / 3 per launch, each rollout
    running on its slice of the batch buffer) and one sn_puct_deal per
    rollout deal the same states from the same Philox streams: a whole PUCT
    search gives identical statistics, histograms and moves"""
    res = {}
    for rb in ("16", "0", "3"):
        monkeypatch.setenv("SECHS_PUCT_DEAL_BATCH", rb)
        env, eng = _engine(B=300, dtype=torch.bfloat16, mc_max=12, mc_per_card=3, seed=17)
        assert eng.deal_batch == int(rb)
        acts = [eng.decide(10).clone()]
        env.step(acts[-1])
        acts.append(eng.decide(9).clone())
        torch.cuda.synchronize()
        res[rb] = (acts, eng.stats.clone(), eng.hist.clone())
    for rb in ("16", "3"):
        assert all(torch.equal(a, b) for a, b in zip(res[rb][0], res["0"][0])), rb
        assert torch.equal(res[rb][1], res["0"][1]) and torch.equal(res[rb][2], res["0"][2]), rb


def test_fused_rollouts_equal_step_launches(monkeypatch):
    """sn_puct_rollouts (whole rollouts per decision group in one kernel,
    logits in LDS) and the launch-per-step loop (sn_puct_mlp_seats +
    sn_puct_step) compute the same logits and draw the same uniforms: a
    whole PUCT search gives identical statistics, histograms and moves --
    4 players (one 16-decision group per 64 seats) and 3 players (48 live
    seat rows per group), a ragged last group"""
    for N, B in [(4, 300), (3, 97)]:
        res = {}
        for rollouts in ("1", "0"):
            monkeypatch.setenv("SECHS_PUCT_ROLLOUTS", rollouts)
            env, eng = _engine(B=B, N=N, dtype=torch.bfloat16, mc_max=12, mc_per_card=3, seed=23)
            assert eng.fused_rollouts == (rollouts == "1")
            acts = [eng.decide(10).clone()]
            env.step(acts[-1])
            acts.append(eng.decide(9).clone())
            torch.cuda.synchronize()
            res[rollouts] = (acts, eng.stats.clone(), eng.hist.clone(), eng.rows_evaluated)
        assert all(torch.equal(a, b) for a, b in zip(res["1"][0], res["0"][0])), N
        assert torch.equal(res["1"][1], res["0"][1]) and torch.equal(res["1"][2], res["0"][2]), N
        assert res["1"][3] == res["0"][3]


def _bf16_forward_bound(x, layers, head_w, head_b, u=2.0 ** -8, l1_roundings=2):
    """first-order bound on |logit(bf16 path) - logit(f64 reference)| for an
    MLP Linear-ReLU-...-Linear evaluated with every input, weight, bias and
    hidden activation rounded to bf16 (unit roundoff u = 2^-8) and f32
    accumulation: e_in = u|x|; per layer |dz| <= |W| e_in + u (|W||x| + |b|)
    + 2u|z| (the product rounded to bf16 once as the seat base and once
    after the card column + ReLU: sn_puct_mlp_seats' two roundings of layer 1,
    one for layer 2); ReLU is 1-Lipschitz; the head adds |w| e + u (|w||h| +
    |b|).  Returns (reference logits, bound), both float64."""
    h, e = x, u * x.abs()
    for i, (w, b) in enumerate(layers):
        z = h @ w.T + b
        e = e @ w.abs().T + u * (h.abs() @ w.abs().T + b.abs()) + (l1_roundings if i == 0 else 1) * u * z.abs()
        h = torch.relu(z)
    logit = h @ head_w + head_b
    e = e @ head_w.abs() + u * (h.abs() @ head_w.abs() + head_b.abs())
    return logit, e


@pytest.mark.parametrize("n", [10, 6, 3])
def test_mlp_seats_kernel_matches_fp32_reference_net(n):
    """VERDICT r04 #2a: sn_puct_mlp_seats -- the MFMA kernel behind every
    rollout logit of config 4 -- on the reference-recorded F8 weights
    (torch.manual_seed(0); PUCTAgent(), utils/nets.py:100-132), at every
    n_cur of rollouts from positions with n cards left, against the f64
    reference forward of the SAME normalised rows (sn_puct_rows in f32 --
    exact vs SechsNimmtStateNormalization, test_root_rows_are_normalised_
    observations): every logit within the derived first-order bf16 bound
    (x 1.25 for the second-order terms), and every candidate's softmax
    probability (mcts.py:219-228) within p * (exp(2 * 1.25 * max bound) - 1).
    (Layer 1 is factored per seat: two bf16 roundings.)"""
    import ctypes

    from rl_6_nimmt import _native as nat

    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    weights = {k: torch.from_numpy(z[k]) for k in z.files if "net" in k}
    env, eng = _engine(B=512, dtype=torch.bfloat16, mc_max=4, mc_per_card=2, seed=31, weights=weights)
    N = env.num_players
    for t in range(10 - n):
        env.step(eng.decide(10 - t))
    net = eng.sync_net()
    w1c, w2p, head, w1s = net.fused()
    q = eng._params(n)
    L, h, st = nat.lib(), env._h, env._stream()
    eng.memorize()
    nat.check(L.sn_puct_deal(h, ctypes.byref(q), st), "deal")
    layers = [(weights["latent_net.0.weight"].double(), weights["latent_net.0.bias"].double()),
              (weights["latent_net.2.weight"].double(), weights["latent_net.2.bias"].double())]
    hw, hb = weights["head_nets.0.0.weight"][0].double(), weights["head_nets.0.0.bias"][0].double()
    worst_dp = 0.0
    for m in range(n, 0, -1):
        R = eng.D * N * m
        rows = torch.empty((R, 48), dtype=torch.float32, device=env.device)
        nat.check(L.sn_puct_rows(h, ctypes.byref(q), m, nat.ptr(rows), 0, st), "rows f32")
        for kern in ("seats",):  # the factored kernel (two layer-1 roundings)
            lg = torch.full((R,), float("nan"), dtype=torch.float32, device=env.device)
            nat.check(L.sn_puct_mlp_seats(h, ctypes.byref(q), m, nat.ptr(w1s), nat.ptr(w1c), nat.ptr(w2p),
                                          nat.ptr(head), nat.ptr(lg), st), "mlp_seats")
            torch.cuda.synchronize()
            ref, bound = _bf16_forward_bound(rows.double().cpu(), layers, hw, hb, l1_roundings=2)
            got = lg.double().cpu()
            assert not torch.isnan(got).any()
            err = (got - ref).abs()
            assert (err <= 1.25 * bound + 1e-6).all(), (kern, m, float((err / bound).max()))
            p, pr = torch.softmax(got.view(-1, m), dim=1), torch.softmax(ref.view(-1, m), dim=1)
            lim = pr * (torch.exp(2 * 1.25 * bound.view(-1, m).max(dim=1, keepdim=True).values) - 1) + 1e-7
            assert ((p - pr).abs() <= lim).all(), (kern, m)
            worst_dp = max(worst_dp, float((p - pr).abs().max()))
    assert worst_dp < 0.02, worst_dp  # the derived bound is loose; the kernel is far inside it


def test_puct_search_statistics_match_reference_in_law():
    """VERDICT r04 #2b, golden F14 (tools/gen_puct_stats.py): G seeded
    reference games of GameSession(PUCTAgent(mc_max=20) with the F8 weights,
    DrunkHamster x 3) -- the batched engine replays the SAME initial deals
    (seat 0 searching with the same weights in bf16, seats 1-3 uniform legal
    moves) and must agree in law, game-paired, within 4 standard errors of
    the paired difference: seat 0's final penalty, and at its first decision
    the PUCT visit distribution (visit-weighted mean hand rank, largest
    visit share) and the chosen card's hand rank (mcts.py:191-323)."""
    d = load("puct_search.json")
    games = d["games"]
    G = len(games)
    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    weights = {k: torch.from_numpy(z[k]) for k in z.files if "net" in k}
    env, eng = _engine(B=G, N=4, mask=1, dtype=torch.bfloat16, mc_max=d["mc_max"], mc_per_card=d["mc_per_card"],
                       seed=2024, weights=weights)
    board = np.full((G, 4, 6), -1, dtype=np.int8)
    hands = np.full((G, 4, 10), -1, dtype=np.int8)
    for g, r in enumerate(games):
        for i, row in enumerate(r["board0"]):
            board[g, i, : len(row)] = row
        hands[g] = np.array(r["hands0"], dtype=np.int8)
    env.reset_to(torch.from_numpy(board), torch.from_numpy(hands))
    total = torch.zeros((G, 4), dtype=torch.int32, device=env.device)
    torch.manual_seed(7)
    for t in range(10):
        acts = eng.decide(10 - t)
        if t == 0:
            visits = eng.stats[:G, 10:20].cpu().numpy().astype(np.float64)
            chosen = acts[:, 0].cpu().numpy()
        acts = torch.where(torch.tensor([True, False, False, False], device=env.device)[None, :], acts,
                           eng._random_moves())
        rew, done, inv = env.step(acts)
        assert (inv.cpu() == -1).all()
        total += rew
    assert bool(done.all())
    ours = {"penalty": -total[:, 0].cpu().numpy().astype(np.float64)}
    ref = {"penalty": np.array([-r["results"][0] for r in games], dtype=np.float64)}
    rv = np.array([r["visits"] for r in games], dtype=np.float64)
    k = np.arange(10, dtype=np.float64)
    assert np.array_equal(visits.sum(axis=1), rv.sum(axis=1))  # 20 playouts per first decision, all backed up
    ours["visit_rank"] = (visits * k).sum(axis=1) / visits.sum(axis=1)
    ref["visit_rank"] = (rv * k).sum(axis=1) / rv.sum(axis=1)
    ours["max_share"] = visits.max(axis=1) / visits.sum(axis=1)
    ref["max_share"] = rv.max(axis=1) / rv.sum(axis=1)
    ours["chosen_rank"] = np.array([list(r["hands0"][0]).index(int(c)) for r, c in zip(games, chosen)], dtype=np.float64)
    ref["chosen_rank"] = np.array([r["legal"].index(r["chosen"]) for r in games], dtype=np.float64)
    report = {}
    for name in ours:
        diff = ours[name] - ref[name]
        se = diff.std(ddof=1) / np.sqrt(G)
        report[name] = (float(ours[name].mean()), float(ref[name].mean()), float(se))
        assert abs(diff.mean()) <= 4 * se, (name, report[name])
    print("F14 (ours, reference, paired s.e.):", report)


def test_puct_search_at_configured_budget_matches_reference_in_law():
    """VERDICT r05 #5, golden F14b (tools/gen_puct_stats.py with
    SECHS_F14_MC_MAX=100): G seeded reference games of GameSession(PUCTAgent
    (mc_max=100 -- the reference's default budget, mcts.py:25 -- with the F8
    weights), DrunkHamster x 3), seat 0's decisions at n = 10, 6 and 3 (the
    min/max/median normalisation and the unvisited-median fill of
    mcts.py:295-315 drive these searches; n = 3 runs 60 playouts).  The
    batched engine replays the same deals and must agree in law, game-paired,
    within 4 standard errors of the paired difference: seat 0's final
    penalty, and at each n the visit-weighted mean hand rank, the largest
    visit share and the chosen card's rank."""
    d = load("puct_search_mc100.json")
    games = d["games"]
    G = len(games)
    assert d["mc_max"] == 100
    z = np.load(os.path.join(GOLDEN, "puct_policy.npz"))
    weights = {k: torch.from_numpy(z[k]) for k in z.files if "net" in k}
    env, eng = _engine(B=G, N=4, mask=1, dtype=torch.bfloat16, mc_max=d["mc_max"], mc_per_card=d["mc_per_card"],
                       seed=2025, weights=weights)
    board = np.full((G, 4, 6), -1, dtype=np.int8)
    hands = np.full((G, 4, 10), -1, dtype=np.int8)
    for g, r in enumerate(games):
        for i, row in enumerate(r["board0"]):
            board[g, i, : len(row)] = row
        hands[g] = np.array(r["hands0"], dtype=np.int8)
    env.reset_to(torch.from_numpy(board), torch.from_numpy(hands))
    total = torch.zeros((G, 4), dtype=torch.int32, device=env.device)
    torch.manual_seed(8)
    ours_dec = {}
    for t in range(10):
        n = 10 - t
        acts = eng.decide(n)
        if str(n) in games[0]["dec"]:
            ours_dec[n] = (eng.stats[:G, 10:10 + n].cpu().numpy().astype(np.float64),
                           eng.best_index[:G].cpu().numpy().astype(np.float64))
        acts = torch.where(torch.tensor([True, False, False, False], device=env.device)[None, :], acts,
                           eng._random_moves())
        rew, done, inv = env.step(acts)
        assert (inv.cpu() == -1).all()
        total += rew
    assert bool(done.all())
    report = {}

    def check(name, ours, ref):
        diff = ours - ref
        se = diff.std(ddof=1) / np.sqrt(len(diff))
        report[name] = (round(float(ours.mean()), 4), round(float(ref.mean()), 4), round(float(se), 4))
        assert abs(diff.mean()) <= 4 * se, (name, report[name])

    check("penalty", -total[:, 0].cpu().numpy().astype(np.float64),
          np.array([-r["results"][0] for r in games], dtype=np.float64))
    for n, (visits, best) in ours_dec.items():
        rv = np.array([r["dec"][str(n)]["visits"] for r in games], dtype=np.float64)
        assert np.array_equal(visits.sum(axis=1), rv.sum(axis=1))  # n_mc playouts per decision, all backed up
        k = np.arange(n, dtype=np.float64)
        check(f"visit_rank@{n}", (visits * k).sum(axis=1) / visits.sum(axis=1), (rv * k).sum(axis=1) / rv.sum(axis=1))
        check(f"max_share@{n}", visits.max(axis=1) / visits.sum(axis=1), rv.max(axis=1) / rv.sum(axis=1))
        check(f"chosen_rank@{n}", best,
              np.array([r["dec"][str(n)]["legal"].index(r["dec"][str(n)]["chosen"]) for r in games], dtype=np.float64))
    print("F14b (ours, reference, paired s.e.):", report)
