"""ACER drop-in agent (agents/actor_critic.py:16-207) against golden F12 on the
host: the recorded sessions' observations are fed straight to the agents (no
env), in GameSession's order (every seat's forward, then every seat's learn:
play.py:38-67), with torch / Python `random` seeded as the generator did.
Moves, log-probs, values, every update's losses and the final weights must
equal the reference's.  The same sessions through the GPU env are in
tests/test_gpu_acer.py; the batched engine's losses are checked against
`acer_losses` there too."""
import json
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def _sessions():
    return json.load(open(os.path.join(GOLDEN, "acer_games.json")))["sessions"]


def _weights():
    return np.load(os.path.join(GOLDEN, "acer_weights.npz"))


def _build(sess, W, si):
    from rl_6_nimmt.agents import BatchedACERAgent

    torch.manual_seed(sess["seed"])
    agents = {}
    for i, c in enumerate(sess["seats"]):
        if c == "A":
            a = BatchedACERAgent(**sess["kwargs"])
            a.train()
            for k, v in a.actor_critic.state_dict().items():
                assert torch.equal(v, torch.from_numpy(W[f"s{si}_a{i}_init_{k}"])), (si, i, k)
            agents[i] = a
    return agents


def _check_weights(agent, W, si, i, games):
    for k, v in agent.actor_critic.state_dict().items():
        got, want = v.detach().numpy(), W[f"s{si}_a{i}_final_{k}"]
        d = np.abs(got - want)
        if k == "head_nets.0.0.bias":  # softmax-invariant: exact gradient 0, Adam scales rounding noise to ~lr
            assert d.max() <= 3e-3 * games, (si, i)
            continue
        # bit-identical on the fixture host; a different CPU rounds the GEMMs
        # differently and Adam amplifies near-cancelling gradients to O(lr)
        assert np.mean(d <= 1e-4) >= 0.5 and d.max() <= 3e-3 * games, (si, i, k, d.max())


@pytest.mark.parametrize("si", range(4))
def test_acer_agent_replays_reference_sessions(si):
    sess, W = _sessions()[si], _weights()
    agents = _build(sess, W, si)
    steps = {i: sess["trace"][str(i)]["steps"] for i in agents}
    losses = {i: [] for i in agents}
    for i, a in agents.items():
        trn = a._train

        def rec(on_policy=True, _t=trn, _i=i):
            out = _t(on_policy)
            losses[_i].append([len(infos[_i]), bool(on_policy)] + list(out))
            return out

        a._train = rec
    infos = {i: [] for i in agents}
    random.seed(sess["seed"])
    T = len(next(iter(steps.values())))
    for j in range(T):
        for i, a in agents.items():
            st = steps[i][j]
            act, info = a(torch.tensor(st["obs"], dtype=torch.float32), legal_actions=list(st["legal"]))
            assert int(act) == st["action"], (si, i, j)
            assert abs(float(info["log_prob"]) - st["log_prob"]) <= 1e-5, (si, i, j)
            assert abs(float(info["value"]) - st["value"]) <= 1e-5, (si, i, j)
            infos[i].append(info)
        for i, a in agents.items():
            st = steps[i][j]
            a.learn(state=torch.tensor(st["obs"], dtype=torch.float32), legal_actions=list(st["legal"]), reward=0,
                    action=st["action"], done=st["done"], next_state=None, next_legal_actions=[],
                    next_reward=np.int32(st["next_reward"]), num_episode=0, episode_end=st["done"], **infos[i][-1])
    for i, a in agents.items():
        want = sess["trace"][str(i)]["losses"]
        got = losses[i]
        assert [g[:2] for g in got] == [w[:2] for w in want], (si, i)
        assert np.allclose([g[2:] for g in got], [w[2:] for w in want], rtol=1e-4, atol=1e-6), (si, i)
        _check_weights(a, W, si, i, sess["games"])


def test_sequential_history_ring_semantics():
    """replay_buffer.py:206-302: len counts the pointer except right after a
    wrap, rollout(n) reads slots [len-n, len), sample uses random.sample"""
    from rl_6_nimmt.utils.history import SequentialHistory

    h = SequentialHistory(max_length=3)
    for s in range(5):
        for t in range(2):
            h.store(x=10 * s + t)
        h.flush()
        assert len(h) == [1, 2, 3, 1, 2][s]
    assert h.rollout(n=1)["x"] == [[40, 41]]  # slot len-1 is always the newest sequence
    assert h.rollout()["first"] == [[True, False], [True, False]]
    h.store(x=50)
    h.flush()
    assert len(h) == 3 and h.rollout(n=1)["x"] == [[50]]
    h.store(x=60)
    h.flush()
    # after a wrap only slots [0, pointer) count: the off-policy sample never
    # sees the older sequences still held in the other slots
    assert len(h) == 1 and h.rollout()["x"] == [[60]]
    h.store(x=70)
    h.flush()
    random.seed(1)
    idx, _, mb = h.sample(2)
    random.seed(1)
    assert idx == random.sample(range(2), k=2)
    assert mb["x"] == [h._slots[k]["x"] for k in idx]


def test_retrace_targets_by_hand():
    """actor_critic.py:195-207 on two sequences, written out"""
    from rl_6_nimmt.agents.actor_critic import retrace_targets

    r = np.array([0.1, -0.2, 0.3, -0.4])
    done = np.array([False, False, False, True])
    first = np.array([True, False, True, False])
    q_a = torch.tensor([[1.0], [2.0], [3.0], [4.0]])
    rho = torch.tensor([[0.5], [1.0], [0.25], [1.0]])
    v = torch.tensor([[0.5], [1.5], [2.5], [3.5]])
    g = 0.9
    got = retrace_targets(r, done, first, q_a, rho, v, g)[:, 0].tolist()
    t3 = -0.4 + g * 0.0
    t2 = 0.3 + g * (1.0 * (t3 - 4.0) + 3.5)
    t1 = -0.2 + g * (1.5 * 1.0)          # restarts from v[1] (row 2 begins a sequence)
    t0 = 0.1 + g * (1.0 * (t1 - 2.0) + 1.5)
    assert np.allclose(got, [t0, t1, t2, t3], atol=1e-6)


class _HostEnv:
    """shape-only stand-in for VecSechsNimmtEnv: BatchedACER's replay and
    loss need no device kernels"""

    def __init__(self, B, N):
        self.num_games, self.num_players, self.device = B, N, torch.device("cpu")


def _fill_replay(eng, episodes, rng):
    D = eng.D
    for e in range(episodes):
        s = e % eng.capacity
        for t in range(10):
            n = 10 - t
            eng.rep_rows[s, t, :, :n] = torch.from_numpy(rng.normal(size=(D, n, 48)).astype(np.float32))
            eng.rep_act[s, t] = torch.from_numpy(rng.integers(0, n, size=D))
            lg = torch.from_numpy(rng.normal(size=(D, n)).astype(np.float32))
            eng.rep_logp[s, t].fill_(-20.0)
            eng.rep_logp[s, t, :, :n] = torch.log_softmax(lg, dim=1)
        eng.rep_rew[s] = torch.from_numpy((rng.integers(-7, 1, size=(10, D)) * eng.r_factor).astype(np.float32))
        eng.episodes += 1


def _reference_loss(eng, slots, chunk_ids):
    """sum over deciders of acer_losses (the drop-in's, = the reference's
    arithmetic) on each decider's concatenated sequences"""
    from rl_6_nimmt.agents.actor_critic import acer_losses

    tot = np.zeros(3)
    chunks = eng.chunks()
    for d in range(eng.D):
        lps, qs, then, acts, rews, done, first = [], [], [], [], [], [], []
        for s, c in zip(slots[d].tolist(), chunk_ids[d].tolist()):
            a, b = chunks[c]
            for t in range(a, b):
                n = 10 - t
                logit, q = eng.actor(eng.rep_rows[s, t, d, :n])
                logit, q = logit.cpu(), q.cpu()
                lp = torch.log(torch.softmax(logit, dim=0).flatten())
                lps.append(torch.nn.functional.pad(lp, (0, 10 - n), value=-20.0))
                qs.append(torch.nn.functional.pad(q.flatten(), (0, 10 - n), value=0.0))
                then.append(eng.rep_logp[s, t, d].cpu())
                acts.append(int(eng.rep_act[s, t, d]))
                rews.append(float(eng.rep_rew[s, t, d]))
                done.append(t == 9)
                first.append(t == a)
        out = acer_losses(torch.stack(lps), torch.stack(qs), torch.stack(then), torch.tensor(acts)[:, None],
                          np.array(rews), np.array(done), np.array(first), eng.gamma, eng.truncate, eng.critic_weight)
        tot += [float(x) for x in out]
    return tot


@pytest.mark.parametrize("rollout_len,truncate", [(10, 1.0), (4, 0.5), (3, 1.0)])
def test_batched_acer_loss_equals_reference_arithmetic(rollout_len, truncate):
    """BatchedACER.loss (vectorised over deciders and sequences, masked
    ragged chunks) == the reference's per-agent update losses summed"""
    from rl_6_nimmt.acer import BatchedACER

    torch.manual_seed(0)
    eng = BatchedACER(_HostEnv(3, 2), net_dtype=torch.float32, rollout_len=rollout_len, truncate=truncate,
                      capacity=2, r_factor=0.1, gamma=0.95, critic_weight=0.7, minibatch=3)
    rng = np.random.default_rng(rollout_len)
    _fill_replay(eng, 3, rng)
    # on-policy (newest sequence of every decider) and off-policy batches
    for batch in (eng.on_policy_batch(len(eng.chunks()) - 1), eng.off_policy_batch(len(eng.chunks()) - 2)):
        total, actor, corr, critic = eng.loss(*batch)
        want = _reference_loss(eng, *batch)
        got = np.array([float(actor), float(corr), float(critic)])
        assert np.allclose(got, want, rtol=1e-4, atol=1e-5), (got, want)
        assert abs(float(total) - want.sum()) <= 1e-4 * max(1.0, abs(want.sum()))
    # the gradient flows into both heads
    total.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in eng.actor.parameters())


def test_batched_acer_replay_bookkeeping():
    from rl_6_nimmt.acer import BatchedACER

    eng = BatchedACER(_HostEnv(2, 2), net_dtype=torch.float32, rollout_len=4, capacity=2, minibatch=2)
    assert eng.chunks() == [(0, 4), (4, 8), (8, 10)]
    _fill_replay(eng, 1, np.random.default_rng(0))
    assert eng.stored_sequences(0) == [(0, 0)]
    _fill_replay(eng, 2, np.random.default_rng(1))  # 3 episodes in 2 slots: slot 1 then 0 hold the newest
    assert eng.stored_sequences() == [(1, 0), (1, 1), (1, 2), (0, 0), (0, 1), (0, 2)]
    assert eng.stored_sequences(1) == [(1, 0), (1, 1), (1, 2), (0, 0), (0, 1)]
    s, c = eng.off_policy_batch(1)
    assert s.shape == (eng.D, 2)
    for d in range(eng.D):
        pairs = list(zip(s[d].tolist(), c[d].tolist()))
        assert len(set(pairs)) == 2 and all(p in eng.stored_sequences(1) for p in pairs)


def test_batched_acer_default_capacity_reaches_warmup():
    """with the reference's defaults (rollout_len 10, warmup 100,
    minibatch 5) the device replay must hold more than max(warmup, minibatch)
    sequences per decider, or learn() never updates (the reference's
    SequentialHistory is unbounded)"""
    from rl_6_nimmt.acer import BatchedACER, default_capacity

    for rl, mb, wu in ((10, 5, 100), (10, 10, 100), (4, 5, 100), (3, 2, 7), (10, 200, 50)):
        cap = default_capacity(rl, mb, wu)
        assert cap * (-(-10 // rl)) > max(wu, mb), (rl, mb, wu, cap)
    eng = BatchedACER(_HostEnv(2, 2), net_dtype=torch.float32)
    assert eng.capacity * len(eng.chunks()) > max(eng.warmup, eng.minibatch)
    # fill past the warmup: the schedule now asks for updates
    _fill_replay(eng, eng.capacity, np.random.default_rng(3))
    assert len(eng.stored_sequences(0)) > max(eng.warmup, eng.minibatch)
    before = [p.detach().clone() for p in eng.actor.parameters()]
    updates = eng.learn(torch.optim.Adam(eng.actor.parameters()))
    assert len(updates) == 2  # one on-policy + one off-policy step, actor_critic.py:146-151
    assert any(not torch.equal(a, b) for a, b in zip(eng.actor.parameters(), before))
    with pytest.warns(UserWarning):
        BatchedACER(_HostEnv(2, 2), net_dtype=torch.float32, capacity=4)


def test_replay_size_is_checked_before_allocating():
    """a replay is capacity x 10 x deciders x 19.7 KB; a size above
    the limit raises a clear error instead of failing in the allocator"""
    from rl_6_nimmt.acer import BatchedACER, replay_bytes

    assert replay_bytes(102, 8192 * 4) > 60 << 30  # the old INTEGRATION example: ~66 GB
    with pytest.raises(ValueError, match="capacity"):
        BatchedACER(_HostEnv(2, 2), net_dtype=torch.float32, capacity=10, max_replay_bytes=replay_bytes(10, 4) - 1)
    BatchedACER(_HostEnv(2, 2), net_dtype=torch.float32, capacity=10, max_replay_bytes=replay_bytes(10, 4))


def test_distinct_off_policy_picks():
    """the tournament ACER's off-policy batch draws distinct sequences per
    seat (random.sample in the reference), uniformly"""
    from rl_6_nimmt.acer import distinct_picks

    g = torch.Generator().manual_seed(0)
    for S, k in ((5, 5), (12, 5), (1000, 10)):
        p = distinct_picks(S, 4000, k, g, torch.device("cpu"))
        assert p.shape == (4000, k) and int(p.min()) >= 0 and int(p.max()) < S
        srt = p.sort(dim=1).values
        assert not (srt[:, 1:] == srt[:, :-1]).any()
        counts = torch.bincount(p.reshape(-1), minlength=S).double()
        exp = 4000 * k / S
        assert float(((counts - exp).abs() / exp ** 0.5).max()) < 5.0
    with pytest.raises(ValueError):
        distinct_picks(3, 2, 4, g, torch.device("cpu"))


def test_decider_chunked_update_equals_one_batch():
    """learn() accumulates the gradient of the decider-summed loss over
    decider chunks (bounded activation memory) before its one Adam step:
    the same update as one batch over every decider"""
    import copy

    from rl_6_nimmt.acer import BatchedACER

    torch.manual_seed(0)
    eng = BatchedACER(_HostEnv(5, 2), net_dtype=torch.float32, rollout_len=10, capacity=3, minibatch=2, warmup=2)
    _fill_replay(eng, 3, np.random.default_rng(7))
    eng2 = copy.deepcopy(eng)
    eng.decider_chunk, eng2.decider_chunk = 3, 10 ** 6
    eng._gen.manual_seed(11)
    eng2._gen.manual_seed(11)  # the same off-policy picks
    o1, o2 = torch.optim.SGD(eng.actor.parameters(), lr=0.1), torch.optim.SGD(eng2.actor.parameters(), lr=0.1)
    u1, u2 = eng.learn(o1), eng2.learn(o2)
    assert len(u1) == len(u2) == 2
    assert np.allclose(np.array(u1), np.array(u2), rtol=1e-5, atol=1e-6)
    for a, b in zip(eng.actor.parameters(), eng2.actor.parameters()):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)


def test_splitk_training_forward_equals_module():
    """train_forward (SplitKLinear: the weight gradient as batched partial
    products over row chunks) gives the module's outputs and, to float64
    rounding, its gradients -- over enough rows for the chunked path"""
    import torch

    from rl_6_nimmt.acer import make_actor_critic, train_forward

    torch.manual_seed(0)
    x = torch.randn(300_000, 48, dtype=torch.float64, requires_grad=True)
    net = make_actor_critic().double()
    grads = []
    for fwd in (lambda r: train_forward(net, r), net):
        out = fwd(x)
        loss = (out[0] ** 2).sum() + (3 * out[1]).sum()
        net.zero_grad()
        x.grad = None
        loss.backward()
        grads.append(([p.grad.clone() for p in net.parameters()], x.grad.clone(), [o.detach() for o in out]))
    (g1, x1, o1), (g2, x2, o2) = grads
    assert all(torch.equal(a, b) for a, b in zip(o1, o2))
    assert torch.equal(x1, x2)
    assert all(torch.allclose(a, b, rtol=1e-12, atol=1e-12 * float(b.abs().max())) for a, b in zip(g1, g2))
