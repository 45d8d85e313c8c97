"""GPU checks of the ACER agent (agents/actor_critic.py:16-207), golden F12.

* drop-in BatchedACERAgent in seeded training GameSessions (GPU env, host
  net like the reference's): every move, log-prob, value, update loss and the
  final weights equal the reference's recordings;
* batched engine (sn_puct_root_rows -> 2-head MLP -> sn_policy_sample, device
  replay): the recorded behaviour log pi == the host formula on the same rows
  (fp32 net, 1e-5), the loss on the device replay == the reference's update
  arithmetic summed over deciders, and learn() runs the reference's update
  schedule.  Samples are Philox (parity unpinned bitwise; the sampler's
  frequency test is test_batched_reinforce_samples_follow_the_policy).
"""
import json
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_dropin_acer_agent_replays_reference_training_sessions():
    from rl_6_nimmt import GameSession
    from rl_6_nimmt.agents import AGENTS, BatchedACERAgent, DrunkHamster

    assert AGENTS["acer"] is BatchedACERAgent
    spec = json.load(open(os.path.join(GOLDEN, "acer_games.json")))
    W = np.load(os.path.join(GOLDEN, "acer_weights.npz"))
    for si, sess in enumerate(spec["sessions"]):
        torch.manual_seed(sess["seed"])
        agents = [BatchedACERAgent(**sess["kwargs"]) if c == "A" else DrunkHamster() for c in sess["seats"]]
        rec = {}
        for i, c in enumerate(sess["seats"]):
            if c != "A":
                continue
            a = agents[i]
            a.train()
            rec[i] = []
            fwd = a.forward

            def fwd_rec(state, legal_actions, *x, _f=fwd, _i=i, **k):
                act, info = _f(state, legal_actions, *x, **k)
                rec[_i].append([int(act), float(info["log_prob"]), float(info["value"])])
                return act, info

            a.forward = fwd_rec
        np.random.seed(sess["seed"])
        random.seed(sess["seed"])
        s = GameSession(*agents)
        for _ in range(sess["games"]):
            s.play_game()
        assert [[int(x) for x in r] for r in s.results] == sess["results"], si
        for i in rec:
            tr = sess["trace"][str(i)]
            got = np.array(rec[i])
            want = np.array([[st["action"], st["log_prob"], st["value"]] for st in tr["steps"]])
            assert np.array_equal(got[:, 0], want[:, 0]), (si, i)
            # host fp32 math on another CPU: floats to 1e-3 (Adam amplifies rounding), moves identical
            assert np.allclose(got[:, 1:], want[:, 1:], rtol=0, atol=1e-3), (si, i)
            assert len(agents[i].last_losses) == len(tr["losses"]), (si, i)
            assert np.allclose(agents[i].last_losses, [w[2:] for w in tr["losses"]], rtol=1e-3, atol=1e-4), (si, i)
            for k, v in agents[i].actor_critic.state_dict().items():
                d = np.abs(v.detach().numpy() - W[f"s{si}_a{i}_final_{k}"])
                if k == "head_nets.0.0.bias":
                    # the policy-logit bias shifts every candidate equally: softmax ignores it, its exact
                    # gradient is 0 and Adam scales the host CPU's rounding noise up to ~lr per step
                    assert d.max() <= 3e-3 * sess["games"], (si, i)
                    continue
                assert np.mean(d <= 1e-4) >= 0.5 and d.max() <= 3e-3 * sess["games"], (si, i, k, d.max())


def _engine(B=32, N=4, mask=None, dtype=torch.float32, seed=5, **kw):
    from rl_6_nimmt.acer import BatchedACER, make_actor_critic
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(B, N, seed=seed, rng="philox")
    torch.manual_seed(0)
    return env, BatchedACER(env, make_actor_critic().to(env.device), seats_mask=mask, net_dtype=dtype, seed=seed, **kw)


@pytest.mark.parametrize("mask", [None, 0b0101])
def test_batched_acer_records_behaviour_policy(mask):
    env, eng = _engine(mask=mask, capacity=2)
    env.reset()
    N = env.num_players
    seats = [p for p in range(N) if mask is None or (mask >> p) & 1]
    for t in range(10):
        n = 10 - t
        hands = env.hands().long()
        acts = eng.decide(n, record=True)
        idx = eng.best_index.long()
        assert ((idx >= 0) & (idx < n)).all()
        want_cards = hands[:, seats, :].reshape(-1, 10).gather(1, idx[:, None])[:, 0]
        assert torch.equal(acts[:, seats].reshape(-1).long(), want_cards)
        rows = eng.rep_rows[0, t, :, :n]
        with torch.no_grad():
            logit, _ = eng.actor(rows.reshape(-1, 48))
        want = torch.log_softmax(logit.reshape(-1, n), dim=1)
        assert torch.allclose(eng.rep_logp[0, t, :, :n], want, atol=1e-5)
        assert (eng.rep_logp[0, t, :, n:] == -20.0).all()
        assert torch.allclose(eng.log_prob, want.gather(1, idx[:, None])[:, 0], atol=1e-5)
        if len(seats) < N:
            keep = torch.tensor([p in seats for p in range(N)], device=env.device)
            acts = torch.where(keep[None, :], acts, eng._random_moves())
        rew, done, inv = env.step(acts)
        assert (inv == -1).all()


def test_batched_acer_loss_on_device_replay_equals_reference_arithmetic():
    from test_acer_cpu import _reference_loss

    env, eng = _engine(B=8, mask=0b0011, rollout_len=4, truncate=0.5, gamma=0.95, capacity=2, minibatch=3)
    for _ in range(3):
        eng.play_episode(record=True)
    for batch in (eng.on_policy_batch(2), eng.off_policy_batch(1)):
        total, actor, corr, critic = eng.loss(*batch)
        want = _reference_loss(eng, *batch)
        got = np.array([float(actor), float(corr), float(critic)])
        assert np.allclose(got, want, rtol=1e-4, atol=1e-5), (got, want)


def test_batched_acer_learn_schedule_and_update():
    env, eng = _engine(B=64, dtype=torch.bfloat16, warmup=2, minibatch=2, capacity=3)
    opt = torch.optim.Adam(eng.actor.parameters())
    before = [p.detach().clone() for p in eng.actor.parameters()]
    counts = []
    for _ in range(4):
        total, _ = eng.play_episode(record=True)
        assert (total <= 0).all()
        counts.append(len(eng.learn(opt)))
    # one sequence per episode (rollout_len 10): updates once more than 2 are stored
    assert counts == [0, 0, 2, 2]
    assert all(np.isfinite(x).all() for x in eng.last_losses)
    assert any(not torch.equal(a, b) for a, b in zip(eng.actor.parameters(), before))
