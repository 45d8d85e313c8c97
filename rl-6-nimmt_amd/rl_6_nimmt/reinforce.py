"""Batched REINFORCE self-play on one MI355X.

Reference: BatchedReinforceAgent (agents/policy.py:109-201), AGENTS["reinforce"].
Every deciding seat of every game acts together: per decision batch one
sn_puct_root_rows launch (normalised `[card, obs]` candidate rows straight
from the device state), one policy-MLP forward (PyTorch-ROCm), one
sn_policy_sample launch (softmax sample with Philox, log-prob, entropy).

Training from stored rows instead of retained graphs (the reference keeps
every forward's autograd graph until the episode ends): per (game, seat),
    rewards r_t  = the reward GameSession hands learn() at step t -- the
                   PREVIOUS step's (play.py:29,57,72), so r_0 = 0 and the
                   last step's reward never reaches the agent -- times r_factor
    returns G_t  = r_t + gamma G_{t+1}        (utils/various.py:41-50)
    actor_loss   = -sum_t gamma^t G_t log pi(a_t | s_t)   (policy.py:183-185)
    entropy_loss = -sum_t H(pi(. | s_t))
    loss         = actor_weight actor_loss + entropy_weight entropy_loss
summed over games (the reference steps Adam after every game).
"""
import numpy as np
import torch

from . import _native as nat
from .puct import ROW, BatchedPUCT, ctypes_ref, decision_forwards, make_actor


class BatchedReinforce(BatchedPUCT):
    def __init__(self, env, actor=None, seats_mask=None, net_dtype=torch.bfloat16, seed=0, gamma=0.99, r_factor=1.0,
                 actor_weight=1.0, entropy_weight=0.0, max_decisions=None):
        super().__init__(env, actor if actor is not None else make_actor(), seed=seed, seats_mask=seats_mask,
                         puct_root=False, net_dtype=net_dtype, max_decisions=max_decisions)
        self.gamma, self.r_factor = float(gamma), float(r_factor)
        self.actor_weight, self.entropy_weight = float(actor_weight), float(entropy_weight)
        D = self.D_max
        self.log_prob = torch.zeros((D,), dtype=torch.float32, device=env.device)
        self.entropy = torch.zeros((D,), dtype=torch.float32, device=env.device)

    def decide(self, n, memorize=False, record=False):
        """sample every deciding seat's card at hand size n: actions [B, N] int32"""
        L, h, st = nat.lib(), self.env._h, self.env._stream()
        if self.D == 0:  # tournament mode: no seat of this agent in the current games
            self.step_id += 1
            return self.actions
        bf16 = int(self.net_dtype == torch.bfloat16)
        q = self._params(n)
        self.sync_net()
        rows = torch.empty((self.D * n, ROW), dtype=self.net_dtype, device=self.env.device)
        nat.check(L.sn_puct_root_rows(h, ctypes_ref(q), nat.ptr(rows), bf16, st), "sn_puct_root_rows")
        logits = self._logits(rows)
        nat.check(L.sn_policy_sample(h, ctypes_ref(q), nat.ptr(logits), nat.ptr(self.actions), nat.ptr(self.best_index),
                                     nat.ptr(self.log_prob), nat.ptr(self.entropy), st), "sn_policy_sample")
        if record:
            self.decisions.append((self._train_rows(q, n, rows), n, self.best_index[: self.D].clone()))
        self.step_id += 1
        return self.actions

    def play_episode(self, others=None, record=False):
        """one whole game of every env game (non-deciding seats: uniform
        moves); returns (summed rewards [B, N] int32, per-step rewards
        [10, B, N] int32)"""
        env = self.env
        env.reset()
        per_step = torch.zeros((10, env.num_games, env.num_players), dtype=torch.int32, device=env.device)
        for t in range(10):
            acts = self.decide(10 - t, record=record)
            if self.M < env.num_players:
                keep = torch.tensor([(self.seats_mask >> p) & 1 for p in range(env.num_players)], device=env.device,
                                    dtype=torch.bool)
                acts = torch.where(keep[None, :], acts, self._random_moves())
            rew, done, inv = env.step(acts)
            per_step[t] = rew
        self.episode_rewards = per_step
        return per_step.sum(dim=0), per_step

    def returns(self, per_step):
        """discounted returns [D, T] of the rewards learn() would see"""
        if self.dec is not None:  # tournament mode: the decision list's seats
            r = per_step.reshape(per_step.shape[0], -1)[:, self.dec.long()].T.double() * self.r_factor
        else:
            seats = [p for p in range(self.env.num_players) if (self.seats_mask >> p) & 1]
            r = per_step[:, :, seats].reshape(per_step.shape[0], -1).T.double() * self.r_factor  # [D, T]
        seen = torch.zeros_like(r)
        seen[:, 1:] = r[:, :-1]  # learn() at step t gets step t-1's reward
        G = torch.zeros_like(seen)
        acc = torch.zeros_like(seen[:, 0])
        for t in range(seen.shape[1] - 1, -1, -1):
            acc = seen[:, t] + self.gamma * acc
            G[:, t] = acc
        return G.float()

    def loss(self, per_step=None, d0=0, d1=None):
        """policy.py:174-196 summed over the games of deciders [d0, d1) (all by
        default), on the recorded rows"""
        per_step = self.episode_rewards if per_step is None else per_step
        dev = self.actor_device()
        logps, ents = [], []
        for (logits,), n, idx in decision_forwards(self.actor, self.decisions, d0, d1, dev):
            logp = torch.log_softmax(logits.reshape(-1, n), dim=1)
            logps.append(logp.gather(1, idx[:, None])[:, 0])
            ents.append(-(logp.exp() * logp).sum(dim=1))
        logps, ents = torch.stack(logps, dim=1), torch.stack(ents, dim=1)  # [D, T]
        T = logps.shape[1]
        G = self.returns(per_step)[d0:d1, :T].to(dev)
        disc = torch.exp(np.log(self.gamma) * torch.linspace(0, T - 1, T)).to(dev)
        actor_loss = -(disc[None, :] * G * logps).sum()
        entropy_loss = -ents.sum()
        return self.actor_weight * actor_loss + self.entropy_weight * entropy_loss
