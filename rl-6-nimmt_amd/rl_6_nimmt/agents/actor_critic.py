"""ACER agent (reference: rl_6_nimmt/agents/actor_critic.py:16-207,
registered as AGENTS["acer"]).

Drop-in host agent, like the reference's: one MultiHeadedMLP(48, (100, 100),
heads (1, 1)) over the normalised `[card, obs]` candidate rows gives a policy
logit and an action value q(s, a) per legal card (actor_critic.py:43-47,
77-96); the move is sampled from exp(clamp(log pi, -20)) over the 10 padded
slots, re-drawn while it lands on a pad slot (:98-106); every step goes into
a `SequentialHistory` and, once a sequence is flushed (rollout_len steps, or
done) and more than max(warmup, minibatch) sequences are stored, one
on-policy and one off-policy ACER update run (:136-151) with truncated
importance weights, the Retrace target q_ret and the bias-correction term
(:153-207).  `acer_losses` is that update's arithmetic on already evaluated
tensors; the batched engine (rl_6_nimmt/acer.py) is tested against it.

The GPU form for many games at once is `acer.BatchedACER` (candidate rows and
sampling in HIP kernels, the net through PyTorch-ROCm, a device replay).
"""
import logging

import numpy as np
import torch
from torch import nn
from torch.distributions import Categorical

from .base import Agent
from ..utils.history import SequentialHistory
from ..utils.nets import MultiHeadedMLP
from ..utils.preprocessing import SechsNimmtStateNormalization

logger = logging.getLogger(__name__)


def retrace_targets(rewards, done, is_first, q_a, rho_bar, v, gamma):
    """actor_critic.py:195-207 over one concatenation of sequences: walking
    backwards, q_ret <- r_i + gamma q_ret is the target of row i, then
    q_ret <- rho_bar_i (q_ret - q_a_i) + v_i; at the first row of a sequence
    (not row 0) it restarts from the previous row's v (0 after done).
    float32 scalars, like the reference's 1-element tensors."""
    q_ret = v[-1] * (1.0 - done[-1])
    out = []
    for i in range(len(rewards) - 1, -1, -1):
        q_ret = rewards[i] + gamma * q_ret
        out.append(q_ret.item())
        q_ret = rho_bar[i] * (q_ret - q_a[i]) + v[i]
        if is_first[i] and i != 0:
            q_ret = v[i - 1] * (1.0 - done[i - 1])
    out.reverse()
    return torch.tensor(out, dtype=torch.float).unsqueeze(1)


def acer_losses(log_probs_now, q, log_probs_then, action_ids, rewards, done, is_first, gamma, truncate, critic_weight):
    """actor_critic.py:157-177: (actor, correction, critic) losses of one
    concatenated batch of T rows ([T, 10] padded log pi / q, [T, 1] action ids)"""
    q_a = q.gather(1, action_ids)
    log_prob_now_a = log_probs_now.gather(1, action_ids)
    v = (q * torch.exp(log_probs_now)).sum(1).unsqueeze(1).detach()
    rho = torch.exp(log_probs_now - log_probs_then).detach()
    rho_bar = rho.gather(1, action_ids).clamp(max=truncate)
    coeff = (1.0 - truncate / rho).clamp(min=0.0)
    q_ret = retrace_targets(rewards, done, is_first, q_a, rho_bar, v, gamma)
    actor = (-rho_bar * log_prob_now_a * (q_ret - v)).mean()
    correction = (-coeff * torch.exp(log_probs_then.detach()) * log_probs_now * (q.detach() - v)).sum(1).mean()
    critic = critic_weight * torch.nn.SmoothL1Loss()(q_a, q_ret)
    return actor, correction, critic


def _flatten(seqs, depth=None):
    """utils/various.py:64-72 iter_flatten: nested lists/tuples/arrays -> items"""
    for e in seqs:
        if isinstance(e, (list, tuple, np.ndarray)) and (depth is None or depth > 0):
            yield from _flatten(e, None if depth is None else depth - 1)
        else:
            yield e


class BatchedActionValueActorCriticAgent(Agent):
    """actor_critic.py:16-116: policy pi(a|s) + action value q(s, a) heads"""

    def __init__(self, env=None, gamma=0.99, optim_kwargs=None, history_length=None, dtype=torch.float,
                 device=torch.device("cpu"), hidden_sizes=(100, 100), activation=nn.ReLU(), max_num_actions=10,
                 log_epsilon=-20.0, *args, **kwargs):
        super().__init__(env, gamma, optim_kwargs, history_length, dtype, device)
        self._init_replay_buffer(history_length)
        self.max_num_actions = max_num_actions
        self.log_epsilon = log_epsilon
        self.preprocessor = SechsNimmtStateNormalization(action=True)
        self.actor_critic = MultiHeadedMLP(1 + self.state_length, hidden_sizes=hidden_sizes, head_sizes=(1, 1),
                                           activation=activation, head_activations=(None, None))
        self.softmax = nn.Softmax(dim=0)

    def _init_replay_buffer(self, history_length):
        pass

    def forward(self, state, legal_actions, **kwargs):
        log_probs, qs = self._evaluate(self._batch_state(state, legal_actions))
        k = self._act(log_probs, legal_actions)
        info = {"action_id": k, "log_probs": log_probs, "log_prob": log_probs[k], "values": qs, "value": qs[k]}
        return legal_actions[k], info

    def evaluate(self, states, legal_actions_list):
        """padded log pi and q per state: ([S, 10], [S, 10])"""
        lps, qs = [], []
        for state, legal in zip(states, legal_actions_list):
            lp, q = self._evaluate(self._batch_state(state, legal))
            lps.append(lp.unsqueeze(0))
            qs.append(q.flatten().unsqueeze(0))
        return torch.cat(lps, dim=0), torch.cat(qs, dim=0)

    def learn(self, *args, **kwargs):
        raise NotImplementedError

    def _batch_state(self, state, legal_actions):
        """candidate rows [n, 48] = [card, obs]"""
        state = torch.as_tensor(state).to(self.device, self.dtype).reshape(-1)
        cards = torch.tensor(list(legal_actions)).to(self.device, self.dtype)[:, None]
        return torch.cat((cards, state[None, :].expand(cards.shape[0], -1)), dim=1)

    def _evaluate(self, rows, pad=True):
        logits, qs = self.actor_critic(self.preprocessor(rows))
        log_probs = torch.log(self.softmax(logits).flatten())
        qs = qs.flatten()
        if pad:
            return self._pad(log_probs), self._pad(qs, value=0.0)
        return log_probs, qs

    def _act(self, log_probs, legal_actions):
        """draw from the padded distribution until the slot is a legal card"""
        dist = Categorical(torch.exp(torch.clamp(log_probs, -20)))
        k = len(legal_actions)
        while k >= len(legal_actions):
            try:
                k = dist.sample()
            except RuntimeError:
                logger.error("Error sampling action! Log probabilities: %s", log_probs)
        return k

    def _pad(self, x, value=None):
        fill = self.log_epsilon if value is None else value
        return torch.nn.functional.pad(x, (0, self.max_num_actions - x.shape[-1]), mode="constant", value=fill)

    def _gradient_step(self, loss):
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()


class BatchedACERAgent(BatchedActionValueActorCriticAgent):
    """actor_critic.py:119-207 (after minimalRL's acer.py)"""

    def __init__(self, *args, rollout_len=10, minibatch=5, truncate=1.0, warmup=100, r_factor=0.1, actor_weight=1.0,
                 critic_weight=1.0, **kwargs):
        self.truncate, self.warmup, self.batchsize = truncate, warmup, minibatch
        self.rollout_len, self.r_factor = rollout_len, r_factor
        self.actor_weight, self.critic_weight = actor_weight, critic_weight
        self.last_losses = []
        super().__init__(*args, **kwargs)

    def _init_replay_buffer(self, history_length):
        self.history = SequentialHistory(max_length=history_length, dtype=self.dtype, device=self.device)

    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, legal_actions,
              *args, **kwargs):
        self.history.store(state=state, legal_actions=legal_actions, log_probs=kwargs["log_probs"],
                           action_id=kwargs["action_id"], next_reward=next_reward * self.r_factor, done=done)
        if self.history.current_sequence_length() >= self.rollout_len or done or episode_end:
            self.history.flush()
            if len(self.history) > max(self.warmup, self.batchsize):
                self.last_losses.append(self._train(on_policy=True))
                self.last_losses.append(self._train(on_policy=False))

    def _train(self, on_policy=True):
        action_ids, done, is_first, legal, log_probs_then, rewards, states = self._rollout(on_policy)
        log_probs_now, q = self.evaluate(states, legal)
        actor, correction, critic = acer_losses(log_probs_now, q, log_probs_then, action_ids, rewards, done, is_first,
                                                self.gamma, self.truncate, self.critic_weight)
        self._gradient_step(actor + correction + critic)
        return actor.item(), correction.item(), critic.item()

    def _rollout(self, on_policy):
        seqs = self.history.rollout(n=1) if on_policy else self.history.sample(self.batchsize)[2]
        states = torch.stack(list(_flatten(seqs["state"])))
        legal = list(_flatten(seqs["legal_actions"], depth=1))
        action_ids = torch.tensor([int(a) for a in _flatten(seqs["action_id"])], dtype=torch.long).unsqueeze(1)
        rewards = np.array(list(_flatten(seqs["next_reward"])))
        log_probs_then = torch.stack(list(_flatten(seqs["log_probs"])))
        done = np.array(list(_flatten(seqs["done"])), dtype=bool)
        is_first = np.array(list(_flatten(seqs["first"])), dtype=bool)
        return action_ids, done, is_first, legal, log_probs_then, rewards, states
