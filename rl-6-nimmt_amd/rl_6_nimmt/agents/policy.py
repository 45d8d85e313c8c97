"""Policy-gradient agent (reference: rl_6_nimmt/agents/policy.py:109-201,
registered as AGENTS["reinforce"]).

`BatchedReinforceAgent` is a drop-in: the same candidate-row policy
(MultiHeadedMLP 48-100-100-1 over `[card, obs]` rows normalised by
SechsNimmtStateNormalization, softmax over the legal cards), the same
torch-RNG sampling, and REINFORCE with discounted returns at episode end.
It is a host-side torch agent like the reference's (its forward is one tiny
MLP call); the GPU form for many games at once is `reinforce.BatchedReinforce`
(candidate rows and sampling in HIP kernels, MLP via PyTorch-ROCm).

The reference's `MaskedReinforceAgent` (policy.py:15-106, 104-way head) is
not registered in AGENTS and fails on list legal actions (`int(action.item())`
on a Python int, policy.py:61), so it is not reproduced.
"""
import numpy as np
import torch
from torch import nn
from torch.distributions import Categorical

from .base import Agent
from ..utils.nets import MultiHeadedMLP
from ..utils.preprocessing import SechsNimmtStateNormalization


def compute_discounted_returns(rewards, gamma, dtype=torch.float, device=torch.device("cpu")):
    """utils/various.py:41-50: G_t = r_t + gamma G_{t+1}, accumulated in float64"""
    if isinstance(rewards, torch.Tensor):
        rewards = rewards.numpy()
    returns = []
    g = 0.0
    for r in rewards[::-1]:
        g = r + gamma * g
        returns.insert(0, g)
    return torch.tensor(returns).to(device, dtype)


class BatchedReinforceAgent(Agent):
    def __init__(self, env=None, gamma=0.99, optim_kwargs=None, history_length=None, dtype=torch.float,
                 device=torch.device("cpu"), hidden_sizes=(100, 100), activation=nn.ReLU(), r_factor=1.0,
                 actor_weight=1.0, entropy_weight=0.0, *args, **kwargs):
        super().__init__(env, gamma, optim_kwargs, history_length, dtype, device)
        self.r_factor = r_factor
        self.actor_weight = actor_weight
        self.entropy_weight = entropy_weight
        self.preprocessor = SechsNimmtStateNormalization(action=True)
        self.actor = MultiHeadedMLP(self.state_length + 1, hidden_sizes=hidden_sizes, head_sizes=(1,),
                                    activation=activation, head_activations=(None,))
        self.softmax = nn.Softmax(dim=0)

    def forward(self, state, legal_actions, **kwargs):
        state = torch.as_tensor(state).to(self.device, self.dtype).reshape(-1)
        cards = torch.tensor(legal_actions, device=self.device).to(self.dtype)[:, None]
        batch = torch.cat((cards, state[None, :].expand(len(legal_actions), -1)), dim=1)
        (logits,) = self.actor(self.preprocessor(batch))
        probs = self.softmax(logits).flatten()
        cat = Categorical(probs)
        action_id = cat.sample()
        return int(legal_actions[action_id]), {"log_prob": cat.log_prob(action_id), "entropy": cat.entropy()}

    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, *args, **kwargs):
        self.history.store(log_prob=kwargs["log_prob"], reward=reward * self.r_factor, entropy=kwargs["entropy"])
        if not episode_end or not self.training:
            return np.zeros(3)
        losses = self._train()
        self.history.clear()
        return losses

    def _train(self):
        rollout = self.history.rollout()
        n = len(self.history)
        log_probs = torch.stack(rollout["log_prob"], dim=0)
        entropies = torch.stack(rollout["entropy"], dim=0)
        returns = compute_discounted_returns(rollout["reward"], self.gamma).to(self.device, self.dtype)
        discounts = torch.exp(np.log(self.gamma) * torch.linspace(0, n - 1, n)).to(self.device, self.dtype)
        actor_loss = -torch.sum(discounts * returns * log_probs)
        entropy_loss = -torch.sum(entropies)
        self._gradient_step(self.actor_weight * actor_loss + self.entropy_weight * entropy_loss)
        return np.array([actor_loss.item(), 0.0, entropy_loss.item()])

    def _gradient_step(self, loss):
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
