"""Agent base class (reference: rl_6_nimmt/agents/base.py:7-62).

An agent is a torch `nn.Module` with
    forward(state: float tensor [47], legal_actions: list[int]) -> (action, info dict)
    learn(state, reward, action, done, next_state, next_reward, episode_end,
          num_episode, legal_actions, **info)
and `train()` creating an Adam optimizer.  The reference reads the action /
observation sizes from a default 4-player env; here they come from the
space descriptors, so building an agent never touches the GPU.
"""
import torch
from torch import nn

from ..spaces import Box, Discrete
from ..vec_env import obs_length
from ..utils.history import History


class Agent(nn.Module):
    def __init__(self, env=None, gamma=0.99, optim_kwargs=None, history_length=None, dtype=torch.float,
                 device=torch.device("cpu")):
        if env is None:
            action_space, state_length = Discrete(104), obs_length(True)
        else:
            action_space, state_length = env.action_space, env.observation_space.shape[0]
        self.gamma = gamma
        self.device = device
        self.dtype = dtype
        self.action_space = action_space
        self.state_length = state_length
        self.num_actions = action_space.n
        self.history = History(max_length=history_length, dtype=dtype, device=device)
        self.optimizer = None
        self.optim_kwargs = optim_kwargs
        super().__init__()

    def train(self, mode=True):
        super().train(mode=mode)
        if mode:
            self.optimizer = torch.optim.Adam(params=self.parameters(), **(self.optim_kwargs or {}))
        return self

    def forward(self, state, legal_actions, *args, **kwargs):
        raise NotImplementedError

    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, legal_actions,
              *args, **kwargs):
        raise NotImplementedError
