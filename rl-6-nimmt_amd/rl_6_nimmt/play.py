"""Drop-in `GameSession` (reference: rl_6_nimmt/play.py:9-87).

Plays whole games between agents through the MI355X `SechsNimmtEnv`.
Behaviour kept from the reference, including its quirks:
  * agents act in seat order, then the env steps, then every agent's
    `learn` runs (play.py:38-67);
  * `learn(reward=...)` receives the *previous* step's reward
    (play.py:29,57,72);
  * `results` collects each game's summed rewards (int32, = -penalties).
"""
import logging

import numpy as np
import torch

from .env import SechsNimmtEnv

logger = logging.getLogger(__name__)


class GameSession:
    def __init__(self, *agents, device=torch.device("cpu"), dtype=torch.float):
        self.device = device
        self.dtype = dtype
        self.agents = [agent.to(self.device, self.dtype) for agent in agents]
        self.num_agents = len(agents)
        self.env = SechsNimmtEnv(self.num_agents)
        self.results = []
        self.game = 0
        self.env._player_names = [getattr(a, "__name__", type(a).__name__) for a in self.agents]

    def play_game(self, render=False):
        states, legal = self.env.reset()
        states = self._tensorize(states)
        n = self.num_agents
        prev_rewards = np.zeros(n, dtype=np.int32)
        total = np.zeros(n, dtype=np.int32)
        if render:
            self.env.render()
        done = False
        while not done:
            actions, infos = [], []
            for agent, state, legal_p in zip(self.agents, states, legal):
                action, info = agent(state, legal_actions=legal_p)
                actions.append(int(action))
                infos.append(info)
            (next_states, next_legal), rewards, done, _ = self.env.step(actions)
            next_states = self._tensorize(next_states)
            if render:
                self.env.render()
            for p, agent in enumerate(self.agents):
                agent.learn(
                    state=states[p],
                    legal_actions=legal[p].copy(),
                    reward=prev_rewards[p],
                    action=actions[p],
                    done=done,
                    next_state=next_states[p],
                    next_legal_actions=next_legal[p].copy(),
                    next_reward=rewards[p],
                    num_episode=self.game,
                    episode_end=done,
                    **infos[p],
                )
            total += np.asarray(rewards)
            states, legal, prev_rewards = next_states, next_legal, rewards
        self.results.append(total)
        self.game += 1

    def _tensorize(self, arrays):
        return [torch.tensor(a).to(self.device, self.dtype) for a in arrays]
