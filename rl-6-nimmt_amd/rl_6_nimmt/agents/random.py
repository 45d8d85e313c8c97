"""DrunkHamster: uniformly random legal move (reference: agents/random.py:5-13).

Draws from numpy's global legacy RNG with the reference's exact call, so a
seeded GameSession replays the reference game for game.  (The batched
engine runs the same policy inside the HIP kernels: VecSechsNimmtEnv.rollout.)
"""
import numpy as np

from .base import Agent


class DrunkHamster(Agent):
    def forward(self, state, legal_actions, **kwargs):
        return np.random.choice(np.array(legal_actions, dtype=np.int32), size=1)[0], {}

    def learn(self, *args, **kwargs):
        return 0.0
