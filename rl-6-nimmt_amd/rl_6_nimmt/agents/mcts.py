"""Monte-Carlo search agents (reference: rl_6_nimmt/agents/mcts.py).

`MCSAgent` is a drop-in for the reference's: same constructor, card memory,
`forward(state, legal_actions) -> (card, {"log_prob": ...})` and `learn`.
Its playouts run on the GPU (sn_mcs_decide_exact): the numpy global RNG
state is copied to the device, one lane runs all n_mc playouts in the
reference's exact draw order, and the advanced state is copied back -- so a
seeded GameSession makes the same choices as the reference.

Deviation: where a legal move received no playout the
reference raises IndexError from a debug f-string (mcts.py:167-170); this
agent returns the best sampled move and logs a warning instead.
"""
import logging
import math

import numpy as np
import torch

from .. import _native as nat
from .base import Agent

logger = logging.getLogger(__name__)

ROWS, THRESHOLD, HAND = 4, 6, 10


class BaseMCAgent(Agent):
    def __init__(self, handsize=10, num_rows=4, num_cards=104, threshold=6, mc_per_card=10, mc_max=100,
                 include_summaries=True, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.num_players = None
        self.handsize = handsize
        self.num_rows = num_rows
        self.num_cards = num_cards
        self.threshold = threshold
        self.mc_per_card = mc_per_card
        self.mc_max = mc_max
        self.include_summaries = include_summaries
        self.available_cards = []

    # ---------------------------------------------------------- card memory (mcts.py:43-89)
    def forward(self, state, legal_actions, *args, **kwargs):
        n = len(legal_actions)
        if n == self.handsize:
            self._initialize_game(state)
        self._memorize_cards(state, legal_actions)
        if n == 1:
            return legal_actions[0], {"log_prob": torch.tensor(0.0).to(self.device, self.dtype)}
        return self._mcts(legal_actions, state)

    def learn(self, state, reward, action, done, next_state, next_reward, episode_end, num_episode, legal_actions,
              *args, **kwargs):
        raise NotImplementedError

    def _initialize_game(self, state):
        self.available_cards = list(range(self.num_cards))
        self.num_players = int(state[10])

    def _memorize_cards(self, state, legal_actions):
        seen = set(int(c) for c in legal_actions) | set(self._board_from_state(state, flatten=True))
        self.available_cards = [c for c in self.available_cards if c not in seen]

    def _board_from_state(self, state, flatten=True):
        if hasattr(state, "detach"):
            state = state.detach().cpu().numpy()
        cells = np.asarray(state[-self.num_rows * self.threshold:], dtype=np.float64).reshape(self.num_rows, self.threshold)
        rows = [[int(v) for v in row if v >= 0.0] for row in cells]
        return [c for row in rows for c in row] if flatten else rows

    def _compute_n_mc(self, n_actions):
        return min(self.mc_max, self.mc_per_card * math.factorial(n_actions))

    def _mcts(self, legal_actions, state):
        raise NotImplementedError


class MCSAgent(BaseMCAgent):
    """Monte-Carlo search with uniformly random playouts for every seat."""

    def learn(self, *args, **kwargs):
        pass

    def _mcts(self, legal_actions, state):
        nat.require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device())
        board = np.full((1, ROWS, THRESHOLD), -1, dtype=np.int8)
        for r, row in enumerate(self._board_from_state(state, flatten=False)):
            board[0, r, : len(row)] = row
        hand = np.full((1, HAND), -1, dtype=np.int8)
        hand[0, : len(legal_actions)] = sorted(int(c) for c in legal_actions)
        words = np.zeros(4, dtype=np.uint64)
        for c in self.available_cards:
            words[c >> 5] |= np.uint64(1) << np.uint64(c & 31)
        st = np.random.get_state()
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
        d_board, d_hand = t(board, torch.int8), t(hand, torch.int8)
        d_avail = t(words.astype(np.uint32).view(np.int32).reshape(1, 4), torch.int32)
        d_key = t(st[1].astype(np.uint32).view(np.int32).reshape(1, 624), torch.int32)
        d_pos = t(np.array([st[2]], dtype=np.int32), torch.int32)
        d_act = torch.zeros(1, dtype=torch.int32, device=dev)
        d_sums = torch.zeros((1, 10), dtype=torch.int32, device=dev)
        d_cnts = torch.zeros((1, 10), dtype=torch.int32, device=dev)
        nat.check(nat.lib().sn_mcs_decide_exact(dev.index, 1, int(self.num_players), nat.ptr(d_board), nat.ptr(d_hand),
                                                nat.ptr(d_avail), int(self.mc_per_card), int(self.mc_max),
                                                nat.ptr(d_key), nat.ptr(d_pos), nat.ptr(d_act), nat.ptr(d_sums),
                                                nat.ptr(d_cnts), nat.stream_handle(dev)), "sn_mcs_decide_exact")
        key = d_key.cpu().numpy().view(np.uint32)[0].copy()
        np.random.set_state((st[0], key, int(d_pos.item()), st[3], st[4]))
        act = int(d_act.item())
        if act < 0:
            act = -act - 2
            logger.warning("MCS: a legal move got no playout (the reference raises IndexError here, quirk Q6)")
        self.last_search = {"sums": d_sums.cpu().numpy()[0], "counts": d_cnts.cpu().numpy()[0]}
        return act, {"log_prob": torch.tensor(0.0).to(self.device, self.dtype)}
