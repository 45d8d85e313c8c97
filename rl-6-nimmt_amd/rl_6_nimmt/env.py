"""Drop-in `SechsNimmtEnv` (reference: rl_6_nimmt/env.py:13-256) on the MI355X engine.

Same constructor, `reset`, `reset_to`, `step`, `render`, return types
(int64 observation arrays of length 47, sorted legal-action lists, int32
rewards) and errors (`AssertionError`, `InvalidMoveException` with the
reference's message).  The game itself lives in device memory: every call
runs the HIP kernels of libsechs.so on a one-game handle.

Randomness follows the reference exactly: `reset()` shuffles the deck with
numpy's *global* legacy RandomState.  The engine pulls that state onto the
GPU (np.random.get_state -> sn_mt_set), deals there and hands the advanced
state back (sn_mt_get -> np.random.set_state), so a seeded script draws the
same cards as with the reference.

Known deviation: hands are card sets on the device, so `reset_to` with an
unsorted hand list yields sorted legal lists (the reference's own callers
always pass sorted hands: env.py:108, agents/mcts.py:118-125).
"""
import ctypes
import logging

import numpy as np
import torch

from . import _native as nat
from .spaces import Box, Discrete
from .vec_env import VecSechsNimmtEnv, obs_length

logger = logging.getLogger(__name__)

ROWS, THRESHOLD, HAND = 4, 6, 10


class InvalidMoveException(Exception):
    """A player tried to play a card that is not in their hand (env.py:9-10)."""


def card_value(card):
    """Bull heads of a card (env.py:224-239); host-side helper for render."""
    c = int(card) + 1
    assert 0 < c <= 104
    if c == 55:
        return 7
    if c % 11 == 0:
        return 5
    if c % 10 == 0:
        return 3
    if c % 10 == 5:
        return 2
    return 1


class SechsNimmtEnv:
    """OpenAI-gym style environment for 6 nimmt! (one game), run on the GPU."""

    metadata = {"render.modes": ["human"]}

    def __init__(self, num_players, num_rows=4, num_cards=104, threshold=6, include_summaries=True,
                 player_names=None, verbose=True):
        assert num_players > 0
        assert num_rows > 0
        assert num_cards >= 10 * num_players + num_rows
        if num_rows != ROWS or threshold != THRESHOLD:
            raise NotImplementedError("the MI355X engine is built for the reference defaults num_rows=4, threshold=6")
        self._num_players = num_players
        self._num_rows = num_rows
        self._num_cards = num_cards
        self._threshold = threshold
        self._include_summaries = include_summaries
        self._player_names = player_names
        self.verbose = verbose

        self.action_space = Discrete(num_cards)
        self.reward_range = (-float("inf"), 0)
        self.observation_space = Box(low=-1.0, high=2.0, shape=(obs_length(include_summaries),), dtype=np.float32)
        self.spec = None

        self._vec = VecSechsNimmtEnv(1, num_players, num_cards, seed=0, rng="numpy", include_summaries=include_summaries)
        # one-game fast path (sn_step1 / sn_reset1): host-side argument and
        # result buffers, one kernel launch + one sync per call
        self._out = np.zeros(2 + 15 * num_players, dtype=np.int32)  # sn_step1's words (include/sechs.h)
        self._acts = np.zeros(num_players, dtype=np.int32)
        self._key = np.zeros(624, dtype=np.uint32)
        self._pos = ctypes.c_int32()
        self._flags = 0 if include_summaries else nat.SN_NO_SUMMARIES
        self._board = [[] for _ in range(num_rows)]
        self._hands = [[] for _ in range(num_players)]
        self._scores = np.zeros(num_players, dtype=np.int32)
        self._obs = None

    # ------------------------------------------------------------ gym API
    def reset(self):
        """Deal a new game from numpy's global RNG (env.py:43-51)."""
        if self.verbose:
            logger.debug("Dealing cards")
        st = np.random.get_state()
        key = np.ascontiguousarray(st[1], dtype=np.uint32)
        nat.check(nat.lib().sn_reset1(self._vec._h, key.ctypes.data_as(ctypes.c_void_p), int(st[2]),
                                      self._key.ctypes.data_as(ctypes.c_void_p), ctypes.byref(self._pos),
                                      self._out.ctypes.data_as(ctypes.c_void_p), self._flags), "sn_reset1")
        np.random.set_state((st[0], self._key.copy(), int(self._pos.value), st[3], st[4]))
        self._unpack()
        return self._create_states()

    def reset_to(self, board, hands):
        """Install a position (env.py:53-62); inputs are copied."""
        assert len(board) == ROWS and len(hands) == self._num_players
        b = np.full((1, ROWS, THRESHOLD), -1, dtype=np.int8)
        h = np.full((1, self._num_players, HAND), -1, dtype=np.int8)
        sizes = {len(x) for x in hands}
        if len(sizes) != 1:
            raise ValueError("every player must hold the same number of cards")
        for r, row in enumerate(board):
            if not 1 <= len(row) <= THRESHOLD - 1:
                raise ValueError("rows must hold 1..5 cards")
            b[0, r, : len(row)] = [self._check_card(c) for c in row]
        for p, hand in enumerate(hands):
            if len(hand) > HAND:
                raise ValueError("at most 10 cards per hand")
            h[0, p, : len(hand)] = [self._check_card(c) for c in hand]
        self._vec.reset_to(torch.from_numpy(b), torch.from_numpy(h))
        self._pull()
        return self._create_states()

    def step(self, action):
        """One simultaneous round (env.py:64-77): ((states, legal), rewards, done, {})."""
        assert len(action) == self._num_players
        acts = np.asarray([int(a) for a in action], dtype=np.int64)
        for p, card in enumerate(acts):  # out-of-range cards can never be in a hand
            if not 0 <= card < self._num_cards:
                self._invalid(p, card)
        self._acts[:] = acts
        nat.check(nat.lib().sn_step1(self._vec._h, self._acts.ctypes.data_as(ctypes.c_void_p),
                                     self._out.ctypes.data_as(ctypes.c_void_p), self._flags), "sn_step1")
        bad = int(self._out[0])
        if bad >= 0:
            self._invalid(bad, acts[bad])
        N = self._num_players
        rewards = self._out[2: 2 + N].copy()
        done = bool(self._out[1])
        self._unpack()
        if self.verbose:  # _play_cards' debug lines, cards ascending (env.py:128,145,165)
            trace = self._out[2 + 14 * N: 2 + 15 * N]
            for card, p in sorted((int(c), p) for p, c in enumerate(acts)):
                logger.debug(f"{self._player_name(p)} plays card {card + 1}")
                w = int(trace[p])
                if w & 4:
                    logger.debug(f"  ...chooses to replace row {(w & 3) + 1}")
                if w & 8:
                    logger.debug(f"  ...and gains {w >> 8} Hornochsen")
        return self._create_states(), rewards, done, dict()

    def render(self, mode="human"):
        """Log the board and the hands (env.py:79-97)."""
        bar = "-" * 120
        logger.info(bar)
        logger.info("Board:")
        for cards in self._board:
            empty = "   _ " * (self._threshold - len(cards) - 1)
            logger.info("  " + " ".join(self._format_card(c) for c in cards) + empty + "   * ")
        logger.info("Players:")
        for p, (score, hand) in enumerate(zip(self._scores, self._hands)):
            cards = "no cards " if not hand else "cards " + " ".join(self._format_card(c) for c in hand)
            logger.info(f"  {self._player_name(p)}: {score:>3d} Hornochsen, " + cards)
        if self._is_done():
            logger.info(
                f"The game is over! {self._player_name(int(np.argmin(self._scores)))} wins, "
                f"{self._player_name(int(np.argmax(self._scores)))} loses. Congratulations!"
            )
        logger.info(bar)

    # ------------------------------------------------------------ internals the reference's callers use
    def _create_states(self):
        """(per-player int64 observations, per-player sorted legal actions), env.py:174-186."""
        states = [self._obs[p].copy() for p in range(self._num_players)]
        legal = [list(h) for h in self._hands]
        return states, legal

    def _is_done(self):
        return len(self._hands[0]) == 0

    @staticmethod
    def _card_value(card):
        return card_value(card)

    def _row_value(self, cards, include_last=False):
        cards = cards if include_last else cards[:-1]
        return sum(card_value(c) for c in cards)

    def _player_name(self, player):
        if self._player_names is None:
            return f"Player {player + 1:d}"
        width = max(len(name) for name in self._player_names)
        return f"{self._player_names[player]:<{width}} (player {player + 1:d})"

    def _format_card(self, card):
        glyph = {1: " ", 2: ".", 3: ":", 5: "+", 7: "#"}[card_value(card)]
        return f"{card + 1:>3d}{glyph}"

    # ------------------------------------------------------------ device <-> mirrors
    def _check_card(self, c):
        c = int(c)
        if not 0 <= c < min(self._num_cards, 104):
            raise ValueError(f"card {c} out of range")
        return c

    def _invalid(self, p, card):
        raise InvalidMoveException(f"Player {p + 1} tried to play card {int(card) + 1}, but their hand is {self._hands[p]}")

    def _unpack(self):
        """Python mirrors from the packed fast-path result (scores, obs rows)."""
        N = self._num_players
        self._scores = self._out[2 + N: 2 + 2 * N].copy()
        rows = self._out[2 + 2 * N: 2 + 14 * N].view(np.int8).reshape(N, 48)
        obs = rows[:, : obs_length(self._include_summaries)].astype(np.int64)
        self._obs = obs
        self._hands = [[int(c) for c in obs[p, :HAND] if c >= 0] for p in range(N)]
        board = obs[0, -ROWS * THRESHOLD:].reshape(ROWS, THRESHOLD)
        self._board = [[int(c) for c in row if c >= 0] for row in board]

    def _pull(self):
        """Copy the device state into the Python mirrors (one obs + one score read)."""
        obs = self._vec.obs(torch.int64)[0].cpu().numpy()
        self._scores = self._vec.scores()[0].cpu().numpy().astype(np.int32)
        self._obs = obs
        self._hands = [[int(c) for c in obs[p, :HAND] if c >= 0] for p in range(self._num_players)]
        board = obs[0, -ROWS * THRESHOLD:].reshape(ROWS, THRESHOLD)
        self._board = [[int(c) for c in row if c >= 0] for row in board]
