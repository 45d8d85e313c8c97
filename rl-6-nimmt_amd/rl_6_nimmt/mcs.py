"""Batched Monte-Carlo search self-play on one MI355X (BASELINE config 3).

Every seat of every game is an MCSAgent (reference: agents/mcts.py:17-188).
One `decide()` call runs, for all B*N (game, seat) decisions at once:
  1. sn_mcs_memorize -- the seat's card memory (mcts.py:62-73, quirk Q5 kept);
  2. sn_mcs_rollouts -- `rollouts` playouts per legal first move, one lane
     per playout (opponents dealt from the memory, every later move uniform,
     mcts.py:108-154);
  3. sn_mcs_choose   -- the move with the best mean (mcts.py:156-165).
The reference draws the first move uniformly and runs min(mc_max,
mc_per_card*n!) playouts; "stratified" mode gives every legal move the same
number of playouts instead, which is BASELINE config 3's "256 uniform
rollouts/action".  Randomness: Philox keyed (seed ^ decision step, game,
seat, move, playout) -- bit-exact against the CPU oracle's restatement.
"""
import torch

from . import _native as nat
from .vec_env import VecSechsNimmtEnv


def rollout_env_steps_per_seat_game(rollouts, hand=10):
    """playout env-steps one seat spends per game: sum over n of rollouts*n*n (n = 2..10)."""
    return sum(rollouts * n * n for n in range(2, hand + 1))


class BatchedMCS:
    def __init__(self, env: VecSechsNimmtEnv, rollouts=256, seed=0, mcs_num_cards=104):
        self.env = env
        self.rollouts = int(rollouts)
        self.seed = int(seed)
        self.mcs_num_cards = int(mcs_num_cards)
        D = env.num_games * env.num_players
        self.avail = torch.zeros((4, D), dtype=torch.int32, device=env.device)  # uint32 card sets
        self.sums = torch.zeros((D, 10), dtype=torch.int32, device=env.device)
        self.actions = torch.zeros((env.num_games, env.num_players), dtype=torch.int32, device=env.device)
        self.step_id = 0

    def decide(self, step_id=None):
        """Choose every seat's card for the current position: int32 [B, N]."""
        sid = self.step_id if step_id is None else int(step_id)
        self.step_id = sid + 1
        h, st = self.env._h, self.env._stream()
        L = nat.lib()
        nat.check(L.sn_mcs_memorize(h, nat.ptr(self.avail), self.mcs_num_cards, st), "sn_mcs_memorize")
        nat.check(L.sn_mcs_rollouts(h, nat.ptr(self.avail), self.rollouts, self.seed & (2**64 - 1), sid & 0xFFFFFFFF,
                                    nat.ptr(self.sums), st), "sn_mcs_rollouts")
        nat.check(L.sn_mcs_choose(h, nat.ptr(self.sums), nat.ptr(self.actions), st), "sn_mcs_choose")
        return self.actions

    def play_episode(self):
        """All seats MCS for one whole game of every env game (reset first).
        Returns the summed rewards [B, N] int32 (GameSession.results)."""
        self.env.reset()
        total = torch.zeros((self.env.num_games, self.env.num_players), dtype=torch.int32, device=self.env.device)
        for _ in range(10):
            acts = self.decide()
            rew, done, inv = self.env.step(acts)
            total += rew
        return total


def play_exact(env: VecSechsNimmtEnv, seats, mc_per_card=10, mc_max=100):
    """Reference-exact GameSession replay (numpy-MT env): seats is a string
    like "MRRR" (M = MCSAgent(mc_per_card, mc_max), R = DrunkHamster).
    Returns (actions [10,B,N], rewards [10,B,N], status [B]); status 1 marks
    games where the reference would have raised IndexError (quirk Q6)."""
    if env.rng != "numpy":
        raise ValueError("reference-exact replay needs rng='numpy'")
    assert len(seats) == env.num_players
    mask = sum(1 << p for p, ch in enumerate(seats) if ch.upper() == "M")
    B, N = env.num_games, env.num_players
    acts = torch.zeros((10, B, N), dtype=torch.int32, device=env.device)
    rews = torch.zeros((10, B, N), dtype=torch.int32, device=env.device)
    status = torch.zeros((B,), dtype=torch.int32, device=env.device)
    nat.check(nat.lib().sn_mcs_play_exact(env._h, mask, int(mc_per_card), int(mc_max), nat.ptr(acts), nat.ptr(rews),
                                          nat.ptr(status), env._stream()), "sn_mcs_play_exact")
    return acts, rews, status
