"""Batched tournament on the MI355X (BASELINE config 5).

Reference: Tournament (rl_6_nimmt/tournament.py:12-262) -- `play_game()`
draws the seats (`_choose_players`, :166-177), plays one GameSession game
(:132-138) and scores it (`score_game`, :140-164: relative positions, first-
argmax winner, order-dependent multiplayer Elo).

Here every slot g of a tournament handle (`sn_league_config`) is one
reference tournament stream: slot g replays

    np.random.seed(seed + game_offset + g)
    t = Tournament(min_players, max_players); t.add_player(name, DrunkHamster()) ...
    t.play_game()  # x games

bit for bit -- seat draw, deal and every move come from the slot's own
numpy MT19937 stream inside the k_play kernel (tests/golden/
tournament_games.json pins it).  All slots play at once; the games of all
slots (and, over RCCL, of all ranks) form one tournament whose scoring is
per game (vectorised here on the device) and whose Elo -- the only
order-dependent part -- is replayed on the host in a canonical order: game
round major, then global slot id (`sn_elo_replay`, C++; multi_elo parity
unpinned, elo.py).

Agents are the reference's DrunkHamster (played in-kernel); a search agent
(MCSAgent, PUCTAgent, ...) in a league plays through the drop-in
`Tournament` instead (host loop over the device env).
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .agents.random import DrunkHamster
from .vec_env import VecSechsNimmtEnv

STAT_GAMES, STAT_SCORE, STAT_POSITION, STAT_WINS = range(4)


def decode_seats(words, max_players):
    """seats word -> (k [..], agent ids [.., max_players], -1 past k)"""
    w = words.to(torch.int64)
    k = w & 15
    p = torch.arange(max_players, device=w.device)
    ids = (w[..., None] >> (4 + 4 * p)) & 15
    ids = torch.where(p < k[..., None], ids, torch.full_like(ids, -1))
    return k, ids


def relative_positions(results, k):
    """Tournament._compute_relative_positions (tournament.py:249-256) per game,
    vectorised: (#lower + (#equal - 1)/2) / (k - 1), seats past k ignored."""
    R = results.to(torch.float64)
    P = R.shape[-1]
    valid = torch.arange(P, device=R.device) < k[..., None]
    a, b = R[..., :, None], R[..., None, :]
    vb = valid[..., None, :]
    lower = ((b < a) & vb).sum(dim=-1).to(torch.float64)
    equal = ((b == a) & vb).sum(dim=-1).to(torch.float64)
    pos = (lower + 0.5 * (equal - 1.0)) / (k[..., None].to(torch.float64) - 1.0)
    return torch.where(valid, pos, torch.zeros_like(pos))


def winners(results, k):
    """winner seat = first argmax of the results (tournament.py:142)"""
    R = results.to(torch.int64)
    P = R.shape[-1]
    valid = torch.arange(P, device=R.device) < k[..., None]
    R = torch.where(valid, R, torch.full_like(R, -(1 << 40)))
    return torch.argmax(R, dim=-1)  # torch.argmax returns the first maximum


class BatchedTournament:
    """A tournament of DrunkHamster agents played by `num_slots` concurrent
    game slots on one GPU (one rank's shard: global slot ids game_offset ..
    game_offset + num_slots - 1)."""

    def __init__(self, num_slots, min_players=2, max_players=4, seed=0, game_offset=0, rng="numpy", device=None,
                 elo_initial=1600, elo_k=32):
        assert 0 < min_players <= max_players
        self.num_slots, self.min_players, self.max_players = int(num_slots), int(min_players), int(max_players)
        self.seed, self.game_offset, self.rng, self.device = int(seed), int(game_offset), rng, device
        self.elo_initial, self.elo_k = float(elo_initial), float(elo_k)
        self.names, self.agents = [], {}
        self.env = None
        self.records = []  # per play_games call: int32 [games, num_slots, 1 + max_players] on the device

    # ------------------------------------------------------------ roster (tournament.py:36-52)
    def add_player(self, name, agent=None):
        assert name not in self.agents and self.env is None, "add every player before the first game"
        agent = DrunkHamster() if agent is None else agent
        if type(agent) is not DrunkHamster:
            raise NotImplementedError("the batched tournament plays DrunkHamster agents in-kernel; leagues with "
                                      "search agents play through rl_6_nimmt.Tournament")
        agent.__name__ = name
        self.names.append(name)
        self.agents[name] = agent

    def __len__(self):
        return len(self.names)

    def _start(self):
        K = len(self.names)
        assert K >= self.max_players, "tournament.py:170: len(self) >= num_players"
        self.env = VecSechsNimmtEnv(self.num_slots, self.max_players, seed=self.seed, game_offset=self.game_offset,
                                    rng=self.rng, device=self.device)
        nat.check(nat.lib().sn_league_config(self.env._h, K, self.min_players, self.max_players), "sn_league_config")
        self.env.reset()  # every slot draws its first seats, then deals

    # ------------------------------------------------------------ games (tournament.py:132-138)
    def play_games(self, games=1, rewards=False):
        """`games` tournament games per slot.  Returns the records int32
        [games, num_slots, 1 + max_players]: seats word (k | agent(seat p)
        << (4 + 4p)), then the results (GameSession.results[0], 0 past k);
        with rewards=True also the per-step rewards [10 games, slots, N]."""
        if self.env is None:
            self._start()
        env = self.env
        T = 10 * int(games)
        rec = torch.empty((games, self.num_slots, 1 + self.max_players), dtype=torch.int32, device=env.device)
        rew = torch.empty((T, self.num_slots, self.max_players), dtype=torch.int32, device=env.device) if rewards else None
        nat.check(nat.lib().sn_league_rollout(env._h, T, nat.ptr(rew), None, None, None, 0, nat.ptr(rec), env._stream()),
                  "sn_league_rollout")
        self.records.append(rec)
        return (rec, rew) if rewards else rec

    def seats(self):
        """(k [slots], agent ids [slots, max_players]) of every slot's next game"""
        out = torch.empty((self.num_slots,), dtype=torch.int32, device=self.env.device)
        nat.check(nat.lib().sn_league_seats(self.env._h, nat.ptr(out), self.env._stream()), "sn_league_seats")
        return decode_seats(out, self.max_players)

    # ------------------------------------------------------------ scoring (tournament.py:140-164)
    def all_records(self):
        """every game played so far, [games, slots, 1 + N] (round major)"""
        return torch.cat(self.records, dim=0) if self.records else torch.zeros(
            (0, self.num_slots, 1 + self.max_players), dtype=torch.int32)

    def agent_stats(self, records=None):
        """per-agent sums float64 [K, 4]: games played, score, relative position, wins"""
        rec = self.all_records() if records is None else records
        return league_agent_stats(rec, len(self.names), self.max_players)

    def replay_elo(self, records=None):
        """Elo of every agent after replaying the games in canonical order
        (round major, then global slot id) -- sn_elo_replay, host C++"""
        rec = self.all_records() if records is None else records
        return replay_league_elo(rec, len(self.names), self.max_players, self.elo_initial, self.elo_k)

    def table(self, stats=None, elos=None):
        """the reference's tournament table (tournament.py:208-238) from the sums"""
        stats = self.agent_stats() if stats is None else stats
        elos = self.replay_elo() if elos is None else elos
        s = stats.cpu().numpy()
        total = int(s[:, STAT_WINS].sum())  # one winner per game
        bar = "-----------------------------------------------------------------"
        out = [f"Tournament after {total} games:", bar,
               " Agent                | Games | Mean score | Win fraction |  ELO ", bar]
        for i, name in enumerate(self.names):
            g = s[i, STAT_GAMES]
            score = f"{s[i, STAT_SCORE] / g:>5.2f}" if g else "-"
            wins = f"{s[i, STAT_WINS] / g:>5.2f}" if g else "-"
            out.append(f" {name:>20s} | {int(g):>5} | {score:>10} | {wins:>12} | {elos[i]:>4.0f} ")
        out.append(bar)
        return "\n".join(out)

    def close(self):
        if self.env is not None:
            self.env.close()
            self.env = None


def league_agent_stats(records, num_agents, max_players):
    """Tournament.score_game's per-agent tallies (tournament.py:140-152) as
    sums over records [..., 1 + N]: float64 [K, 4] = games played, score,
    relative position, wins (all_reduce-able across ranks)"""
    K, N = num_agents, max_players
    rec = records.reshape(-1, 1 + N)
    k, ids = decode_seats(rec[:, 0], N)
    res = rec[:, 1:]
    rel = relative_positions(res, k)
    win = winners(res, k)
    valid = ids >= 0
    is_win = torch.arange(N, device=rec.device)[None, :] == win[:, None]
    vals = torch.stack((valid.to(torch.float64), res.to(torch.float64), rel, is_win.to(torch.float64)), dim=-1)
    # one-hot [seatings, K] x [seatings, 4]: a GEMM instead of float64
    # atomics on K addresses (index_add_ serialises millions of them)
    onehot = ((ids.reshape(-1, 1) == torch.arange(K, device=rec.device)[None, :]) & valid.reshape(-1, 1)).to(torch.float64)
    return onehot.T @ vals.reshape(-1, 4)


def replay_league_elo(records, num_agents, max_players, elo_initial=1600.0, elo_k=32.0):
    """sn_elo_replay over records [..., 1 + max_players] in row order"""
    rec = np.ascontiguousarray(records.reshape(-1, 1 + max_players).cpu().numpy(), dtype=np.int32)
    elos = np.full(num_agents, float(elo_initial), dtype=np.float64)
    nat.check(nat.lib().sn_elo_replay(rec.ctypes.data_as(ctypes.c_void_p), rec.shape[0], max_players, num_agents,
                                      float(elo_k), elos.ctypes.data_as(ctypes.c_void_p)), "sn_elo_replay")
    return elos
