"""Drop-in `Tournament` (reference: rl_6_nimmt/tournament.py:12-262).

A league of agents: random seatings of min..max players, per-game scoring
(relative position, win, multiplayer Elo), baseline evaluations and
evolutionary cloning / pruning.  Games are played by the drop-in
`GameSession` on the MI355X env.  Behaviour kept: `np.random.choice` for
the seat draw (tournament.py:166-177, same global-RNG calls), first-argmax
winner, `_compute_absolute_positions` returning 1-based ranks despite its
docstring (quirk Q10).  Elo: see elo.py (parity unpinned).
"""
import copy
import io
import logging

import numpy as np
import torch

from . import elo
from .play import GameSession

logger = logging.getLogger(__name__)

_PER_AGENT = ("active", "elos", "descendants", "played_games", "tournament_scores", "tournament_positions",
              "tournament_wins", "baseline_scores", "baseline_positions", "baseline_wins")


class Tournament:
    def __init__(self, min_players=2, max_players=4, baseline_agents=None, baseline_num_games=1, baseline_condition=10,
                 elo_initial=1600, elo_k=32):
        assert 0 < min_players <= max_players
        self.min_players, self.max_players = min_players, max_players
        self.baseline_agents = baseline_agents
        self.baseline_num_games = baseline_num_games
        self.baseline_condition = baseline_condition
        self.elo_initial, self.elo_k = elo_initial, elo_k
        self.total_games = 0
        self.agents = {}
        for name in _PER_AGENT:
            setattr(self, name, {})

    # ------------------------------------------------------------ roster
    def add_player(self, name, agent):
        assert name not in self.agents
        agent.__name__ = name  # the reference names agents this way (tournament.py:40)
        self.agents[name] = agent
        self.descendants[name] = name
        self.active[name] = True
        self.played_games[name] = 0
        for d in ("tournament_scores", "tournament_positions", "tournament_wins", "baseline_scores",
                  "baseline_positions", "baseline_wins"):
            getattr(self, d)[name] = []
        self.elos[name] = [self.elo_initial]

    def copy_player(self, old_name, new_name):
        for d in _PER_AGENT:
            getattr(self, d)[new_name] = copy.deepcopy(getattr(self, d)[old_name])
        # the reference round-trips the module through temp_model.pt in the
        # CWD because deepcopy failed on torch modules of its day; deepcopy
        # works now, with an in-memory save/load as the fallback
        try:
            clone = copy.deepcopy(self.agents[old_name])
        except Exception:
            buf = io.BytesIO()
            torch.save(self.agents[old_name], buf)
            buf.seek(0)
            clone = torch.load(buf, weights_only=False)  # our own object, serialised just above
        clone.__name__ = new_name
        self.agents[new_name] = clone

    def remove_player(self, name, full_delete=False):
        if not full_delete:
            self.active[name] = False
            return
        del self.agents[name]
        for d in _PER_AGENT:
            del getattr(self, d)[name]

    def active_agents(self):
        return [name for name in self.agents if self.active[name]]

    def __len__(self):
        return len(self.active_agents())

    # ------------------------------------------------------------ evolution (tournament.py:78-130)
    def evolve(self, copies=(2,), max_players=None, max_per_descendant=2, metric="elo"):
        table = {
            "tournament_scores": (self.tournament_scores, True, True),
            "tournament_positions": (self.tournament_positions, False, True),
            "tournament_wins": (self.tournament_wins, False, True),
            "elo": (self.elos, True, False),
        }
        if metric not in table:
            raise NotImplementedError(metric)
        scores, reverse, use_mean = table[metric]

        def key(name):
            vals = scores[name]
            if not vals:
                return 0.0
            return np.mean(vals) if use_mean else vals[-1]

        ranking = sorted(self.active_agents(), key=key, reverse=reverse)
        kept, per_family = 0, {}
        for pos, name in enumerate(ranking):
            family = self.descendants[name]
            per_family.setdefault(family, 0)
            if pos < len(copies):
                n_copies = copies[pos]
                logger.info(f"Copying player {name} into {n_copies} instances!")
            elif max_players is not None and kept >= max_players:
                n_copies = 0
                logger.info(f"Removing player {name}")
            elif max_per_descendant is not None and per_family[family] >= max_per_descendant:
                n_copies = 0
                logger.info(f"Removing player {name}")
            else:
                n_copies = 1
            for c in range(n_copies):
                self.copy_player(name, f"{name}_{c}")
            self.remove_player(name, full_delete=n_copies > 0)
            kept += n_copies
            per_family[family] += n_copies

    # ------------------------------------------------------------ games
    def play_game(self, num_players=None):
        names, agents = self._choose_players(num_players)
        session = GameSession(*agents)
        session.play_game(render=False)
        self.score_game(names, session.results[0])

    def score_game(self, agent_names, scores):
        rel = self._compute_relative_positions(scores)
        winner = agent_names[int(np.argmax(scores))]
        new_elos = self._compute_elos(agent_names, scores)
        self.total_games += 1
        for name, score, rp, e in zip(agent_names, scores, rel, new_elos):
            self.played_games[name] += 1
            self.tournament_scores[name].append(score)
            self.tournament_positions[name].append(rp)
            self.tournament_wins[name].append(1.0 if name == winner else 0.0)
            self.elos[name].append(e)
            if self.played_games[name] % self.baseline_condition == 0:
                self.baseline_eval(name)

    def _compute_elos(self, agent_names, scores):
        places = self._compute_absolute_positions(scores)
        players = [elo.EloPlayer(place=pl, elo=self.elos[n][-1]) for pl, n in zip(places, agent_names)]
        return elo.calc_elo(players, self.elo_k)

    def _choose_players(self, num_players):
        if num_players is None:
            num_players = np.random.choice(list(range(self.min_players, self.max_players + 1)), size=1)[0]
        assert len(self) >= num_players
        active = self.active_agents()
        idx = np.random.choice(len(active), size=num_players, replace=False)
        names = [active[i] for i in idx]
        return names, [self.agents[n] for n in names]

    def baseline_eval(self, agent_name):
        if self.baseline_agents is None:
            return
        session = GameSession(self.agents[agent_name], *self.baseline_agents)
        for _ in range(self.baseline_num_games):
            session.play_game(render=False)
        scores = np.mean(np.array(session.results), axis=0)
        rel = self._compute_relative_positions(scores)
        self.baseline_scores[agent_name].append(scores[0])
        self.baseline_positions[agent_name].append(rel[0])
        self.baseline_wins[agent_name].append(float(np.argmax(scores) == 0))

    def winner(self):
        best, best_agent = -float("inf"), None
        for name, agent in self.agents.items():
            m = np.mean(self.tournament_positions[name])
            if m > best:
                best, best_agent = m, agent
        return best_agent

    # ------------------------------------------------------------ table (tournament.py:208-238)
    def __str__(self):
        bar = "-----------------------------------------------------------------"
        out = [f"Tournament after {self.total_games} games:", bar,
               " Agent                | Games | Mean score | Win fraction |  ELO ", bar]

        def row(name):
            sc = self.tournament_scores[name]
            wn = self.tournament_wins[name]
            score = f"{np.mean(sc):>5.2f}" if sc else "-"
            wins = f"{np.mean(wn):>5.2f}" if wn else "-"
            return f" {name:>20s} | {self.played_games[name]:>5} | {score:>10} | {wins:>12} | {self.elos[name][-1]:>4.0f} "

        out += [row(n) for n in self.agents if self.active[n]]
        out.append(bar)
        out += [row(n) for n in self.agents if not self.active[n]]
        if out[-1] != bar:
            out.append(bar)
        return "\n".join(out)

    def __repr__(self):
        return self.__str__()

    # ------------------------------------------------------------ positions (tournament.py:240-256)
    @staticmethod
    def _compute_absolute_positions(scores):
        """1-based ranks, best first, ties averaged (the docstring upstream says 0-based; quirk Q10)."""
        s = np.asarray(scores, dtype=np.float64)
        neg = np.sort(-s)
        left = np.searchsorted(neg, -s - 0.5)
        right = 1.0 + np.searchsorted(neg, -s + 0.5)
        return (0.5 * (left + right)).astype(np.float32)

    @staticmethod
    def _compute_relative_positions(scores):
        """1 = best, 0 = worst, ties averaged."""
        s = np.asarray(scores, dtype=np.float64)
        srt = np.sort(s)
        left = np.searchsorted(srt, s + 0.5).astype(np.float32)
        right = 1.0 + np.searchsorted(srt, s - 0.5).astype(np.float32)
        pos = 0.5 * (left + right)
        return (pos - 1) / (len(s) - 1)
