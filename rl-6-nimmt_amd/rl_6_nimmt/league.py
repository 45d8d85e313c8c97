"""Batched tournament on the MI355X (BASELINE config 5).

Reference: Tournament (rl_6_nimmt/tournament.py:12-262) -- `play_game()`
draws the seats (`_choose_players`, :166-177), plays one GameSession game
(:132-138) and scores it (`score_game`, :140-164: relative positions, first-
argmax winner, order-dependent multiplayer Elo); `evolve` / `copy_player`
(:54-130) clone and prune the roster between games.

Here every slot g of a tournament handle (`sn_league_config`) is one
reference tournament stream: slot g replays

    np.random.seed(seed + game_offset + g)
    t = Tournament(min_players, max_players); t.add_player(name, agent) ...
    t.play_game()  # x games

All slots play at once; the games of all slots (and, over RCCL, of all
ranks) form one tournament whose scoring is per game (vectorised on the
device) and whose Elo -- the only order-dependent part -- is replayed on the
host in a canonical order: game round major, then global slot id
(`sn_elo_replay`, C++; multi_elo parity unpinned, elo.py).

Agents (the pool of run.py:20-40):
  * DrunkHamster -- drawn in-kernel from the slot's numpy stream;
  * MCSAgent -- card memory + the reference-exact search on the slot's
    stream (sn_league_step), so a league of DrunkHamster and MCSAgent seats
    replays the reference's seeded Tournament bit for bit (golden F11);
  * PUCTAgent / PolicyMCSAgent, PUCTCustomedAgent, BatchedACERAgent -- one
    batched engine per agent (puct.BatchedPUCT / BatchedPUCTCustomed,
    acer.BatchedACER) over the decision list of its seats in the slots'
    current games (sn_puct.dec_list); the policy net runs on PyTorch-ROCm.
    Their random draws are Philox, not torch's CPU generator (parity
    unpinned, like the engines themselves), and they consume no numpy words
    (the reference's _draw_env shuffles do), so a league with net agents is
    the reference's in law, not draw for draw.
All-DrunkHamster leagues play whole games per launch (sn_league_rollout,
`fused`); every other league plays sn_reset (seat draw + deal) then 10
sn_league_step launches per game round.

Training (train=True, like run.py's agent.train()): after each round every
net agent takes one Adam step on its loss summed over the round's games
(the reference steps once per game: puct.py / acer.py document the batched
losses).  Nets move to the tournament's device.
"""
import copy
import ctypes
import io
import logging

import numpy as np
import torch

from . import _native as nat
from .vec_env import VecSechsNimmtEnv

logger = logging.getLogger(__name__)

STAT_GAMES, STAT_SCORE, STAT_POSITION, STAT_WINS = range(4)
KIND_RANDOM, KIND_MCS, KIND_PUCT, KIND_CUSTOMED, KIND_ACER = "random", "mcs", "puct", "customed", "acer"
KIND_REINFORCE = "reinforce"
NET_KINDS = (KIND_PUCT, KIND_CUSTOMED, KIND_ACER, KIND_REINFORCE)
T_STEPS = 10


def agent_kind(agent):
    """the batched engine that plays `agent` (tournament.py seats any Agent)"""
    from .agents import BatchedACERAgent, BatchedReinforceAgent, DrunkHamster, MCSAgent, PolicyMCSAgent, PUCTCustomedAgent

    if isinstance(agent, PUCTCustomedAgent):
        return KIND_CUSTOMED
    if isinstance(agent, PolicyMCSAgent):  # PUCTAgent included
        return KIND_PUCT
    if isinstance(agent, MCSAgent):
        return KIND_MCS
    if isinstance(agent, BatchedACERAgent):
        return KIND_ACER
    if isinstance(agent, BatchedReinforceAgent):
        return KIND_REINFORCE
    if isinstance(agent, DrunkHamster):
        return KIND_RANDOM
    raise NotImplementedError(f"the batched tournament has no engine for {type(agent).__name__}")


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
    """A tournament played by `num_slots` concurrent game slots on one GPU
    (one rank's shard: global slot ids game_offset .. game_offset + num_slots - 1)."""

    def __init__(self, num_slots, min_players=2, max_players=4, seed=0, game_offset=0, rng="numpy", device=None,
                 elo_initial=1600, elo_k=32, net_dtype=torch.bfloat16, train=False, fused=True, distributed=False,
                 baseline_agents=None, baseline_num_games=1, baseline_condition=10, updates_per_round=1):
        """distributed=True: this handle is one rank's shard of ONE tournament
        over the initialised process group (every rank constructs it with the
        same roster and calls the same methods): the tallies and Elo that
        evolve / agent_stats / replay_elo use are folded from every rank's
        records (all_gather, canonical order), so every rank keeps the same
        roster.  Every accessor that folds records -- evolve, agent_stats,
        replay_elo, winner, table / __str__, copy_player, remove_player,
        clear_records -- is then a COLLECTIVE: all ranks must call it, in the
        same order (one rank alone blocks in the all_gather).  total_games
        counts every rank's games, and baseline evaluations draw from
        rank-independent streams, so the ranks' baseline lists agree.
        False: the tallies are this rank's own (reduce them with
        distributed.reduce_agent_stats), and evolve refuses to run on more
        than one rank.

        updates_per_round (train=True): Adam steps each PUCT / PUCTCustomed /
        REINFORCE agent takes per round.  The reference steps once per GAME
        the agent played (learn() at episode end, play.py:52-67,
        mcts.py:230-261); a round plays every slot's game at once, so its
        games' losses are split into k contiguous chunks (by slot) with one
        step each: 1 (default) = one step on the whole round's loss, "games"
        = one step per game played (the reference's count; every game's
        search still used the round's starting weights).  ACER keeps its own
        update schedule (acer.py).  optimizer_steps[name] counts the steps."""
        assert 0 < min_players <= max_players
        if updates_per_round != "games" and not (isinstance(updates_per_round, int) and updates_per_round >= 1):
            raise ValueError('updates_per_round must be an int >= 1 or "games"')
        self.updates_per_round = updates_per_round
        self.optimizer_steps = {}
        self._inherit = {}  # clone name -> its parent's engine (copy_player), until the clone's engine exists
        self._dirty = False  # the roster changed since the handle was configured
        self.num_slots, self.min_players, self.max_players = int(num_slots), int(min_players), int(max_players)
        self.seed, self.game_offset, self.rng, self.device = int(seed), int(game_offset), rng, device
        self.elo_initial, self.elo_k = float(elo_initial), float(elo_k)
        self.net_dtype, self.train, self.fused = net_dtype, bool(train), bool(fused)
        self.distributed = bool(distributed)
        # baseline evaluations (tournament.py:13-24,147-155,182-195): each time an
        # agent's played-game count reaches a multiple of baseline_condition, one
        # GameSession(agent, *baseline_agents) of baseline_num_games games;
        # played here as batched sessions on their own handle (see _baselines)
        self.baseline_agents = list(baseline_agents) if baseline_agents is not None else None
        self.baseline_num_games, self.baseline_condition = int(baseline_num_games), int(baseline_condition)
        self.baseline_scores, self.baseline_positions, self.baseline_wins = {}, {}, {}
        self._baseline_calls = 0
        # phase_timing = True: _round records HIP events around its phases on
        # the stream (no synchronisation in between) and sums them, with the
        # host's enqueue time of each phase, into phase_ms / phase_host_ms
        self.phase_timing = False
        self.phase_ms, self.phase_host_ms = {}, {}
        # the roster, in the reference's dict order (tournament.py:25-35)
        self.names, self.agents, self.active, self.descendants, self.kinds = [], {}, {}, {}, {}
        self.env = None
        self.mode = None  # "fused" (all DrunkHamster, sn_league_rollout) or "step" (sn_league_step)
        self.engines = {}  # net agent name -> batched engine
        self.records = []  # (int32 [games, slots, 1 + N] on the device, roster index of each active agent)
        self.record_names = []  # the active agents' names of each records block (roster indices shift on deletes)
        self.stats = np.zeros((0, 4), dtype=np.float64)  # per roster agent: games, score, position, wins
        self.elos = np.zeros((0,), dtype=np.float64)     # current Elo per roster agent
        # per roster agent, its relative positions as the reference keeps them
        # (float32, tournament.py:249-256) in play order -- (round, global
        # slot) order here: evolve's "tournament_positions" key and winner()
        # are np.mean over exactly this sequence, as the reference's are
        self.positions = {}
        self.total_games = 0
        self.q6_slot_rounds = 0  # (slot, round) pairs with an MCS decision where a legal move got no playout (Q6)
        self._seen = 0  # records already folded into stats / elos

    # ------------------------------------------------------------ roster (tournament.py:36-76)
    def add_player(self, name, agent=None):
        from .agents.random import DrunkHamster

        assert name not in self.agents
        if self.mode == "fused":
            raise NotImplementedError("the fused all-DrunkHamster league has drawn its next seats already; add every "
                                      "player before the first game (or use fused=False)")
        agent = DrunkHamster() if agent is None else agent
        kind = agent_kind(agent)
        agent.__name__ = name  # tournament.py:40
        self.names.append(name)
        self.agents[name], self.kinds[name] = agent, kind
        self.active[name], self.descendants[name] = True, name
        self.stats = np.concatenate((self.stats, np.zeros((1, 4))), axis=0)
        self.elos = np.concatenate((self.elos, [self.elo_initial]))
        self.positions[name] = []
        self.baseline_scores[name], self.baseline_positions[name], self.baseline_wins[name] = [], [], []
        if self.env is not None:
            self._configure()

    def copy_player(self, old_name, new_name, _defer=False):
        """tournament.py:54-60: the clone inherits the tallies, Elo, family and
        (ACER) replay (the reference round-trips the module through
        temp_model.pt); it plays from the next game on"""
        if self.mode == "fused" and not _defer:
            raise NotImplementedError("the fused all-DrunkHamster league has drawn its next seats already; change the "
                                      "roster before the first game (or use fused=False)")
        self._fold()
        try:
            clone = copy.deepcopy(self.agents[old_name])
        except Exception:
            buf = io.BytesIO()
            torch.save(self.agents[old_name], buf)
            buf.seek(0)
            clone = torch.load(buf, weights_only=False)  # our own object, serialised just above
        i = self.names.index(old_name)
        clone.__name__ = new_name
        self.names.append(new_name)
        self.agents[new_name], self.kinds[new_name] = clone, self.kinds[old_name]
        self.active[new_name], self.descendants[new_name] = self.active[old_name], self.descendants[old_name]
        self.stats = np.concatenate((self.stats, self.stats[i: i + 1]), axis=0)
        self.elos = np.concatenate((self.elos, self.elos[i: i + 1]))
        self.positions[new_name] = list(self.positions[old_name])
        for d in (self.baseline_scores, self.baseline_positions, self.baseline_wins):
            d[new_name] = list(d[old_name])
        if old_name in self.engines:  # the clone's engine (made at the next _configure) inherits its replay
            self._inherit[new_name] = self.engines[old_name]
        self._dirty = True  # the handle is reconfigured before the next game

    def remove_player(self, name, full_delete=False, _defer=False):
        """tournament.py:62-76 (from the next game on)"""
        if self.mode == "fused" and not _defer:
            raise NotImplementedError("the fused all-DrunkHamster league has drawn its next seats already; change the "
                                      "roster before the first game (or use fused=False)")
        self._fold()
        if full_delete:
            i = self.names.index(name)
            self.names.pop(i)
            for d in (self.agents, self.kinds, self.active, self.descendants, self.positions, self.baseline_scores,
                      self.baseline_positions, self.baseline_wins):
                del d[name]
            self.stats = np.delete(self.stats, i, axis=0)
            self.elos = np.delete(self.elos, i)
            self.engines.pop(name, None)
        else:
            self.active[name] = False
        self._dirty = True  # the handle is reconfigured before the next game

    def active_agents(self):
        return [n for n in self.names if self.active[n]]

    def __len__(self):
        return len(self.active_agents())

    def evolve(self, copies=(2,), max_players=None, max_per_descendant=2, metric="elo"):
        """tournament.py:78-130 on the batched tallies: rank the active agents
        by `metric`, clone the top ones, prune past max_players / per family.
        The next round's seats are drawn over the new active list."""
        if self.mode == "fused":
            raise NotImplementedError("evolve needs the per-game round (BatchedTournament(..., fused=False)): the fused "
                                      "rollout draws each slot's next seats at the end of the game before")
        from .distributed import world_size

        if world_size() > 1 and not self.distributed:
            raise RuntimeError("evolve on one rank's shard would rank the agents by that rank's games only and let "
                               "the ranks' rosters diverge: construct the tournament with distributed=True")
        self._fold()
        s = self.stats
        table = {"tournament_scores": (STAT_SCORE, True, True), "tournament_positions": (STAT_POSITION, False, True),
                 "tournament_wins": (STAT_WINS, False, True), "elo": (None, True, False)}
        if metric not in table:
            raise NotImplementedError(metric)
        col, reverse, use_mean = table[metric]

        def key(name):
            # the reference's keys (tournament.py:98-101): np.mean of the
            # agent's list, 0. when empty; Elo: the latest value.  Scores and
            # wins are integers / 0-1 floats, so their float64 mean is the sum
            # over the count exactly; positions are float32 values whose
            # float32 np.mean depends on their order, kept in self.positions
            i = self.names.index(name)
            if not use_mean:
                return float(self.elos[i])  # the latest Elo (never empty)
            g = s[i, STAT_GAMES]
            if g == 0:
                return 0.0
            if col == STAT_POSITION:
                return np.mean(np.concatenate(self.positions[name]))
            return float(s[i, col] / g)

        ranking = sorted(self.active_agents(), key=key, reverse=reverse)
        kept, per_family = 0, {}
        for pos, name in enumerate(ranking):
            fam = self.descendants[name]
            per_family.setdefault(fam, 0)
            if pos < len(copies):
                n_copies = copies[pos]
                logger.info(f"Copying player {name} into {n_copies} instances!")
            elif max_players is not None and kept >= max_players:
                n_copies = 0
                logger.info(f"Removing player {name}")
            elif max_per_descendant is not None and per_family[fam] >= max_per_descendant:
                n_copies = 0
                logger.info(f"Removing player {name}")
            else:
                n_copies = 1
            for c in range(n_copies):
                self.copy_player(name, f"{name}_{c}", _defer=True)
            self.remove_player(name, full_delete=n_copies > 0, _defer=True)
            kept += n_copies
            per_family[fam] += n_copies
        if self.env is not None:
            self._configure()

    # ------------------------------------------------------------ the handle
    def _start(self):
        K = len(self)
        assert K >= self.max_players, "tournament.py:170: len(self) >= num_players"
        all_random = all(self.kinds[n] == KIND_RANDOM for n in self.active_agents())
        self.mode = "fused" if (self.fused and all_random) else "step"
        if self.mode == "step" and self.rng != "numpy":
            raise NotImplementedError("mixed leagues play numpy-MT tournament streams (rng='numpy')")
        self.env = VecSechsNimmtEnv(self.num_slots, self.max_players, seed=self.seed, game_offset=self.game_offset,
                                    rng=self.rng, device=self.device)
        self._configure()
        if self.mode == "fused":
            self.env.reset()  # every slot draws its first seats, then deals

    def _configure(self):
        """(re)configure the handle for the current active roster"""
        act = self.active_agents()
        K = len(act)
        if K > 16:
            raise NotImplementedError("a tournament handle seats at most 16 active agents")
        L = nat.lib()
        nat.check(L.sn_league_config(self.env._h, K, self.min_players, self.max_players), "sn_league_config")
        kind_code = {KIND_RANDOM: nat.SN_AGENT_RANDOM, KIND_MCS: nat.SN_AGENT_MCS}
        kinds = np.array([kind_code.get(self.kinds[n], nat.SN_AGENT_EXTERNAL) for n in act], dtype=np.int32)
        mpc = np.array([getattr(self.agents[n], "mc_per_card", 10) for n in act], dtype=np.int32)
        mmax = np.array([getattr(self.agents[n], "mc_max", 100) for n in act], dtype=np.int32)
        P = ctypes.c_void_p
        nat.check(L.sn_league_agents(self.env._h, P(kinds.ctypes.data), P(mpc.ctypes.data), P(mmax.ctypes.data)),
                  "sn_league_agents")
        self._ids = torch.tensor([self.names.index(n) for n in act], dtype=torch.long)
        self._dirty = False
        keep = {}
        for n in act:
            if self.kinds[n] in NET_KINDS:
                eng = self.engines.get(n)
                if eng is None:
                    eng = self._engine(n)
                    parent = self._inherit.pop(n, None)
                    if parent is not None:
                        inherit_replay(eng, parent)
                keep[n] = eng
        self.engines = keep
        self._inherit.clear()

    def _engine(self, name):
        """the batched engine of one net agent over this handle (decision-list mode)"""
        from .acer import BatchedACER
        from .puct import BatchedPUCT, BatchedPUCTCustomed
        from .reinforce import BatchedReinforce

        agent, kind, env = self.agents[name], self.kinds[name], self.env
        agent.to(env.device)
        agent.device = env.device
        seed = (self.seed * 1000003 + self.names.index(name) * 7919 + self.game_offset) & (2**62 - 1)
        B = self.num_slots
        if kind == KIND_PUCT:
            return BatchedPUCT(env, agent.actor, mc_per_card=agent.mc_per_card, mc_max=agent.mc_max,
                               c_puct=getattr(agent, "c_puct", 2.0), seed=seed, puct_root=agent._puct_root,
                               net_dtype=self.net_dtype, mcs_num_cards=agent.num_cards, max_decisions=B)
            # whole rollouts per kernel (sn_puct_rollouts) since round 6: 0.783 vs 0.822-0.827 s per run.py
            # league round against a launch per step (gpurun_out/r06_mixed3)
        if kind == KIND_CUSTOMED:
            return BatchedPUCTCustomed(env, agent.actor, net_dtype=self.net_dtype, seed=seed, max_decisions=B)
        if kind == KIND_REINFORCE:
            return BatchedReinforce(env, agent.actor, net_dtype=self.net_dtype, seed=seed, gamma=agent.gamma,
                                    r_factor=agent.r_factor, actor_weight=agent.actor_weight,
                                    entropy_weight=agent.entropy_weight, max_decisions=B)
        # replay rounds: enough that the stored sequences (every seat of the
        # agent in each kept round, ceil(10 / rollout_len) per seat) pass
        # max(warmup, minibatch), from the expected seats per round
        K = max(1, len(self.active_agents()))
        seats = B * (self.min_players + self.max_players) / 2.0 / K
        chunks = -(-T_STEPS // int(agent.rollout_len))
        need = max(int(agent.warmup), int(agent.batchsize)) + 1
        capacity = max(2, int(-(-need // max(1.0, seats * chunks))) + 1)
        return BatchedACER(env, agent.actor_critic, net_dtype=self.net_dtype, seed=seed, gamma=agent.gamma,
                           rollout_len=agent.rollout_len, minibatch=agent.batchsize, truncate=agent.truncate,
                           warmup=agent.warmup, r_factor=agent.r_factor, critic_weight=agent.critic_weight,
                           capacity=capacity, log_epsilon=agent.log_epsilon, max_decisions=B)

    # ------------------------------------------------------------ games (tournament.py:132-138)
    def play_games(self, games=1, rewards=False):
        """`games` tournament games per slot.  Returns the records int32
        [games, num_slots, 1 + max_players]: seats word (k | active agent
        index of seat p << (4 + 4p)), then the results (GameSession.results[0],
        0 past k); with rewards=True also the per-step rewards [10 games, slots, N]."""
        if self.env is None:
            self._start()
        elif self._dirty:
            self._configure()  # copy_player / remove_player since the last game (tournament.py:170 asserts here)
        env = self.env
        if self.mode == "fused":
            T = T_STEPS * int(games)
            rec = torch.empty((games, self.num_slots, 1 + self.max_players), dtype=torch.int32, device=env.device)
            rew = torch.empty((T, self.num_slots, self.max_players), dtype=torch.int32, device=env.device) if rewards else None
            nat.check(nat.lib().sn_league_rollout(env._h, T, nat.ptr(rew), None, None, None, 0, nat.ptr(rec), env._stream()),
                      "sn_league_rollout")
        else:
            recs, rews = [], []
            for _ in range(int(games)):
                r, w = self._round()
                recs.append(r)
                rews.append(w)
            rec = torch.stack(recs, dim=0)
            rew = torch.cat(rews, dim=0) if rewards else None
        self.records.append((rec, self._ids.clone()))
        self.record_names.append(tuple(self.active_agents()))
        world = 1
        if self.distributed:
            from .distributed import world_size

            world = world_size()  # every rank plays the same number of slots per round
        self.total_games += int(games) * self.num_slots * world
        return (rec, rew) if rewards else rec

    def _phase(self, name):
        """context of one timed phase of _round (no-op unless phase_timing)"""
        import contextlib
        import time

        if not self.phase_timing:
            return contextlib.nullcontext()
        t = self

        class _P:
            def __enter__(self):
                self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                self.ev[0].record()
                self.h = time.perf_counter()

            def __exit__(self, *exc):
                self.ev[1].record()
                t._phase_events.append((name, self.ev))
                t.phase_host_ms[name] = t.phase_host_ms.get(name, 0.0) + (time.perf_counter() - self.h) * 1e3
                return False

        return _P()

    def _phase_collect(self):
        if self.phase_timing and getattr(self, "_phase_events", None):
            torch.cuda.synchronize(self.env.device)
            for name, (a, b) in self._phase_events:
                self.phase_ms[name] = self.phase_ms.get(name, 0.0) + a.elapsed_time(b)
        self._phase_events = []

    def _round(self):
        """one game per slot: sn_reset (seat draw + deal), then 10 x [net
        agents' engines on their seats -> sn_league_step]"""
        env, L, st = self.env, nat.lib(), self.env._stream()
        B, N, dev = self.num_slots, self.max_players, env.device
        self._phase_events = []
        with self._phase("reset (seat draw + deal) + decision lists"):
            nat.check(L.sn_reset(env._h, None, st), "sn_reset")  # Tournament.play_game: seats, then the deal
            self._use_decisions()
        acts = torch.zeros((B, N), dtype=torch.int32, device=dev)
        per_step = torch.zeros((T_STEPS, B, N), dtype=torch.int32, device=dev)
        rec = torch.zeros((B, 1 + N), dtype=torch.int32, device=dev)
        invalid = torch.empty((T_STEPS, B), dtype=torch.int32, device=dev)
        status = torch.zeros((B,), dtype=torch.int32, device=dev)
        flat_acts = acts.view(-1)
        for t in range(T_STEPS):
            n = T_STEPS - t
            for name, eng in self.engines.items():
                if eng.D == 0:
                    continue
                with self._phase(f"decide {name}"):
                    a = eng.decide(n, record=self.train)
                    idx = eng.dec.long()
                    flat_acts[idx] = a.reshape(-1)[idx]
            with self._phase("league step (MCS + DrunkHamster seats, resolution)"):
                nat.check(L.sn_league_step(env._h, nat.ptr(acts), nat.ptr(per_step[t]), None,
                                           nat.ptr(rec) if t == T_STEPS - 1 else None, nat.ptr(invalid[t]),
                                           nat.ptr(status), st), "sn_league_step")
        if self.engines:  # external seats played: an illegal card fails the round (sechs.h) -- checked once
            # per round, not per step: a host read-back per step kept the host from enqueueing the next
            # step's searches while the GPU ran this one
            bad = (invalid >= 0).sum(dim=1).cpu()
            if int(bad.sum()):
                t = int(torch.nonzero(bad).flatten()[0])
                raise RuntimeError(f"sn_league_step: {int(bad[t])} illegal moves of the net agents' engines at step {t}")
        q6 = int(status.sum())
        if q6:
            self.q6_slot_rounds += q6
            logger.warning("MCS: a legal move got no playout (the reference raises IndexError here, quirk Q6)")
        if self.train:
            self._learn(per_step)
        self._phase_collect()
        return rec, per_step

    def _use_decisions(self):
        if self.engines:
            k, ids = self.seats()
            flat = ids.reshape(-1)
            act = self.active_agents()
            for name, eng in self.engines.items():
                eng.use_decisions(torch.nonzero(flat == act.index(name)).flatten())
                eng.decisions = []

    def _learn(self, per_step):
        """one Adam step per net agent on its loss over the round's games"""
        from .acer import BatchedACER
        from .puct import BatchedPUCTCustomed
        from .reinforce import BatchedReinforce

        for name, eng in self.engines.items():
            agent = self.agents[name]
            if agent.optimizer is None:
                agent.train()
            with self._phase(f"learn {name}"):
                if isinstance(eng, BatchedACER):
                    if eng.D:
                        eng.record_rewards(per_step)
                        eng.learn(agent.optimizer)
                    continue
                if eng.D == 0 or not eng.decisions:
                    continue
                # one decider per game of this agent (a game seats distinct agents):
                # k contiguous decider ranges = k chunks of games
                D = int(eng.D)
                k = D if self.updates_per_round == "games" else min(int(self.updates_per_round), D)
                bounds = [D * c // k for c in range(k + 1)]
                for d0, d1 in zip(bounds[:-1], bounds[1:]):
                    if isinstance(eng, (BatchedPUCTCustomed, BatchedReinforce)):
                        loss = eng.loss(per_step, d0, d1) if k > 1 else eng.loss(per_step)
                    else:
                        loss = eng.policy_loss(d0, d1) if k > 1 else eng.policy_loss()
                    agent.optimizer.zero_grad()
                    loss.backward()
                    agent.optimizer.step()
                    self.optimizer_steps[name] = self.optimizer_steps.get(name, 0) + 1
                eng.decisions = []

    def seats(self):
        """(k [slots], active agent index [slots, max_players]) of every slot's current game"""
        out = torch.empty((self.num_slots,), dtype=torch.int32, device=self.env.device)
        nat.check(nat.lib().sn_league_seats(self.env._h, nat.ptr(out), self.env._stream()), "sn_league_seats")
        return decode_seats(out, self.max_players)

    # ------------------------------------------------------------ scoring (tournament.py:140-164)
    def _fold(self):
        """fold records not yet seen into the per-agent tallies and Elo (in
        play order: the Elo is sequential, tournament.py:157-164)"""
        while self._seen < len(self.records):
            rec, ids = self.records[self._seen]
            if self.distributed:  # every rank's games of this block, in global slot order
                from .distributed import gather_league_records

                rec = gather_league_records(rec)
            K = int(ids.numel())
            s = league_agent_stats(rec, K, self.max_players).cpu().numpy()
            played_before = self.stats[ids.numpy(), STAT_GAMES].copy()
            np.add.at(self.stats, ids.numpy(), s)
            if self.baseline_agents is not None:
                c = self.baseline_condition
                evals = (self.stats[ids.numpy(), STAT_GAMES] // c - played_before // c).astype(np.int64)
                for name, k in zip(self.record_names[self._seen], evals):
                    if k > 0:
                        self._baselines(name, int(k))
            for name, pos in zip(self.record_names[self._seen], league_positions32(rec, K, self.max_players)):
                self.positions[name].append(pos)
            sub = replay_league_elo(rec, K, self.max_players, 0.0, self.elo_k, initial=self.elos[ids.numpy()])
            self.elos[ids.numpy()] = sub
            self._seen += 1

    def all_records(self):
        """every game played so far, [games, slots, 1 + N] (round major).
        Seat ids index the active list of their round, so the blocks of
        rounds played under different rosters (evolve, copy_player,
        remove_player in between) cannot share one tensor: use
        `records_by_roster()` then."""
        if not self.records:
            return torch.zeros((0, self.num_slots, 1 + self.max_players), dtype=torch.int32)
        ids0 = self.records[0][1]
        if any(not torch.equal(ids, ids0) for _, ids in self.records[1:]):
            raise ValueError("the records span a roster change (seat ids index each round's active list): use "
                             "records_by_roster()")
        return torch.cat([r for r, _ in self.records], dim=0)

    def _baselines(self, name, evals):
        """`evals` baseline evaluations of agent `name` (tournament.py:182-195):
        each one GameSession(agent, *baseline_agents).play_game() x
        baseline_num_games; scores = the per-seat mean over those games,
        relative positions and the win flag in that seat order (the agent
        first).  Batched: one slot per evaluation on a tournament handle of
        its own whose every game seats all 1 + len(baseline_agents) agents; a
        slot's seat order is a drawn permutation and the per-seat means are
        taken back into the agent-first order, so the evaluation is the
        reference's in law (the game treats seats alike), and its games draw
        from their own streams -- the reference's draw from the tournament's
        global stream, so with baseline agents a slot's later games are no
        longer the seeded reference tournament's draw for draw."""
        from .tournament import Tournament

        K = 1 + len(self.baseline_agents)
        self._baseline_calls += 1
        # a distributed tournament folds the same records on every rank and so
        # runs the same evaluations there: their streams must not depend on
        # the rank's slot offset, or the ranks' baseline lists would diverge
        shard_off = 0 if self.distributed else self.game_offset
        off = (0x40000000 + self._baseline_calls * 0x10000 + shard_off) & 0x7FFFFFFF
        bt = BatchedTournament(evals, K, K, seed=self.seed, game_offset=off, rng="numpy", device=self.device,
                               net_dtype=self.net_dtype, train=False)
        seated = [self.agents[name]] + self.baseline_agents
        names = [getattr(a, "__name__", None) for a in seated]
        for j, a in enumerate(seated):
            bt.add_player("agent" if j == 0 else f"baseline{j - 1}", a)
        rec = bt.play_games(self.baseline_num_games)
        bt.close()
        for a, n in zip(seated, names):  # add_player renamed them (tournament.py:40); the evaluation does not
            if n is not None:
                a.__name__ = n
        k, ids = decode_seats(rec[..., 0], K)
        res = rec[..., 1:].to(torch.float64)  # [games, evals, seat]
        by_agent = torch.zeros_like(res).scatter_(-1, ids.clamp(min=0), res)  # seat -> agent order
        means = by_agent.mean(dim=0).cpu().numpy()  # np.mean over the session's results, per agent
        for sc in means:
            rel = Tournament._compute_relative_positions(sc)
            self.baseline_scores[name].append(sc[0])
            self.baseline_positions[name].append(rel[0])
            self.baseline_wins[name].append(float(np.argmax(sc) == 0))

    def clear_records(self):
        """fold the records so far into the tallies, then drop them (the
        tallies, Elo and position lists keep every game)"""
        self._fold()
        self.records.clear()
        self.record_names.clear()
        self._seen = 0

    def records_by_roster(self):
        """[(records [games, slots, 1 + N], the names of the active agents the
        seat ids of those records index)] -- one entry per play_games call"""
        return [(r, list(names)) for (r, _), names in zip(self.records, self.record_names)]

    def winner(self):
        """tournament.py:197-206: the agent (active or not) with the best mean
        relative position, first in roster order on ties; agents without
        games have a NaN mean and never win"""
        self._fold()
        best, best_agent = -float("inf"), None
        for name in self.names:
            p = self.positions[name]
            with np.errstate(all="ignore"):
                m = np.mean(np.concatenate(p)) if p else np.float64("nan")
            if m > best:
                best, best_agent = m, self.agents[name]
        return best_agent

    def _to_roster(self, active_vals, fill):
        """values per active agent (this roster's current active list) -> roster rows"""
        out = np.full((len(self.names),) + tuple(active_vals.shape[1:]), fill, dtype=np.float64)
        out[self._active_ids().numpy()] = active_vals
        return out

    def _active_ids(self):
        return torch.tensor([self.names.index(n) for n in self.active_agents()], dtype=torch.long)

    def agent_stats(self, records=None):
        """per-agent sums float64 [roster, 4]: games played, score, relative
        position, wins.  `records` (seat ids indexing the CURRENT active
        list) are mapped onto the roster rows through it."""
        if records is not None:
            K = len(self.active_agents())
            s = league_agent_stats(records, K, self.max_players).cpu().numpy()
            return torch.from_numpy(self._to_roster(s, 0.0))
        self._fold()
        return torch.from_numpy(self.stats.copy())

    def replay_elo(self, records=None):
        """Elo of every roster agent after the games so far (round major, then
        global slot id -- sn_elo_replay, host C++).  With `records` (seat ids
        indexing the current active list): the Elo those games alone give,
        every agent starting from elo_initial."""
        if records is not None:
            K = len(self.active_agents())
            e = replay_league_elo(records, K, self.max_players, self.elo_initial, self.elo_k)
            return self._to_roster(e, self.elo_initial)
        self._fold()
        return self.elos.copy()

    def table(self, stats=None, elos=None):
        """the reference's tournament table (tournament.py:208-238) from the sums"""
        stats = self.agent_stats() if stats is None else stats
        elos = self.replay_elo() if elos is None else elos
        s = stats.cpu().numpy() if hasattr(stats, "cpu") else np.asarray(stats)
        total = self.total_games  # tournament.py:211 (clones inherit tallies: a sum over rows would double count)
        bar = "-----------------------------------------------------------------"
        out = [f"Tournament after {total} games:", bar,
               " Agent                | Games | Mean score | Win fraction |  ELO ", bar]

        def row(i, name):
            g = s[i, STAT_GAMES]
            score = f"{s[i, STAT_SCORE] / g:>5.2f}" if g else "-"
            wins = f"{s[i, STAT_WINS] / g:>5.2f}" if g else "-"
            return f" {name:>20s} | {int(g):>5} | {score:>10} | {wins:>12} | {elos[i]:>4.0f} "

        out += [row(i, n) for i, n in enumerate(self.names) if self.active[n]]
        out.append(bar)
        out += [row(i, n) for i, n in enumerate(self.names) if not self.active[n]]
        if out[-1] != bar:
            out.append(bar)
        return "\n".join(out)

    def __str__(self):
        return self.table()

    def close(self):
        if self.env is not None:
            self.env.close()
            self.env = None


def inherit_replay(dst, src):
    """a clone's ACER engine starts from its parent's replay, as the
    reference's copy_player carries the agent's history through its
    torch.save round trip (tournament.py:54-60, the agent's
    SequentialHistory): the parent's most recent episodes, oldest first, up
    to the clone's capacity.  Other engines keep nothing across rounds."""
    from .acer import BatchedACER

    if not (isinstance(dst, BatchedACER) and isinstance(src, BatchedACER)):
        return
    if dst.rep_rows.shape[1:] != src.rep_rows.shape[1:]:
        return
    n = min(src.episodes, src.capacity, dst.capacity)
    with torch.no_grad():
        for k in range(n):
            e = src.episodes - n + k
            a, b = e % src.capacity, k % dst.capacity
            dst.rep_rows[b].copy_(src.rep_rows[a])
            dst.rep_act[b].copy_(src.rep_act[a])
            dst.rep_logp[b].copy_(src.rep_logp[a])
            dst.rep_rew[b].copy_(src.rep_rew[a])
            dst.rep_nd[b] = src.rep_nd[a]
    dst.episodes = n


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


def league_positions32(records, num_agents, max_players):
    """per active agent id, the float32 relative positions of its seats in
    records [..., 1 + N], in row order (the reference's tournament_positions
    entries: _compute_relative_positions in float32, tournament.py:249-256)"""
    rec = records.reshape(-1, 1 + max_players)
    k, ids = decode_seats(rec[:, 0], max_players)
    rel = relative_positions(rec[:, 1:], k).to(torch.float32).cpu().numpy()
    ids = ids.cpu().numpy()
    return [rel[ids == a] for a in range(num_agents)]


def replay_league_elo(records, num_agents, max_players, elo_initial=1600.0, elo_k=32.0, initial=None):
    """sn_elo_replay over records [..., 1 + max_players] in row order
    (starting from `initial` [num_agents] if given)"""
    rec = np.ascontiguousarray(records.reshape(-1, 1 + max_players).cpu().numpy(), dtype=np.int32)
    if initial is None:
        elos = np.full(num_agents, float(elo_initial), dtype=np.float64)
    else:
        elos = np.ascontiguousarray(initial, dtype=np.float64).copy()
    nat.check(nat.lib().sn_elo_replay(rec.ctypes.data_as(ctypes.c_void_p), rec.shape[0], max_players, num_agents,
                                      float(elo_k), elos.ctypes.data_as(ctypes.c_void_p)), "sn_elo_replay")
    return elos
