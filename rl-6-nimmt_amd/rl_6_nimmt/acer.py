"""Batched ACER self-play and training on one MI355X.

Reference: BatchedACERAgent (agents/actor_critic.py:119-207), AGENTS["acer"].
Every deciding seat of every game acts together: per decision batch one
sn_puct_root_rows launch (normalised `[card, obs]` candidate rows straight
from the device state), one forward of the 2-head net (policy logit, q) on
PyTorch-ROCm, one sn_policy_sample launch (Philox softmax sample over the
legal cards, log pi).  The reference draws from exp(clamp(log pi, -20)) over
10 padded slots and re-draws pad hits, i.e. from softmax over the legal cards
except that a card below e^-20 keeps e^-20: the sampler here is the exact
softmax (Philox: parity unpinned bitwise, frequency-tested).

Replay on the device (the reference's SequentialHistory of Python lists):
`capacity` episodes x 10 steps x D deciders of padded candidate rows (fp32,
the rows the training forward sees), chosen slot, behaviour log pi (padded
with log_epsilon = -20 like actor_critic.py:108-111) and reward x r_factor.
A decider's episode splits into sequences of rollout_len steps (the last one
ends at done), exactly where the reference flushes (actor_critic.py:146).

Training (actor_critic.py:153-207), per decider d over a batch of its
sequences, vectorised over deciders and sequences:
    v      = sum_a q(a) pi(a)                 rho = pi_now / pi_then
    q_ret  = Retrace target, walked backwards within each sequence
    actor  = mean -min(rho_a, c) log pi(a) (q_ret - v)
    corr   = mean sum_a -max(0, 1 - c/rho) pi_then log pi (q - v)
    critic = critic_weight * mean SmoothL1(q(a), q_ret)
and the batch loss is the sum over deciders of actor + corr + critic (the
reference takes one Adam step per agent and sequence batch).  `learn()`
follows the reference's schedule: after every flushed sequence, once more
than max(warmup, minibatch) sequences are stored, one on-policy update (the
newest sequence of every decider) and one off-policy update (`minibatch`
stored sequences per decider, drawn without replacement on the device).
"""
import os
import warnings

import torch
from torch import nn

from . import _native as nat
from .puct import ROW, BatchedPUCT, ctypes_ref
from .splitk import SplitKLinear, splitk_wgrad, train_forward  # noqa: F401  (re-exported)
from .utils.nets import MultiHeadedMLP

T_STEPS = 10


def default_capacity(rollout_len=10, minibatch=5, warmup=100):
    """replay episodes that let learn() start: the reference's SequentialHistory
    is unbounded (agents/base.py history_length=None), so its warmup of
    `warmup` sequences is always reached; a ring of C episodes stores
    C * ceil(10 / rollout_len) sequences, which must exceed max(warmup, minibatch)"""
    chunks = -(-T_STEPS // int(rollout_len))
    need = max(int(warmup), int(minibatch)) + 1
    return max(4, -(-need // chunks) + 1)


def replay_bytes(capacity, decisions):
    """device bytes of a replay of `capacity` episodes x 10 steps x
    `decisions` deciders: fp32 candidate rows [10][48], chosen slot (int64),
    behaviour log pi [10] and reward (fp32)"""
    return int(capacity) * T_STEPS * int(decisions) * (10 * ROW * 4 + 8 + 10 * 4 + 4)


MAX_REPLAY_BYTES = 128 << 30  # default cap on one engine's replay (and at most 80 % of the free device memory)


def make_actor_critic(hidden_sizes=(100, 100), activation=None):
    """the reference's net (actor_critic.py:44-46): MultiHeadedMLP(48, (100, 100), (1, 1)) -- policy logit, q"""
    return MultiHeadedMLP(ROW, hidden_sizes=hidden_sizes, head_sizes=(1, 1), activation=activation or nn.ReLU(),
                          head_activations=(None, None))


def distinct_picks(S, rows, k, gen, dev):
    """[rows, k] indices into range(S), each row k DISTINCT uniform picks
    (random.sample per row, as the reference draws its off-policy batch):
    pick j is uniform over the S - j values not picked yet -- x uniform in
    [0, S - j), then stepped past the row's earlier picks in ascending order
    (x + 1 for each one <= x) -- so every ordered k-tuple of distinct values
    is equally likely.  A fixed amount of device work, no host sync (the
    round-5 rejection loop read a duplicate count back every round)."""
    if k > S:
        raise ValueError(f"sample of {k} distinct sequences from {S}")
    cols, taken = [], None  # taken: the row's picks so far, ascending
    for j in range(k):
        x = torch.randint(0, S - j, (rows, 1), generator=gen, device=dev)
        if taken is not None:
            for m in range(j):  # ascending: each earlier pick at or below x shifts it up by one
                x = x + (x >= taken[:, m:m + 1]).to(x.dtype)
        cols.append(x)
        taken = x if taken is None else torch.cat((taken, x), dim=1).sort(dim=1).values
    return torch.cat(cols, dim=1)


class BatchedACER(BatchedPUCT):
    def __init__(self, env, actor=None, seats_mask=None, net_dtype=torch.bfloat16, seed=0, gamma=0.99, rollout_len=10,
                 minibatch=5, truncate=1.0, warmup=100, r_factor=0.1, critic_weight=1.0, capacity=None,
                 log_epsilon=-20.0, max_decisions=None, max_replay_bytes=None):
        super().__init__(env, actor if actor is not None else make_actor_critic(), seed=seed, seats_mask=seats_mask,
                         puct_root=False, net_dtype=net_dtype, max_decisions=max_decisions)
        self.gamma, self.truncate, self.r_factor = float(gamma), float(truncate), float(r_factor)
        self.rollout_len, self.minibatch, self.warmup = int(rollout_len), int(minibatch), int(warmup)
        self.critic_weight, self.log_epsilon = float(critic_weight), float(log_epsilon)
        self.capacity = default_capacity(rollout_len, minibatch, warmup) if capacity is None else int(capacity)
        # (tournament mode stores every seat of a round: one round passes the warmup)
        if max_decisions is None and self.capacity * len(self.chunks()) <= max(self.warmup, self.minibatch):
            warnings.warn(f"BatchedACER: capacity {self.capacity} episodes hold {self.capacity * len(self.chunks())} "
                          f"sequences per decider, so learn() never passes warmup {max(self.warmup, self.minibatch)} "
                          f"(capacity >= {default_capacity(rollout_len, minibatch, warmup)} learns)")
        D, dev = self.D_max, env.device
        # the replay grows with capacity x deciders: refuse a size that would
        # not fit instead of failing inside the allocator (the default
        # capacity reaches warmup = 100 sequences: ~102 episodes)
        need = replay_bytes(self.capacity, D)
        cap = MAX_REPLAY_BYTES if max_replay_bytes is None else int(max_replay_bytes)
        if dev.type == "cuda":
            free, _ = torch.cuda.mem_get_info(dev)
            cap = min(cap, int(0.8 * free))
        if need > cap:
            raise ValueError(f"BatchedACER: a replay of {self.capacity} episodes x {D} deciders needs {need / 2**30:.1f} "
                             f"GiB (limit {cap / 2**30:.1f} GiB): pass a smaller capacity (each episode holds "
                             f"{len(self.chunks())} sequences per decider; learn() starts past max(warmup, minibatch) = "
                             f"{max(self.warmup, self.minibatch)} stored sequences) or fewer games")
        self.log_prob = torch.zeros((D,), dtype=torch.float32, device=dev)
        self.entropy = torch.zeros((D,), dtype=torch.float32, device=dev)
        C = self.capacity
        self.rep_rows = torch.zeros((C, T_STEPS, D, 10, ROW), dtype=torch.float32, device=dev)
        self.rep_act = torch.zeros((C, T_STEPS, D), dtype=torch.long, device=dev)
        self.rep_logp = torch.full((C, T_STEPS, D, 10), self.log_epsilon, dtype=torch.float32, device=dev)
        self.rep_rew = torch.zeros((C, T_STEPS, D), dtype=torch.float32, device=dev)
        self.episodes = 0  # episodes written (slot = episodes % capacity)
        self.rep_nd = [0] * C  # deciders stored in each slot (tournament mode: the round's seats of this agent)
        self._t = 0
        # deciders per backward pass of an update (learn): bounds the activations
        # (~1.6 KB per candidate row of the fp32 forward + backward).  Larger
        # chunks run fewer, larger fp32 GEMMs: the run.py league's ACER update
        # took 406 / 320 / 286 ms per round at 4096 / 16384 / 65536 deciders
        # (profiles/r04_handoff_and_mlp_ab.txt); a quarter of the free memory
        # at construction caps it
        per_decider = max(self.minibatch, 1) * self.rollout_len * 10 * 1600
        budget = (torch.cuda.mem_get_info(dev)[0] // 4) if dev.type == "cuda" else (8 << 30)
        self.decider_chunk = int(os.environ.get("SECHS_ACER_DECIDER_CHUNK",
                                                max(1024, min(65536, budget // per_decider))))
        self._gen = torch.Generator(device=dev)
        self._gen.manual_seed(self.seed ^ 0xACE5)
        self.last_losses = []

    # ------------------------------------------------------------ acting
    def decide(self, n, memorize=False, record=False):
        """sample every deciding seat's card at hand size n: actions [B, N] int32"""
        L, h, st = nat.lib(), self.env._h, self.env._stream()
        if self.D == 0:
            self.step_id += 1
            return self.actions
        bf16 = int(self.net_dtype == torch.bfloat16)
        q = self._params(n)
        # recording with the actor on this device: the training-precision
        # forward (fp32 rows) is the one sampled from, so the behaviour log pi
        # is that forward's and no second, inference-dtype pass is needed
        train_fwd = record and self.net_dtype != torch.float32 and self.actor_device() == self.env.device
        if train_fwd:
            r32 = self._train_rows(q, n, None)
            with torch.no_grad():
                lt, _ = self.actor(r32)
            logits = lt.reshape(-1).float().contiguous()
            self.rows_evaluated += r32.shape[0]
        else:
            self.sync_net()
            rows = torch.empty((self.D * n, ROW), dtype=self.net_dtype, device=self.env.device)
            nat.check(L.sn_puct_root_rows(h, ctypes_ref(q), nat.ptr(rows), bf16, st), "sn_puct_root_rows")
            with torch.no_grad():
                logit, _ = self._net(rows)
            self.rows_evaluated += rows.shape[0]
            logits = logit.reshape(-1).float().contiguous()
        nat.check(L.sn_policy_sample(h, ctypes_ref(q), nat.ptr(logits), nat.ptr(self.actions), nat.ptr(self.best_index),
                                     nat.ptr(self.log_prob), nat.ptr(self.entropy), st), "sn_policy_sample")
        if record:
            s, t, D = self.episodes % self.capacity, T_STEPS - n, self.D
            if not train_fwd:
                r32 = self._train_rows(q, n, rows)
            self.rep_rows[s, t, :D, :n] = r32.view(D, n, ROW)
            self.rep_rows[s, t, :D, n:] = 0.0
            self.rep_act[s, t, :D] = self.best_index[:D].long()
            self.rep_logp[s, t, :D].fill_(self.log_epsilon)
            # behaviour log pi in the training forward's precision (fp32), so that
            # rho = pi_now / pi_then is exactly 1 on-policy as in the reference
            # (the bf16 inference logits differ from it by rounding)
            if self.net_dtype == torch.float32 or train_fwd:
                lt = logits.view(self.D, n)
            else:
                with torch.no_grad():
                    lt, _ = self.actor(r32.to(self.actor_device()))
                lt = lt.reshape(self.D, n).to(self.env.device)
            self.rep_logp[s, t, :D, :n] = torch.log_softmax(lt.float(), dim=1)
        self.step_id += 1
        return self.actions

    def play_episode(self, others=None, record=True):
        """one whole game of every env game (non-deciding seats: uniform moves);
        with record, the episode goes into replay slot episodes % capacity.
        Returns (summed rewards [B, N] int32, per-step rewards [10, B, N])."""
        env = self.env
        env.reset()
        per_step = torch.zeros((T_STEPS, env.num_games, env.num_players), dtype=torch.int32, device=env.device)
        for t in range(T_STEPS):
            acts = self.decide(T_STEPS - t, record=record)
            if self.M < env.num_players:
                keep = torch.tensor([(self.seats_mask >> p) & 1 for p in range(env.num_players)], device=env.device,
                                    dtype=torch.bool)
                acts = torch.where(keep[None, :], acts, self._random_moves())
            rew, done, inv = env.step(acts)
            per_step[t] = rew
        if record:
            seats = [p for p in range(env.num_players) if (self.seats_mask >> p) & 1]
            # learn(next_reward=r_t) of the step's own reward, x r_factor in float64 (actor_critic.py:142)
            r = per_step[:, :, seats].reshape(T_STEPS, -1).double() * self.r_factor
            self.rep_rew[self.episodes % self.capacity] = r.float()
            self.rep_nd[self.episodes % self.capacity] = self.D
            self.episodes += 1
        self.episode_rewards = per_step
        return per_step.sum(dim=0), per_step

    def record_rewards(self, per_step):
        """tournament mode: close the round's episode -- the rewards of this
        agent's seats (per_step [10, B, N] int32, learn(next_reward=r_t) of
        the step's own reward x r_factor, actor_critic.py:142)"""
        s = self.episodes % self.capacity
        r = per_step.reshape(T_STEPS, -1)[:, self.dec.long()].double() * self.r_factor
        self.rep_rew[s, :, : self.D] = r.float()
        self.rep_nd[s] = self.D
        self.episodes += 1

    # ------------------------------------------------------------ sequences in the replay
    def chunks(self):
        """step ranges of one episode's sequences (flush at rollout_len or done)"""
        L = self.rollout_len
        return [(c, min(T_STEPS, c + L)) for c in range(0, T_STEPS, L)]

    def _chunk_tables(self):
        """chunks() as device tensors (start, length), built once per rollout_len:
        a host list copied per loss() call would wait for the stream each time"""
        key = (self.rollout_len, str(self.env.device))
        if getattr(self, "_chunk_tab", (None,))[0] != key:
            ch = torch.tensor([c for c, _ in self.chunks()], device=self.env.device)
            ln = torch.tensor([e - c for c, e in self.chunks()], device=self.env.device)
            self._chunk_tab = (key, ch, ln)
        return self._chunk_tab[1], self._chunk_tab[2]

    def stored_sequences(self, upto_chunk=None):
        """(slot, chunk index) of every stored sequence, oldest episode first;
        the newest episode only up to `upto_chunk` (inclusive)"""
        nch = len(self.chunks())
        full = min(self.episodes, self.capacity)
        newest = (self.episodes - 1) % self.capacity
        out = []
        for e in range(self.episodes - full, self.episodes):
            s = e % self.capacity
            last = nch - 1 if (upto_chunk is None or s != newest) else upto_chunk
            out += [(s, c) for c in range(last + 1)]
        return out

    # ------------------------------------------------------------ the ACER loss
    def loss(self, slots, chunk_ids, decs=None):
        """sum over deciders of the reference's ACER loss on a batch of each
        decider's sequences: `slots`, `chunk_ids` [D, K] long (sequence k of
        decider d = replay slot slots[d, k], chunk chunk_ids[d, k], decider
        index decs[d, k] within the slot -- default d).
        Returns (total, actor, correction, critic) -- components summed over
        deciders, total carrying the gradient."""
        dev = self.actor_device()
        D, K = slots.shape
        L = self.rollout_len
        ch, ln = self._chunk_tables()
        j = torch.arange(L, device=self.env.device)
        t = ch[chunk_ids][:, :, None] + j  # [D, K, L]
        valid = j < ln[chunk_ids][:, :, None]
        t = torch.where(valid, t, torch.zeros_like(t))
        if decs is None:
            d = torch.arange(D, device=self.env.device)[:, None, None].expand(D, K, L)
        else:
            d = decs[:, :, None].expand(D, K, L)
        s = slots[:, :, None].expand(D, K, L)
        act = self.rep_act[s, t, d].to(dev)
        logp_then = self.rep_logp[s, t, d].to(dev)
        rew = self.rep_rew[s, t, d].to(dev)
        done = (t == T_STEPS - 1).to(dev)
        n = (T_STEPS - t).to(dev)
        valid = valid.to(dev)
        legal = torch.arange(10, device=dev) < n[..., None]
        # the net runs on the legal candidates' rows only (a step with n cards has n of the 10
        # slots: 55 % of them over an episode); the padded slots' logits are -inf and their
        # q 0 -- what masking the padded rows' outputs gave -- so they carry no gradient either
        lg_idx = legal.reshape(-1).nonzero()[:, 0]  # one host sync per loss call (sizes the batch)
        r_idx = lg_idx // 10
        rows = self.rep_rows[s.reshape(-1)[r_idx], t.reshape(-1)[r_idx], d.reshape(-1)[r_idx], lg_idx % 10]
        lg_sel, q_sel = train_forward(self.actor, rows.to(dev))
        logit = torch.full((D * K * L * 10,), float("-inf"), dtype=lg_sel.dtype, device=dev)
        logit = logit.index_copy(0, lg_idx.to(dev), lg_sel.reshape(-1)).reshape(D, K, L, 10)
        q = torch.zeros((D * K * L * 10,), dtype=q_sel.dtype, device=dev)
        q = q.index_copy(0, lg_idx.to(dev), q_sel.reshape(-1)).reshape(D, K, L, 10)
        logp = torch.log_softmax(logit, dim=-1).masked_fill(~legal, self.log_epsilon)
        a = act[..., None]
        q_a = q.gather(-1, a)[..., 0]
        logp_a = logp.gather(-1, a)[..., 0]
        v = (q * logp.exp()).sum(-1).detach()
        rho = (logp - logp_then).exp().detach()
        rho_bar = rho.gather(-1, a)[..., 0].clamp(max=self.truncate)
        coeff = (1.0 - self.truncate / rho).clamp(min=0.0)
        # Retrace targets, backwards within each sequence (actor_critic.py:195-207)
        last = (ln[chunk_ids] - 1).to(dev)  # [D, K]
        q_ret = torch.zeros((D, K), dtype=torch.float32, device=dev)
        qa_d = q_a.detach()
        targets = torch.zeros((D, K, L), dtype=torch.float32, device=dev)
        for i in range(L - 1, -1, -1):
            start = last == i
            q_ret = torch.where(start, v[:, :, i] * (1.0 - done[:, :, i].float()), q_ret)
            tgt = rew[:, :, i] + self.gamma * q_ret
            targets[:, :, i] = tgt
            q_ret = torch.where(valid[:, :, i], rho_bar[:, :, i] * (tgt - qa_d[:, :, i]) + v[:, :, i], q_ret)
        w = valid.float()
        rows_per_d = w.sum(dim=(1, 2))  # [D]

        def per_decider(x):
            return ((x * w).sum(dim=(1, 2)) / rows_per_d).sum()

        actor = per_decider(-rho_bar * logp_a * (targets - v))
        corr = per_decider((-coeff * logp_then.exp() * logp * (q.detach() - v[..., None])).sum(-1))
        err = (q_a - targets).abs()
        critic = self.critic_weight * per_decider(torch.where(err < 1.0, 0.5 * err * err, err - 0.5))
        return actor + corr + critic, actor.detach(), corr.detach(), critic.detach()

    def on_policy_batch(self, chunk):
        """every decider's newest sequence: [D, 1] slots / chunk ids"""
        D, dev = self.D, self.env.device
        s = (self.episodes - 1) % self.capacity
        return (torch.full((D, 1), s, dtype=torch.long, device=dev),
                torch.full((D, 1), chunk, dtype=torch.long, device=dev))

    def off_policy_batch(self, upto_chunk):
        """`minibatch` distinct stored sequences per decider, uniform"""
        seqs = self.stored_sequences(upto_chunk)
        S, dev = len(seqs), self.env.device
        pick = torch.rand((self.D, S), generator=self._gen, device=dev).argsort(dim=1)[:, : self.minibatch]
        # [S, 2] built on the device: a host tensor copied per call would wait for the stream
        sl = torch.tensor([q for q, _ in seqs], dtype=torch.long).pin_memory().to(dev, non_blocking=True) \
            if dev.type == "cuda" else torch.tensor([q for q, _ in seqs], dtype=torch.long)
        ch = torch.tensor([c for _, c in seqs], dtype=torch.long).pin_memory().to(dev, non_blocking=True) \
            if dev.type == "cuda" else torch.tensor([c for _, c in seqs], dtype=torch.long)
        return sl[pick], ch[pick]

    # ------------------------------------------------------------ tournament mode (decision lists)
    def league_batches(self, chunk):
        """(slots, chunk ids, decider indices) of the on-policy batch (every
        seat of the newest episode: its sequence `chunk`) and the off-policy
        batch (`minibatch` distinct stored sequences per seat, uniform over
        every stored (slot, chunk, seat) of this agent -- the reference's
        random.sample over its whole history, here over the replay's last
        `capacity` rounds)"""
        dev = self.env.device
        s_new = (self.episodes - 1) % self.capacity
        Dn = self.rep_nd[s_new]
        on = (torch.full((Dn, 1), s_new, dtype=torch.long, device=dev),
              torch.full((Dn, 1), chunk, dtype=torch.long, device=dev),
              torch.arange(Dn, device=dev)[:, None])
        # built on the device (a host tensor copied per call would wait for the stream)
        tab = []
        for sl, c in self.stored_sequences(chunk):
            nd = self.rep_nd[sl]
            tab.append(torch.stack((torch.full((nd,), sl, device=dev), torch.full((nd,), c, device=dev),
                                    torch.arange(nd, device=dev)), dim=1))
        tab = torch.cat(tab, dim=0)
        pick = distinct_picks(tab.shape[0], Dn, self.minibatch, self._gen, dev)
        off = (tab[pick, 0], tab[pick, 1], tab[pick, 2])
        return on, off

    def stored_count(self, upto_chunk):
        """sequences stored (tournament mode: over every seat of every stored episode)"""
        if self.dec is None:
            return len(self.stored_sequences(upto_chunk))
        return sum(self.rep_nd[sl] for sl, _ in self.stored_sequences(upto_chunk))

    def learn(self, optimizer):
        """the reference's update schedule for the episode just played: per
        flushed sequence, if more than max(warmup, minibatch) are stored, one
        on-policy and one off-policy Adam step (actor_critic.py:146-151)"""
        done_updates = []
        for c in range(len(self.chunks())):
            if self.stored_count(c) <= max(self.warmup, self.minibatch):
                continue
            batches = self.league_batches(c) if self.dec is not None else (self.on_policy_batch(c), self.off_policy_batch(c))
            for batch in batches:
                # the loss is a sum over deciders: its gradient accumulates over
                # decider chunks (bounded activation memory: a 65 536-slot
                # league's off-policy batch is ~4e7 candidate rows), then one step
                optimizer.zero_grad()
                D = batch[0].shape[0]
                if len(batch) == 2:  # explicit decider indices: a chunk's row d is decider d0 + d
                    batch = (*batch, torch.arange(D, device=batch[0].device)[:, None].expand_as(batch[0]))
                tot = None  # loss components stay on the device: no host sync per decider chunk
                for d0 in range(0, D, self.decider_chunk):
                    part = tuple(x[d0: d0 + self.decider_chunk] for x in batch)
                    total, actor, corr, critic = self.loss(*part)
                    total.backward()
                    comp = torch.stack((actor, corr, critic))
                    tot = comp if tot is None else tot + comp
                optimizer.step()
                done_updates.append(tot)
        # one transfer for the whole schedule
        done_updates = [tuple(float(v) for v in u) for u in torch.stack(done_updates).cpu()] if done_updates else []
        self.last_losses += done_updates
        return done_updates
