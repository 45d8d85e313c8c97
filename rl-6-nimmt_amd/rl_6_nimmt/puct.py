"""Batched "Alpha0.5" PUCT search on one MI355X (BASELINE config 4).

Reference: PUCTAgent / PolicyMCSAgent (agents/mcts.py:191-323).  A decision
runs n_mc = min(mc_max, mc_per_card * n!) rollouts; at each rollout's first
step the deciding seat picks its move by PUCT over the statistics so far,
every other move is sampled from the policy net, and the return is backed
up to the root move; finally the move with the best mean return is played.

Here all decisions of a batch (every deciding seat of every game) advance
together: for each rollout r and rollout step t, the HIP kernels emit the
normalised candidate rows of every seat, the policy MLP (PyTorch-ROCm,
bf16 by default) turns them into logits, and sn_puct_step selects / samples,
plays the step and, at the end, backs up.  Rollouts of one decision stay a
sequential chain, exactly as in the reference.
"""
import math
import os

import torch
from torch import nn

from . import _native as nat
from .splitk import train_forward
from .utils.nets import MultiHeadedMLP

ROW = 48


def make_actor(hidden_sizes=(100, 100), activation=None):
    """the reference's policy net: MultiHeadedMLP(48, (100, 100), (1,), ReLU, (None,))"""
    return MultiHeadedMLP(ROW, hidden_sizes=hidden_sizes, head_sizes=(1,), activation=activation or nn.ReLU(),
                          head_activations=(None,))


class FusedMLP:
    """Inference form of MultiHeadedMLP(48, hidden, heads, ReLU, (None,)) on
    PyTorch-ROCm (north_star: the net runs through PyTorch): every hidden
    layer one hipBLASLt GEMM with the bias + ReLU fused into its epilogue
    (torch._addmm_activation: no separate clamp pass over the [rows, 100]
    activations), the heads one GEMM over the head rows zero-padded to 16
    outputs (a [rows,100]x[100,1] GEMV runs 2x slower than the padded GEMM on
    gfx950).  Measured on 1.31 M bf16 rows: 1091 -> 839 us (tools/mlp_bench.py).
    Other layouts fall back to the module."""

    def __init__(self, module, layers, head_w, head_b, head_sizes):
        self.module, self.layers = module, layers
        self.head_w, self.head_b, self.head_sizes = head_w, head_b, head_sizes

    @classmethod
    def of(cls, net):
        lat = list(net.latent_net)
        heads = list(net.head_nets)
        ok = len(lat) % 2 == 0 and all(isinstance(m, nn.Linear) for m in lat[0::2]) and \
            all(isinstance(m, nn.ReLU) for m in lat[1::2]) and \
            all(len(h) == 1 and isinstance(h[0], nn.Linear) for h in heads)
        if not ok:
            return cls(net, None, None, None, None)
        layers = [(m.weight.detach(), m.bias.detach()) for m in lat[0::2]]
        w = torch.cat([h[0].weight.detach() for h in heads], dim=0)
        b = torch.cat([h[0].bias.detach() for h in heads], dim=0)
        pad = max(16, -(-w.shape[0] // 16) * 16)
        wp = torch.zeros((pad, w.shape[1]), dtype=w.dtype, device=w.device)
        bp = torch.zeros((pad,), dtype=b.dtype, device=b.device)
        wp[: w.shape[0]], bp[: b.shape[0]] = w, b
        return cls(net, layers, wp.t().contiguous(), bp, [h[0].out_features for h in heads])

    def refresh_from(self, actor):
        """copy new weights of the same architecture into this net's tensors
        in place (every derived tensor too): addresses stay, so captured
        hipGraphs stay valid.  False if the layout differs."""
        src, dst = dict(actor.named_parameters()), dict(self.module.named_parameters())
        if src.keys() != dst.keys() or any(src[k].shape != dst[k].shape for k in dst):
            return False
        with torch.no_grad():
            for k, v in dst.items():
                v.copy_(src[k])
            if self.layers is not None:
                fresh = FusedMLP.of(self.module)
                self.head_w.copy_(fresh.head_w)
                self.head_b.copy_(fresh.head_b)
                if getattr(self, "_fused", None) is not None:
                    for old, new in zip(self._fused, fresh.fused()):
                        old.copy_(new)
        return True

    def fused(self):
        """the one-kernel rollout form (sn_puct_mlp_seats / sn_puct_rollouts)
        for MultiHeadedMLP(48, (H, H2), (1,)) in bf16 with H <= 111, H2 <= 127:
        w1c [112] f32 (W1[:, 0], then 0), W2 [128][112] bf16 ([W2 | b2 | 0]
        rows, the ones pass-through row H2), head [128] f32 ([wh | bh | 0]),
        w1s [128][64] bf16 ([W1 | b1 | 0] rows, 1 at (H, 48): the ones
        feature); None for other layouts (they run sn_puct_rows + __call__)"""
        if getattr(self, "_fused", "unset") != "unset":
            return self._fused
        self._fused = None
        if self.layers is None or len(self.layers) != 2 or self.head_sizes != [1] or \
                self.layers[0][0].shape[1] != ROW or self.layers[0][0].dtype != torch.bfloat16:
            return None
        w1, b1 = self.layers[0]
        H = w1.shape[0]
        w2, b2 = self.layers[1]
        H2 = w2.shape[0]
        if H > 111 or H2 > 127 or w2.shape[1] != H:
            return None
        dev = w1.device
        c = torch.zeros((112,), dtype=torch.float32, device=dev)
        c[:H] = w1[:, 0].float()
        w2p = torch.zeros((128, 112), dtype=torch.bfloat16, device=dev)
        w2p[:H2, :H], w2p[:H2, H], w2p[H2, H] = w2, b2, 1.0
        head = torch.zeros((128,), dtype=torch.float32, device=dev)
        head[:H2] = self.head_w[:, 0].float()
        head[H2] = self.head_b[0].float()
        w1s = torch.zeros((128, 64), dtype=torch.bfloat16, device=dev)  # [W1 | b1 | 0] rows
        w1s[:H, :ROW], w1s[:H, ROW] = w1, b1
        w1s[H, ROW] = 1.0
        self._fused = (c, w2p, head, w1s)
        return self._fused

    def __call__(self, rows):
        if self.layers is None:
            return self.module(rows)
        h = rows
        for w, b in self.layers:
            h = torch._addmm_activation(b, h, w.t())
        out = torch.addmm(self.head_b, h, self.head_w)
        res, c = [], 0
        for n in self.head_sizes:
            res.append(out[:, c: c + n])
            c += n
        return res


class BatchedPUCT:
    def __init__(self, env, actor, mc_per_card=10, mc_max=100, c_puct=2.0, seed=0, seats_mask=None, puct_root=True,
                 net_dtype=torch.bfloat16, mcs_num_cards=104, graph=False, max_decisions=None, fused_rollouts=None):
        # `actor` stays where the caller keeps it (the drop-in agents run it
        # on the host): inference uses a device copy in net_dtype (sync_net),
        # the training losses run on the actor's own device (actor_device).
        self.env, self.actor = env, actor
        self.mc_per_card, self.mc_max, self.c_puct = mc_per_card, mc_max, float(c_puct)
        self.seed = int(seed)
        self.puct_root = bool(puct_root)
        self.net_dtype = net_dtype
        self.mcs_num_cards = mcs_num_cards
        B, N, dev = env.num_games, env.num_players, env.device
        self.seats_mask = ((1 << N) - 1) if seats_mask is None else int(seats_mask)
        self.M = bin(self.seats_mask & ((1 << N) - 1)).count("1")
        self.D = B * self.M
        # tournament mode (max_decisions given): the deciding seats are a
        # decision list (use_decisions: g * N + p of this agent's seats in the
        # slots' current games), at most max_decisions of them
        self.dec = None
        if max_decisions is not None:
            self.D = 0
        self.D_max = B * self.M if max_decisions is None else int(max_decisions)
        D = self.D_max
        self.avail = torch.zeros((4, B * N), dtype=torch.int32, device=dev)
        self.ro = torch.zeros((D, 48), dtype=torch.int32, device=dev)
        self.stats = torch.zeros((D, 24), dtype=torch.int32, device=dev)
        self.hist = torch.zeros((D, 172), dtype=torch.int32, device=dev)
        self.root_probs = torch.zeros((D, 10), dtype=torch.float32, device=dev)
        self.best_index = torch.zeros((D,), dtype=torch.int32, device=dev)
        self.actions = torch.zeros((B, N), dtype=torch.int32, device=dev)
        self.step_id = 0
        self.decisions = []  # (root rows, best index) per decision batch, for learn()
        self._net = None
        self._net_version = None
        self.rows_evaluated = 0
        # graph=True: a decision's rollout chain (n_mc x [deal, n x (rows,
        # MLP, step)] launches) is captured once per hand size as a hipGraph
        # (torch.cuda.CUDAGraph) and replayed for every decision; the kernels
        # read the decision counter from step_dev, new weights are copied
        # into the captured tensors in place (FusedMLP.refresh_from).
        # graph_after: uses of a shape that run eagerly before it is captured
        # (1 for one-game drop-in agents, whose one-off shapes would cost a
        # capture each)
        self.graph = bool(graph) and max_decisions is None
        self.graph_after = 0
        self._graphs, self._graphs_seen = {}, {}
        # bf16 nets of the reference's shape (FusedMLP.fused) run the rollout MLP as one MFMA
        # kernel (sn_puct_mlp_seats / sn_puct_rollouts); other nets run sn_puct_rows + the net
        # the rollout loop deals this many rollouts per launch
        # (sn_puct_deal_batch into a [deal_batch][D][48] buffer, each rollout
        # then running on its slice); 0: one sn_puct_deal per rollout (A/B, tests)
        self.deal_batch = int(os.environ.get("SECHS_PUCT_DEAL_BATCH", "16"))
        # whole rollouts in one kernel per deal batch (sn_puct_rollouts: a wave per group of 8
        # decisions, logits in LDS; round 6: 1.10 G playout env-steps/s on config 4, and the
        # tournament's engines too) or a launch per step (fused_rollouts=False);
        # SECHS_PUCT_ROLLOUTS=0 / 1 overrides (A/B runs, tests)
        env_ro = os.environ.get("SECHS_PUCT_ROLLOUTS")
        self.fused_rollouts = (env_ro != "0") if env_ro is not None else (True if fused_rollouts is None
                                                                            else bool(fused_rollouts))
        self._step_dev = torch.zeros((1,), dtype=torch.int32, device=dev)

    # ------------------------------------------------------------ policy net on the device
    def sync_net(self):
        """(re)build the device copy of the actor in net_dtype"""
        version = tuple(p._version for p in self.actor.parameters())
        if self._net is not None and version != self._net_version and self._net.refresh_from(self.actor):
            self._net_version = version  # updated in place: the captured graphs still hold
        if self._net is None or version != self._net_version:
            import copy

            self._graphs = {}

            net = copy.deepcopy(self.actor).to(self.env.device, self.net_dtype)
            net.eval()
            self._net, self._net_version = FusedMLP.of(net), version
            if self._net.fused() is not None:  # built here: a graph capture may not allocate
                self._fused_bufs()
        return self._net

    def actor_device(self):
        return next(self.actor.parameters()).device

    def _logits(self, rows):
        with torch.no_grad():
            (out,) = self._net(rows)
        self.rows_evaluated += rows.shape[0]
        return out.reshape(-1).float().contiguous()

    def n_mc(self, n):
        return min(self.mc_max, self.mc_per_card * math.factorial(n))

    def use_decisions(self, dec):
        """tournament mode: the seats to decide for, int32 [D] = g * N + p on
        the device (sn_puct.dec_list); a game of k players rolls out k seats"""
        dec = torch.as_tensor(dec, device=self.env.device).to(torch.int32).contiguous()
        assert dec.numel() <= self.D_max, "more decisions than max_decisions"
        self.dec, self.D = dec, int(dec.numel())

    def _params(self, n, rollout=0, step_dev=False):
        q = nat.SnPuct()
        if self.dec is not None:
            q.dec_list, q.num_dec = self.dec.data_ptr(), self.D
        q.step_dev = self._step_dev.data_ptr() if step_dev else None
        q.seats_mask, q.n, q.puct_root, q.c_puct = self.seats_mask, n, int(self.puct_root), self.c_puct
        q.seed, q.step, q.rollout = self.seed & (2**64 - 1), self.step_id & 0xFFFFFFFF, rollout
        q.avail, q.rollouts, q.stats = self.avail.data_ptr(), self.ro.data_ptr(), self.stats.data_ptr()
        q.hist, q.root_probs = self.hist.data_ptr(), self.root_probs.data_ptr()
        return q

    # ------------------------------------------------------------ one decision per deciding seat
    def memorize(self):
        nat.check(nat.lib().sn_mcs_memorize(self.env._h, nat.ptr(self.avail), self.mcs_num_cards, self.env._stream()),
                  "sn_mcs_memorize")

    def decide(self, n, memorize=True, record=False):
        """Search every deciding seat at hand size n; returns actions [B, N]
        (int32, deciding seats filled in)."""
        L, h, st = nat.lib(), self.env._h, self.env._stream()
        if memorize:
            self.memorize()
        if self.D == 0:  # tournament mode: this agent has no seat in any current game
            self.step_id += 1
            return self.actions
        bf16 = int(self.net_dtype == torch.bfloat16)
        q = self._params(n)
        if n > 1:
            self.sync_net()
            rows = torch.empty((self.D * n, ROW), dtype=self.net_dtype, device=self.env.device)
            nat.check(L.sn_puct_root_rows(h, ctypes_ref(q), nat.ptr(rows), bf16, st), "sn_puct_root_rows")
            nat.check(L.sn_puct_init(h, ctypes_ref(q), nat.ptr(self._logits(rows)), st), "sn_puct_init")
            if self.graph:
                # the same 32-bit counter as the eager path's q.step, as int32 bits
                sid = self.step_id & 0xFFFFFFFF
                self._step_dev.fill_(sid - (1 << 32) if sid >= (1 << 31) else sid)
                key = (n, self.n_mc(n), self.c_puct, self.puct_root, self.D)  # everything a capture bakes in
                g = self._graphs.get(key)
                if g is None and self._graphs_seen.get(key, 0) >= self.graph_after:
                    g = self._capture(n)
                    self._graphs[key] = g
                if g is None:
                    self._graphs_seen[key] = self._graphs_seen.get(key, 0) + 1
                    self._rollouts(n, q)
                else:
                    g[0].replay()
                    self.rows_evaluated += g[1]
            else:
                self._rollouts(n, q)
        nat.check(L.sn_puct_choose(h, ctypes_ref(q), nat.ptr(self.actions), nat.ptr(self.best_index), st),
                  "sn_puct_choose")
        if record and n > 1:
            self.decisions.append((self._train_rows(q, n, rows), n, self.best_index[: self.D].clone()))
        self.step_id += 1
        return self.actions

    def _train_rows(self, q, n, rows):
        """the root rows of a recorded decision in fp32, as the reference's
        training forward sees them (inference may run on bf16 rows)"""
        if rows is not None and rows.dtype == torch.float32:
            return rows.clone()
        r32 = torch.empty((self.D * n, ROW), dtype=torch.float32, device=self.env.device)
        nat.check(nat.lib().sn_puct_root_rows(self.env._h, ctypes_ref(q), nat.ptr(r32), 0, self.env._stream()),
                  "sn_puct_root_rows")
        return r32

    def _rollouts(self, n, q):
        """the decision's rollout chain: n_mc x [deal, n x (rows, MLP, step)]"""
        L, h, st = nat.lib(), self.env._h, self.env._stream()
        bf16 = int(self.net_dtype == torch.bfloat16)
        N = self.env.num_players
        fz = self._net.fused()
        if fz is not None:
            # the reference-shaped bf16 net: per rollout step the seats' [0, obs, 1] rows, layer 1's
            # per-seat part on MFMA, the card column + ReLU, layer 2 + ReLU and the head in one MFMA
            # kernel (f32 logits, packed) -- no activation tensor in HBM
            w1c, w2p, head, w1s = fz
            S = self.D * N
            logits = self._fused_bufs()
            # the arguments built once (the league's engines run this loop eagerly: host time per launch)
            qr, deal, step, mlp = ctypes_ref(q), L.sn_puct_deal, L.sn_puct_step, L.sn_puct_mlp_seats
            wargs = (nat.ptr(w1s), nat.ptr(w1c), nat.ptr(w2p), nat.ptr(head), nat.ptr(logits), st)
            lp = nat.ptr(logits)
            RB, nmc = self.deal_batch, self.n_mc(n)
            if self.fused_rollouts and RB > 0 and 3 <= N <= 8:
                rob = self._deal_buf(RB)
                for r0 in range(0, nmc, RB):
                    nr = min(RB, nmc - r0)
                    nat.check(L.sn_puct_deal_batch(h, qr, r0, nr, rob.data_ptr(), st), "sn_puct_deal_batch")
                    nat.check(L.sn_puct_rollouts(h, qr, r0, nr, rob.data_ptr(), nat.ptr(w1s), nat.ptr(w1c),
                                                 nat.ptr(w2p), nat.ptr(head), st), "sn_puct_rollouts")
                self.rows_evaluated += nmc * S * (n * (n + 1) // 2)
                return
            if RB > 0:
                rob = self._deal_buf(RB)
                stride = self.D * 48 * 4  # bytes of one rollout's states
            for r in range(nmc):
                q.rollout = r
                if RB > 0:
                    if r % RB == 0:
                        nat.check(L.sn_puct_deal_batch(h, qr, r, min(RB, nmc - r), rob.data_ptr(), st),
                                  "sn_puct_deal_batch")
                    q.rollouts = rob.data_ptr() + (r % RB) * stride
                else:
                    nat.check(deal(h, qr, st), "sn_puct_deal")
                for t in range(n):
                    nat.check(mlp(h, qr, n - t, *wargs), "sn_puct_mlp_seats")
                    nat.check(step(h, qr, lp, t, n - t, st), "sn_puct_step")
            q.rollouts = self.ro.data_ptr()
            self.rows_evaluated += nmc * S * (n * (n + 1) // 2)
            return
        # any other net (fp32, other widths or depths): the candidate rows + the net's forward
        bufs = self._bufs(n)
        views = {m: bufs[m][: self.D * N * m] for m in range(1, n + 1)}  # this batch's decisions
        for r in range(self.n_mc(n)):
            q.rollout = r
            nat.check(L.sn_puct_deal(h, ctypes_ref(q), st), "sn_puct_deal")
            for t in range(n):
                m = n - t
                nat.check(L.sn_puct_rows(h, ctypes_ref(q), m, nat.ptr(views[m]), bf16, st), "sn_puct_rows")
                nat.check(L.sn_puct_step(h, ctypes_ref(q), nat.ptr(self._logits(views[m])), t, m, st), "sn_puct_step")

    def _deal_buf(self, RB):
        """[RB][D_max][48] int32: the initial states of RB rollouts (sn_puct_deal_batch)"""
        if getattr(self, "_robuf", None) is None or self._robuf.shape[0] != RB:
            self._robuf = torch.zeros((RB, self.D_max, 48), dtype=torch.int32, device=self.env.device)
        return self._robuf

    def _fused_bufs(self):
        """the rollout logits [D_max*N*10] f32 of sn_puct_mlp_seats"""
        S = self.D_max * self.env.num_players
        if getattr(self, "_fbufs", None) is None or self._fbufs.shape[0] != S * 10:
            self._fbufs = torch.empty((S * 10,), dtype=torch.float32, device=self.env.device)
        return self._fbufs

    def _bufs(self, n):
        N = self.env.num_players
        if not hasattr(self, "_rowbufs"):
            self._rowbufs = {}
        for m in range(1, n + 1):
            if m not in self._rowbufs:
                self._rowbufs[m] = torch.empty((self.D_max * N * m, ROW), dtype=self.net_dtype, device=self.env.device)
        return self._rowbufs

    def _capture(self, n):
        """capture _rollouts(n) with the decision counter read from step_dev"""
        q = self._params(n, step_dev=True)
        self._bufs(n)
        before = self.rows_evaluated
        torch.cuda.synchronize(self.env.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._rollouts(n, q)
        rows = self.rows_evaluated - before
        self.rows_evaluated = before
        return g, rows

    def play_episode(self, others=None, record=False):
        """One whole game of every env game; deciding seats search, the other
        seats (if any) play DrunkHamster moves in-kernel.  Returns the summed
        rewards [B, N] int32."""
        env = self.env
        env.reset()
        total = torch.zeros((env.num_games, env.num_players), dtype=torch.int32, device=env.device)
        for t in range(10):
            acts = self.decide(10 - t, record=record)
            if self.M < env.num_players:
                rnd = self._random_moves()
                keep = torch.tensor([(self.seats_mask >> p) & 1 for p in range(env.num_players)], device=env.device,
                                    dtype=torch.bool)
                acts = torch.where(keep[None, :], acts, rnd)
            rew, done, inv = env.step(acts)
            total += rew
        return total

    def _random_moves(self):
        """uniform legal moves for the non-deciding seats (host-side torch RNG)"""
        hands = self.env.hands().long()
        n = (hands >= 0).sum(dim=2)
        k = (torch.rand(hands.shape[:2], device=hands.device) * n).long().clamp(max=9)
        return hands.gather(2, k[..., None])[..., 0].to(torch.int32)

    # ------------------------------------------------------------ training (mcts.py:230-261)
    def policy_loss(self, d0=0, d1=None):
        """-sum over recorded decisions of log pi(chosen root move) under the
        current weights (the reference stores log(probs[best]) from the
        rollout that first chose it -- same weights during an episode, so the
        same value).  n == 1 decisions play without search and add log 1 = 0
        (mcts.py:50-51), so they are not recorded.  [d0, d1): the deciders
        (games) whose terms are summed -- one decider's term is the
        reference's per-episode loss (mcts.py:244-255)."""
        dev = self.actor_device()
        loss = torch.zeros((), device=dev)
        for (logits,), n, best in decision_forwards(self.actor, self.decisions, d0, d1, dev):
            logp = torch.log_softmax(logits.reshape(-1, n), dim=1)
            loss = loss - logp.gather(1, best[:, None]).sum()
        return loss


def decision_forwards(actor, decisions, d0, d1, dev):
    """the training forward of every recorded decision batch's root rows in ONE
    pass (the batches' rows concatenated: one GEMM chain forward and backward
    instead of one per hand size), split back per batch: yields (the net's
    outputs, n, chosen indices) of deciders [d0, d1) per decision batch"""
    parts, segs = [], []
    for rows, n, best in decisions:
        e = best.shape[0] if d1 is None else d1
        parts.append(rows[d0 * n: e * n])
        segs.append((n, (e - d0) * n, best[d0:e].to(dev).long()))
    if not parts:
        return
    outs = train_forward(actor, torch.cat(parts).to(dev))
    off = 0
    for n, m, best in segs:
        yield [o[off: off + m] for o in outs], n, best
        off += m


def make_actor_value(hidden_sizes=(100, 100), activation=None):
    """PUCTCustomedAgent's net (mcts.py:334-335): MultiHeadedMLP(48, (100, 100), (2,)) -- column 0 the
    policy logit, column 1 the value"""
    return MultiHeadedMLP(ROW, hidden_sizes=hidden_sizes, head_sizes=(2,), activation=activation or nn.ReLU(),
                          head_activations=(None,))


class BatchedPUCTCustomed(BatchedPUCT):
    """PUCTCustomedAgent (agents/mcts.py:325-451) for every deciding seat of
    a batch of games.  The reference's "search" draws an environment and
    evaluates the 2-head net once on the root candidates -- no rollouts
    (_play_out_with_NN, mcts.py:366-376): the move is the first argmax of
    the value head, its log-probability comes from the policy head and the
    chosen value is the step's outcome.  Per decision batch: one
    sn_puct_root_rows launch (normalised rows straight from the device
    state), one MLP forward (PyTorch-ROCm), one sn_pcv_choose launch.

    Training (mcts.py:421-451) from stored rows instead of retained graphs:
    per (game, deciding seat), loss = MSE(values of the chosen moves,
    reward_sum) - sum(log pi(chosen)), with reward_sum = the rewards of the
    first 9 steps (GameSession hands learn() the previous step's reward,
    play.py:29,57,72, so the last step's never reaches the agent); the batch
    loss is the sum over games (the reference steps Adam after every game)."""

    def __init__(self, env, actor, seats_mask=None, net_dtype=torch.bfloat16, seed=0, max_decisions=None):
        super().__init__(env, actor, seed=seed, seats_mask=seats_mask, puct_root=False, net_dtype=net_dtype,
                         max_decisions=max_decisions)
        D = self.D_max
        self.log_prob = torch.zeros((D,), dtype=torch.float32, device=env.device)
        self.value = torch.zeros((D,), dtype=torch.float32, device=env.device)

    def decide(self, n, memorize=False, record=False):
        """every deciding seat at hand size n; returns actions [B, N] int32"""
        L, h, st = nat.lib(), self.env._h, self.env._stream()
        if self.D == 0:
            self.step_id += 1
            return self.actions
        bf16 = int(self.net_dtype == torch.bfloat16)
        q = self._params(n)
        self.sync_net()
        rows = torch.empty((self.D * n, ROW), dtype=self.net_dtype, device=self.env.device)
        nat.check(L.sn_puct_root_rows(h, ctypes_ref(q), nat.ptr(rows), bf16, st), "sn_puct_root_rows")
        with torch.no_grad():
            (heads,) = self._net(rows)
        self.rows_evaluated += rows.shape[0]
        heads = heads.float().contiguous()
        nat.check(L.sn_pcv_choose(h, ctypes_ref(q), nat.ptr(heads), nat.ptr(self.actions), nat.ptr(self.best_index),
                                  nat.ptr(self.log_prob), nat.ptr(self.value), st), "sn_pcv_choose")
        if record:
            self.decisions.append((self._train_rows(q, n, rows), n, self.best_index[: self.D].clone()))
        self.step_id += 1
        return self.actions

    def play_episode(self, others=None, record=False):
        """one whole game of every env game; returns (summed rewards [B, N]
        int32, per-step rewards [10, B, N] int32)"""
        env = self.env
        env.reset()
        per_step = torch.zeros((10, env.num_games, env.num_players), dtype=torch.int32, device=env.device)
        for t in range(10):
            acts = self.decide(10 - t, record=record)
            if self.M < env.num_players:
                keep = torch.tensor([(self.seats_mask >> p) & 1 for p in range(env.num_players)], device=env.device,
                                    dtype=torch.bool)
                acts = torch.where(keep[None, :], acts, self._random_moves())
            rew, done, inv = env.step(acts)
            per_step[t] = rew
        self.episode_rewards = per_step
        return per_step.sum(dim=0), per_step

    def _decider_rewards(self, per_step):
        if self.dec is not None:  # tournament mode: the decision list's seats
            return per_step.reshape(per_step.shape[0], -1)[:, self.dec.long()]
        seats = [p for p in range(self.env.num_players) if (self.seats_mask >> p) & 1]
        return per_step[:, :, seats].reshape(per_step.shape[0], -1)  # [10, D] in decision order

    def loss(self, per_step=None, d0=0, d1=None):
        """reference loss of the recorded episode (mcts.py:431-451), summed over
        the games of deciders [d0, d1) (all by default)"""
        per_step = self.episode_rewards if per_step is None else per_step
        dev = self.actor_device()
        target = self._decider_rewards(per_step)[:-1].sum(dim=0).float().to(dev)  # [D]
        target = target[d0:d1]
        logps, values = [], []
        for (out,), n, best in decision_forwards(self.actor, self.decisions, d0, d1, dev):
            out = out.reshape(-1, n, 2)
            best = best[:, None]
            logp = torch.log_softmax(out[:, :, 0], dim=1)
            logps.append(logp.gather(1, best)[:, 0])
            values.append(out[:, :, 1].gather(1, best)[:, 0])
        logps, values = torch.stack(logps, dim=1), torch.stack(values, dim=1)  # [D, steps]
        outcome_loss = ((values - target[:, None]) ** 2).mean(dim=1)
        policy_loss = -logps.sum(dim=1)
        return (outcome_loss + policy_loss).sum()


def ctypes_ref(q):
    import ctypes

    return ctypes.byref(q)
