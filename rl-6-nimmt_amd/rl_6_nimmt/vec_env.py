"""Batched 6 nimmt! environment on one MI355X: B independent games, one per lane.

This is the MI355X-native form of `SechsNimmtEnv` (rl_6_nimmt/env.py:13-256
in the reference): every call enqueues one HIP kernel on torch's current
stream and exchanges torch tensors that stay in HBM.

    env = VecSechsNimmtEnv(65536, num_players=4, seed=0, rng="numpy")
    env.reset()
    out = env.rollout(10)          # one episode of DrunkHamster self-play
    out["rewards"]                 # int32 [10, 65536, 4]

RNG modes (both bit-exact against the CPU oracle):
  "numpy"  -- game g owns a numpy legacy MT19937 seeded seed + global id, so
              game g replays `np.random.seed(seed+g); GameSession(DrunkHamster()
              x N).play_game()` of the reference exactly, episode after episode.
  "philox" -- counter-based Philox4x32-10 keyed (seed, global game id): no
              per-game state in HBM; same draw structure (numpy's masked
              rejection interval), different words.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat

RNG_MODES = {"philox": nat.SN_RNG_PHILOX, "numpy": nat.SN_RNG_NUMPY_MT}
ROWS, THRESHOLD, HAND = 4, 6, 10


def obs_length(include_summaries=True):
    return 10 + 1 + (3 * ROWS if include_summaries else 0) + ROWS * THRESHOLD


class VecSechsNimmtEnv:
    def __init__(self, num_games, num_players=4, num_cards=104, seed=0, game_offset=0, rng="numpy", device=None,
                 include_summaries=True):
        nat.require_gpu()
        if rng not in RNG_MODES:
            raise ValueError(f"rng must be one of {sorted(RNG_MODES)}")
        if device is None:
            idx = torch.cuda.current_device()
        else:
            d = torch.device(device)
            idx = d.index if d.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.num_games, self.num_players, self.num_cards = int(num_games), int(num_players), int(num_cards)
        self.seed, self.game_offset, self.rng = int(seed), int(game_offset), rng
        self.include_summaries = bool(include_summaries)
        self.obs_len = obs_length(self.include_summaries)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(
                nat.lib().sn_create(ctypes.byref(h), self.device.index, self.num_games, self.num_players, self.num_cards,
                                    self.seed & (2**64 - 1), self.game_offset, RNG_MODES[rng]),
                "sn_create",
            )
        self._h = h

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            nat.lib().sn_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _flags(self, auto_reset=False):
        f = 0 if self.include_summaries else nat.SN_NO_SUMMARIES
        return f | (nat.SN_AUTO_RESET if auto_reset else 0)

    def _stream(self):
        return nat.stream_handle(self.device)

    def _empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    # ------------------------------------------------------------ env API
    def reset(self, decks=None):
        """env.py:43-51.  decks: optional uint8 [B, C] permutations."""
        if decks is not None:
            decks = torch.as_tensor(decks, dtype=torch.uint8, device=self.device).contiguous()
            assert decks.shape == (self.num_games, self.num_cards)
        nat.check(nat.lib().sn_reset(self._h, nat.ptr(decks), self._stream()), "sn_reset")

    def reset_to(self, board, hands):
        """env.py:53-62.  board int8 [B,4,6] (-1 pad), hands int8 [B,N,10] (-1 pad)."""
        board = torch.as_tensor(board, dtype=torch.int8, device=self.device).contiguous()
        hands = torch.as_tensor(hands, dtype=torch.int8, device=self.device).contiguous()
        assert board.shape == (self.num_games, ROWS, THRESHOLD) and hands.shape == (self.num_games, self.num_players, HAND)
        nat.check(nat.lib().sn_reset_to(self._h, nat.ptr(board), nat.ptr(hands), self._stream()), "sn_reset_to")
        self._keep = (board, hands)  # kernel reads them asynchronously

    def step(self, actions=None, auto_reset=False):
        """env.py:64-77 for every game.  actions int [B,N] (None = in-kernel
        DrunkHamster).  Returns (rewards int32 [B,N], done bool [B],
        invalid int32 [B] = first illegal seat or -1)."""
        B, N = self.num_games, self.num_players
        if actions is not None:
            actions = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
            assert actions.shape == (B, N)
        rew = self._empty((B, N), torch.int32)
        done = self._empty((B,), torch.uint8)
        inv = self._empty((B,), torch.int32)
        nat.check(nat.lib().sn_step(self._h, nat.ptr(actions), nat.ptr(rew), nat.ptr(done), nat.ptr(inv),
                                    self._flags(auto_reset), self._stream()), "sn_step")
        return rew, done.bool(), inv

    def rollout(self, steps, want_rewards=True, want_done=True, want_actions=False, want_obs=False, obs_stride=None,
                out=None, check=False):
        """Fused DrunkHamster self-play for `steps` env-steps with auto-reset.
        Returns dict of tensors: rewards int32 [T,B,N], done uint8 [T,B],
        actions uint8 [T,B,N], obs int8 [T,B,N,obs_stride] (pre-action).

        numpy mode: a pipelined draw past the twisted words (probability
        < 1e-25 per game and launch pair) raises
        PipeOverrunError -- at the next call without a sync (the library
        mirrors the count to pinned host memory), or at once with
        check=True (synchronises)."""
        B, N, T = self.num_games, self.num_players, int(steps)
        stride = obs_stride or ((self.obs_len + 15) // 16 * 16)
        if out is None:
            out = {}
            if want_rewards:
                out["rewards"] = self._empty((T, B, N), torch.int32)
            if want_done:
                out["done"] = self._empty((T, B), torch.uint8)
            if want_actions:
                out["actions"] = self._empty((T, B, N), torch.uint8)
            if want_obs:
                out["obs"] = self._empty((T, B, N, stride), torch.int8)
        if "obs" in out:
            stride = out["obs"].shape[-1]
        nat.check(
            nat.lib().sn_rollout(self._h, T, nat.ptr(out.get("rewards")), nat.ptr(out.get("done")),
                                 nat.ptr(out.get("actions")), nat.ptr(out.get("obs")), stride,
                                 self._flags(True), self._stream()),
            "sn_rollout",
        )
        if check and self.rng == "numpy":
            n = self.pipe_errors()
            if n:
                raise nat.PipeOverrunError(f"sn_rollout: {n} pipelined MT19937 draws ran past the twisted words")
        return out

    # ------------------------------------------------------------ views
    _DT = {torch.int8: nat.SN_I8, torch.int16: nat.SN_I16, torch.int32: nat.SN_I32, torch.int64: nat.SN_I64,
           torch.float32: nat.SN_F32}

    def obs(self, dtype=torch.int8, stride=None):
        """env.py:174-212 observations [B, N, L] (L = 47, or 35 without summaries)."""
        stride = stride or self.obs_len
        o = self._empty((self.num_games, self.num_players, stride), dtype)
        nat.check(nat.lib().sn_obs(self._h, nat.ptr(o), self._DT[dtype], stride, self._flags(), self._stream()), "sn_obs")
        return o

    def hands(self):
        """legal actions: int8 [B, N, 10], ascending, -1 padded."""
        h = self._empty((self.num_games, self.num_players, HAND), torch.int8)
        nat.check(nat.lib().sn_hands(self._h, nat.ptr(h), self._stream()), "sn_hands")
        return h

    def board(self):
        b = self._empty((self.num_games, ROWS, THRESHOLD), torch.int8)
        nat.check(nat.lib().sn_board(self._h, nat.ptr(b), self._stream()), "sn_board")
        return b

    def scores(self):
        s = self._empty((self.num_games, self.num_players), torch.int32)
        nat.check(nat.lib().sn_scores(self._h, nat.ptr(s), self._stream()), "sn_scores")
        return s

    def results(self):
        """(sum of finished episodes' final scores [B,N] int32, episodes [B] int32)"""
        s = self._empty((self.num_games, self.num_players), torch.int32)
        e = self._empty((self.num_games,), torch.int32)
        nat.check(nat.lib().sn_results(self._h, nat.ptr(s), nat.ptr(e), self._stream()), "sn_results")
        return s, e

    def clear_results(self):
        nat.check(nat.lib().sn_clear_results(self._h, self._stream()), "sn_clear_results")

    # ------------------------------------------------------------ numpy RNG bridge
    def set_option(self, ring_words=None, chunk_steps=None, pipeline=None, pipe_gpw=None, pipe_lead=None,
                   play_split=None, twist_round=None, twist_every=None, twist_skip=None, pipe_dec=None):
        """rollout tuning (include/sechs.h SN_OPT_*; all numpy-compat only except play_split,
        the role-split kernel of philox handles; twist_round: whole-round MT twists in
        k_mt_ahead; twist_every: one twist-ahead launch per K = 1 .. 5 play launches; pipe_dec:
        decode-ahead, k_decode + k_play from the records); results never
        depend on it (except the test knobs pipe_lead < 600 and twist_skip = 1, which make
        overruns -- PipeOverrunError -- likely / certain)"""
        if pipe_lead is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_PIPE_LEAD, int(pipe_lead)), "sn_set_option")
        if pipe_gpw is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_PIPE_GPW, int(pipe_gpw)), "sn_set_option")
        if play_split is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_PLAY_SPLIT, int(play_split)), "sn_set_option")
        if twist_every is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_TWIST_EVERY, int(twist_every)), "sn_set_option")
        if twist_round is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_TWIST_ROUND, int(twist_round)), "sn_set_option")
        if pipe_dec is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_PIPE_DEC, int(pipe_dec)), "sn_set_option")
        if twist_skip is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_TWIST_SKIP, int(twist_skip)), "sn_set_option")
        if pipeline is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_PIPELINE, int(bool(pipeline))), "sn_set_option")
        if ring_words is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_RING_WORDS, int(ring_words)), "sn_set_option")
        if chunk_steps is not None:
            nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_CHUNK_STEPS, int(chunk_steps)), "sn_set_option")

    def time_kernels(self, launches):
        """record HIP events around the next `launches` pipelined k_play /
        k_mt_ahead launches, each on its own stream (0 = off)"""
        nat.check(nat.lib().sn_set_option(self._h, nat.SN_OPT_TIMING, int(launches)), "sn_set_option")

    def kernel_times(self, with_decode=False):
        """(mean k_play ms, mean k_mt_ahead ms, launches recorded) [sync];
        with_decode: (k_play, k_mt_ahead, k_decode ms, launches)"""
        a, b, c, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_float(), ctypes.c_int32()
        nat.check(nat.lib().sn_kernel_times_dec(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                                ctypes.byref(n)), "sn_kernel_times_dec")
        return (a.value, b.value, c.value, n.value) if with_decode else (a.value, b.value, n.value)

    def pipe_errors(self):
        """draws of pipelined rollouts that ran past the twisted words (must be 0) [sync]"""
        c = ctypes.c_uint32()
        nat.check(nat.lib().sn_pipe_errors(self._h, ctypes.byref(c)), "sn_pipe_errors")
        return c.value

    def get_mt_state(self, game=0):
        key = np.zeros(624, dtype=np.uint32)
        pos = ctypes.c_int32()
        torch.cuda.current_stream(self.device).synchronize()
        nat.check(nat.lib().sn_mt_get(self._h, game, key.ctypes.data_as(ctypes.c_void_p), ctypes.byref(pos)), "sn_mt_get")
        return key, int(pos.value)

    def set_mt_state(self, key, pos, game=0):
        key = np.ascontiguousarray(key, dtype=np.uint32)
        assert key.shape == (624,)
        torch.cuda.current_stream(self.device).synchronize()
        nat.check(nat.lib().sn_mt_set(self._h, game, key.ctypes.data_as(ctypes.c_void_p), int(pos)), "sn_mt_set")

    def philox_counter(self, game=0):
        c = ctypes.c_uint64()
        torch.cuda.current_stream(self.device).synchronize()
        nat.check(nat.lib().sn_philox_counter(self._h, game, ctypes.byref(c)), "sn_philox_counter")
        return int(c.value)
