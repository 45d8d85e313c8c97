"""ctypes binding of the CPU oracle (oracle/sechs_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  The oracle is
pinned against the reference's own outputs (tests/golden/, see
tests/test_oracle_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SECHS_ORACLE_LIB: another build of the same sources (liboracle_asan.so, tools/asan_cpu.sh)
_LIB = os.environ.get("SECHS_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")

RNG_PHILOX = 0
RNG_NUMPY_MT = 1
MAX_PLAYERS = 10
ROWS, THRESHOLD, HAND, MAX_CARDS = 4, 6, 10, 104


def build(force=False):
    if os.environ.get("SECHS_ORACLE_LIB"):
        return _LIB  # prebuilt variant (make -C oracle asan)
    src = os.path.join(_HERE, "sechs_oracle.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(
        os.path.getmtime(src), os.path.getmtime(os.path.join(_HERE, "sechs_oracle.h"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE, "-B", "liboracle.so"])
    return _LIB


def obs_len(include_summaries=True):
    return 10 + 1 + (3 * ROWS if include_summaries else 0) + ROWS * THRESHOLD


class _Rng(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int),
        ("mt", ctypes.c_uint32 * 624),
        ("pos", ctypes.c_int),
        ("key", ctypes.c_uint32 * 2),
        ("stream", ctypes.c_uint64),
        ("ctr", ctypes.c_uint64),
    ]


class _Game(ctypes.Structure):
    _fields_ = [
        ("num_players", ctypes.c_int),
        ("num_cards", ctypes.c_int),
        ("row_len", ctypes.c_int * ROWS),
        ("rows", (ctypes.c_int * THRESHOLD) * ROWS),
        ("hand_len", ctypes.c_int * MAX_PLAYERS),
        ("hands", (ctypes.c_int * HAND) * MAX_PLAYERS),
        ("scores", ctypes.c_int32 * MAX_PLAYERS),
    ]


class _Vec(ctypes.Structure):
    _fields_ = [
        ("num_games", ctypes.c_int),
        ("num_players", ctypes.c_int),
        ("num_cards", ctypes.c_int),
        ("rng_mode", ctypes.c_int),
        ("seed", ctypes.c_uint64),
        ("game_offset", ctypes.c_uint64),
        ("games", ctypes.POINTER(_Game)),
        ("rngs", ctypes.POINTER(_Rng)),
        ("sum_results", ctypes.POINTER(ctypes.c_int32)),
        ("episodes", ctypes.POINTER(ctypes.c_int32)),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        L.or_rng_init_mt.argtypes = [ctypes.POINTER(_Rng), ctypes.c_uint32]
        L.or_rng_init_philox.argtypes = [ctypes.POINTER(_Rng), ctypes.c_uint64, ctypes.c_uint64]
        L.or_rng_next.argtypes = [ctypes.POINTER(_Rng)]
        L.or_rng_next.restype = ctypes.c_uint32
        L.or_rng_interval.argtypes = [ctypes.POINTER(_Rng), ctypes.c_uint32]
        L.or_rng_interval.restype = ctypes.c_uint32
        L.or_shuffle_int.argtypes = [ctypes.POINTER(_Rng), P, ctypes.c_int]
        L.or_philox4x32_10.argtypes = [P, P, P]
        L.or_card_heads.argtypes = [ctypes.c_int]
        L.or_deal_from_deck.argtypes = [ctypes.POINTER(_Game), ctypes.c_int, ctypes.c_int, P]
        L.or_reset.argtypes = [ctypes.POINTER(_Game), ctypes.c_int, ctypes.c_int, ctypes.POINTER(_Rng)]
        L.or_step.argtypes = [ctypes.POINTER(_Game), P, P]
        L.or_is_done.argtypes = [ctypes.POINTER(_Game)]
        L.or_obs.argtypes = [ctypes.POINTER(_Game), ctypes.c_int, ctypes.c_int, P]
        L.or_random_policy.argtypes = [ctypes.POINTER(_Rng), ctypes.POINTER(_Game), ctypes.c_int]
        L.or_vec_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        L.or_vec_create.restype = ctypes.POINTER(_Vec)
        L.or_vec_destroy.argtypes = [ctypes.POINTER(_Vec)]
        L.or_vec_reset.argtypes = [ctypes.POINTER(_Vec)]
        L.or_vec_rollout.argtypes = [ctypes.POINTER(_Vec), ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int]
        L.or_vec_step.argtypes = [ctypes.POINTER(_Vec), P, P, P, P, ctypes.c_int]
        L.or_vec_step.restype = ctypes.c_int
        L.or_vec_obs.argtypes = [ctypes.POINTER(_Vec), ctypes.c_int, P]
        L.or_vec_scores.argtypes = [ctypes.POINTER(_Vec), P]
        L.or_mcs_game.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, P, P]
        L.or_mcs_game.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- RNG
class Rng:
    def __init__(self, mode=RNG_NUMPY_MT, seed=0, stream=0):
        self.s = _Rng()
        if mode == RNG_NUMPY_MT:
            lib().or_rng_init_mt(ctypes.byref(self.s), seed & 0xFFFFFFFF)
        else:
            lib().or_rng_init_philox(ctypes.byref(self.s), seed, stream)

    def next(self):
        return lib().or_rng_next(ctypes.byref(self.s))

    def interval(self, m):
        return lib().or_rng_interval(ctypes.byref(self.s), m)

    def shuffle(self, arr):
        a = np.ascontiguousarray(arr, dtype=np.int32)
        lib().or_shuffle_int(ctypes.byref(self.s), _p(a), len(a))
        return a

    @property
    def key(self):
        return np.ctypeslib.as_array(self.s.mt).copy()


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().or_philox4x32_10(_p(c), _p(k), _p(o))
    return o


def card_heads(c):
    return lib().or_card_heads(int(c))


# ---------------------------------------------------------------- single game
class Game:
    """Scalar game mirroring SechsNimmtEnv (env.py) on the oracle."""

    def __init__(self, num_players, num_cards=104):
        self.g = _Game()
        self.n, self.c = num_players, num_cards

    def deal(self, deck):
        d = np.ascontiguousarray(deck, dtype=np.int32)
        lib().or_deal_from_deck(ctypes.byref(self.g), self.n, self.c, _p(d))

    def reset(self, rng):
        lib().or_reset(ctypes.byref(self.g), self.n, self.c, ctypes.byref(rng.s))

    def set_position(self, board, hands):
        g = self.g
        g.num_players, g.num_cards = len(hands), self.c
        for r in range(ROWS):
            g.row_len[r] = len(board[r])
            for i, c in enumerate(board[r]):
                g.rows[r][i] = c
        for p, h in enumerate(hands):
            g.hand_len[p] = len(h)
            for i, c in enumerate(h):
                g.hands[p][i] = c
            g.scores[p] = 0

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        r = np.zeros(self.n, dtype=np.int32)
        bad = lib().or_step(ctypes.byref(self.g), _p(a), _p(r))
        return bad, r

    def done(self):
        return bool(lib().or_is_done(ctypes.byref(self.g)))

    def obs(self, p, include_summaries=True):
        o = np.zeros(64, dtype=np.int64)
        lib().or_obs(ctypes.byref(self.g), p, int(include_summaries), _p(o))
        return o[: obs_len(include_summaries)]

    def random_action(self, rng, p):
        return lib().or_random_policy(ctypes.byref(rng.s), ctypes.byref(self.g), p)

    @property
    def board(self):
        return [[self.g.rows[r][i] for i in range(self.g.row_len[r])] for r in range(ROWS)]

    @property
    def hands(self):
        return [[self.g.hands[p][i] for i in range(self.g.hand_len[p])] for p in range(self.n)]

    @property
    def scores(self):
        return [self.g.scores[p] for p in range(self.n)]


# ---------------------------------------------------------------- batched
class VecOracle:
    """Batched random-policy self-play with the sn_rollout contract."""

    def __init__(self, num_games, num_players=4, num_cards=104, rng_mode=RNG_NUMPY_MT, seed=0, game_offset=0):
        self.B, self.N, self.C = num_games, num_players, num_cards
        self.v = lib().or_vec_create(num_games, num_players, num_cards, rng_mode, seed, game_offset)

    def __del__(self):
        if getattr(self, "v", None) is not None and _lib is not None:
            _lib.or_vec_destroy(self.v)
            self.v = None

    def reset(self):
        lib().or_vec_reset(self.v)

    def rollout(self, steps, include_summaries=True, want_obs=False, want_actions=True, nthreads=1):
        B, N = self.B, self.N
        rew = np.zeros((steps, B, N), dtype=np.int32)
        done = np.zeros((steps, B), dtype=np.uint8)
        act = np.zeros((steps, B, N), dtype=np.uint8) if want_actions else None
        obs = np.zeros((steps, B, N, obs_len(include_summaries)), dtype=np.int8) if want_obs else None
        lib().or_vec_rollout(self.v, steps, int(include_summaries), _p(rew), _p(done), _p(act), _p(obs), nthreads)
        return rew, done, act, obs

    def step(self, actions, auto_reset=True):
        B, N = self.B, self.N
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(B, N)
        rew = np.zeros((B, N), dtype=np.int32)
        done = np.zeros(B, dtype=np.uint8)
        inv = np.zeros(B, dtype=np.int32)
        lib().or_vec_step(self.v, _p(a), _p(rew), _p(done), _p(inv), int(auto_reset))
        return rew, done, inv

    def obs(self, include_summaries=True):
        o = np.zeros((self.B, self.N, obs_len(include_summaries)), dtype=np.int8)
        lib().or_vec_obs(self.v, int(include_summaries), _p(o))
        return o

    def scores(self):
        s = np.zeros((self.B, self.N), dtype=np.int32)
        lib().or_vec_scores(self.v, _p(s))
        return s

    def hands(self):
        """[B][N] lists of sorted cards"""
        out = []
        for g in range(self.B):
            G = self.v.contents.games[g]
            out.append([[G.hands[p][i] for i in range(G.hand_len[p])] for p in range(self.N)])
        return out

    def sum_results(self):
        return np.ctypeslib.as_array(self.v.contents.sum_results, shape=(self.B * self.N,)).reshape(self.B, self.N).copy()

    def episodes(self):
        return np.ctypeslib.as_array(self.v.contents.episodes, shape=(self.B,)).copy()


def mcs_game(seats, mc_per_card, mc_max, seed):
    n = len(seats)
    a = np.zeros((10, n), dtype=np.int32)
    r = np.zeros((10, n), dtype=np.int32)
    rc = lib().or_mcs_game(seats.encode(), n, mc_per_card, mc_max, seed & 0xFFFFFFFF, _p(a), _p(r))
    return rc, a, r


def mcs_memorize(avail, game, seat, mcs_cards=104):
    a = np.zeros(MAX_CARDS, dtype=np.int32)
    a[: len(avail)] = avail
    lib().or_mcs_memorize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(_Game), ctypes.c_int, ctypes.c_int]
    n = lib().or_mcs_memorize(_p(a), len(avail), ctypes.byref(game.g), seat, mcs_cards)
    return [int(x) for x in a[:n]]


def mcs_stratified(game, seat, avail, rollouts, seed, step, gid):
    a = np.ascontiguousarray(avail, dtype=np.int32)
    s = np.zeros(HAND, dtype=np.int32)
    L = lib()
    L.or_mcs_stratified.argtypes = [ctypes.POINTER(_Game), ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
    L.or_mcs_stratified(ctypes.byref(game.g), seat, _p(a), len(a), rollouts, seed, step, gid, _p(s))
    return s


# ---------------------------------------------------------------- tournament
def league_records(num_agents, min_players, max_players, seed=0, game_offset=0, slots=1, games=1):
    """DrunkHamster tournament streams (tournament.py:132-177 over K
    DrunkHamster agents, play.py:23-75): slot g replays np.random.seed(seed +
    game_offset + g); Tournament(min, max); play_game() x games -- per game
    _choose_players (num_players = lo + random_interval(hi - lo), agents =
    permutation(K)[:k]), env.reset() and 10 DrunkHamster steps.  Returns
    int32 [games, slots, 1 + max_players] in the device's record format
    (seats word k | agent(seat p) << (4 + 4p), then -penalties, 0 past k)."""
    K, N = int(num_agents), int(max_players)
    out = np.zeros((games, slots, 1 + N), dtype=np.int32)
    for j in range(slots):
        rng = Rng(RNG_NUMPY_MT, seed + game_offset + j)
        for e in range(games):
            k = min_players + rng.interval(max_players - min_players)
            seats = rng.shuffle(np.arange(K))[:k]
            g = Game(k)
            g.reset(rng)
            while not g.done():
                acts = [g.random_action(rng, p) for p in range(k)]
                g.step(acts)
            w = k
            for p, a in enumerate(seats):
                w |= int(a) << (4 + 4 * p)
            out[e, j, 0] = w  # < 2^28: K <= 16 agents, k <= 6 seats
            out[e, j, 1: 1 + k] = [-s for s in g.scores]
    return out


def league_mixed_records(kinds, min_players, max_players, mc_per_card=10, mc_max=100, seed=0, game_offset=0, slots=1,
                         games=1, nthreads=None):
    """Tournament streams of DrunkHamster ('R') and MCSAgent ('M') agents
    (tournament.py:132-177, mcts.py:43-188): slot g replays np.random.seed(
    seed + game_offset + g); Tournament(min, max) over the agents in `kinds`;
    play_game() x games -- the MCS seats search on the same global stream,
    in seat order.  Returns (records int32 [games, slots, 1 + max_players] in
    the device's format, q6 int32 [slots]: MCS decisions where a legal move
    got no playout -- quirk Q6, the best sampled move is played)."""
    K = len(kinds)
    mpc = np.ascontiguousarray(np.broadcast_to(np.asarray(mc_per_card, dtype=np.int32), (K,)))
    mmx = np.ascontiguousarray(np.broadcast_to(np.asarray(mc_max, dtype=np.int32), (K,)))
    rec = np.zeros((games, slots, 1 + max_players), dtype=np.int32)
    st = np.zeros(slots, dtype=np.int32)
    L = lib()
    P = ctypes.c_void_p
    L.or_league_mixed.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_uint64,
                                  ctypes.c_uint64, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int]
    if nthreads is None:
        nthreads = max(1, min(16, len(os.sched_getaffinity(0))))
    L.or_league_mixed(kinds.encode(), K, min_players, max_players, _p(mpc), _p(mmx), seed, game_offset, slots, games,
                      _p(rec), _p(st), nthreads)
    return rec, st
