"""GPU parity: libsechs.so kernels vs the CPU oracle and the reference's golden vectors.

Bit-exact for everything (integer/index work): rewards, done flags,
actions, observations, hands, board, scores, RNG streams.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RNG = {"numpy": O.RNG_NUMPY_MT, "philox": O.RNG_PHILOX}


def venv(*a, **k):
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(*a, **k)
    # SECHS_TEST_TWIST_EVERY=2 / 3: the same parity tests with one twist-ahead per 2 / 3 play launches
    # SECHS_TEST_TWIST_ROUND=0: with exact-lead (partial) twists instead of whole rounds
    if env.rng == "numpy" and os.environ.get("SECHS_TEST_TWIST_EVERY"):
        env.set_option(twist_every=int(os.environ["SECHS_TEST_TWIST_EVERY"]))
    if env.rng == "numpy" and os.environ.get("SECHS_TEST_TWIST_ROUND"):
        env.set_option(twist_round=int(os.environ["SECHS_TEST_TWIST_ROUND"]))
    return env


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("rng", ["numpy", "philox"])
@pytest.mark.parametrize("N,C,summ", [(4, 104, True), (2, 104, True), (3, 40, True), (10, 104, True), (1, 104, True),
                                      (5, 104, False), (7, 80, True)])
def test_rollout_matches_oracle(rng, N, C, summ):
    B, T = 1000, 23  # ragged B (not a multiple of 256), episodes cross launch boundaries
    seed = 12345
    env = venv(B, N, C, seed=seed, rng=rng, include_summaries=summ)
    env.reset()
    ref = O.VecOracle(B, N, C, rng_mode=RNG[rng], seed=seed)
    ref.reset()
    L = O.obs_len(summ)
    for chunk in (T, 1, 16):
        out = env.rollout(chunk, want_actions=True, want_obs=True)
        rr, rd, ra, ro = ref.rollout(chunk, include_summaries=summ, want_obs=True)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra)
        assert np.array_equal(out["rewards"].cpu().numpy(), rr)
        assert np.array_equal(out["done"].cpu().numpy(), rd)
        o = out["obs"].cpu().numpy()
        assert np.array_equal(o[..., :L], ro)
        assert not o[..., L:].any()
    assert np.array_equal(env.hands().cpu().numpy(), _pad_hands(ref.hands(), N))
    assert np.array_equal(env.scores().cpu().numpy(), ref.scores())
    s, e = env.results()
    assert np.array_equal(s.cpu().numpy(), ref.sum_results())
    assert np.array_equal(e.cpu().numpy(), ref.episodes())
    for dt in (torch.int8, torch.int16, torch.int64, torch.float32):
        assert np.array_equal(env.obs(dt).cpu().numpy(), ref.obs(summ).astype(np.int64).astype(dt_np(dt)))
    if rng == "numpy":
        assert env.pipe_errors() == 0


def dt_np(dt):
    return {torch.int8: np.int8, torch.int16: np.int16, torch.int64: np.int64, torch.float32: np.float32}[dt]


def _pad_hands(hands, N):
    out = np.full((len(hands), N, 10), -1, dtype=np.int8)
    for g, hs in enumerate(hands):
        for p, h in enumerate(hs):
            out[g, p, : len(h)] = h
    return out


@pytest.mark.parametrize("rng", ["numpy", "philox"])
def test_full_size_episode_matches_oracle(rng):
    """BASELINE config 2 size: 65 536 x 4-player games, one full episode with
    the int8 observations the headline emits, bit-exact."""
    B, N = 65536, 4
    env = venv(B, N, seed=0, rng=rng)
    env.reset()
    out = env.rollout(10, want_actions=True, want_obs=True, check=True)
    ref = O.VecOracle(B, N, rng_mode=RNG[rng], seed=0)
    ref.reset()
    rr, rd, ra, ro = ref.rollout(10, want_obs=True, nthreads=16)
    torch.cuda.synchronize()
    assert np.array_equal(out["actions"].cpu().numpy(), ra)
    assert np.array_equal(out["rewards"].cpu().numpy(), rr)
    assert np.array_equal(out["done"].cpu().numpy(), rd)
    o = out["obs"].cpu().numpy()
    assert np.array_equal(o[..., :47], ro)
    assert not o[..., 47:].any()
    del o, ro
    # size-independent properties: every game ends after exactly 10 steps, the
    # 104-card deck holds 171 heads, so no episode can cost more than that
    d = out["done"].cpu().numpy()
    assert d[9].all() and not d[:9].any()
    tot = -out["rewards"].cpu().numpy().sum(axis=(0, 2))
    assert tot.min() >= 0 and tot.max() <= 171


def test_bench_lanes_replay_reference_sessions():
    """game g seeded g, 100 episodes back to back == reference GameSession(DrunkHamster x4)."""
    d = load("random_sessions.json")
    recs = [r for r in d["sessions"] if r.get("episodes") == 100]
    B = 65536
    env = venv(B, 4, seed=0, rng="numpy")
    env.reset()
    last = None
    for ep in range(100):
        out = env.rollout(10)
        last = out["rewards"]
    s, e = env.results()
    s, e = s.cpu().numpy(), e.cpu().numpy()
    last = last.sum(dim=0).cpu().numpy()
    for r in recs:
        g = r["seed"]
        assert e[g] == 100
        assert s[g].tolist() == r["results_sum"]
        assert last[g].tolist() == r["results_last"]


def test_multi_episode_sessions_all_sizes():
    d = load("random_sessions.json")
    for r in d["sessions"]:
        if "results" not in r:
            continue
        n, eps = r["num_players"], len(r["results"])
        env = venv(1, n, seed=r["seed"], rng="numpy")
        env.reset()
        out = env.rollout(10 * eps)
        per_ep = out["rewards"][:, 0, :].reshape(eps, 10, n).sum(dim=1).cpu().numpy()
        assert per_ep.tolist() == r["results"]


def test_random_games_golden_obs():
    meta = load("random_games_meta.json")
    z = np.load(os.path.join(GOLDEN, "random_games.npz"))
    for cfg in meta["configs"]:
        k, n, c, summ, S = cfg["key"], cfg["num_players"], cfg["num_cards"], cfg["include_summaries"], cfg["seeds"]
        L = cfg["obs_len"]
        # game g of a handle with seed 0 is np.random.seed(g)
        env = venv(S, n, c, seed=0, rng="numpy", include_summaries=summ)
        env.reset()
        out = env.rollout(10, want_actions=True, want_obs=True)
        assert np.array_equal(out["actions"].cpu().numpy().transpose(1, 0, 2), z[k + "_actions"])
        assert np.array_equal(out["rewards"].cpu().numpy().transpose(1, 0, 2), z[k + "_rewards"])
        assert np.array_equal(out["obs"].cpu().numpy()[..., :L].transpose(1, 0, 2, 3), z[k + "_obs"][:, :10])


def test_reset_to_edge_cases_golden():
    d = load("edge_cases.json")
    by_n = {}
    for case in d["cases"]:
        if case.get("error", {}).get("type") == "AssertionError":
            continue
        by_n.setdefault((len(case["hands"]), case["include_summaries"]), []).append(case)
    for (n, summ), cases in by_n.items():
        B = len(cases)
        board = np.full((B, 4, 6), -1, dtype=np.int8)
        hands = np.full((B, n, 10), -1, dtype=np.int8)
        acts = np.zeros((B, n), dtype=np.int32)
        for g, c in enumerate(cases):
            for r, row in enumerate(c["board"]):
                board[g, r, : len(row)] = row
            for p, h in enumerate(c["hands"]):
                hands[g, p, : len(h)] = h
            acts[g] = c["actions"]
        env = venv(B, n, seed=0, rng="philox", include_summaries=summ)
        env.reset_to(board, hands)
        L = O.obs_len(summ)
        obs0 = env.obs(torch.int64).cpu().numpy()
        rew, done, inv = env.step(torch.from_numpy(acts))
        obs1 = env.obs(torch.int64).cpu().numpy()
        b1, h1, s1 = env.board().cpu().numpy(), env.hands().cpu().numpy(), env.scores().cpu().numpy()
        rew, done, inv = rew.cpu().numpy(), done.cpu().numpy(), inv.cpu().numpy()
        for g, c in enumerate(cases):
            # hands are card sets on the device: reset_to with an unsorted hand
            # list yields the sorted legal list (the reference's own callers
            # always pass sorted hands, env.py:108 and mcts.py:118-125)
            canon = lambda o: [sorted(x for x in row[:10] if x >= 0) + [-1] * sum(1 for x in row[:10] if x < 0) + row[10:] for row in o]
            assert obs0[g, :, :L].tolist() == canon(c["obs0"]), c["label"]
            if "error" in c:
                assert inv[g] >= 0, c["label"]
                assert c["error"]["message"].startswith(f"Player {inv[g] + 1} tried")
                continue
            e = c["expect"]
            assert inv[g] == -1, c["label"]
            assert rew[g].tolist() == e["rewards"], c["label"]
            assert bool(done[g]) == e["done"]
            assert [[x for x in row if x >= 0] for row in b1[g].tolist()] == e["board"], c["label"]
            assert [[x for x in h if x >= 0] for h in h1[g].tolist()] == [sorted(h) for h in e["hands"]]
            assert s1[g].tolist() == e["scores"]
            assert obs1[g, :, :L].tolist() == canon(e["obs"]), c["label"]


def test_notebook_games_through_step_api():
    d = load("notebook_games.json")
    games = d["games"]
    B = len(games)
    board = np.full((B, 4, 6), -1, dtype=np.int8)
    hands = np.full((B, 2, 10), -1, dtype=np.int8)
    for g, G in enumerate(games):
        for r, row in enumerate(G["board"]):
            board[g, r, : len(row)] = row
        for p, h in enumerate(G["hands"]):
            hands[g, p, : len(h)] = h
    env = venv(B, 2, seed=0, rng="philox")
    env.reset_to(board, hands)
    for t in range(10):
        acts = torch.tensor([G["actions"][t] for G in games], dtype=torch.int32)
        rew, done, inv = env.step(acts)
        obs = env.obs(torch.int64).cpu().numpy()
        for g, G in enumerate(games):
            assert inv[g].item() == -1
            assert rew[g].tolist() == G["steps"][t]["rewards"]
            assert obs[g].tolist() == G["steps"][t]["obs"]
            assert bool(done[g]) == G["steps"][t]["done"]
    assert (-env.scores().cpu().numpy()).tolist() == [G["final_scores"] for G in games]


@pytest.mark.parametrize("rng", ["numpy", "philox"])
def test_step_api_external_actions_vs_oracle(rng):
    B, N = 3000, 4
    env = venv(B, N, seed=77, rng=rng)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=RNG[rng], seed=77)
    ref.reset()
    gen = np.random.RandomState(5)
    for t in range(25):
        h = env.hands().cpu().numpy()
        n = (h[:, 0] >= 0).sum(axis=1)
        pick = (gen.rand(B, N) * n[:, None]).astype(np.int64)
        acts = np.take_along_axis(h, pick[..., None], axis=2)[..., 0].astype(np.int32)
        bad = gen.rand(B) < 0.02  # sprinkle illegal moves
        acts[bad, 1] = 103 - acts[bad, 1]
        rew, done, inv = env.step(torch.from_numpy(acts), auto_reset=True)
        r_rew, r_done, r_inv = ref.step(acts, auto_reset=True)
        assert np.array_equal(inv.cpu().numpy(), r_inv)
        assert np.array_equal(rew.cpu().numpy(), r_rew)
        assert np.array_equal(done.cpu().numpy().astype(np.uint8), r_done)
        assert np.array_equal(env.obs().cpu().numpy(), ref.obs())


def test_numpy_rng_bridge_roundtrip():
    env = venv(2, 4, seed=0, rng="numpy")
    env.reset()
    env.rollout(7)
    key, pos = env.get_mt_state(1)
    rs = np.random.RandomState(1)
    gs = O.VecOracle(2, 4, rng_mode=O.RNG_NUMPY_MT, seed=0)
    gs.reset()
    gs.rollout(7)
    # the exported state must continue the stream exactly like numpy
    rs.set_state(("MT19937", key, pos, 0, 0.0))
    nxt = rs.randint(0, 2**32, size=1000, dtype=np.uint64)
    r = gs.v.contents.rngs[1]
    ora = O.Rng.__new__(O.Rng)
    ora.s = r
    assert [int(x) for x in nxt] == [ora.next() for _ in range(1000)]
    # import a numpy state and draw on the device
    rs = np.random.RandomState(99)
    rs.randint(0, 10, size=37)
    st = rs.get_state()
    env.set_mt_state(st[1], st[2], game=0)
    env.reset()
    deck = np.arange(104)
    rs.shuffle(deck)
    b = env.board().cpu().numpy()[0]
    assert [int(x) for x in b[:, 0]] == [int(deck[103 - r]) for r in range(4)]
    k2, p2 = env.get_mt_state(0)
    assert np.array_equal(k2, rs.get_state()[1]) and p2 == rs.get_state()[2]


def _np_form(key, pos):
    """(key, pos) with a pending twist applied, so equal streams compare equal."""
    key = np.array(key, dtype=np.uint32)
    if pos < 624:
        return key, pos
    rs = np.random.RandomState()
    rs.set_state(("MT19937", key, 624, 0, 0.0))
    rs.randint(0, 2**32, size=1, dtype=np.uint64)  # forces the twist, consumes word 0
    k2, p2 = rs.get_state()[1:3]
    return np.array(k2, dtype=np.uint32), p2 - 1


def test_mt_state_across_round_boundaries_every_step():
    """Single-step launches: after every env-step the exported MT19937 state
    of every game equals the oracle's numpy state, across several 624-word
    rounds (launches end mid-straddle for some games), and after importing a
    mid-round numpy state that runs out during the next episodes."""
    B, N, seed = 64, 4, 7
    env = venv(B, N, seed=seed, rng="numpy")
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    rngs = ref.v.contents.rngs
    for t in range(90):
        if t == 45:  # import a state 20 words before the end of its round into games 0..7
            rs = np.random.RandomState(1234 + t)
            rs.randint(0, 2**32, size=604, dtype=np.uint64)
            key, pos = rs.get_state()[1:3]
            for g in range(8):
                env.set_mt_state(key, pos, game=g)
                for i in range(624):
                    rngs[g].mt[i] = int(key[i])
                rngs[g].pos = int(pos)
        out = env.rollout(1, want_actions=True)
        rr, rd, ra, _ = ref.rollout(1)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra), t
        assert np.array_equal(out["rewards"].cpu().numpy(), rr), t
        for g in range(B):
            k, p = _np_form(*env.get_mt_state(g))
            rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
            assert p == rp and np.array_equal(k, rk), (t, g)


@pytest.mark.parametrize("ring_words,chunk_steps,pipeline,gpw", [(0, 10, 0, 64), (64, 10, 0, 64), (64, 1, 0, 64),
                                                                  (128, 3, 0, 64), (512, 25, 0, 64), (256, 7, 0, 64),
                                                                  (256, 10, 1, 64), (256, 3, 1, 64), (0, 1, 1, 64),
                                                                  (512, 25, 1, 64), (256, 10, 1, 32), (0, 3, 1, 32),
                                                                  (0, 25, 1, 32)])
def test_ring_options_do_not_change_results(ring_words, chunk_steps, pipeline, gpw):
    """The twist-ahead paths are optimisations only: every ring size (0 =
    lazy per-lane MT19937; 64 runs k_mt_prep's ring dry inside every
    episode, so the slow path continues mid-launch), launch chunking, and
    the pipelined k_mt_ahead (concurrent with the previous k_play) give the
    oracle's actions, rewards, obs and final numpy MT states."""
    B, N, T, seed = 300, 4, 37, 21
    env = venv(B, N, seed=seed, rng="numpy")
    env.set_option(ring_words=ring_words, chunk_steps=chunk_steps, pipeline=pipeline, pipe_gpw=gpw)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    out = env.rollout(T, want_actions=True, want_obs=True)
    rr, rd, ra, ro = ref.rollout(T, want_obs=True)
    torch.cuda.synchronize()
    assert np.array_equal(out["actions"].cpu().numpy(), ra)
    assert np.array_equal(out["rewards"].cpu().numpy(), rr)
    assert np.array_equal(out["done"].cpu().numpy(), rd)
    assert np.array_equal(out["obs"].cpu().numpy()[..., :47], ro)
    rngs = ref.v.contents.rngs
    for g in range(0, B, 7):
        k, p = _np_form(*env.get_mt_state(g))
        rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
        assert p == rp and np.array_equal(k, rk), g
    assert env.pipe_errors() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("rng,split", [("numpy", 0), ("philox", 0), ("philox", 1)])
@pytest.mark.parametrize("N", [2, 4])
def test_play_split_modes_match_oracle(rng, split, N):
    """SN_OPT_PLAY_SPLIT (role-split k_play of philox handles: producer waves
    decode every random decision into LDS) changes nothing observable: ragged B, launches
    that start mid-episode (3 then 10-step chunks: the deal falls inside a
    launch), obs/actions/rewards/done and the final RNG states equal the
    oracle's."""
    B, T0, T, seed = 300, 3, 37, 5
    env = venv(B, N, seed=seed, rng=rng)
    env.set_option(play_split=split)
    env.reset()
    mode = O.RNG_NUMPY_MT if rng == "numpy" else O.RNG_PHILOX
    ref = O.VecOracle(B, N, rng_mode=mode, seed=seed)
    ref.reset()
    for t in (T0, T):
        out = env.rollout(t, want_actions=True, want_obs=True)
        rr, rd, ra, ro = ref.rollout(t, want_obs=True)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra)
        assert np.array_equal(out["rewards"].cpu().numpy(), rr)
        assert np.array_equal(out["done"].cpu().numpy(), rd)
        assert np.array_equal(out["obs"].cpu().numpy()[..., :47], ro)
    if rng == "numpy":
        rngs = ref.v.contents.rngs
        for g in range(0, B, 13):
            k, p = _np_form(*env.get_mt_state(g))
            rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
            assert p == rp and np.array_equal(k, rk), g
        assert env.pipe_errors() == 0


def test_ring_option_validation():
    env = venv(4, 4, rng="numpy")
    for bad in (-64, 32, 576):
        with pytest.raises(ValueError):
            env.set_option(ring_words=bad)
    with pytest.raises(ValueError):
        env.set_option(chunk_steps=0)
    penv = venv(4, 4, rng="philox")
    with pytest.raises(ValueError):
        penv.set_option(ring_words=256)


def test_kernel_timing_is_observational():
    """SN_OPT_TIMING only records events: rollouts stay bit-exact with the
    oracle, every timed launch is counted (capped at the requested number)
    and both kernels report a positive duration."""
    B, N, seed = 500, 4, 9
    env = venv(B, N, seed=seed, rng="numpy")
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    env.time_kernels(3)
    for T in (10, 10, 10, 10):
        out = env.rollout(T, want_actions=True)
        rr, rd, ra, _ = ref.rollout(T)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra)
        assert np.array_equal(out["rewards"].cpu().numpy(), rr)
    play_ms, ahead_ms, n = env.kernel_times()
    assert n == 3 and play_ms > 0 and ahead_ms > 0
    env.time_kernels(0)
    assert env.kernel_times()[2] == 0
    with pytest.raises(ValueError):
        env.time_kernels(-1)
    assert env.pipe_errors() == 0


def test_pipeline_then_other_paths_interleave():
    """The pipelined twist-ahead state (ring, a k_mt_ahead in flight) is
    folded back into the MT state whenever anything else touches the stream
    (per-step API with external actions, reset, the k_mt_prep path, numpy
    state import): every mix stays bit-exact with the oracle."""
    B, N, seed = 130, 4, 5
    env = venv(B, N, seed=seed, rng="numpy")
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    rngs = ref.v.contents.rngs
    plan = [("roll", 13), ("step", 1), ("roll", 4), ("reset", 0), ("roll", 9), ("prep", 6), ("roll", 21),
            ("import", 0), ("roll", 12), ("roll", 1), ("roll", 30)]
    for what, T in plan:
        if what == "roll":
            env.set_option(pipeline=1)
            out = env.rollout(T, want_actions=True)
            rr, rd, ra, _ = ref.rollout(T)
            torch.cuda.synchronize()
            assert np.array_equal(out["actions"].cpu().numpy(), ra), what
            assert np.array_equal(out["rewards"].cpu().numpy(), rr), what
        elif what == "prep":
            env.set_option(pipeline=0)
            out = env.rollout(T, want_actions=True)
            rr, rd, ra, _ = ref.rollout(T)
            torch.cuda.synchronize()
            assert np.array_equal(out["actions"].cpu().numpy(), ra), what
        elif what == "step":  # external actions (lazy MtGen path; deals of finished games draw words)
            for _ in range(12):
                acts = env.hands().cpu().numpy()[:, :, 0].astype(np.int32)
                rew, done, inv = env.step(torch.from_numpy(acts), auto_reset=True)
                r_rew, r_done, r_inv = ref.step(acts, auto_reset=True)
                assert np.array_equal(rew.cpu().numpy(), r_rew)
        elif what == "reset":
            env.reset()
            ref.reset()
        elif what == "import":
            rs = np.random.RandomState(77)
            rs.randint(0, 2**32, size=300, dtype=np.uint64)
            key, pos = rs.get_state()[1:3]
            for g in (0, 5, 129):
                env.set_mt_state(key, pos, game=g)
                for i in range(624):
                    rngs[g].mt[i] = int(key[i])
                rngs[g].pos = int(pos)
    for g in range(0, B, 3):
        k, p = _np_form(*env.get_mt_state(g))
        rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
        assert p == rp and np.array_equal(k, rk), g


@pytest.mark.parametrize("N", [9, 10])
def test_pipelined_many_players_full_size(N):
    """The default pipelined numpy-MT path at 65 536 games and 9 / 10
    players without observations (the case whose LDS fits the pipelined
    k_play and whose launch pairs draw the most words): 3 episodes = 6
    launches (5 env-steps each at N >= 5, sechs_env.hip pipe_max_chunk),
    bit-exact against the oracle, no overrun."""
    B, seed = 65536, 3
    env = venv(B, N, seed=seed, rng="numpy")
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    for ep in range(3):
        out = env.rollout(10, want_actions=True, check=True)
        rr, rd, ra, _ = ref.rollout(10, nthreads=16)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra), ep
        assert np.array_equal(out["rewards"].cpu().numpy(), rr), ep
        assert np.array_equal(out["done"].cpu().numpy(), rd), ep
    assert env.pipe_errors() == 0
    s, e = env.results()
    assert np.array_equal(s.cpu().numpy(), ref.sum_results())


@pytest.mark.parametrize("N,chunk", [(9, 10), (10, 10), (10, 3), (5, 7), (6, 10)])
def test_pipelined_many_players_chunks(N, chunk):
    """pipelined rollouts at N >= 5 with requested launch lengths above and
    below the per-N cap: bit-exact, final numpy MT states equal, no overrun"""
    B, T, seed = 2000, 37, 8
    env = venv(B, N, seed=seed, rng="numpy")
    env.set_option(chunk_steps=chunk, pipeline=1)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    out = env.rollout(T, want_actions=True, check=True)
    rr, rd, ra, _ = ref.rollout(T)
    torch.cuda.synchronize()
    assert np.array_equal(out["actions"].cpu().numpy(), ra)
    assert np.array_equal(out["rewards"].cpu().numpy(), rr)
    rngs = ref.v.contents.rngs
    for g in range(0, B, 97):
        k, p = _np_form(*env.get_mt_state(g))
        rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
        assert p == rp and np.array_equal(k, rk), g
    assert env.pipe_errors() == 0


@pytest.mark.parametrize("N,lead", [(10, 128), (4, 96)])
def test_pipelined_overrun_is_an_error(N, lead):
    """With the lead lowered below a launch pair's draws (test knob), lanes
    overrun: the count is nonzero, rollout(check=True) raises at once, and
    the next rollout raises from the asynchronous mirror (sticky)."""
    from rl_6_nimmt._native import PipeOverrunError

    env = venv(4096, N, seed=1, rng="numpy")
    # exact-lead twists beside every launch: whole-round ones overshoot a short lead by up
    # to a round, so the first launches would not run dry -- the detection is the same;
    # the default schedule's own case is test_default_schedule_overrun_is_an_error
    env.set_option(pipe_lead=lead, twist_round=0, twist_every=1)
    env.reset()
    with pytest.raises(PipeOverrunError):
        env.rollout(20, check=True)
    assert env.pipe_errors() > 0
    with pytest.raises(PipeOverrunError):
        env.rollout(10)


@pytest.mark.parametrize("N", [4, 10])
def test_default_schedule_overrun_is_an_error(N):
    """VERDICT r05 #1a: the overrun detector under the DEFAULT pipeline (whole-
    round twists, one twist per four play launches, 10-step launches at
    N <= 4): SN_OPT_TWIST_SKIP makes every steady twist after the first
    group's twist nothing, so the consumers run past the words the start-up
    twist left (600 K = 2 400 words, ~12 episodes at N = 4) -- the play lanes
    count perr, rollout(check=True) raises, sn_pipe_errors > 0, and the next
    rollout raises from the sticky host mirror.  Until then the games equal
    the oracle (the detector does not fire early)."""
    from rl_6_nimmt._native import PipeOverrunError

    B = 2048
    env = venv(B, N, seed=3, rng="numpy")
    env.set_option(twist_skip=1)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=3)
    ref.reset()
    out = env.rollout(40, want_actions=True, check=True)  # within the start-up lead: exact
    rr, rd, ra, _ = ref.rollout(40)
    assert np.array_equal(out["actions"].cpu().numpy(), ra) and np.array_equal(out["rewards"].cpu().numpy(), rr)
    assert env.pipe_errors() == 0
    with pytest.raises(PipeOverrunError):
        env.rollout(200, check=True)
    assert env.pipe_errors() > 0
    with pytest.raises(PipeOverrunError):
        env.rollout(10)
    env.close()


@pytest.mark.parametrize("plan", [(10, 10, 10, 10), (25, 1, 1, 7, 30), (3, 10, 10)])
def test_pipelined_launch_plans_match_oracle(plan):
    """several pipelined launches per call and 1-step launches: each launch's
    twist-ahead hands its ring to the next play launch (events both ways) --
    actions, rewards, obs and final MT states equal the oracle's"""
    B, N, seed = 300, 4, 31
    env = venv(B, N, seed=seed, rng="numpy")
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    for T in plan:
        out = env.rollout(T, want_actions=True, want_obs=True)
        rr, rd, ra, ro = ref.rollout(T, want_obs=True)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra), T
        assert np.array_equal(out["rewards"].cpu().numpy(), rr), T
        assert np.array_equal(out["obs"].cpu().numpy()[..., :47], ro), T
    rngs = ref.v.contents.rngs
    for g in range(0, B, 11):
        k, p = _np_form(*env.get_mt_state(g))
        rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
        assert p == rp and np.array_equal(k, rk), g
    assert env.pipe_errors() == 0


@pytest.mark.parametrize("N,C,summ", [(4, 104, True), (2, 104, False), (3, 40, True), (1, 104, True)])
def test_decode_ahead_equals_ring_play(N, C, summ):
    """SN_OPT_PIPE_DEC (round 6, the default where it applies): k_decode
    walks the ring a group ahead and k_play<RNG_NUMPY_DEC> plays from its
    records -- the same outputs as k_play drawing from the ring itself
    (pipe_dec=0), launch plans that start mid-episode and cross deals
    (25 / 1 / 7 / 3 / 30 / 10 steps: records of two episodes per launch),
    the pipeline restarted after a mid-rollout MT export (phi0 > 0 at the
    new start), K = 1 / 4 groups; then the same exported numpy states, the
    same results, and the oracle agrees on the first rollouts."""
    B, seed = 1500, 5
    outs = {}
    for dec in (1, 0):
        for K in (4, 1):
            env = venv(B, N, num_cards=C, seed=seed, rng="numpy", include_summaries=summ)
            env.set_option(pipe_dec=dec, twist_every=K)
            env.reset()
            got = []
            for i, T in enumerate((25, 1, 7, 3, 30, 10)):
                o = env.rollout(T, want_actions=True, want_obs=True, check=True)
                got.append({k: v.cpu().numpy() for k, v in o.items()})
                if i == 2:  # a sync in the middle: the pipeline restarts at step 3 of an episode
                    got.append({"mt": np.append(*env.get_mt_state(B // 2))})
            s_, e_ = env.results()
            got.append({"sums": s_.cpu().numpy(), "eps": e_.cpu().numpy(), "hands": env.hands().cpu().numpy()})
            got.append({f"mt{g}": np.append(*env.get_mt_state(g)) for g in (0, 777, B - 1)})
            assert env.pipe_errors() == 0
            outs[(dec, K)] = got
            env.close()
    for key in ((1, 4), (1, 1), (0, 1)):
        for a, b in zip(outs[key], outs[(0, 4)]):
            assert a.keys() == b.keys()
            for k in a:
                assert np.array_equal(a[k], b[k]), (key, k)
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed, num_cards=C)
    ref.reset()
    rr, rd, ra, ro = ref.rollout(25, include_summaries=summ, want_obs=True)
    assert np.array_equal(outs[(1, 4)][0]["rewards"], rr) and np.array_equal(outs[(1, 4)][0]["actions"], ra)
    assert np.array_equal(outs[(1, 4)][0]["obs"][..., : O.obs_len(summ)], ro)


def test_pipelined_full_size_across_streams():
    """65 536 games, 12 back-to-back episodes of the pipeline with the
    caller's stream switching between rollouts (the library orders a new
    stream behind the last play launch): every episode equals the oracle
    (checked on 16 sampled games' own oracle streams) and no lane overran"""
    B, N, seed = 65536, 4, 3
    env = venv(B, N, seed=seed, rng="numpy")
    env.reset()
    idx = np.arange(0, B, 64)
    refs = [O.VecOracle(1, N, rng_mode=O.RNG_NUMPY_MT, seed=seed, game_offset=int(g)) for g in idx[:16]]
    for r in refs:
        r.reset()
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    for e in range(12):
        with torch.cuda.stream(streams[e % 3]):
            out = env.rollout(10, want_actions=True)
            torch.cuda.current_stream().synchronize()
        acts = out["actions"].cpu().numpy()
        for j, r in enumerate(refs):
            _, _, ra, _ = r.rollout(10)
            assert np.array_equal(acts[:, idx[j]], ra[:, 0]), (e, j)
    torch.cuda.synchronize()
    assert env.pipe_errors() == 0


_DEBUG_WORKLOAD = r"""
import ctypes, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from rl_6_nimmt import _native as nat
from rl_6_nimmt.vec_env import VecSechsNimmtEnv
from rl_6_nimmt import SechsNimmtEnv
from rl_6_nimmt.league import BatchedTournament
from rl_6_nimmt.agents import MCSAgent
L = nat.lib()
cnt, line = ctypes.c_uint32(), ctypes.c_uint32()
nat.check(L.sn_debug_failures(ctypes.byref(cnt), ctypes.byref(line), 1), "selftest")
assert cnt.value == 1, cnt.value  # the deliberately failing check was counted
for rng in ("numpy", "philox"):
    env = VecSechsNimmtEnv(8192, 4, seed=5, rng=rng)
    env.reset()
    for T in (10, 3, 17):
        env.rollout(T, want_actions=True, want_obs=True, check=rng == "numpy")
    env.close()
env = VecSechsNimmtEnv(1000, 3, seed=2, rng="numpy")
env.reset()
env.rollout(25, want_obs=True)
env.close()
np.random.seed(1)
e1 = SechsNimmtEnv(4, verbose=False)
for g in range(20):
    (st, legal) = e1.reset()
    done = False
    while not done:
        (st, legal), r, done, _ = e1.step([l[np.random.randint(len(l))] for l in legal])
t = BatchedTournament(512, 2, 4, seed=1, rng="numpy", fused=False)
for i in range(3):
    t.add_player(f"r{i}")
t.add_player("m", MCSAgent(mc_max=20))
t.play_games(2)
t.close()
torch.cuda.synchronize()
nat.check(L.sn_debug_failures(ctypes.byref(cnt), ctypes.byref(line), 0), "failures")
print("debug failures", cnt.value, "first line", line.value)
assert cnt.value == 0, (cnt.value, line.value)
"""


def test_debug_library_invariants_hold():
    """SURVEY §5 / VERDICT r04 #8: libsechs_debug.so (-DSECHS_DEBUG: SN_DASSERT
    invariant checks counted on the device) runs numpy / philox rollouts with
    both play kernels, ragged 3-player handles, drop-in games and a league
    with an MCS seat in one process: the self-test's deliberate failure is
    counted (the checks are live), the workload's count is 0."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "rl-6-nimmt_amd", "libsechs_debug.so")
    assert os.path.exists(lib), "make -C rl-6-nimmt_amd libsechs_debug.so"
    envv = dict(os.environ, SECHS_LIB=lib)
    r = subprocess.run([sys.executable, "-c", _DEBUG_WORKLOAD, os.path.join(root, "rl-6-nimmt_amd")], env=envv,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "debug failures 0" in r.stdout
