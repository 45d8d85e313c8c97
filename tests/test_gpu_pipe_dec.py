"""Decode-ahead pipeline (SN_OPT_PIPE_DEC, k_play_dec): a launch plays from
per-game records of its draws and deal that the launch before decoded from
the ring, and decodes the next launch in other waves.  It is an optimisation
only: against the oracle (oracle/sechs_oracle.c, the restatement of env.py +
DrunkHamster + numpy's legacy MT19937) every action, reward, done flag,
observation and final numpy state is identical, through launch patterns that
make the speculative decode of a rollout's last launch right or wrong."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rl_6_nimmt.vec_env import VecSechsNimmtEnv

pytestmark = pytest.mark.gpu


def venv(B, N, seed, dec=1):
    env = VecSechsNimmtEnv(B, N, seed=seed, rng="numpy", device="cuda:0")
    env.set_option(pipe_dec=dec)
    return env


def _np_form(key, pos):
    key = np.asarray(key, dtype=np.uint32)
    return key, int(pos)


def _check_states(env, ref, games):
    rngs = ref.v.contents.rngs
    for g in games:
        k, p = _np_form(*env.get_mt_state(g))
        rk, rp = _np_form(np.frombuffer(bytes(rngs[g].mt), dtype=np.uint32), rngs[g].pos)
        assert p == rp and np.array_equal(k, rk), g


@pytest.mark.parametrize("N", [2, 3, 4])
@pytest.mark.parametrize("plan", [(10, 10, 10), (25, 7, 3, 10, 10), (1, 1, 2, 10), (37,)])
def test_pipe_dec_rollouts_match_oracle(N, plan):
    B, seed = 300, 17
    env = venv(B, N, seed)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    for T in plan:
        out = env.rollout(T, want_actions=True, want_obs=True, check=True)
        rr, rd, ra, ro = ref.rollout(T, want_obs=True)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra), T
        assert np.array_equal(out["rewards"].cpu().numpy(), rr), T
        assert np.array_equal(out["done"].cpu().numpy(), rd), T
        assert np.array_equal(out["obs"].cpu().numpy()[..., :47], ro), T
    _check_states(env, ref, range(0, B, 11))
    s, e = env.results()
    assert np.array_equal(s.cpu().numpy(), ref.sum_results())
    assert env.pipe_errors() == 0


def test_pipe_dec_interleaves_with_every_other_path():
    """A pending speculative decode is dropped by whatever else touches the
    handle: external-action steps, reset, reset_to, numpy state import /
    export, the non-decode pipeline, option changes."""
    B, N, seed = 130, 4, 5
    env = venv(B, N, seed)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    rngs = ref.v.contents.rngs
    plan = [("roll", 13), ("step", 1), ("roll", 4), ("reset", 0), ("roll", 9), ("plain", 6), ("roll", 21),
            ("import", 0), ("roll", 12), ("export", 0), ("roll", 10), ("reset_to", 0), ("roll", 10), ("roll", 1),
            ("roll", 30)]
    for what, T in plan:
        if what in ("roll", "plain"):
            env.set_option(pipe_dec=int(what == "roll"))
            out = env.rollout(T, want_actions=True)
            rr, rd, ra, _ = ref.rollout(T)
            torch.cuda.synchronize()
            assert np.array_equal(out["actions"].cpu().numpy(), ra), what
            assert np.array_equal(out["rewards"].cpu().numpy(), rr), what
            assert np.array_equal(out["done"].cpu().numpy(), rd), what
        elif what == "step":
            for _ in range(12):
                acts = env.hands().cpu().numpy()[:, :, 0].astype(np.int32)
                rew, done, inv = env.step(torch.from_numpy(acts), auto_reset=True)
                r_rew, r_done, r_inv = ref.step(acts, auto_reset=True)
                assert np.array_equal(rew.cpu().numpy(), r_rew)
        elif what == "reset":
            env.reset()
            ref.reset()
        elif what == "reset_to":  # every game to the oracle's own current state (hands/board unchanged)
            board = env.board().cpu().numpy()
            hands = env.hands().cpu().numpy()
            env.reset_to(board, hands)
        elif what == "export":
            _check_states(env, ref, range(0, B, 9))
        elif what == "import":
            rs = np.random.RandomState(77)
            rs.randint(0, 2**32, size=300, dtype=np.uint64)
            key, pos = rs.get_state()[1:3]
            for g in (0, 5, 129):
                env.set_mt_state(key, pos, game=g)
                for i in range(624):
                    rngs[g].mt[i] = int(key[i])
                rngs[g].pos = int(pos)
    _check_states(env, ref, range(0, B, 3))
    assert env.pipe_errors() == 0


def test_pipe_dec_full_size_headline():
    """The bench's workload (65 536 x 4 players, one episode per rollout(10),
    int8 obs) for 3 episodes: bit-exact, no overrun, and the same as the
    one-wave pipeline (pipe_dec 0) on a second handle."""
    B, N, seed = 65536, 4, 0
    env = venv(B, N, seed)
    env.reset()
    ref = O.VecOracle(B, N, rng_mode=O.RNG_NUMPY_MT, seed=seed)
    ref.reset()
    for ep in range(3):
        out = env.rollout(10, want_actions=True, want_obs=True, check=True)
        rr, rd, ra, ro = ref.rollout(10, want_obs=True, nthreads=16)
        torch.cuda.synchronize()
        assert np.array_equal(out["actions"].cpu().numpy(), ra), ep
        assert np.array_equal(out["rewards"].cpu().numpy(), rr), ep
        assert np.array_equal(out["done"].cpu().numpy(), rd), ep
        assert np.array_equal(out["obs"].cpu().numpy()[..., :47], ro), ep
    assert env.pipe_errors() == 0
    _check_states(env, ref, range(0, B, 4099))
