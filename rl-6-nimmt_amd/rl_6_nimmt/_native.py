"""ctypes binding of libsechs.so (include/sechs.h).

The library is built in-tree (rl-6-nimmt_amd/libsechs.so, `make -C
rl-6-nimmt_amd`).  There is no CPU fallback: if the library or a GPU is
missing, every entry point raises.

torch is imported first so that libsechs.so binds to the HIP runtime torch
already loaded (both carry the soname libamdhip64.so.7); device pointers and
streams are then shared with torch tensors.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below, see module doc)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SECHS_LIB", os.path.join(_PKG_ROOT, "libsechs.so"))

SN_OK, SN_EINVAL, SN_EHIP, SN_ENOMEM, SN_EUNSUPPORTED, SN_ERNG = 0, 1, 2, 3, 4, 5
SN_RNG_PHILOX, SN_RNG_NUMPY_MT = 0, 1
SN_I8, SN_I16, SN_I32, SN_I64, SN_F32 = 1, 2, 3, 4, 5
SN_AUTO_RESET, SN_NO_SUMMARIES = 1, 2
SN_OPT_RING_WORDS, SN_OPT_CHUNK_STEPS, SN_OPT_PIPELINE, SN_OPT_TIMING, SN_OPT_PIPE_GPW, SN_OPT_PIPE_LEAD = 1, 2, 3, 4, 5, 6
SN_OPT_PLAY_SPLIT = 7
SN_OPT_TWIST_ROUND = 9
SN_OPT_TWIST_EVERY = 10
SN_OPT_TWIST_SKIP = 12  # test knob: the default schedule runs its ring dry
SN_OPT_PIPE_DEC = 13
SN_AGENT_RANDOM, SN_AGENT_MCS, SN_AGENT_EXTERNAL = 0, 1, 2

class SnPuct(ctypes.Structure):
    """sn_puct (include/sechs.h)"""

    _fields_ = [
        ("seats_mask", ctypes.c_uint32),
        ("n", ctypes.c_int),
        ("puct_root", ctypes.c_int),
        ("c_puct", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("step", ctypes.c_uint32),
        ("rollout", ctypes.c_uint32),
        ("avail", ctypes.c_void_p),
        ("rollouts", ctypes.c_void_p),
        ("stats", ctypes.c_void_p),
        ("hist", ctypes.c_void_p),
        ("root_probs", ctypes.c_void_p),
        ("step_dev", ctypes.c_void_p),
        ("dec_list", ctypes.c_void_p),
        ("num_dec", ctypes.c_int64),
        ("logit_stride", ctypes.c_int32),
        ("logit_bf16", ctypes.c_int32),
    ]


# every symbol include/sechs.h declares, with its ctypes signature
_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
SIGNATURES = {
    "sn_last_error": ([], ctypes.c_char_p),
    "sn_version": ([], ctypes.c_char_p),
    "sn_create": ([ctypes.POINTER(_P), _I, _I64, _I, _I, _U64, _U64, _I], _I),
    "sn_destroy": ([_P], _I),
    "sn_info": ([_P, _P, _P, _P, _P], _I),
    "sn_reset": ([_P, _P, _P], _I),
    "sn_reset_to": ([_P, _P, _P, _P], _I),
    "sn_step": ([_P, _P, _P, _P, _P, _I, _P], _I),
    "sn_rollout": ([_P, _I, _P, _P, _P, _P, _I, _I, _P], _I),
    "sn_obs": ([_P, _P, _I, _I, _I, _P], _I),
    "sn_hands": ([_P, _P, _P], _I),
    "sn_board": ([_P, _P, _P], _I),
    "sn_scores": ([_P, _P, _P], _I),
    "sn_results": ([_P, _P, _P, _P], _I),
    "sn_clear_results": ([_P, _P], _I),
    "sn_mt_get": ([_P, _I64, _P, _P], _I),
    "sn_mt_set": ([_P, _I64, _P, ctypes.c_int32], _I),
    "sn_philox_counter": ([_P, _I64, _P], _I),
    "sn_set_option": ([_P, _I, _I], _I),
    "sn_pipe_errors": ([_P, _P], _I),
    "sn_kernel_times": ([_P, _P, _P, _P], _I),
    "sn_kernel_times_dec": ([_P, _P, _P, _P, _P], _I),
    "sn_debug_phases": ([_P, _I], _I),
    "sn_debug_puct_phases": ([_P, _I], _I),
    "sn_debug_pipe_words": ([_P, _I, _I, _P], _I),
    "sn_debug_failures": ([_P, _P, _I], _I),
    "sn_step1": ([_P, _P, _P, _I], _I),
    "sn_reset1": ([_P, _P, ctypes.c_int32, _P, _P, _P, _I], _I),
    "sn_league_config": ([_P, _I, _I, _I], _I),
    "sn_league_rollout": ([_P, _I, _P, _P, _P, _P, _I, _P, _P], _I),
    "sn_league_seats": ([_P, _P, _P], _I),
    "sn_league_agents": ([_P, _P, _P, _P], _I),
    "sn_league_step": ([_P, _P, _P, _P, _P, _P, _P, _P], _I),
    "sn_elo_replay": ([_P, _I64, _I, _I, ctypes.c_double, _P], _I),
    "sn_mcs_memorize": ([_P, _P, _I, _P], _I),
    "sn_mcs_rollouts": ([_P, _P, _I, _U64, ctypes.c_uint32, _P, _P], _I),
    "sn_mcs_rollouts_ex": ([_P, _P, _I, _U64, ctypes.c_uint32, _P, _P, _P], _I),
    "sn_mcs_choose": ([_P, _P, _P, _P], _I),
    "sn_mcs_play_exact": ([_P, ctypes.c_uint32, _I, _I, _P, _P, _P, _P], _I),
    "sn_mcs_decide_exact": ([_I, _I64, _I, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P], _I),
    "sn_puct_root_rows": ([_P, _P, _P, _I, _P], _I),
    "sn_puct_init": ([_P, _P, _P, _P], _I),
    "sn_puct_deal": ([_P, _P, _P], _I),
    "sn_puct_deal_batch": ([_P, _P, _I, _I, _P, _P], _I),
    "sn_puct_rollouts": ([_P, _P, _I, _I, _P, _P, _P, _P, _P, _P], _I),
    "sn_puct_rows": ([_P, _P, _I, _P, _I, _P], _I),
    "sn_puct_step": ([_P, _P, _P, _I, _I, _P], _I),
    "sn_puct_mlp_seats": ([_P, _P, _I, _P, _P, _P, _P, _P, _P], _I),
    "sn_puct_choose": ([_P, _P, _P, _P, _P], _I),
    "sn_pcv_choose": ([_P, _P, _P, _P, _P, _P, _P, _P], _I),
    "sn_policy_sample": ([_P, _P, _P, _P, _P, _P, _P, _P], _I),
    "sn_puct_score": ([_I64, _P, _P, _P, _P, ctypes.c_double, _P, _P, _P], _I),
}


class NativeError(RuntimeError):
    pass


class PipeOverrunError(NativeError):
    """A pipelined numpy-MT draw ran past the twisted words (SN_ERNG): the
    handle's rollouts from that launch on are not the reference's."""


_lib = None


def lib():
    """Load libsechs.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"libsechs.so not found at {LIB_PATH}; build it with `make -C {_PKG_ROOT}` "
                "(or __graft_entry__.build()). There is no CPU fallback."
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(status, what=""):
    if status != SN_OK:
        msg = lib().sn_last_error().decode(errors="replace")
        if status == SN_EINVAL:
            raise ValueError(f"{what}: {msg}")
        if status == SN_EUNSUPPORTED:
            raise NotImplementedError(f"{what}: {msg}")
        if status == SN_ERNG:
            raise PipeOverrunError(f"{what}: {msg}")
        raise NativeError(f"{what} failed ({status}): {msg}")


def require_gpu():
    if not torch.cuda.is_available():
        raise NativeError("no HIP device visible: the 6 nimmt! engine runs only on the GPU (no CPU fallback)")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
