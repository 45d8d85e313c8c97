"""MI355X-native drop-in for coolo/rl-6-nimmt's hot path.

Same import surface as the reference package (rl_6_nimmt/__init__.py):
    from rl_6_nimmt import SechsNimmtEnv, GameSession, Tournament
plus the batched engine:
    from rl_6_nimmt import VecSechsNimmtEnv
The game rules run in HIP kernels (libsechs.so); there is no CPU fallback.
"""
__version__ = "0.1.0"

_LAZY = {
    "SechsNimmtEnv": ".env",
    "InvalidMoveException": ".env",
    "GameSession": ".play",
    "Tournament": ".tournament",
    "VecSechsNimmtEnv": ".vec_env",
}


def __getattr__(name):
    if name in _LAZY:
        import importlib

        mod = importlib.import_module(_LAZY[name], __name__)
        return getattr(mod, name)
    raise AttributeError(name)


__all__ = list(_LAZY)
