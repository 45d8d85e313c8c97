"""CPU-side checks of the drop-in boundary: libsechs.so loads and exports
every symbol include/sechs.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import PKG_ROOT, ROOT

HEADER = os.path.join(ROOT, "include", "sechs.h")
LIB = os.path.join(PKG_ROOT, "libsechs.so")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sn_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["sn_create", "sn_destroy", "sn_reset", "sn_reset_to", "sn_step", "sn_rollout", "sn_obs", "sn_hands",
              "sn_board", "sn_scores", "sn_results", "sn_mt_get", "sn_mt_set", "sn_last_error"]:
        assert s in syms


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsechs.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  share torch's HIP runtime

    lib = ctypes.CDLL(LIB)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    from rl_6_nimmt import _native

    assert sorted(_native.SIGNATURES) == declared_symbols()
    assert _native.lib().sn_version().decode().startswith("sechs-mi355x")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsechs.so not built")
def test_library_is_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_product_never_imports_the_oracle():
    pkg = os.path.join(PKG_ROOT, "rl_6_nimmt")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle|liboracle|sechs_oracle", src, flags=re.M), f
