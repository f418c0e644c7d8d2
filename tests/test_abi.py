"""CPU checks of the C ABI boundary: the library loads, exports every symbol
declared in include/midiseq.h, and the ctypes table mirrors the header."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "midiseq.h")


def _declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(msq_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def built():
    import midiseq._build as b
    return b.build()


def test_library_exports_every_declared_symbol(built):
    lib = ctypes.CDLL(built)
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    from midiseq import _lib
    assert set(_lib.SIGNATURES) == set(_declared())


def test_error_plumbing(built):
    from midiseq import _lib
    L = _lib.lib()
    assert L.msq_version() >= 1
    # argument validation runs on the host, no GPU needed
    rc = L.msq_gemm(7, 0, 0, 1, 1, 1, None, 1, 0, None, 1, 0, None, 0, 1, 0, 1, 0, None, None, 0, 0, 0, None)
    assert rc == -1 and b"dtype" in L.msq_last_error()
    rc = L.msq_layernorm_fwd(None, 0, None, None, None, None, None, 4, 6, 1e-5, 0, 0, None)
    assert rc == -1
