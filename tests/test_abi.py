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


def test_colstats_applies_at_descriptor_boundary(built):
    """msq_gemm_bias_colstats_applies (host-only): the lm_head statistics
    epilogue is used only where the persistent 256 tile's descriptors cover C
    ((M-1) * ldc + N) * 2 < 0xFFFF0000 and the partials; beyond that (e.g. the
    real vocab v_pad = 17920 at B * T >= 59 * 2048 rows) the caller falls back
    to the plain bias GEMM instead of failing (ops.gemm_bias_colstats)."""
    from midiseq import _lib
    L = _lib.lib()
    base = 1 << 40  # any 16-B aligned address: nothing is dereferenced
    N, K, pld = 17920, 1024, 17920

    def applies(M, ldc=N, c=base):
        return L.msq_gemm_bias_colstats_applies(0, M, N, K, base, K, base, K, c, ldc, base, base, pld)

    m_max = (0xFFFF0000 // 2 - N) // N + 1  # largest M with the C extent in range
    m_ok = m_max // 256 * 256
    assert applies(32 * 2048)
    assert applies(m_ok)
    assert not applies(m_ok + 256)
    assert not applies(59 * 2048)
    assert not applies(32 * 2048, c=base + 8)  # C not 16-B aligned
    assert not applies(32 * 2048 + 128)  # M % 256
    L.msq_gemm_set_route(_lib.ROUTE_TILE128)
    try:
        assert not applies(32 * 2048)
    finally:
        L.msq_gemm_set_route(_lib.ROUTE_DEFAULT)
