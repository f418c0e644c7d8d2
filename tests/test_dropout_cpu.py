"""CPU checks of the dropout keep-mask oracle (oracle/dropout.py): rate, site
and seed independence, and that p = 0 leaves the oracle forward unchanged."""
import numpy as np
import pytest
import torch

from midiseq import _lib as L

from oracle import dropout as odrop
from oracle import transformer as otr


def test_keep_rate_and_independence():
    for p in (0.01, 0.1, 0.5):
        k = odrop.keep(1, odrop.PROJ, 256, 1024, p)
        n = k.size
        assert abs((1 - k.mean()) - p) < 6 * np.sqrt(p * (1 - p) / n)
    a = odrop.keep(1, odrop.PROJ, 64, 64, 0.5)
    b = odrop.keep(1, odrop.FFN, 64, 64, 0.5)
    c = odrop.keep(2, odrop.PROJ, 64, 64, 0.5)
    assert np.array_equal(a, odrop.keep(1, odrop.PROJ, 64, 64, 0.5))
    assert 0.4 < (a == b).mean() < 0.6 and 0.4 < (a == c).mean() < 0.6


def test_threshold_and_scale_match_kernel_formula():
    assert odrop.threshold(0.0) == 0
    assert odrop.threshold(0.01) == int(float(np.float32(0.01)) * 2 ** 32 + 0.5)
    assert abs(odrop.scale(0.01) - 1 / 0.99) < 1e-6


def test_attn_keep_layout():
    k = odrop.attn_keep(3, 1, 2, 2, 40, 0.2)
    assert k.shape == (2, 2, 40, 40)
    assert np.array_equal(k[1, 0], odrop.attn_keep_site(3, odrop.ATTN + 65536 + 2, 40, 0.2))
    assert odrop.attn_keep(3, 1, 1, 1, 70, 0.0).all()


@pytest.mark.parametrize("p", [0.0, 0.01, 0.1, 0.2, 0.5, 0.9])
def test_attn_table_matches_library(p):
    """The Binomial(64, p) thresholds of the attention keep words: the oracle's
    float64 restatement equals the library's host table bit for bit."""
    out = np.zeros(64, dtype=np.uint32)
    assert L.lib().msq_dropout_attn_table(float(p), out.ctypes.data) == 0
    assert np.array_equal(out, odrop.attn_table(p))
    if p > 0:
        from math import comb
        q = float(np.float32(p))  # the library takes p as a float
        cdf = np.cumsum([comb(64, t) * q ** t * (1 - q) ** (64 - t) for t in range(64)])
        assert np.abs(out.astype(np.float64) / 2 ** 32 - np.minimum(cdf, 1.0)).max() < 1e-9


@pytest.mark.parametrize("p", [0.01, 0.1, 0.5])
def test_attn_keep_words_rate_position_and_pairs(p):
    """Keep words: each of the 64 positions is dropped at rate p, and two
    positions of a word independently (pair rate p^2), over 2^17 words."""
    rk = odrop.row_key(odrop.base(7, odrop.ATTN + 3), np.arange(1 << 15, dtype=np.uint64).astype(np.uint32))
    words = np.concatenate([odrop.attn_words(rk, jb, odrop.attn_table(p)) for jb in range(4)])
    bits = ((words[:, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)) == 0  # dropped
    n = bits.shape[0]
    per_pos = bits.mean(0)
    assert np.abs(per_pos - p).max() < 6 * np.sqrt(p * (1 - p) / n)
    pair = (bits[:, 3] & bits[:, 40]).mean()
    assert abs(pair - p * p) < 6 * np.sqrt(p * p * (1 - p * p) / n) + 1e-5
    cnt = bits.sum(1)
    assert abs(cnt.var() - 64 * p * (1 - p)) < 0.05 * 64 * p * (1 - p) + 0.02


def test_zero_p_forward_unchanged():
    shapes = otr.param_shapes(32, 4, 2, 16, 34, 568)
    p = otr.filled_params(shapes)
    idx = torch.randint(0, 34, (2, 16), generator=torch.Generator().manual_seed(0))
    meta = torch.randint(0, 568, (2, 6), generator=torch.Generator().manual_seed(1))
    a = otr.forward(p, idx, meta, 2, 4)
    b = otr.forward(p, idx, meta, 2, 4, drop=(5, 0.0))
    assert torch.equal(a, b)
