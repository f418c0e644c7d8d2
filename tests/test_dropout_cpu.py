"""CPU checks of the dropout keep-mask oracle (oracle/dropout.py): rate, site
and seed independence, and that p = 0 leaves the oracle forward unchanged."""
import numpy as np
import torch

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
    assert np.array_equal(k[1, 0], odrop.keep(3, odrop.ATTN + 65536 + 2, 40, 40, 0.2))


def test_zero_p_forward_unchanged():
    shapes = otr.param_shapes(32, 4, 2, 16, 34, 568)
    p = otr.filled_params(shapes)
    idx = torch.randint(0, 34, (2, 16), generator=torch.Generator().manual_seed(0))
    meta = torch.randint(0, 568, (2, 6), generator=torch.Generator().manual_seed(1))
    a = otr.forward(p, idx, meta, 2, 4)
    b = otr.forward(p, idx, meta, 2, 4, drop=(5, 0.0))
    assert torch.equal(a, b)
