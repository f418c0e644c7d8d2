"""Element-level gradient pins against the golden files (make_golden.py:197-198
and :322-323 record, per gradient tensor, [signed sum, |g| sum, sum of
squares] and 64 strided elements g.reshape(-1)[::max(1, n // 64)][:64]).

check_grad compares all four: the signed sum (within tol of the |g| sum, so
a sign error cannot hide behind a matching magnitude), the |g| sum and the
sum of squares (relative), and every picked element (within tol of the
largest picked magnitude). Analytically-zero gradients (the loss is
invariant to a per-(b, v) shift along T) are round-off noise in both runs
and are checked by the callers against an absolute floor instead."""
import numpy as np


def picks(g):
    gf = np.asarray(g, dtype=np.float64).reshape(-1)
    return gf[:: max(1, gf.size // 64)][:64]


def check_grad(name, g, gsum, gpick, tol):
    gf = np.asarray(g, dtype=np.float64).reshape(-1)
    s, a, q = gf.sum(), np.abs(gf).sum(), (gf * gf).sum()
    assert abs(a - gsum[1]) <= tol * abs(gsum[1]) + 1e-9, (name, "abs sum", a, gsum[1])
    assert abs(q - gsum[2]) <= 2 * tol * abs(gsum[2]) + 1e-12, (name, "sum sq", q, gsum[2])
    assert abs(s - gsum[0]) <= tol * abs(gsum[1]) + 1e-9, (name, "signed sum", s, gsum[0], gsum[1])
    p, r = picks(gf), np.asarray(gpick, dtype=np.float64)
    assert p.shape == r.shape, (name, p.shape, r.shape)
    err = np.abs(p - r).max()
    assert err <= tol * np.abs(r).max() + 1e-9, (name, "picked elements", err, np.abs(r).max())
