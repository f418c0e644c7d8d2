"""CPU ORACLE (test infra): dropout keep masks of nn.Dropout
(model_transformer.py:51 proj, :80 attention probabilities, :101 FFN output)
as drawn by this build.

The reference draws its masks from torch's Philox stream; that stream cannot
be reproduced outside torch, so the build uses a counter-based hash instead and
parity is checked with the oracle applying the SAME mask. This module restates
the hash of csrc/common.h (drop_mix / drop_base / drop_row / drop_bits, and
for the attention probabilities the keep-word draw attn_word_key /
attn_drop_draw / attn_drop_table) bit-exactly in numpy uint32 / float64
arithmetic. The semantics follow nn.Dropout: an element is kept
with probability 1-p and kept values are scaled by 1/(1-p).

Sites (engine convention, transformer.py): attention of layer l, batch b, head h
= ATTN + l*65536 + b*H + h (rows i = query, cols j = key); proj output of layer
l = PROJ + l; FFN output = FFN + l (rows = flat B*S row, cols = feature).
"""
import numpy as np

ATTN, PROJ, FFN = 1 << 28, 2 << 28, 3 << 28

_U = np.uint32


def mix(x):
    x = np.asarray(x, dtype=_U)
    with np.errstate(over="ignore"):
        x = x ^ (x >> _U(16))
        x = (x * _U(0x7FEB352D)).astype(_U)
        x = x ^ (x >> _U(15))
    return x


def base(seed, site):
    with np.errstate(over="ignore"):
        return mix(_U(seed) ^ mix(_U((int(site) + 0x9E3779B9) & 0xFFFFFFFF)))


def row_key(b, rows):
    with np.errstate(over="ignore"):
        return mix((_U(b) + np.asarray(rows, dtype=_U) * _U(0x9E3779B9)).astype(_U))


def bits(rk, cols):
    with np.errstate(over="ignore"):
        return mix(np.asarray(rk, dtype=_U) ^ (np.asarray(cols, dtype=_U) * _U(0x85EBCA6B)).astype(_U))


def threshold(p):
    t = float(np.float32(p)) * 4294967296.0
    return 0 if t <= 0 else (0xFFFFFFFF if t >= 4294967295.0 else int(t + 0.5))


def keep(seed, site, n_rows, n_cols, p):
    """bool [n_rows, n_cols] keep mask of one site."""
    rk = row_key(base(seed, site), np.arange(n_rows, dtype=np.uint64).astype(_U))
    return bits(rk[:, None], np.arange(n_cols, dtype=np.uint64).astype(_U)[None, :]) >= _U(threshold(p))


def attn_table(p):
    """uint32 [64]: T[t] = round(2^32 P(K <= t)), K ~ Binomial(64, p) (common.h
    attn_drop_table: the same float64 operations in the same order)."""
    q = float(np.float32(p))
    r = q / (1.0 - q)
    pmf = 1.0 - q
    for _ in range(6):
        pmf = pmf * pmf
    cdf = 0.0
    out = np.empty(64, dtype=np.uint64)
    for t in range(64):
        cdf = cdf + pmf
        sc = cdf * 4294967296.0
        rd = sc + 0.5
        out[t] = 0xFFFFFFFF if (q <= 0.0 or rd >= 4294967295.0) else int(rd)
        pmf = pmf * float(64 - t)
        pmf = pmf / float(t + 1)
        pmf = pmf * r
    return out.astype(_U)


def _nth_set_bit(w, n):
    """bit index of the n-th set bit of each uint64 w (n < popcount(w))"""
    w = w.copy()
    n = n.astype(np.int64).copy()
    pos = np.zeros(w.shape, dtype=np.int64)
    for sh in (32, 16, 8, 4, 2, 1):
        c = np.bitwise_count(w & np.uint64((1 << sh) - 1)).astype(np.int64)
        up = n >= c
        n = np.where(up, n - c, n)
        w = np.where(up, w >> np.uint64(sh), w)
        pos = np.where(up, pos + sh, pos)
    return pos


def attn_words(rowkeys, jb, table, on=True):
    """uint64 keep words of the rows with these row keys over keys 64 jb .. +63
    (common.h attn_word_key: bit c = key 64 jb + c kept)."""
    with np.errstate(over="ignore"):
        key = mix(np.asarray(rowkeys, dtype=_U) ^ _U(((jb + 1) * 0xC2B2AE35) & 0xFFFFFFFF))
    k = (key[:, None] >= table[None, :]).sum(1) if on else np.zeros(key.shape, dtype=np.int64)
    w = np.full(key.shape, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    for s in range(int(k.max()) if k.size else 0):
        with np.errstate(over="ignore"):
            d = mix((key + _U(((s + 1) * 0x9E3779B9) & 0xFFFFFFFF)).astype(_U))
        n = (d.astype(np.uint64) * np.uint64(64 - s)) >> np.uint64(32)
        pos = _nth_set_bit(w, n)
        act = k > s
        w = np.where(act, w & ~(np.uint64(1) << pos.astype(np.uint64)), w)
    return w


def attn_keep_site(seed, site, S, p):
    """bool [S, S] keep mask of one (layer, b, h) attention site: row i, key j."""
    table = attn_table(p)
    nb = (S + 63) // 64
    rk = row_key(base(seed, site), np.arange(nb * 64, dtype=np.uint64).astype(_U))
    out = np.empty((nb * 64, nb * 64), dtype=bool)
    for jb in range(nb):
        w = attn_words(rk, jb, table, on=p > 0)
        out[:, jb * 64:(jb + 1) * 64] = ((w[:, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)) != 0
    return out[:S, :S]


def attn_keep(seed, layer, B, H, S, p):
    """bool [B, H, S, S] keep mask of the attention probabilities of one layer."""
    out = np.empty((B, H, S, S), dtype=bool)
    for b in range(B):
        for h in range(H):
            out[b, h] = attn_keep_site(seed, ATTN + layer * 65536 + b * H + h, S, p)
    return out


def scale(p):
    return float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
