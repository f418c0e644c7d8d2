"""CPU ORACLE (test infra): dropout keep masks of nn.Dropout
(model_transformer.py:51 proj, :80 attention probabilities, :101 FFN output)
as drawn by this build.

The reference draws its masks from torch's Philox stream; that stream cannot
be reproduced outside torch, so the build uses a counter-based hash instead and
parity is checked with the oracle applying the SAME mask. This module restates
the hash of csrc/common.h (drop_mix / drop_base / drop_row / drop_bits) bit-exactly
in numpy uint32 arithmetic. The semantics follow nn.Dropout: an element is kept
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


def attn_keep(seed, layer, B, H, S, p):
    """bool [B, H, S, S] keep mask of the attention probabilities of one layer."""
    out = np.empty((B, H, S, S), dtype=bool)
    for b in range(B):
        for h in range(H):
            out[b, h] = keep(seed, ATTN + layer * 65536 + b * H + h, S, S, p)
    return out


def scale(p):
    return float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
