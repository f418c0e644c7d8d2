"""CPU oracle (test infra): the training-window cut and data augmentation of
processing/dataset.py (SequenceDataset.__getitem__ :171-195 and
data_augementation :134-168 with its helpers :18-39), restated in numpy.
Pinned by tests/golden/g6_data.npz (the reference's own functions run in the
build container, tests/golden/make_g6_data.py)."""
import numpy as np


def window(seq, T, ix):
    """dataset.py:174-183: pad with zeros to T+1 tokens, or take [ix, ix+T+1)."""
    seq = np.asarray(seq, dtype=np.int64)
    n = T + 1
    if n > len(seq):
        return np.concatenate([seq, np.zeros(n - len(seq), dtype=np.int64)])
    if len(seq) > n:
        return seq[ix:ix + n].copy()
    return seq.copy()


def shift(seq, r, lb, ub):
    """dataset.py:18-22 shift_sequence."""
    out = seq.copy()
    m = (seq >= lb) & (seq < ub)
    out[m] = np.clip(seq[m] + r, lb, ub - 1)
    return out


def shift_drums(seq, r, lb, ub, P):
    """dataset.py:24-33 shift_sequence_drums."""
    out = seq.copy()
    m = (seq >= lb) & (seq < ub)
    sel = seq[m]
    out[m] = (sel // P) * P + np.clip(sel % P + r, 0, P - 1)
    return out


def multiply(seq, f, lb, ub):
    """dataset.py:35-39 multiply_sequence: float32 arithmetic, int64 truncation."""
    out = seq.copy()
    m = (seq >= lb) & (seq < ub)
    v = (seq[m] - lb).astype(np.float32) * np.float32(f) + np.float32(lb)
    out[m] = np.clip(v, np.float32(lb), np.float32(ub - 1)).astype(np.int64)
    return out


def augment(seq, note_r, vel_r, f, disc):
    """dataset.py:134-168; disc = (pitch, channel, dyn, length, time, tempo)."""
    P, C, D, L, Tm, Tp = disc
    dyn0 = P * C
    len0, time0 = dyn0 + D, dyn0 + D + L
    tempo0 = time0 + Tm
    seq = shift_drums(seq, note_r, 0, P * C - 1, P)
    seq = shift(seq, vel_r, dyn0, dyn0 + D - 1)
    seq = multiply(seq, f, time0, time0 + Tm - 1)
    seq = multiply(seq, f, len0, len0 + L - 1)
    return multiply(seq, f, tempo0, tempo0 + Tp - 1)


def sample(seq, T, ix, aug=None, disc=None):
    """(src, trg) of one training sample; aug = (note_r, vel_r, f) or None."""
    w = window(seq, T, ix)
    if aug is not None:
        w = augment(w, aug[0], aug[1], aug[2], disc)
    return w[:-1], w[1:]
