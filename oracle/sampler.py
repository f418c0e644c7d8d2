"""CPU oracle (test infra): the sliding-window autoregressive sampler of
scripts/generate.py:14-95, with torch.multinomial replaced by inverse-CDF
sampling on caller-supplied uniforms (SURVEY.md §7 hard part (d)).
"""
import random
from collections import Counter

import torch

from . import loss as oloss
from .fill import Vocab


def recent_window(cur, v: Vocab):
    """generate.py:36-45. Walk the history backwards summing time-shift values;
    stop at the first reversed position j where the sum reaches 64*16. The
    window is cur[-j:] (so j == 0 means the whole history)."""
    t0, t1 = v.start["time"], v.start["tempo"]
    acc = 0
    j = 0
    for j, tok in enumerate(reversed(cur)):
        if t0 <= tok < t1:
            acc += tok - t0
        if acc >= 64 * 16:
            break
    return cur[-j:]


def choose_k(last: int, v: Vocab, rng: random.Random) -> int:
    """generate.py:47-56 — consumes the Python RNG only for tempo/dyn/pitch."""
    s = v.start
    if last >= s["tempo"]:
        return rng.choice([1, 1, 1, 2, 2])
    if last >= s["time"] or last >= s["length"]:
        return 1
    if last >= s["dyn"]:
        return rng.choice([1, 3])
    return rng.choice([1, 2])


def penalise(z_row: torch.Tensor, recent, v: Vocab):
    """generate.py:58-71 — divide the filtered logit of every pitch (dyn) token
    present in the window by min(1.01**count, 1.2) (min(1.02**count, 1.2))."""
    s = v.start
    for tok, cnt in Counter(recent).items():
        if tok >= s["length"]:
            continue
        pen = min(1.02 ** cnt, 1.2) if tok >= s["dyn"] else min(1.01 ** cnt, 1.2)
        z_row[tok] /= pen


def inverse_cdf(probs: torch.Tensor, u: float) -> int:
    c = torch.cumsum(probs, 0)
    hit = (c > u).nonzero()
    return int(hit[0, 0]) if hit.numel() else probs.numel() - 1


def generate(model_fn, context_len, token_ids, meta_ids, num_tokens, v: Vocab, rng: random.Random, uniforms,
             trace=None):
    """model_fn(idx[B,T], meta[B,6]) -> logits[B,T,V] (fp32). ``uniforms`` is an
    iterator of floats in [0,1) consumed once per (step, row), rows in order."""
    B, _ = token_ids.shape
    hist = [list(map(int, r)) for r in token_ids]
    window = token_ids.clone()
    for step in range(num_tokens):
        if window.shape[1] > context_len:
            window = window[:, -context_len:]
        with torch.no_grad():
            logits = model_fn(window, meta_ids)
        z_last = oloss.filtered_logit(window, logits, v)[:, -1, :].clone()
        ks = []
        for i in range(B):
            recent = recent_window(hist[i], v)
            ks.append(choose_k(hist[i][-1], v, rng))
            penalise(z_last[i], recent, v)
        new = []
        for i in range(B):
            vals, idx = torch.topk(z_last[i], ks[i])
            p = vals / vals.sum()
            pick = inverse_cdf(p, next(uniforms))
            tok = int(idx[pick])
            if trace is not None:
                trace.append((step, i, ks[i], idx.tolist(), p.tolist(), tok))
            new.append(tok)
            hist[i].append(tok)
        window = torch.cat([window, torch.tensor(new, dtype=window.dtype)[:, None]], dim=1)
    return hist
