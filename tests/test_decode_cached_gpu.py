"""The Transformer's cached decode (generate(mode="cached"), BASELINE cfg 5
"KV-cache AR decode") against its own oracle restatement
(oracle/transformer.py CachedTransformer; an approximation of the reference's
full forward per token, scripts/generate.py:26-31, documented in
midiseq/generate.py).

* fp32 engine: token ids bit-exact against the oracle sampler driven by
  CachedTransformer on the same uniforms and Python RNG, with the window
  growing, full and sliding (prompt shorter than / equal to the context).
* the first sampled token equals the exact mode's (the prefill is exact).
* bf16 engine (hs = 128, msq_relattn_decode's bf16 path): the cached logits
  rows of a teacher-forced run within 3e-2 of max against the fp32 oracle."""
import random

import numpy as np
import pytest
import torch

from oracle import transformer as otr
from oracle import sampler as osamp
from oracle.fill import TINY, REAL, grammar_tokens
from midiseq.transformer import Transformer, TransformerConfig
from midiseq.generate import generate
from midiseq.config import Grammar, Discretization

pytestmark = pytest.mark.gpu


def grammar_for(v):
    d = v.disc
    return Grammar(Discretization(pitch=d["pitch"], channel=d["channel"], dyn=d["dyn"], length=d["length"],
                                  time=d["time"], tempo=d["tempo"]))


def _model(vocab, mv, hp, precision):
    cfg = TransformerConfig(vocab_size=vocab.size, metadata_vocab_size=mv, precision=precision, dropout=0.0, **hp)
    m = Transformer(cfg).to("cuda").eval()
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], vocab.size, mv)
    p = otr.filled_params(shapes)
    m.load_state_dict(p)
    return m, p


CASES = {"tiny": (TINY, 10, dict(n_embd=32, n_heads=4, n_layer=2, block_len=16)),
         "small": (REAL, 568, dict(n_embd=64, n_heads=4, n_layer=2, block_len=48))}


@pytest.mark.parametrize("tag,T0,steps", [("tiny", 16, 12), ("tiny", 9, 14), ("small", 48, 10), ("small", 30, 25)])
def test_cached_fp32_ids_match_oracle(tag, T0, steps):
    vocab, mv, hp = CASES[tag]
    m, p = _model(vocab, mv, hp, "fp32")
    rng = np.random.default_rng(T0 + steps)
    B = 2
    src = torch.from_numpy(np.stack([grammar_tokens(rng, vocab, T0) for _ in range(B)]))
    meta = torch.from_numpy(rng.integers(0, mv, size=(B, 6)))
    us = rng.random(B * steps).tolist()
    got = generate(m, hp["block_len"], src, meta, num_tokens=steps, rng=random.Random(7), uniforms=iter(us),
                   grammar=grammar_for(vocab), mode="cached")
    oracle_model = otr.CachedTransformer(p, hp["n_layer"], hp["n_heads"], hp["block_len"])
    ref = osamp.generate(oracle_model, hp["block_len"], src, meta, steps, vocab, random.Random(7), iter(us))
    np.testing.assert_array_equal(np.array(got), np.array(ref))


def test_cached_fp32_ids_ctx2048_multiblock():
    """The benched context (cfg 5: 2048 = 32 ring blocks of msq_ring_lse's
    RB = 64 rows). Prefill 1900 tokens, then 300 steps: the window fills at step
    148 and slides for 152 more, so every step recomputes only its slot's block
    (blk_lo..blk_hi) and, at the block crossings (slots 1920, 1984, the wrap
    2047 -> 0, 64, 128), the previous row's block (the ``extra`` branch), and
    the merge runs over all 32 partials. hs = 128 like the default model; the
    tiny vocabulary keeps the oracle's per-step filtered_logit over the whole
    window cheap. Token ids bit-exact against the oracle sampler."""
    vocab, mv = TINY, 10
    hp = dict(n_embd=256, n_heads=2, n_layer=1, block_len=2048)
    m, p = _model(vocab, mv, hp, "fp32")
    eng = m.engine
    rng = np.random.default_rng(2048)
    B, T0, steps = 2, 1900, 300
    src = torch.from_numpy(np.stack([grammar_tokens(rng, vocab, T0) for _ in range(B)]))
    meta = torch.from_numpy(rng.integers(0, mv, size=(B, 6)))
    us = rng.random(B * steps).tolist()
    got = generate(m, hp["block_len"], src, meta, num_tokens=steps, rng=random.Random(11), uniforms=iter(us),
                   grammar=grammar_for(vocab), mode="cached")
    oracle_model = otr.CachedTransformer(p, hp["n_layer"], hp["n_heads"], hp["block_len"])
    ref = osamp.generate(oracle_model, hp["block_len"], src, meta, steps, vocab, random.Random(11), iter(us))
    np.testing.assert_array_equal(np.array(got), np.array(ref))
    assert eng is m.engine


def test_cached_bf16_ring_lse_ctx2000():
    """bf16 engine, real vocabulary, context 2000 (31 full ring blocks + one of
    16 rows): prefill 1950, 120 teacher-forced steps (the window slides after
    50). Checks the ring rows and cache.lse — the time-axis LSE over the
    window's other rows that msq_ring_lse assembles from per-block partials —
    against CachedTransformer's fp32 rows, within 3e-2 of max."""
    hp = dict(n_embd=256, n_heads=2, n_layer=1, block_len=2000)
    m, p = _model(REAL, 568, hp, "bf16")
    eng = m.engine
    rng = np.random.default_rng(5)
    B, T0, steps, ctx = 2, 1950, 120, hp["block_len"]
    toks = torch.from_numpy(np.stack([grammar_tokens(rng, REAL, T0 + steps) for _ in range(B)]))
    meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]])
    cache = eng.decode_cache(B, ctx)
    with torch.no_grad():
        eng.forward(toks[:, :T0].cuda(), meta.cuda(), save=False, cache=cache)
        for t in range(T0, T0 + steps):
            eng.step(toks[:, t].contiguous().cuda(), cache)
    torch.cuda.synchronize()
    ref = otr.CachedTransformer(p, hp["n_layer"], hp["n_heads"], ctx)
    win = toks[:, :T0]
    with torch.no_grad():
        rows = ref(win, meta)
        for t in range(T0, T0 + steps):
            win = torch.cat([win, toks[:, t:t + 1]], 1)[:, -ctx:]
            rows = ref(win, meta)
    n = T0 + steps
    first = n - ctx
    order = [(first + r) % ctx for r in range(ctx)]
    got = cache.ring[:, order, :REAL.size].float().cpu()
    scale = rows.abs().max()
    assert ((got - rows).abs().max() / scale).item() < 3e-2
    # cache.lse after the last step: LSE over the window's rows except the newest
    ref_lse = torch.logsumexp(rows[:, :-1], dim=1)
    lse = cache.lse.cpu()
    assert torch.isfinite(lse).all()
    assert ((lse - ref_lse).abs().max() / scale).item() < 3e-2
    assert torch.equal(cache.tokens[:, order].cpu(), toks[:, first:n])


def test_first_cached_token_equals_exact():
    vocab, mv, hp = CASES["small"]
    m, _ = _model(vocab, mv, hp, "fp32")
    rng = np.random.default_rng(1)
    src = torch.from_numpy(np.stack([grammar_tokens(rng, vocab, 48) for _ in range(3)]))
    meta = torch.from_numpy(rng.integers(0, mv, size=(3, 6)))
    us = rng.random(3).tolist()
    a = generate(m, 48, src, meta, num_tokens=1, rng=random.Random(0), uniforms=iter(us), grammar=grammar_for(vocab))
    b = generate(m, 48, src, meta, num_tokens=1, rng=random.Random(0), uniforms=iter(us), grammar=grammar_for(vocab),
                 mode="cached")
    assert a == b


def test_cached_bf16_rows_against_oracle():
    """Teacher-forced: prefill a 60-token prompt, then 30 steps (the window of
    64 slides after 4) on fixed tokens; the window's logits rows (bf16 ring)
    against CachedTransformer's fp32 rows."""
    hp = dict(n_embd=256, n_heads=2, n_layer=2, block_len=64)
    m, p = _model(REAL, 568, hp, "bf16")
    eng = m.engine
    rng = np.random.default_rng(3)
    B, T0, steps = 2, 60, 30
    toks = torch.from_numpy(np.stack([grammar_tokens(rng, REAL, T0 + steps) for _ in range(B)]))
    meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]])
    cache = eng.decode_cache(B, hp["block_len"])
    with torch.no_grad():
        eng.forward(toks[:, :T0].cuda(), meta.cuda(), save=False, cache=cache)
        for t in range(T0, T0 + steps):
            eng.step(toks[:, t].contiguous().cuda(), cache)
    torch.cuda.synchronize()
    ref = otr.CachedTransformer(p, hp["n_layer"], hp["n_heads"], hp["block_len"])
    win = toks[:, :T0]
    rows = ref(win, meta)
    for t in range(T0, T0 + steps):
        win = torch.cat([win, toks[:, t:t + 1]], 1)[:, -hp["block_len"]:]
        rows = ref(win, meta)
    # ring slot of window row r: (first + r) % ctx
    n = T0 + steps
    first = n - hp["block_len"]
    order = [(first + r) % hp["block_len"] for r in range(hp["block_len"])]
    got = cache.ring[:, order, :REAL.size].float().cpu()
    err = ((got - rows).abs().max() / rows.abs().max()).item()
    assert err < 3e-2, err
    assert torch.equal(cache.tokens[:, order].cpu(), toks[:, first:n])
