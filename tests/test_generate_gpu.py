"""Decode parity: the MI355X sampler (exact sliding-window mode, fp32 model)
reproduces the token ids the REFERENCE's generate() produced (golden G4:
scripts/generate.py run by make_golden.py with torch.multinomial replaced by
inverse-CDF on recorded uniforms and random.seed(1234)). Bit-exact ids."""
import random
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import transformer as otr
from oracle.fill import TINY, REAL
from midiseq.transformer import Transformer, TransformerConfig
from midiseq.generate import generate
from midiseq.config import Grammar, Discretization

pytestmark = pytest.mark.gpu
G = Path(__file__).parent / "golden"
GCASES = {"tiny": (TINY, 10, dict(n_embd=32, n_heads=4, n_layer=2, block_len=16), 12),
          "small": (REAL, 568, dict(n_embd=64, n_heads=4, n_layer=2, block_len=48), 8)}


def grammar_for(v):
    d = v.disc
    return Grammar(Discretization(pitch=d["pitch"], channel=d["channel"], dyn=d["dyn"], length=d["length"],
                                  time=d["time"], tempo=d["tempo"]))


@pytest.mark.parametrize("tag", ["tiny", "small"])
def test_generate_matches_reference(tag):
    g4 = np.load(G / "g4_generate.npz")
    vocab, mv, hp, steps = GCASES[tag]
    cfg = TransformerConfig(vocab_size=vocab.size, metadata_vocab_size=mv, precision="fp32", **hp)
    m = Transformer(cfg).to("cuda")
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], vocab.size, mv)
    m.load_state_dict(otr.filled_params(shapes))
    seqs = generate(m, hp["block_len"], torch.from_numpy(g4[f"{tag}_src"]), torch.from_numpy(g4[f"{tag}_meta"]),
                    num_tokens=steps, rng=random.Random(1234), uniforms=iter(g4[f"{tag}_uniforms"].tolist()),
                    grammar=grammar_for(vocab))
    np.testing.assert_array_equal(np.array(seqs), g4[f"{tag}_seqs"])


def test_generate_bf16_runs_and_respects_grammar():
    cfg = TransformerConfig(n_embd=256, n_heads=2, n_layer=2, block_len=64, precision="bf16")
    m = Transformer(cfg).to("cuda")
    rng = np.random.default_rng(0)
    from oracle.fill import grammar_tokens
    src = torch.from_numpy(np.stack([grammar_tokens(rng, REAL, 64) for _ in range(3)]))
    meta = torch.tensor([[519, 279, 202, 202, 202, 178]] * 3)
    seqs = generate(m, 64, src, meta, num_tokens=6, rng=random.Random(0))
    assert np.array(seqs).shape == (3, 70)
    assert all(0 <= t < REAL.size for row in seqs for t in row)


def test_default_sampling_leaves_python_rng_to_the_k_choice():
    """Without injected uniforms the device sampler is seeded from torch's RNG
    (the reference's torch.multinomial stream), so the caller's Python
    ``random`` only feeds the k choice of scripts/generate.py:47-56: replaying
    choose_k over the generated rows with a fresh Random(seed) ends in the same
    generator state as the one generate() consumed."""
    from midiseq.generate import choose_k
    vocab, mv, hp, steps = GCASES["small"]
    cfg = TransformerConfig(vocab_size=vocab.size, metadata_vocab_size=mv, precision="fp32", **hp)
    m = Transformer(cfg).to("cuda")
    g4 = np.load(G / "g4_generate.npz")
    src, meta = torch.from_numpy(g4["small_src"]), torch.from_numpy(g4["small_meta"])
    rng = random.Random(77)
    torch.manual_seed(5)
    seqs = np.array(generate(m, hp["block_len"], src, meta, num_tokens=steps, rng=rng, grammar=grammar_for(vocab)))
    replay = random.Random(77)
    T0 = src.shape[1]
    start = grammar_for(vocab).disc.start_idx
    for s in range(steps):
        choose_k(seqs[:, T0 + s - 1].tolist(), start, replay)
    assert rng.getstate() == replay.getstate()
