"""Pins the CPU oracle against golden vectors recorded from the reference's own
code (tests/golden/make_golden.py). CPU only."""
import random
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import loss as oloss
from oracle import sampler as osamp
from oracle import transformer as otr
from oracle.fill import TINY, REAL, Vocab, hash_uniform
from golden_check import check_grad

G = Path(__file__).parent / "golden"


def _proj(V, k=8, salt=7):
    return torch.from_numpy(hash_uniform(V * k, salt).reshape(V, k).astype(np.float32))


@pytest.fixture(scope="module")
def g12():
    return np.load(G / "g1g2_loss.npz")


@pytest.fixture(scope="module")
def g3():
    return np.load(G / "g3_transformer.npz")


@pytest.fixture(scope="module")
def g4():
    return np.load(G / "g4_generate.npz")


@pytest.mark.parametrize("tag,vocab", [("tiny", TINY), ("real", REAL)])
def test_weight_table_and_buckets(g12, tag, vocab):
    tab = oloss.weight_table(vocab).reshape(-1)
    nz = np.nonzero(tab)[0]
    np.testing.assert_array_equal(nz, g12[f"{tag}_table_nz_idx"])
    np.testing.assert_array_equal(tab[nz], g12[f"{tag}_table_nz_val"])  # bit-exact
    np.testing.assert_array_equal(oloss.bucket_of(g12[f"{tag}_edge_tokens"], vocab), g12[f"{tag}_edge_buckets"])


def test_real_edge_buckets_survey():
    toks = np.array([0, 16510, 16511, 16512, 16638, 16639, 16640, 17150, 17151, 17152, 17662, 17663, 17664, 17913])
    np.testing.assert_array_equal(oloss.bucket_of(toks, REAL), [0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4])


@pytest.mark.parametrize("tag,vocab", [("tiny", TINY), ("real", REAL)])
def test_filtered_ce(g12, tag, vocab):
    B, T = 2, 16
    logits = torch.from_numpy((4.0 * hash_uniform(B * T * vocab.size, 99)).astype(np.float32)).reshape(
        B, T, vocab.size).requires_grad_(True)
    src = torch.from_numpy(g12[f"{tag}_ce_src"])
    trg = torch.from_numpy(g12[f"{tag}_ce_trg"])
    z = oloss.filtered_logit(src, logits, vocab)
    l = oloss.loss(src, trg, logits, vocab)
    l.backward()
    assert abs(l.item() - float(g12[f"{tag}_ce_loss"])) < 1e-5
    if tag == "tiny":
        np.testing.assert_allclose(z.detach().numpy(), g12["tiny_ce_z"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(logits.grad.numpy(), g12["tiny_ce_dlogits"], rtol=1e-4, atol=1e-8)
    else:
        P = _proj(vocab.size)
        np.testing.assert_allclose((z.detach() @ P).numpy(), g12["real_ce_z_proj"], rtol=1e-4, atol=1e-3)
        np.testing.assert_allclose(z.detach()[:, [0, T - 1]].numpy(), g12["real_ce_z_rows"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(logits.grad[:, [0, 7, T - 1]].numpy(), g12["real_ce_dlogits_rows"],
                                   rtol=1e-4, atol=1e-10)


CASES = {"tiny": (TINY, 10, dict(n_embd=32, n_heads=4, n_layer=2, block_len=16)),
         "small": (REAL, 568, dict(n_embd=128, n_heads=8, n_layer=2, block_len=64))}


@pytest.mark.parametrize("tag", ["tiny", "small"])
def test_transformer_fwd_bwd(g3, tag):
    vocab, mv, hp = CASES[tag]
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], vocab.size, mv)
    p = {k: v.requires_grad_(True) for k, v in otr.filled_params(shapes).items()}
    src, trg, meta = (torch.from_numpy(g3[f"{tag}_{n}"]) for n in ("src", "trg", "meta"))
    logits = otr.forward(p, src, meta, hp["n_layer"], hp["n_heads"])
    l = oloss.loss(src, trg, logits, vocab)
    l.backward()
    assert abs(l.item() - float(g3[f"{tag}_loss"])) < 2e-5 * max(1.0, abs(float(g3[f"{tag}_loss"])))
    if tag == "tiny":
        np.testing.assert_allclose(logits.detach().numpy(), g3["tiny_logits"], rtol=1e-4, atol=1e-4)
        for k, t in p.items():
            ref = g3[f"tiny_grad:{k}"]
            # ln_f.bias / lm_head.bias grads are ~0: log-softmax over T is
            # invariant to a per-column constant, so use an absolute floor
            scale = np.abs(ref).max()
            assert np.abs(t.grad.numpy() - ref).max() <= 1e-3 * scale + 1e-6, k
    else:
        P = _proj(vocab.size)
        np.testing.assert_allclose((logits.detach() @ P).numpy(), g3["small_logits_proj"], rtol=1e-3, atol=2e-3)
        T = src.shape[1]
        np.testing.assert_allclose(logits.detach()[:, [0, T // 2, T - 1]].numpy(), g3["small_logits_rows"],
                                   rtol=1e-4, atol=1e-4)
        for k, t in p.items():
            if k in ("ln_f.bias", "lm_head.bias"):  # analytically zero (shift invariance along T)
                assert t.grad.abs().max().item() < 1e-4 * p["lm_head.weight"].grad.abs().max().item(), k
                continue
            check_grad(k, t.grad.numpy(), g3[f"small_gsum:{k}"], g3[f"small_gpick:{k}"], 1e-3)
    # length anchoring: the shorter window changes the prefix logits
    with torch.no_grad():
        short = otr.forward(p, src[:, :-1], meta, hp["n_layer"], hp["n_heads"])
    d = (short - logits.detach()[:, :-1]).abs().max().item()
    assert abs(d - float(g3[f"{tag}_anchor_maxdiff"])) < 1e-3 * max(1.0, d)
    np.testing.assert_allclose(short[:, 0].numpy(), g3[f"{tag}_anchor_short_logits_row0"], rtol=1e-4, atol=1e-4)


GCASES = {"tiny": (TINY, 10, dict(n_embd=32, n_heads=4, n_layer=2, block_len=16), 12),
          "small": (REAL, 568, dict(n_embd=64, n_heads=4, n_layer=2, block_len=48), 8)}


@pytest.mark.parametrize("tag", ["tiny", "small"])
def test_generate(g4, tag):
    vocab, mv, hp, steps = GCASES[tag]
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], vocab.size, mv)
    p = otr.filled_params(shapes)
    src = torch.from_numpy(g4[f"{tag}_src"])
    meta = torch.from_numpy(g4[f"{tag}_meta"])
    rng = random.Random(1234)
    trace = []
    seqs = osamp.generate(lambda i, m: otr.forward(p, i, m, hp["n_layer"], hp["n_heads"]), hp["block_len"],
                          src, meta, steps, vocab, rng, iter(g4[f"{tag}_uniforms"].tolist()), trace)
    np.testing.assert_array_equal(np.array(seqs), g4[f"{tag}_seqs"])  # bit-exact sampled ids
    np.testing.assert_array_equal([t[2] for t in trace], g4[f"{tag}_k"])
    for n, t in enumerate(trace):
        k = t[2]
        np.testing.assert_array_equal(t[3], g4[f"{tag}_topk_idx"][n, :k])
