"""bf16 sampler agreement. G4 pins the sampler bit-exactly
in fp32; the bf16 engine (the cfg-5 configuration) cannot be bit-exact on its
logits, so this test bounds how often its top-k candidate set differs from the
fp32 oracle's (scripts/generate.py:58-85: filtered logit of the last row,
repetition penalties, top-k, renormalised inverse-CDF draw).

Teacher-forced on the bf16 engine's own trajectory, so both sides see the same
prefix at every step: generate() runs the bf16 engine with recorded uniforms
and a seeded Python RNG; then for every (row, step) the oracle's fp32 forward
of the same window and the engine's bf16 forward each give a penalised
filtered-logit row, and the two top-k index sets (k replayed from the same RNG
stream) are compared. Also checked: the token the engine sampled is the
inverse-CDF pick over ITS OWN top-k with that step's uniform.
Shape: the smallest bf16 flash-path model (hs = 128) with the reference
vocabulary; G4's own shapes (hs = 16) have no bf16 path. 12 rows x 56 steps
= 672 draws (past block_len, so the window slides). Measured (round 6):
665 / 672 = 0.9896, each of the 7 misses a near-tie (fp32 gap 0.002-0.05 between
the k-th and (k+1)-th filtered logit). The test asserts that every miss is a
near-tie (gap within the bound on how far bf16 rounding moved the two tokens'
filtered logits), the rate >= 0.98 and the engine's own draws >= 0.99."""
import random

import numpy as np
import pytest
import torch

from oracle import loss as oloss, sampler as osamp, transformer as otr
from oracle.fill import REAL, grammar_tokens
from midiseq.transformer import Transformer, TransformerConfig
from midiseq.generate import generate

pytestmark = pytest.mark.gpu
RATE_MIN = 0.98


def test_bf16_topk_sets_agree_with_fp32_oracle():
    hp = dict(n_embd=256, n_heads=2, n_layer=2, block_len=64)
    B, T0, steps, mv = 12, 40, 56, 568  # 672 (row, step) draws; the window slides past block_len
    cfg = TransformerConfig(vocab_size=REAL.size, metadata_vocab_size=mv, precision="bf16", dropout=0.0, **hp)
    m = Transformer(cfg).to("cuda").eval()
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], REAL.size, mv)
    p = otr.filled_params(shapes)
    m.load_state_dict(p, strict=False)
    rng = np.random.default_rng(3)
    src = torch.from_numpy(np.stack([grammar_tokens(rng, REAL, T0) for _ in range(B)]))
    meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173],
                         [437, 279, 272, 202, 202, 180], [452, 272, 202, 202, 202, 184],
                         [508, 272, 202, 202, 202, 184], [519, 279, 202, 202, 202, 178]]).repeat(2, 1)
    us = np.random.default_rng(11).random(B * steps).tolist()
    seqs = np.array(generate(m, hp["block_len"], src, meta, num_tokens=steps, rng=random.Random(5),
                             uniforms=iter(us)))
    kr = random.Random(5)
    agree = total = picks = 0
    worst = []
    for s in range(steps):
        cur = T0 + s
        W = min(cur, hp["block_len"])
        window = torch.from_numpy(seqs[:, cur - W:cur].copy())
        with torch.no_grad():
            ref_logits = otr.forward(p, window, meta, hp["n_layer"], hp["n_heads"])
            eng_logits = m(window.cuda(), meta.cuda()).float().cpu()
        z_ref = oloss.filtered_logit(window, ref_logits, REAL)[:, -1, :].clone()
        z_eng = oloss.filtered_logit(window, eng_logits, REAL)[:, -1, :].clone()
        wrow = oloss.weight_table_torch(REAL)[torch.from_numpy(oloss.bucket_of(window[:, -1].numpy(), REAL))].abs()
        for i in range(B):
            k = osamp.choose_k(int(seqs[i, cur - 1]), REAL, kr)
            recent = osamp.recent_window(seqs[i, :cur].tolist(), REAL)
            osamp.penalise(z_ref[i], recent, REAL)
            osamp.penalise(z_eng[i], recent, REAL)
            vr, ir = torch.topk(z_ref[i], k)
            ve, ie = torch.topk(z_eng[i], k)
            same = set(ir.tolist()) == set(ie.tolist())
            agree += same
            total += 1
            if not same:
                # a token of the fp32 top-k left out by the bf16 engine (a) and the one
                # it took instead (b): z_ref[a] >= z_ref[b], z_eng[b] >= z_eng[a], so
                # z_ref[a] - z_ref[b] <= |dz_a| + |dz_b|; z = -(l[T-1] - logsumexp_t l[t]) w
                # (train.py:133-138, w the bucket weight of the row) moves by at most
                # 2 w times the largest |bf16 - fp32| logit difference in its column
                # (the penalty only divides by >= 1)
                def dz(tok):
                    return 2 * float(wrow[i, tok]) * float((eng_logits[i, :, tok] - ref_logits[i, :, tok]).abs().max())
                for a_ in set(ir.tolist()) - set(ie.tolist()):
                    for b_ in set(ie.tolist()) - set(ir.tolist()):
                        worst.append((s, i, k, float(z_ref[i][a_] - z_ref[i][b_]), dz(a_) + dz(b_)))
            # the engine's draw: inverse CDF over its own top-k on this step's uniform
            # (the device computed its filtered logits from the same bf16 logits,
            # so this agrees up to fp32 rounding of the filtered-logit pass)
            pick = int(ie[osamp.inverse_cdf(ve / ve.sum(), us[s * B + i])])
            picks += pick == int(seqs[i, cur])
    rate = agree / total
    print(f"\nbf16 vs fp32 top-k set agreement: {agree}/{total} = {rate:.4f}; engine draws reproduced "
          f"{picks}/{total}; disagreements (step, row, k, fp32 gap of the swapped pair, bound on their bf16 "
          f"movement): {worst}")
    # every disagreement is a near-tie: the fp32 gap of each swapped pair is
    # within the bound on how far the two tokens' bf16 filtered logits can move
    # (a larger gap could not swap); the rate itself is reported and must stay
    # >= RATE_MIN (672 draws: 13 near-ties allowed)
    ties = [w for w in worst if w[3] <= w[4]]
    assert len(ties) == len(worst), [w for w in worst if w not in ties]
    assert rate >= RATE_MIN, (rate, worst)
    assert picks / total >= 0.99, (picks, total)
