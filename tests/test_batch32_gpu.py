"""Value check at the benched batch: bench.py times the
default Transformer at B = 32, T = 2048 (BASELINE cfg 2; the reference trains
on batch_size rows, train_parallel.py:173-183). Every other value test runs
B <= 4, so the B-indexed paths are pinned here: the XCD block order of the
attention kernels over b, the lm_head column-statistics partials
[B*T/128, 2, V_pad], the loss's per-b column ranges, the sorted embedding
backward over B*S rows, the dropout keep words of b > 3.

One TrainStep (lr = 0: Adam leaves the parameters as they are) on a B = 32
synthetic batch against 32 TrainSteps of the same model on each row alone:
* the loss (CrossEntropyLoss mean over B*T, train_parallel.py:179) equals the
  mean of the 32 per-row losses (1e-4 relative);
* the flat gradient equals the mean of the 32 per-row gradients (norm-relative
  < 1e-2, cosine > 0.9999: the per-row products are the same kernels, the
  weight gradients sum the rows in another order);
* the logits rows of b = 0 and b = 31 equal their B = 1 forwards (1e-3 of max),
  except the last (B*S) % 256 window positions of b = 31: those rows of the
  layer products fall in the persistent GEMM's partial last round, which sums
  them over K slices (csrc/gemm256p.hip), in another order than the B = 1
  run's whole tiles, so they (and the logits they feed) agree to bf16
  rounding through 8 layers (2e-2 of max); causal attention keeps every
  earlier position's logits within 1e-3.
Then the attention keep words of b = 31 (dropout p = 0.01, S = 2054) against
oracle/dropout.py bit for bit."""
import numpy as np
import pytest
import torch

from oracle import dropout as odrop
from midiseq import ops
from midiseq.config import N_META
from midiseq.transformer import Transformer, TransformerConfig, DROP_ATTN
from midiseq.train_parallel import TrainStep, SyntheticMIDI

pytestmark = pytest.mark.gpu
dev = "cuda"


def test_b32_step_equals_mean_of_rows():
    B, T = 32, 2048
    m = Transformer(TransformerConfig(precision="bf16", dropout=0.0)).to(dev)
    src, trg, meta = next(iter(SyntheticMIDI(B, T, dev, n_batches=1)))
    st = TrainStep(m, lr=0.0)
    loss = st(src, trg, meta).item()
    g32 = st.grads.clone()
    logits32 = m.engine.acts(B, T).logits.view(B, T, -1)[:, :, :m.cfg.vocab_size]
    rows = {b: logits32[b].float().clone() for b in (0, B - 1)}
    S = T + N_META
    t_cut = T - (B * S) % 256  # the partial-round rows of b = B-1 start at this token position
    gsum = torch.zeros_like(g32)
    losses = []
    lerr = {}
    for b in range(B):
        losses.append(st(src[b:b + 1], trg[b:b + 1], meta[b:b + 1]).item())
        gsum += st.grads
        if b in rows:
            l1 = m.engine.acts(1, T).logits.view(1, T, -1)[0, :, :m.cfg.vocab_size].float()
            scale = rows[b].abs().max()
            lerr[b] = ((l1[:t_cut] - rows[b][:t_cut]).abs().max() / scale).item()
            if b == B - 1:
                lerr["tail"] = ((l1[t_cut:] - rows[b][t_cut:]).abs().max() / scale).item()
    torch.cuda.synchronize()
    gmean = gsum / B
    d = (g32.double() - gmean.double())
    nr = (d.norm() / gmean.double().norm()).item()
    cos = (g32.double() @ gmean.double() / (g32.double().norm() * gmean.double().norm())).item()
    lm = float(np.mean(losses))
    print(f"\nB=32 step: loss {loss:.6f} vs mean of rows {lm:.6f}; grad norm-rel {nr:.2e}, cos {cos:.7f}; "
          f"logit rows err {lerr}")
    assert abs(loss - lm) <= 1e-4 * abs(lm)
    assert nr < 1e-2 and cos > 0.9999, (nr, cos)
    assert lerr[0] <= 1e-3 and lerr[B - 1] <= 1e-3 and lerr["tail"] <= 2e-2, lerr


def test_attn_keep_words_at_b31():
    B, H, S, p, layer, seed = 32, 8, 2054, 0.01, 3, 24680
    nb = (S + 63) // 64
    mw = ops.dropout_attn_mask(B, H, S, seed, DROP_ATTN + layer * 65536, p, dev)
    torch.cuda.synchronize()
    b = B - 1
    tri = np.tril(np.ones((S, S), dtype=bool))
    for h in (0, H - 1):
        words = mw[0].view(B, H, nb, nb, 64, 2)[b, h].permute(0, 2, 1, 3).reshape(nb * 64, nb * 2)
        w = words.cpu().numpy().view(np.uint32)
        bits = (((w[..., None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(nb * 64, -1)[:S, :S]).astype(bool)
        ref = odrop.attn_keep_site(seed, odrop.ATTN + layer * 65536 + b * H + h, S, p)
        assert np.array_equal(bits[tri], ref[tri]), (b, h)
