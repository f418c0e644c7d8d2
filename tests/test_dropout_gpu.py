"""Dropout (nn.Dropout(p) at model_transformer.py:51 proj, :80 attention
probabilities, :101 FFN output; active in train() mode) on the MI355X path.

The reference draws its masks from torch's Philox stream, which cannot be
reproduced outside torch; the build draws them from a counter-based hash
(csrc/common.h) and the oracle (oracle/dropout.py) restates that hash
bit-exactly. Parity is therefore: the same masks, and every other number as in
the dropout-free parity tests (fp32 exact mode: logits 1e-4, loss 1e-4 rel,
grads 2e-3 of max; bf16 mode: loss 2e-2 rel, grads norm-rel < 1e-1, cos > 0.99).
"""
import numpy as np
import pytest
import torch

from oracle import dropout as odrop
from oracle import loss as oloss
from oracle import transformer as otr
from oracle.fill import REAL, grammar_tokens
from midiseq import ops
from midiseq import _lib as L
from midiseq.transformer import Transformer, TransformerConfig, DROP_ATTN
from midiseq.loss import filtered_cross_entropy

pytestmark = pytest.mark.gpu
dev = "cuda"


def unpack(words, S):
    """uint32 words [..., ld] -> bits [..., ld*32][:S]"""
    w = words.cpu().numpy().view(np.uint32)
    b = (w[..., None] >> np.arange(32, dtype=np.uint32)) & 1
    return b.reshape(*w.shape[:-1], -1)[..., :S].astype(bool)


@pytest.mark.parametrize("S,p", [(70, 0.1), (200, 0.01), (2054, 0.01)])
def test_attn_mask_bits_match_oracle(S, p):
    B, H, seed, layer = 2, 3, 987654321, 5
    if S > 1000:
        B, H = 1, 2
    nb = (S + 63) // 64
    m = ops.dropout_attn_mask(B, H, S, seed, DROP_ATTN + layer * 65536, p, dev)
    torch.cuda.synchronize()
    assert m.shape[1] == L.lib().msq_dropout_mask_words(B, H, S) == B * H * nb * nb * 128

    def dense(words):   # block-transposed [B,H,nb(r),nb(c),64(r%64),2] -> [B,H,r,c words]
        w = words.view(B, H, nb, nb, 64, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, H, nb * 64, nb * 2)
        return unpack(w[:, :, :S], S)
    rows = dense(m[0])          # [B,H,i,j]
    cols = dense(m[1])          # [B,H,j,i]
    ref = odrop.attn_keep(seed, layer, B, H, S, p)
    tri = np.tril(np.ones((S, S), dtype=bool))
    assert np.array_equal(rows[..., tri], ref[..., tri])
    assert np.array_equal(cols.transpose(0, 1, 3, 2)[..., tri], ref[..., tri])
    rate = 1 - ref[..., tri].mean()
    assert abs(rate - p) < 6 * np.sqrt(p * (1 - p) / ref[..., tri].size) + 1e-4


def _model(hp, precision, p):
    cfg = TransformerConfig(vocab_size=REAL.size, metadata_vocab_size=568, precision=precision, dropout=p, **hp)
    m = Transformer(cfg).to(dev)
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], REAL.size, 568)
    prm = otr.filled_params(shapes)
    m.load_state_dict(prm, strict=True)
    return m, prm


def _batch(B, T, seed):
    rng = np.random.default_rng(seed)
    w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
    meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]][:B])
    return torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy()), meta


def _run(m, prm, src, trg, meta, p, n_layer, n_heads):
    torch.manual_seed(11)
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    torch.manual_seed(11)  # the module draws the same seed for its forward
    logits = m(src.to(dev), meta.to(dev))
    loss = filtered_cross_entropy(src.to(dev), logits, trg.to(dev))
    loss.backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in prm.items()}
    ref_logits = otr.forward(pr, src, meta, n_layer, n_heads, drop=(seed, p))
    ref_loss = oloss.loss(src, trg, ref_logits, REAL)
    ref_loss.backward()
    return logits, loss, pr, ref_logits, ref_loss


def test_fp32_train_mode_matches_oracle():
    hp = dict(n_embd=128, n_heads=8, n_layer=2, block_len=64)
    p = 0.1
    m, prm = _model(hp, "fp32", p)
    src, trg, meta = _batch(2, 64, 4)
    logits, loss, pr, ref_logits, ref_loss = _run(m, prm, src, trg, meta, p, 2, 8)
    np.testing.assert_allclose(logits.detach().cpu().numpy(), ref_logits.detach().numpy(), rtol=1e-4, atol=1e-4)
    assert abs(loss.item() - ref_loss.item()) < 1e-4 * max(1.0, abs(ref_loss.item()))
    for k, g in m.grad_dict().items():
        r = pr[k].grad.numpy()
        err = np.abs(g.cpu().numpy() - r).max()
        assert err <= 2e-3 * np.abs(r).max() + 1e-6, (k, err)
    # dropout really acted: the undropped forward differs
    no = otr.forward(prm, src, meta, 2, 8)
    assert (no - ref_logits.detach()).abs().max().item() > 1e-2


def test_eval_mode_has_no_dropout():
    hp = dict(n_embd=128, n_heads=8, n_layer=2, block_len=64)
    m, prm = _model(hp, "fp32", 0.1)
    m.eval()
    src, _, meta = _batch(2, 64, 5)
    with torch.no_grad():
        logits = m(src.to(dev), meta.to(dev))
    ref = otr.forward(prm, src, meta, 2, 8)
    np.testing.assert_allclose(logits.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


def test_bf16_train_mode_matches_oracle():
    hp = dict(n_embd=256, n_heads=2, n_layer=2, block_len=128)
    p = 0.1
    m, prm = _model(hp, "bf16", p)
    src, trg, meta = _batch(2, 128, 9)
    logits, loss, pr, ref_logits, ref_loss = _run(m, prm, src, trg, meta, p, 2, 2)
    err = (logits.detach().float().cpu() - ref_logits.detach()).abs().max().item()
    assert err < 5e-2 * max(1.0, ref_logits.abs().max().item()), err
    assert abs(loss.item() - ref_loss.item()) < 2e-2 * abs(ref_loss.item())
    gd = m.grad_dict()
    gmax = gd["lm_head.weight"].abs().max().item()
    for k, g in gd.items():
        g = g.cpu().double().reshape(-1)
        if k in ("ln_f.bias", "lm_head.bias"):
            assert g.abs().max().item() < 5e-3 * gmax, k
            continue
        r = pr[k].grad.double().reshape(-1)
        nr = ((g - r).norm() / r.norm()).item()
        cos = (g @ r / (g.norm() * r.norm())).item()
        assert nr < 1e-1 and cos > 0.99, (k, nr, cos)
