"""Parity at the benched sizes: the bf16 kernels at
the shapes bench.py times, against the fp32 CPU oracle on the same inputs.

* relative attention fwd + bwd at S = 2054 (= block_len 2048 + 6 metadata),
  H = 8, hs = 128 (model_transformer.py:54-90), tolerance 2e-2 of max|ref| as
  the smaller attention cases (bf16 operands and outputs);
* the default Transformer (d 1024, 8 heads, 8 layers, T 2048, V 17 914) at
  B = 1: loss, three logit rows, and norm-relative gradients of one tensor per
  kind (model_transformer.py:136-168, train.py:133-138);
* Mamba (d 1024, 2 layers) at T = 4096 (cfg 3's length: 65 SSD chunks of the
  pass / reverse-pass kernels) against oracle.mamba2 (mamba.py:27-35).
Tolerances are the small-config ones of test_transformer_gpu.py /
test_mamba_gpu.py; each test prints the measured errors."""
import numpy as np
import pytest
import torch

from oracle import loss as oloss
from oracle.fill import REAL, grammar_tokens
from oracle.transformer import rel_attention

pytestmark = pytest.mark.gpu
dev = "cuda"
META = torch.tensor([[519, 279, 202, 202, 202, 178]])


def _nrcos(g, r):
    g, r = g.double().reshape(-1), r.double().reshape(-1)
    return ((g - r).norm() / r.norm()).item(), (g @ r / (g.norm() * r.norm())).item()


def test_relattn_bf16_at_bench_length():
    from midiseq import attention as att
    B, S, H, hs = 1, 2054, 8, 128
    scale = (H * hs) ** -0.5
    g = torch.Generator().manual_seed(2054)
    qkv = (torch.randn(B * S, 3 * H * hs, generator=g) * 0.5).bfloat16()
    R = (torch.randn(H, S, hs, generator=g) * 0.5).bfloat16()
    dout = torch.randn(B * S, H * hs, generator=g).bfloat16()
    out, lse = att.relattn_fwd(qkv.to(dev), R.to(dev), B, S, H, hs, scale)
    dqkv, dR = att.relattn_bwd(dout.to(dev), out, lse, qkv.to(dev), R.to(dev), B, S, H, hs, scale)
    torch.cuda.synchronize()
    qf = qkv.float().clone().requires_grad_(True)
    Rf = R.float().clone().requires_grad_(True)
    x = qf.view(B, S, 3, H, hs)
    ref = torch.cat([rel_attention(x[:, :, 0, h], x[:, :, 1, h], x[:, :, 2, h], Rf[h], scale) for h in range(H)],
                    dim=-1).reshape(B * S, H * hs)
    ref.backward(dout.float())

    def rel(a, b):
        return ((a.float().cpu() - b).abs().max() / b.abs().max()).item()
    errs = {"out": rel(out, ref.detach()), "dR": rel(dR, Rf.grad)}
    nq = H * hs
    for name, sl in (("dq", slice(0, nq)), ("dk", slice(nq, 2 * nq)), ("dv", slice(2 * nq, 3 * nq))):
        errs[name] = rel(dqkv[:, sl], qf.grad[:, sl])
    print("relattn S=2054 errors (of max):", errs)
    assert all(v < 2e-2 for v in errs.values()), errs


def test_default_transformer_bf16_b1_t2048():
    from oracle import transformer as otr
    from midiseq.transformer import Transformer, TransformerConfig
    from midiseq.loss import filtered_cross_entropy
    torch.set_num_threads(min(16, torch.get_num_threads()))
    m = Transformer(TransformerConfig(precision="bf16", dropout=0.0)).to(dev)
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items() if not k.endswith("tril")}
    rng = np.random.default_rng(2048)
    T = 2048
    w = grammar_tokens(rng, REAL, T + 1)[None]
    src, trg = torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy())
    logits = m(src.to(dev), META.to(dev))
    loss = filtered_cross_entropy(src.to(dev), logits, trg.to(dev))
    loss.backward()
    rl = otr.forward(p, src, META, 8, 8)
    rloss = oloss.loss(src, trg, rl, REAL)
    rloss.backward()
    lerr = abs(loss.item() - rloss.item()) / abs(rloss.item())
    rows = [0, T // 2, T - 1]
    xerr = ((logits.detach()[:, rows].float().cpu() - rl.detach()[:, rows]).abs().max() / rl.detach().abs().max()).item()
    gd = m.grad_dict()
    res = {}
    for k in ("token_embedding_table.weight", "metadata_embedding_table.weight", "blocks.0.sa.heads.0.query.weight",
              "blocks.3.sa.heads.5.key.weight", "blocks.7.sa.heads.7.value.weight", "blocks.0.sa.heads.2.rel_pos_emb",
              "blocks.6.sa.heads.1.rel_pos_emb", "blocks.4.sa.proj.weight", "blocks.2.ffwd.net.0.weight",
              "blocks.5.ffwd.net.2.weight", "blocks.1.ln1.weight", "blocks.7.ln2.bias", "lm_head.weight",
              "ln_f.weight"):
        res[k] = _nrcos(gd[k].cpu(), p[k].grad)
    print(f"default model B=1 T=2048: loss {loss.item():.6f} vs {rloss.item():.6f} (rel {lerr:.2e}), "
          f"logit rows err {xerr:.2e} of max;", res)
    assert lerr < 1e-2
    assert xerr < 5e-2
    for k, (nr, cos) in res.items():
        assert nr < 8e-2 and cos > 0.995, (k, nr, cos)


def test_mamba_bf16_t4096():
    from oracle import mamba2 as om
    from midiseq.mamba import Mamba
    from midiseq.loss import filtered_cross_entropy
    torch.set_num_threads(min(16, torch.get_num_threads()))
    m = Mamba(d_model=1024, n_layers=2, precision="bf16").to(dev)
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    rng = np.random.default_rng(4096)
    T = 4096
    w = grammar_tokens(rng, REAL, T + 1)[None]
    src, trg = torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy())
    logits = m(src.to(dev), META.to(dev))
    loss = filtered_cross_entropy(src.to(dev), logits, trg.to(dev))
    loss.backward()
    rl = om.forward(p, src, META, 2, chunked=True)
    rloss = oloss.loss(src, trg, rl, REAL)
    rloss.backward()
    lerr = abs(loss.item() - rloss.item()) / abs(rloss.item())
    gd = m.grad_dict()
    res = {}
    for k in ("token_embedding.weight", "layers.0.in_proj.weight", "layers.1.in_proj.weight", "layers.0.out_proj.weight",
              "layers.1.conv1d.weight", "layers.0.conv1d.bias", "layers.1.dt_bias", "layers.0.A_log", "layers.1.D",
              "layers.0.norm.weight", "output_layer.weight", "norm.weight"):
        res[k] = _nrcos(gd[k].cpu(), p[k].grad)
    print(f"mamba d=1024 L=2 T=4096: loss {loss.item():.6f} vs {rloss.item():.6f} (rel {lerr:.2e});", res)
    assert lerr < 2e-2
    for k, (nr, cos) in res.items():
        assert nr < 0.1 and cos > 0.99, (k, nr, cos)
