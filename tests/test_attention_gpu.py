"""GPU parity of the relative-position attention (fwd + bwd) against the CPU
oracle (oracle/transformer.py:rel_attention, pinned to model_transformer.py).

exact fp32 path: rtol 1e-4 on outputs and grads.
bf16 flash path (MFMA, hs=128): inputs rounded to bf16, compared against the
fp32 oracle on the SAME rounded inputs; tolerance 2e-2 of max|ref| (bf16 P/V
operands and bf16 outputs)."""
import pytest
import torch

from oracle.transformer import rel_attention
from midiseq import attention as att

pytestmark = pytest.mark.gpu
dev = "cuda"


def _mk(B, S, H, hs, S_max, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    qkv = (torch.randn(B * S, 3 * H * hs, generator=g) * 0.5).to(dtype)
    R = (torch.randn(H, S_max, hs, generator=g) * 0.5).to(dtype)
    dout = torch.randn(B * S, H * hs, generator=g).to(dtype)
    return qkv, R, dout


def _ref(qkv, R, dout, B, S, H, hs, scale):
    qkv = qkv.float().clone().requires_grad_(True)
    Rf = R.float().clone().requires_grad_(True)
    x = qkv.view(B, S, 3, H, hs)
    outs = []
    for h in range(H):
        outs.append(rel_attention(x[:, :, 0, h], x[:, :, 1, h], x[:, :, 2, h], Rf[h], scale))
    out = torch.cat(outs, dim=-1).reshape(B * S, H * hs)
    out.backward(dout.float())
    return out.detach(), qkv.grad, Rf.grad


def _rel(a, b):
    return ((a.float().cpu() - b).abs().max() / (b.abs().max() + 1e-12)).item()


@pytest.mark.parametrize("dtype,B,S,H,hs", [
    (torch.float32, 2, 23, 2, 8),
    (torch.float32, 1, 70, 3, 16),
    (torch.bfloat16, 2, 134, 2, 128),
    (torch.bfloat16, 1, 262, 1, 128),
    (torch.bfloat16, 1, 7, 1, 128),
    (torch.bfloat16, 2, 1030, 2, 128),
])
def test_relattn_fwd_bwd(dtype, B, S, H, hs):
    S_max = S + 5
    scale = (H * hs) ** -0.5
    qkv, R, dout = _mk(B, S, H, hs, S_max, dtype, seed=S)
    ref_out, ref_dqkv, ref_dR = _ref(qkv, R, dout, B, S, H, hs, scale)
    out, lse = att.relattn_fwd(qkv.to(dev), R.to(dev), B, S, H, hs, scale)
    dqkv, dR = att.relattn_bwd(dout.to(dev), out, lse, qkv.to(dev), R.to(dev), B, S, H, hs, scale)
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref_out) < tol
    nq = H * hs
    for name, sl in (("dq", slice(0, nq)), ("dk", slice(nq, 2 * nq)), ("dv", slice(2 * nq, 3 * nq))):
        assert _rel(dqkv[:, sl], ref_dqkv[:, sl]) < tol, name
    assert _rel(dR[:, :S], ref_dR[:, :S]) < tol
    assert dR[:, S:].abs().max().item() == 0.0


@pytest.mark.parametrize("dtype,B,S,H,hs,p", [
    (torch.float32, 2, 70, 2, 16, 0.2),
    (torch.bfloat16, 2, 390, 2, 128, 0.1),
    (torch.bfloat16, 1, 600, 1, 128, 0.01),
])
def test_relattn_dropout_fwd_bwd(dtype, B, S, H, hs, p):
    """nn.Dropout on the attention probabilities (model_transformer.py:80): the
    kernels' keep bits (msq_dropout_attn_mask) applied by the oracle."""
    from oracle import dropout as odrop
    from midiseq import ops
    S_max = S + 3
    scale = (H * hs) ** -0.5
    qkv, R, dout = _mk(B, S, H, hs, S_max, dtype, seed=S + 1)
    seed, layer = 4242, 3
    masks = ops.dropout_attn_mask(B, H, S, seed, odrop.ATTN + layer * 65536, p, dev)
    keep = torch.from_numpy(odrop.attn_keep(seed, layer, B, H, S, p))
    qf = qkv.float().clone().requires_grad_(True)
    Rf = R.float().clone().requires_grad_(True)
    x = qf.view(B, S, 3, H, hs)
    ref_out = torch.cat([rel_attention(x[:, :, 0, h], x[:, :, 1, h], x[:, :, 2, h], Rf[h], scale, keep[:, h],
                                       odrop.scale(p)) for h in range(H)], dim=-1).reshape(B * S, H * hs)
    ref_out.backward(dout.float())
    out, lse = att.relattn_fwd(qkv.to(dev), R.to(dev), B, S, H, hs, scale, drop=(masks, p))
    dqkv, dR = att.relattn_bwd(dout.to(dev), out, lse, qkv.to(dev), R.to(dev), B, S, H, hs, scale,
                               drop=(masks, p))
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref_out.detach()) < tol
    nq = H * hs
    for name, sl in (("dq", slice(0, nq)), ("dk", slice(nq, 2 * nq)), ("dv", slice(2 * nq, 3 * nq))):
        assert _rel(dqkv[:, sl], qf.grad[:, sl]) < tol, name
    assert _rel(dR[:, :S], Rf.grad[:, :S]) < tol
