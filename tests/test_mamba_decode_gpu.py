"""Mamba cached decode: the recurrent step
(msq_mamba_conv_step / msq_mamba_ssd_step through MambaEngine.step) after a
prefill (msq_mamba_ssd_fwd_state) reproduces the last row of the full forward
over the grown sequence, and generate(mode="cached") reproduces the exact
sliding-window loop's token ids (scripts/generate.py:14-95 semantics),
including the fallback once the window slides. The full forward is pinned by
G5 / the CPU oracle (tests/test_mamba_gpu.py); the step is also checked
against the oracle's sequential recurrence (oracle/mamba2.py) directly.
Tolerances: fp32 1e-4 relative to the logit scale, bf16 3e-2."""
import random

import numpy as np
import pytest
import torch

from oracle import mamba2 as om
from oracle.fill import REAL, grammar_tokens
from midiseq.mamba import Mamba
from midiseq.generate import generate

pytestmark = pytest.mark.gpu
META = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173],
                     [437, 279, 272, 202, 202, 180]])


def build(d_model, n_layers, precision):
    m = Mamba(d_model=d_model, n_layers=n_layers, precision=precision).to("cuda")
    p = om.filled_params(om.param_shapes(d_model, n_layers, REAL.size, 568))
    m.load_state_dict(p)
    return m, p


def tokens(B, T, seed):
    rng = np.random.default_rng(seed)
    return torch.from_numpy(np.stack([grammar_tokens(rng, REAL, T) for _ in range(B)]))


@pytest.mark.parametrize("precision,d,T0,steps,tol", [("fp32", 128, 70, 6, 1e-4), ("bf16", 256, 130, 4, 3e-2)])
def test_step_matches_full_forward(precision, d, T0, steps, tol):
    m, p = build(d, 2, precision)
    eng = m.engine
    B = 3
    seq = tokens(B, T0 + steps, 7).cuda()
    meta = META[:B].cuda()
    V = eng.cfg.vocab_size
    cache = eng.decode_cache(B)
    with torch.no_grad():
        full0 = eng.forward(seq[:, :T0].contiguous(), meta, save=False, cache=cache)[:, -1].float().clone()
        ref0 = eng.forward(seq[:, :T0].contiguous(), meta, save=False)[:, -1].float()
        assert torch.equal(full0, ref0)  # the prefill hook changes nothing
        assert cache.length == T0
        for s in range(steps):
            tok = seq[:, T0 + s].contiguous()
            got = eng.step(tok, cache)[:, :V].float().clone()
            want = eng.forward(seq[:, :T0 + s + 1].contiguous(), meta, save=False)[:, -1].float()
            scale = want.abs().max().item()
            err = (got - want).abs().max().item()
            assert err <= tol * scale, (s, err, scale)
    if precision == "fp32":  # the step against the oracle's sequential recurrence
        ref = om.forward(p, seq.cpu(), META[:B], 2)[:, -1]
        assert (got.cpu() - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()


def test_filtered_step_matches_window_lse():
    """Running LSE + z of the step equal msq_filtered_logit's last row over the grown window."""
    from midiseq import _lib as L
    from midiseq._lib import ptr, call, stream, dt
    from midiseq.loss import grammar_table
    from midiseq.config import Grammar
    from midiseq.ops import workspace
    m, _ = build(128, 2, "fp32")
    eng = m.engine
    B, T0 = 2, 40
    seq = tokens(B, T0 + 1, 3).cuda()
    meta = META[:B].cuda()
    V = eng.cfg.vocab_size
    gram = Grammar()
    wtab, bd = grammar_table(seq.device, gram), gram.bounds
    ldz = (V + 3) // 4 * 4
    cache = eng.decode_cache(B)

    def window_z(W, col_lse):
        win = seq[:, :W].contiguous()
        eng.forward(win, meta, save=False, cache=cache if col_lse is cache.lse else None)
        A = eng.acts(B, W, save=False)
        z = torch.empty(B, 1, ldz, device="cuda")
        ws = workspace(L.lib().msq_filtered_workspace(B, W, V), seq.device, "loss")
        call("msq_filtered_logit", ptr(z), ldz, ptr(A.logits), dt(A.logits), eng.cfg.v_pad, ptr(win), ptr(wtab),
             bd[0], bd[1], bd[2], bd[3], B, W, V, W - 1, ptr(col_lse), ptr(ws), stream())
        return z

    with torch.no_grad():
        window_z(T0, cache.lse)
        tok = seq[:, T0].contiguous()
        logits = eng.step(tok, cache)
        z = torch.empty(B, 1, ldz, device="cuda")
        call("msq_filtered_logit_step", ptr(z), ldz, ptr(cache.lse), ptr(logits), dt(logits), eng.cfg.v_pad,
             ptr(tok), ptr(wtab), bd[0], bd[1], bd[2], bd[3], B, V, stream())
        lse_ref = torch.empty(B, V, device="cuda")
        z_ref = window_z(T0 + 1, lse_ref)
    torch.cuda.synchronize()
    assert (cache.lse - lse_ref).abs().max().item() < 1e-4 * lse_ref.abs().max().item()
    assert (z[..., :V] - z_ref[..., :V]).abs().max().item() < 1e-4 * z_ref[..., :V].abs().max().item() + 1e-5


@pytest.mark.parametrize("T0,ctx,n", [(30, 64, 12), (30, 36, 12)])
def test_generate_cached_matches_exact(T0, ctx, n):
    """(30, 36): the window starts sliding at step 7 -> exact fallback for the rest."""
    m, _ = build(128, 2, "fp32")
    B = 3
    src = tokens(B, T0, 11)
    u = np.random.default_rng(5).random(B * n).tolist()
    out = {}
    for mode in ("exact", "cached"):
        out[mode] = generate(m, ctx, src, META[:B], num_tokens=n, rng=random.Random(99), uniforms=iter(u),
                             mode=mode)
    np.testing.assert_array_equal(np.array(out["cached"]), np.array(out["exact"]))


def test_unknown_mode_rejected():
    from midiseq.transformer import Transformer, TransformerConfig
    m = Transformer(TransformerConfig(n_embd=64, n_heads=4, n_layer=1, block_len=16, precision="fp32")).to("cuda")
    with pytest.raises(ValueError):
        generate(m, 16, tokens(1, 8, 0), META[:1], num_tokens=2, mode="kv")


@pytest.mark.parametrize("B,d_model", [(1, 256), (37, 1024), (64, 1024), (65, 512), (8, 1536)])
def test_in_proj_conv_step_matches_two_launches(B, d_model):
    """msq_mamba_in_proj_conv_step (the conv step in the skinny in_proj's
    epilogue for B <= 64, d_model <= 1024; the two launches past that) against
    msq_gemm + msq_mamba_conv_step on the same inputs: zx and the shifted conv
    state bitwise, the conv output within one bf16 step (the two kernels may
    contract the tap sum into FMAs differently)."""
    from midiseq import _lib as L, ops
    from midiseq._lib import call, ptr
    torch.manual_seed(B)
    H = 32
    di, cd = H * 64, H * 64 + 128
    dp = di + cd + H
    x = torch.randn(B, d_model, device="cuda").bfloat16()
    w = (torch.randn(dp, d_model, device="cuda") * d_model ** -0.5).bfloat16()
    cw = torch.randn(cd, 4, device="cuda") * 0.5
    cb = torch.randn(cd, device="cuda") * 0.1
    st0 = torch.randn(B, 3, cd, device="cuda")
    zx_a, xc_a, st_a = torch.empty(B, dp, device="cuda", dtype=torch.bfloat16), torch.empty(B, cd, device="cuda", dtype=torch.bfloat16), st0.clone()
    zx_b, xc_b, st_b = torch.empty_like(zx_a), torch.empty_like(xc_a), st0.clone()
    s = ops.stream()
    call("msq_mamba_in_proj_conv_step", ptr(zx_a), dp, ptr(xc_a), cd, ptr(st_a), ptr(x), d_model, ptr(w), d_model,
         ptr(cw), ptr(cb), B, d_model, dp, di, H, s)
    ops.gemm(x, w, out=zx_b)
    call("msq_mamba_conv_step", ptr(xc_b), cd, ptr(st_b), ptr(zx_b), dp, L.BF16, ptr(cw), ptr(cb), B, di, H, s)
    torch.cuda.synchronize()
    assert torch.equal(zx_a, zx_b)
    assert torch.equal(st_a, st_b)
    assert torch.equal(st_a[:, :2], st0[:, 1:])  # the window shifted by one row
    d = (xc_a.float() - xc_b.float()).abs()
    assert d.max().item() <= 2 ** -7 * max(1.0, xc_b.float().abs().max().item()), d.max().item()
