"""lm_head forward with the filtered loss's time-axis column statistics in its
epilogue (msq_gemm_bias_colstats + msq_filtered_ce_bias_part; model_transformer.py:147,
train.py:133-138 log_softmax over the time axis).

* the GEMM output is bitwise the plain bias GEMM's (same persistent tile and
  main loop; only the epilogue adds the statistics);
* the merged (max, sum exp) partials give the column logsumexp of the stored
  bf16 logits: against msq_filtered_colstats on the same logits, 1e-5 relative;
* loss and dlogits through the partials equal the streaming loss's own
  colstats pass within round-off (loss 1e-5 relative, dlogits 1e-2 of max in
  bf16) and the oracle on the same bf16 logits (loss 1e-4 relative);
* a whole TrainStep with the head statistics on and off: same loss (1e-5)."""
import numpy as np
import pytest
import torch

from oracle import loss as oloss
from oracle.fill import REAL, grammar_tokens
from midiseq import ops
from midiseq import _lib as L
from midiseq._lib import ptr, call, stream
from midiseq.loss import ce_forward_backward

pytestmark = pytest.mark.gpu
dev = "cuda"


def _head(B, T, K, seed):
    g = torch.Generator().manual_seed(seed)
    V = REAL.size
    Vp = (V + 255) // 256 * 256
    A = (torch.randn(B * T, K, generator=g)).bfloat16().to(dev)
    W = (torch.randn(Vp, K, generator=g) * K ** -0.5 * 3).bfloat16()
    W[V:] = 0
    bias = torch.randn(Vp, generator=g) * 0.5
    bias[V:] = 0
    return A, W.to(dev), bias.to(dev), V, Vp


@pytest.mark.parametrize("B,T", [(1, 512), (2, 2048)])
def test_colstats_epilogue_matches_plain_gemm_and_colstats(B, T):
    A, W, bias, V, Vp = _head(B, T, 1024, B * T)
    plain = torch.empty(B * T, Vp, device=dev, dtype=torch.bfloat16)
    ops.gemm(A, W, out=plain, epilogue=L.EPI_BIAS, bias=bias)
    out = torch.empty_like(plain)
    part = torch.full((B * T // 128, 2, Vp), float("nan"), device=dev)
    assert ops.gemm_bias_colstats(A, W, out, bias, part)
    torch.cuda.synchronize()
    assert torch.equal(out, plain)
    # merge the partials on the host (fp64) and compare with the colstats kernel
    p = part.double().cpu().view(B, T // 128, 2, Vp)[..., :V]
    m = p[:, :, 0].max(dim=1).values
    s = (p[:, :, 1] * torch.exp(p[:, :, 0] - m[:, None])).sum(dim=1)
    lse_part = m + torch.log(s)
    col = torch.empty(B, V, device=dev)
    ws = torch.empty(L.lib().msq_filtered_workspace(B, T, V), device=dev, dtype=torch.uint8)
    call("msq_filtered_colstats", ptr(col), ptr(out), L.BF16, Vp, B, T, V, ptr(ws), stream())
    x = out.double().cpu().view(B, T, Vp)[:, :, :V]
    lse_ref = torch.logsumexp(x, dim=1)
    assert ((lse_part - lse_ref).abs().max() / lse_ref.abs().max()).item() < 1e-6
    assert ((col.double().cpu() - lse_ref).abs().max() / lse_ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("B,T", [(2, 512)])
def test_loss_through_partials(B, T):
    A, W, bias, V, Vp = _head(B, T, 1024, 11)
    logits = torch.empty(B * T, Vp, device=dev, dtype=torch.bfloat16)
    part = torch.empty(B * T // 128, 2, Vp, device=dev)
    assert ops.gemm_bias_colstats(A, W, logits, bias, part)
    rng = np.random.default_rng(3)
    w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
    src, trg = torch.from_numpy(w[:, :-1].copy()).to(dev), torch.from_numpy(w[:, 1:].copy()).to(dev)
    x = logits.view(B, T, Vp)
    dl1 = torch.zeros_like(x)
    db1 = torch.zeros(V, device=dev)
    loss1, _ = ce_forward_backward(src, x, trg, V, dlogits=dl1, dbias=db1, colpart=part)
    dl2 = torch.zeros_like(x)
    db2 = torch.zeros(V, device=dev)
    loss2, _ = ce_forward_backward(src, x, trg, V, dlogits=dl2, dbias=db2)
    torch.cuda.synchronize()
    assert abs(loss1.item() - loss2.item()) < 1e-5 * abs(loss2.item())
    d1, d2 = dl1.float(), dl2.float()
    assert ((d1 - d2).abs().max() / d2.abs().max()).item() < 1e-2
    # the output-bias gradient is analytically zero (the loss is invariant to a
    # per-(b, v) constant along T): both at round-off level
    assert db1.abs().max().item() < 1e-5 and db2.abs().max().item() < 1e-5
    lr = x[:, :, :V].float().cpu().requires_grad_(True)
    ref = oloss.loss(src.cpu(), trg.cpu(), lr, REAL)
    assert abs(loss1.item() - ref.item()) < 1e-4 * abs(ref.item())


def test_train_step_head_stats_on_off():
    from midiseq.transformer import Transformer, TransformerConfig
    from midiseq.train_parallel import TrainStep, SyntheticMIDI
    losses = []
    for on in (True, False):
        torch.manual_seed(0)
        cfg = TransformerConfig(n_layer=2, block_len=512, precision="bf16", dropout=0.0)
        model = Transformer(cfg).to(dev)
        step = TrainStep(model)
        step.eng.head_stats = on
        src, trg, meta = next(iter(SyntheticMIDI(2, 512, dev)))
        loss = step(src, trg, meta)
        A = step.eng.acts(2, 512)
        assert A.colpart_valid == on
        losses.append((loss.item(), model.flat.data.double().norm().item()))
    assert abs(losses[0][0] - losses[1][0]) < 1e-5 * abs(losses[1][0])
    assert abs(losses[0][1] - losses[1][1]) < 1e-6 * abs(losses[1][1])
