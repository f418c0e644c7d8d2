"""Drop-in for train.py's loss surface (train.py:79-138 / train_parallel.py:
83-141 + torch.nn.CrossEntropyLoss) on the HIP kernels of csrc/loss.hip.

* ``filtered_logit(input, output)`` returns Z = -log_softmax(output, dim=1) *
  W[bucket(input)] exactly like the reference (autograd supported);
* ``filtered_cross_entropy(src, logits, trg)`` fuses filtered_logit and the
  cross-entropy (mean over B*T, no ignore_index) into one pass and produces
  d(loss)/d(logits) in the same pass when gradients are needed.
No [B,T,V] weight tensor is ever materialised."""
import torch

from . import _lib as L
from ._lib import ptr, call, stream, dt
from .config import Grammar
from .ops import workspace

_tables = {}


def grammar_table(device, grammar: Grammar = None):
    grammar = grammar or Grammar()
    key = (str(device), grammar.disc.vocab_size, grammar.bounds)
    t = _tables.get(key)
    if t is None:
        t = grammar.table(device).contiguous()
        _tables[key] = t
    return t


def _ws(B, T, V, device):
    return workspace(L.lib().msq_filtered_workspace(B, T, V), device, "loss")


def ce_forward_backward(src, logits, trg, V, grammar=None, dlogits=None, grad_scale=None, col_lse=None, dbias=None,
                        colpart=None):
    """logits [B,T,ld] (fp32/bf16, ld >= V). Returns (loss scalar tensor,
    dlogits or None). grad_scale defaults to 1/(B*T) (gradient of the mean).
    dbias (fp32 [V], with dlogits): += column sums of dlogits (the output
    layer's bias gradient) in the same pass. colpart ([B*T/128, 2, ld] fp32,
    with dlogits): the time-axis column (max, sum exp) partials the lm_head
    GEMM epilogue produced (ops.gemm_bias_colstats); the loss then skips its
    own pass over the logits for them."""
    grammar = grammar or Grammar()
    B, T = src.shape
    ld = logits.stride(1)
    assert logits.stride(2) == 1 and logits.stride(0) == T * ld, "logits must be [B,T,ld] row-major"
    wtab = grammar_table(logits.device, grammar)
    loss = torch.empty((), device=logits.device, dtype=torch.float32)
    if col_lse is None:
        col_lse = torch.empty(B, V, device=logits.device, dtype=torch.float32)
    gs = (1.0 / (B * T)) if grad_scale is None else float(grad_scale)
    b = grammar.bounds
    if colpart is not None:
        assert dlogits is not None and colpart.shape[0] == B * T // 128
        call("msq_filtered_ce_bias_part", ptr(loss), ptr(dlogits), dlogits.stride(1), ptr(dbias), ptr(logits),
             dt(logits), ld, ptr(src), ptr(trg), ptr(wtab), b[0], b[1], b[2], b[3], B, T, V, gs, ptr(col_lse),
             ptr(colpart), T // 128, colpart.stride(1), ptr(_ws(B, T, V, logits.device)), stream())
        return loss, dlogits
    call("msq_filtered_ce_bias", ptr(loss), ptr(dlogits), dlogits.stride(1) if dlogits is not None else 0,
         ptr(dbias), ptr(logits), dt(logits), ld, ptr(src), ptr(trg), ptr(wtab), b[0], b[1], b[2], b[3], B, T, V, gs,
         ptr(col_lse), ptr(_ws(B, T, V, logits.device)), stream())
    return loss, dlogits


class _FilteredCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, src, trg, grammar):
        B, T, V = logits.shape
        x = logits if logits.stride(2) == 1 and logits.stride(1) % 4 == 0 and logits.stride(0) == T * logits.stride(1) \
            else _padded(logits)
        need = logits.requires_grad
        dl = torch.empty(B, T, x.stride(1), device=x.device, dtype=x.dtype)[:, :, :V] if need else None
        loss, dl = ce_forward_backward(src.contiguous(), x, trg.contiguous(), V, grammar, dl)
        ctx.save_for_backward(dl if need else None)
        return loss

    @staticmethod
    def backward(ctx, gout):
        (dl,) = ctx.saved_tensors
        return (dl * gout.to(dl.dtype)) if dl is not None else None, None, None, None


def filtered_cross_entropy(src, logits, trg, grammar: Grammar = None):
    """== CrossEntropyLoss()(filtered_logit(src, logits).reshape(-1,V), trg.view(-1))."""
    return _FilteredCE.apply(logits, src, trg, grammar)


class _FilteredLogit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, src, grammar):
        grammar = grammar or Grammar()
        B, T, V = logits.shape
        x = logits if logits.stride(2) == 1 and logits.stride(1) % 4 == 0 and logits.stride(0) == T * logits.stride(1) \
            else _padded(logits)
        wtab = grammar_table(x.device, grammar)
        col_lse = torch.empty(B, V, device=x.device, dtype=torch.float32)
        ldz = (V + 3) // 4 * 4
        z = torch.empty(B, T, ldz, device=x.device, dtype=torch.float32)
        b = grammar.bounds
        src = src.contiguous()
        call("msq_filtered_logit", ptr(z), ldz, ptr(x), dt(x), x.stride(1), ptr(src), ptr(wtab), b[0], b[1], b[2],
             b[3], B, T, V, 0, ptr(col_lse), ptr(_ws(B, T, V, x.device)), stream())
        ctx.save_for_backward(x, src, col_lse)
        ctx.grammar = grammar
        ctx.V = V
        return z[:, :, :V]

    @staticmethod
    def backward(ctx, dz):
        x, src, col_lse = ctx.saved_tensors
        g, V = ctx.grammar, ctx.V
        B, T = src.shape
        ldz = (V + 3) // 4 * 4
        dzp = torch.zeros(B, T, ldz, device=x.device, dtype=torch.float32)
        dzp[:, :, :V] = dz
        dl = torch.empty(B, T, x.stride(1), device=x.device, dtype=x.dtype)
        b = g.bounds
        call("msq_filtered_logit_bwd", ptr(dl), dl.stride(1), ptr(dzp), ldz, ptr(x), dt(x), x.stride(1), ptr(src),
             ptr(grammar_table(x.device, g)), b[0], b[1], b[2], b[3], B, T, V, ptr(col_lse),
             ptr(_ws(B, T, V, x.device)), stream())
        return dl[:, :, :V], None, None


def _padded(t):
    B, T, V = t.shape
    ld = (V + 3) // 4 * 4
    p = torch.empty(B, T, ld, device=t.device, dtype=t.dtype)
    p[:, :, :V] = t
    return p[:, :, :V]


def filtered_logit(input, output, grammar: Grammar = None):
    """train.py:133-138 drop-in: -log_softmax(output, dim=1) * weights[bucket(input)]."""
    return _FilteredLogit.apply(output, input, grammar)
