"""Thin tensor-level wrappers over the libmidiseq C ABI (no autograd here).

Every function launches on torch's current stream and raises on failure;
there is no fallback path.
"""
import torch

from . import _lib as L
from ._lib import ptr, call, stream, dt


def _mat(t, trans):
    """(rows, cols, ld, batch_stride, batch) of a 2-D/3-D row-major tensor."""
    assert t.stride(-1) == 1, "innermost dim must be contiguous"
    r, c = t.shape[-2], t.shape[-1]
    ld = t.stride(-2)
    if t.dim() == 3:
        return r, c, ld, t.stride(0), t.shape[0]
    return r, c, ld, 0, 1


def gemm(A, B, *, ta=False, tb=False, out=None, out_dtype=None, epilogue=L.EPI_NONE, bias=None, aux=None,
         drop=None, role=None):
    """C = op(A) . op(B).  ta: A stored [K,M]; tb: B stored [K,N] (else [N,K]).
    drop=(seed, site, p): epilogue BIAS_RESID becomes aux + dropout(acc + bias).
    role: what the product is for (e.g. "gemm_dX"), seen by launch observers
    (midiseq._lib.TAP, bench.py's per-class timing); no effect on the launch."""
    ar, ac, lda, sA, ba = _mat(A, ta)
    br, bc, ldb, sB, bb = _mat(B, tb)
    M, K = (ac, ar) if ta else (ar, ac)
    N, K2 = (bc, br) if tb else (br, bc)
    assert K == K2, f"K mismatch {K} vs {K2}"
    assert A.dtype == B.dtype
    batch = max(ba, bb)
    if out is None:
        odt = out_dtype or A.dtype
        out = torch.empty((batch, M, N) if batch > 1 or A.dim() == 3 else (M, N), device=A.device, dtype=odt)
    cr, cc, ldc, sC, bcnt = _mat(out, False)
    assert (cr, cc) == (M, N), f"out shape {(cr, cc)} != {(M, N)}"
    ldx = sX = 0
    axd = L.F32
    if aux is not None:
        _, _, ldx, sX, _ = _mat(aux, False)
        axd = dt(aux)
    seed, site, p = 0, 0, 0.0
    if drop is not None and drop[2] > 0:
        assert epilogue == L.EPI_BIAS_RESID, "dropout is fused into the bias+residual epilogue only"
        epilogue = L.EPI_BIAS_DROP_RESID
        seed, site, p = int(drop[0]), int(drop[1]), float(drop[2])
    # split-K partials (weight gradients) / the split-K tail of a wave-quantisation split
    nws = L.lib().msq_gemm_workspace_size(dt(A), int(ta), int(tb), M, N, K, lda, ldb, batch, epilogue)
    ws = _splitk_ws(A.device, nws) if nws > 0 else None
    L.ROLE = role
    try:
        call("msq_gemm_ex", dt(A), int(ta), int(tb), M, N, K, ptr(A), lda, sA, ptr(B), ldb, sB, ptr(out), dt(out),
             ldc, sC, batch, epilogue, ptr(bias), ptr(aux), axd, ldx, sX, seed, site, p, ptr(ws),
             nws if ws is not None else 0, stream())
    finally:
        L.ROLE = None
    return out


class gemm_route:
    """with ops.gemm_route(L.ROUTE_TILE256): ... runs the large bf16 products
    on that kernel family (msq_gemm_set_route; tests and A/B tools)."""

    def __init__(self, route):
        self.route = route

    def __enter__(self):
        self.prev = L.lib().msq_gemm_set_route(self.route)
        if self.prev < 0:
            raise RuntimeError(L.lib().msq_last_error().decode())
        return self

    def __exit__(self, *exc):
        L.lib().msq_gemm_set_route(self.prev)


def gemm_colsum(A, B, out, dbias, *, ta=False, tb=False, epilogue=L.EPI_NONE, aux=None, accumulate=False):
    """out = epi(op(A) . op(B)) (bf16, epilogue NONE / RELU_MASK) and
    dbias (+)= its column sums (fp32, fused into the GEMM epilogue)."""
    if A.dtype != torch.bfloat16:  # fp32 engine: the unfused pair
        gemm(A, B, ta=ta, tb=tb, out=out, epilogue=epilogue, aux=aux)
        return colsum(out, dbias, accumulate=accumulate)
    ar, ac, lda, _, _ = _mat(A, ta)
    br, bc, ldb, _, _ = _mat(B, tb)
    M, K = (ac, ar) if ta else (ar, ac)
    N = bc if tb else br
    assert out.shape == (M, N) and out.dtype == torch.bfloat16 and B.dtype == torch.bfloat16
    ws = workspace(L.lib().msq_gemm_colsum_workspace(M, N), A.device, "gemm_colsum")
    ldx = aux.stride(0) if aux is not None else 0
    call("msq_gemm_colsum", int(ta), int(tb), M, N, K, ptr(A), lda, ptr(B), ldb, ptr(out), out.stride(0), epilogue,
         ptr(aux), dt(aux) if aux is not None else L.F32, ldx, ptr(dbias), int(accumulate), ptr(ws), ws.numel(),
         stream())
    return out


def gemm_resid_ln(A, W, out, bias, aux, gamma, beta, y, eps=1e-5):
    """out = aux + A . W^T + bias (fp32) and y = LayerNorm(out rows) (msq_gemm_resid_ln:
    the decode step's residual product and the next LayerNorm, the norm fused
    into the split-K reduce for <= 64 bf16 rows)."""
    M, K = A.shape
    N = W.shape[0]
    assert out.shape == (M, N) and out.dtype == torch.float32 and aux.shape == (M, N) and y.shape == (M, N)
    nws = L.lib().msq_gemm_resid_ln_workspace(dt(A), M, N, K, A.stride(0), W.stride(0))
    ws = workspace(nws, A.device, "resid_ln")
    call("msq_gemm_resid_ln", dt(A), M, N, K, ptr(A), A.stride(0), ptr(W), W.stride(0), ptr(out), out.stride(0),
         ptr(bias), ptr(aux), aux.stride(0), ptr(gamma), ptr(beta), float(eps), ptr(y), dt(y), y.stride(0), ptr(ws),
         ws.numel(), stream())
    return out


def gemm_bias_colstats(A, W, out, bias, part):
    """out = A . W^T + bias (bf16; W [N, K] as nn.Linear.weight) and the
    column (max, sum exp) partials of out per 128 rows into part
    (msq_gemm_bias_colstats; [M / 128, 2, ld] fp32). Returns False when the
    shape is outside the kernel (the caller runs the plain GEMM)."""
    M, K = A.shape
    N = W.shape[0]
    if A.dtype != torch.bfloat16 or out.shape != (M, N):
        return False
    # the kernel's own preconditions (persistent 256 tile, descriptor extents of
    # C and of the partials, 16-B alignment, GEMM route), asked without a launch
    if not L.lib().msq_gemm_bias_colstats_applies(0, M, N, K, ptr(A), A.stride(0), ptr(W), W.stride(0), ptr(out),
                                                   out.stride(0), ptr(bias), ptr(part), part.stride(-2)):
        return False
    call("msq_gemm_bias_colstats", 0, M, N, K, ptr(A), A.stride(0), ptr(W), W.stride(0), ptr(out), out.stride(0),
         ptr(bias), ptr(part), part.stride(-2), stream())
    return True


class SideStream:
    """Weight-gradient launches of a backward on a second stream. Weight
    gradients (dW GEMMs, bias column sums of a bf16 branch gradient) feed only
    the optimizer, never the next layer's backward, so they can overlap the
    dX / normalisation / mixer chain of the main stream: each side launch
    waits for the main stream's producer of its inputs (an event recorded at
    the call), and the main stream waits for the side launch that reads a
    shared buffer before it overwrites it (before_write). With enabled=False
    every launch runs in place on the current stream (the one-stream
    backward). `hook` (the DDP bucket callback) runs on the side stream after
    both streams' work of the bucket (layer_done); finish() joins the streams
    before the optimizer reads the gradients."""

    _streams = {}

    def __init__(self, device, enabled, hook=None):
        self.main = torch.cuda.current_stream(device)
        self.enabled = enabled
        if enabled and device not in SideStream._streams:
            SideStream._streams[device] = torch.cuda.Stream(device=device)
        self.side = SideStream._streams[device] if enabled else self.main
        self.hook = hook
        self.pending = {}

    def run(self, key, fn):
        if not self.enabled:
            fn()
            return
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            fn()
        done = torch.cuda.Event()
        done.record(self.side)
        self.pending[key] = done

    def before_write(self, key):
        ev = self.pending.pop(key, None)
        if ev is not None:
            self.main.wait_event(ev)

    def layer_done(self, key):
        if self.hook is None:
            return
        if not self.enabled:
            self.hook(key)
            return
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):  # the bucket's event then follows both streams
            self.hook(key)

    def finish(self):
        if self.enabled:
            self.main.wait_stream(self.side)  # the optimizer reads every gradient
        self.pending.clear()


_WS = {}


def _splitk_ws(device, nbytes):
    """Split-K partial workspace of the weight-gradient GEMMs, one per
    (device, stream): kept and grown, owned by torch's caching allocator."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 64 << 20), device=device, dtype=torch.uint8)
        _WS[key] = ws
    return ws


def layernorm_fwd(x, gamma, beta, eps=1e-5, out_dtype=torch.float32, out=None, mean=None, rstd=None, seg=(0, 0)):
    """seg=(seg_len, seg_skip): normalise only rows skip..skip+seg_len-1 of every
    (seg_len+seg_skip)-row segment of x into a compact output."""
    d = x.shape[-1]
    rows = x.numel() // d
    if seg[1]:
        rows = rows // (seg[0] + seg[1]) * seg[0]
    y = out if out is not None else torch.empty((rows, d), device=x.device, dtype=out_dtype)
    mean = mean if mean is not None else torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = rstd if rstd is not None else torch.empty(rows, device=x.device, dtype=torch.float32)
    call("msq_layernorm_fwd", ptr(y), dt(y), ptr(mean), ptr(rstd), ptr(x), ptr(gamma), ptr(beta), rows, d,
         float(eps), seg[0], seg[1], stream())
    return y, mean, rstd


_ws_cache = {}


def workspace(nbytes, device, tag="ws"):
    """Scratch buffer of a launch, one per (tag, device, stream): launches on
    different streams never share one."""
    key = (tag, device, torch.cuda.current_stream(device).cuda_stream)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), device=device, dtype=torch.uint8)
        _ws_cache[key] = buf
    return buf


def layernorm_bwd(dx_acc, dy, x, mean, rstd, gamma, dgamma, dbeta, dx_copy=None, seg=(0, 0), drop=None,
                  dbias=None, ordered=True):
    """dx_acc[map(r)] += LN'(dy[r]); dgamma/dbeta += ...; optional copy of the updated rows
    (drop=(seed, site, p): the copy is masked by that site's dropout keep mask and scaled);
    dbias += column sums of the written rows (the copy, else dx_acc).
    ordered=True: rows in a fixed order, so the parameter-gradient sums are bitwise
    reproducible (the ln_f beta gradient is analytically-zero round-off that Adam
    normalises); ordered=False: rows from a work queue (timing decides the last bits;
    measured slower since the kernel keeps two rows in flight per wave)."""
    d = x.shape[-1]
    rows = mean.numel()
    ws = workspace(L.lib().msq_layernorm_bwd_workspace(rows, d), x.device, "ln")
    seed, site, p = drop if drop is not None else (0, 0, 0.0)
    call("msq_layernorm_bwd_bias", ptr(dx_acc), ptr(dx_copy), dt(dx_copy) if dx_copy is not None else L.F32,
         ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(dy), dt(dy), ptr(x), ptr(mean), ptr(rstd), ptr(gamma), rows, d,
         seg[0], seg[1], int(seed), int(site), float(p), 0 if ordered else 1, ptr(ws), stream())


def colsum(x2d, out, accumulate=False):
    rows, cols = x2d.shape
    ws = workspace(L.lib().msq_colsum_workspace(rows, cols), x2d.device, "colsum")
    call("msq_colsum", ptr(out), int(accumulate), ptr(x2d), dt(x2d), rows, cols, x2d.stride(0), ptr(ws), stream())
    return out


def embed_fwd(x, tok_table, meta_table, idx, meta):
    B, T = idx.shape
    call("msq_embed_fwd", ptr(x), ptr(tok_table), ptr(meta_table), ptr(idx), ptr(meta), B, T, meta.shape[1],
         tok_table.shape[1], stream())
    return x


def embed_bwd(g_tok, g_meta, dx, idx, meta, deterministic=True):
    """g_tok[idx] += dx token rows, g_meta[meta] += dx metadata rows. deterministic:
    sorted segment sums (bitwise reproducible); else fp32 atomics."""
    B, T = idx.shape
    nm, d = meta.shape[1], g_tok.shape[1]
    if not deterministic:
        call("msq_embed_bwd", ptr(g_tok), ptr(g_meta), ptr(dx), ptr(idx), ptr(meta), B, T, nm, d, stream())
        return
    Vt, Vm = g_tok.shape[0], g_meta.shape[0]
    ws = workspace(L.lib().msq_embed_bwd_workspace(B, T, nm, d, Vt, Vm), dx.device, "embed")
    call("msq_embed_bwd_sorted", ptr(g_tok), ptr(g_meta), ptr(dx), ptr(idx), ptr(meta), B, T, nm, d, Vt, Vm,
         ptr(ws), stream())


def cast(dst, src):
    call("msq_cast", ptr(dst), dt(dst), ptr(src), dt(src), src.numel(), stream())
    return dst


def adam_step(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, shadow=None, grad_scale=1.0):
    call("msq_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), ptr(shadow), p.numel(), float(lr), float(beta1),
         float(beta2), float(eps), int(step), float(grad_scale), stream())


def dropout_attn_mask(B, H, S, seed, site0, p, device, out=None):
    """(rowmask, colmask) keep bits of one layer's attention dropout (msq_dropout_attn_mask)."""
    if out is None:
        out = torch.zeros(2, L.lib().msq_dropout_mask_words(B, H, S), device=device, dtype=torch.int32)
    call("msq_dropout_attn_mask", ptr(out[0]), ptr(out[1]), B, H, S, int(seed), int(site0), float(p), stream())
    return out
