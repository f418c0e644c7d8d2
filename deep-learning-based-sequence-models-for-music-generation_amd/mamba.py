"""Drop-in for models/mamba/mamba.py:8-35 (``Mamba(d_model=1024, n_layers=10)``)
over the HIP kernels: 10 stacked Mamba2 mixers with NO residual and no
per-layer norm, a final LayerNorm and the output head, sliced [:, 6:].

Same engine structure as the Transformer: one flat fp32 parameter buffer
(reference state_dict keys map onto views of it), a bf16 shadow for the MFMA
GEMMs (in_proj 1024->4256, out_proj 2048->1024, the 17 914-way head), the SSD
scan in fp32 from chunk-entry states kept in HBM for the backward."""
import math
import os
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from ._lib import ptr, call, stream
from .config import N_META, VOCAB_SIZE, METADATA_VOCAB_SIZE
from .transformer import TransformerEngine, _align, _select, dx_gemm

D_STATE, D_CONV, HEADDIM = 64, 4, 64


def _keep_casts():
    """MSQ_MAMBA_CASTS=1: fp32 layer outputs / input gradients plus a cast
    launch (the round-2 form; A/B switch)."""
    return os.environ.get("MSQ_MAMBA_CASTS") == "1"


@dataclass
class MambaConfig:
    d_model: int = 1024
    n_layers: int = 10
    vocab_size: int = VOCAB_SIZE
    metadata_vocab_size: int = METADATA_VOCAB_SIZE
    precision: str = "bf16"
    norm_eps: float = 1e-5  # RMSNormGated eps of mamba_ssm.Mamba2

    @property
    def d_inner(self):
        return 2 * self.d_model

    @property
    def nheads(self):
        return self.d_inner // HEADDIM

    @property
    def conv_dim(self):
        return self.d_inner + 2 * D_STATE

    @property
    def d_in_proj(self):
        return 2 * self.d_inner + 2 * D_STATE + self.nheads

    @property
    def v_pad(self):
        return (self.vocab_size + 7) // 8 * 8


class MambaLayout:
    def __init__(self, cfg: MambaConfig):
        d, di, H, cd = cfg.d_model, cfg.d_inner, cfg.nheads, cfg.conv_dim
        entries = [("tok_emb", (cfg.vocab_size, d)), ("meta_emb", (cfg.metadata_vocab_size, d))]
        for l in range(cfg.n_layers):
            entries += [(f"{l}.in_w", (cfg.d_in_proj, d)), (f"{l}.conv_w", (cd, D_CONV)), (f"{l}.conv_b", (cd,)),
                        (f"{l}.dt_bias", (H,)), (f"{l}.A_log", (H,)), (f"{l}.D", (H,)), (f"{l}.norm_w", (di,)),
                        (f"{l}.out_w", (d, di))]
        entries += [("lnf_w", (d,)), ("lnf_b", (d,)), ("lm_w", (cfg.v_pad, d)), ("lm_b", (cfg.v_pad,))]
        self.offsets, off = {}, 0
        for name, shape in entries:
            self.offsets[name] = (off, shape)
            off += _align(math.prod(shape))
        self.numel = off

    def views(self, flat):
        return {n: flat[o:o + math.prod(s)].view(s) for n, (o, s) in self.offsets.items()}

    def layer_range(self, l):
        s = self.offsets[f"{l}.in_w"][0]
        o, sh = self.offsets[f"{l}.out_w"]
        return s, o + _align(math.prod(sh))


def reference_keys(cfg: MambaConfig):
    m = OrderedDict()
    m["token_embedding.weight"] = ("tok_emb", None)
    m["metadata_embedding.weight"] = ("meta_emb", None)
    m["output_layer.weight"] = ("lm_w", ("rows", 0, cfg.vocab_size))
    m["output_layer.bias"] = ("lm_b", ("rows", 0, cfg.vocab_size))
    for l in range(cfg.n_layers):
        p = f"layers.{l}."
        m[p + "dt_bias"] = (f"{l}.dt_bias", None)
        m[p + "A_log"] = (f"{l}.A_log", None)
        m[p + "D"] = (f"{l}.D", None)
        m[p + "in_proj.weight"] = (f"{l}.in_w", None)
        m[p + "conv1d.weight"] = (f"{l}.conv_w", ("conv",))
        m[p + "conv1d.bias"] = (f"{l}.conv_b", None)
        m[p + "norm.weight"] = (f"{l}.norm_w", None)
        m[p + "out_proj.weight"] = (f"{l}.out_w", None)
    m["norm.weight"] = ("lnf_w", None)
    m["norm.bias"] = ("lnf_b", None)
    return m


def _sel(t, sel):
    if sel is not None and sel[0] == "conv":
        return t.view(t.shape[0], 1, t.shape[1])
    return _select(t, sel)


class _MActs:
    def __init__(self, cfg, B, T, device, act, save):
        L_ = T + N_META
        M = B * L_
        n = cfg.n_layers if save else 1
        f32 = torch.float32
        e = lambda *s, dt=act: torch.empty(*s, device=device, dtype=dt)  # noqa: E731
        self.B, self.T, self.L, self.M, self.save = B, T, L_, M, save
        self.x = e(2, M, cfg.d_model, dt=f32)                # fp32 layer output ping-pong
        self.xa = e(n + 1 if save else 2, M, cfg.d_model)    # act copies (in_proj inputs)
        self.zx = e(n, M, cfg.d_in_proj)
        self.xc = e(n, M, cfg.conv_dim)
        self.y = e(n, M, cfg.d_inner)                        # SSD output, compute dtype
        self.yn = e(n, M, cfg.d_inner)
        self.rstd = e(n, M, dt=f32)
        nst = L.lib().msq_mamba_states_size(B, L_, cfg.nheads) // 4
        self.states = e(n, nst, dt=f32)
        self.xlast = e(M, cfg.d_model, dt=f32)
        self.f = e(B * T, cfg.d_model)
        self.stf = e(2, B * T, dt=f32)
        self.logits = e(B * T, cfg.v_pad)
        self.gen = 0
        self._bwd = None

    def bwd(self, cfg, device, act):
        if self._bwd is None:
            M = self.M
            f32 = torch.float32
            e = lambda *s, dt=act: torch.empty(*s, device=device, dtype=dt)  # noqa: E731
            self._bwd = dict(gx=e(M, cfg.d_model, dt=f32), gxb=e(M, cfg.d_model), dyn=e(M, cfg.d_inner, dt=f32),
                             dy=e(M, cfg.d_inner), dzx=e(M, cfg.d_in_proj), dxc=e(M, cfg.conv_dim, dt=f32),
                             df=e(self.B * self.T, cfg.d_model), dlogits=torch.zeros(self.B * self.T, cfg.v_pad, device=device, dtype=act))
        return self._bwd


class DecodeCache:
    """Recurrent state of the cached decode for B rows:
    per layer the conv window (fp32 [B, 3, conv_dim], last three pre-conv xBC
    rows) and the SSM state (fp32 [B, H, 64, 64]); the running time-axis LSE
    of the logits (fp32 [B, V]); step buffers for one position."""

    def __init__(self, cfg, B, device, act):
        f32 = torch.float32
        e = lambda *s, dt=act: torch.empty(*s, device=device, dtype=dt)  # noqa: E731
        self.B = B
        self.conv = torch.zeros(cfg.n_layers, B, D_CONV - 1, cfg.conv_dim, device=device, dtype=f32)
        self.ssm = torch.zeros(cfg.n_layers, B, cfg.nheads, HEADDIM, D_STATE, device=device, dtype=f32)
        self.lse = e(B, cfg.vocab_size, dt=f32)
        self.x = e(B, cfg.d_model, dt=f32)
        self.xa = e(B, cfg.d_model)
        self.zx = e(B, cfg.d_in_proj)
        self.xc = e(B, cfg.conv_dim)
        self.y = e(B, cfg.d_inner)
        self.yn = e(B, cfg.d_inner)
        self.rstd = e(B, dt=f32)
        self.f = e(B, cfg.d_model)
        self.stf = e(2, B, dt=f32)
        self.logits = e(B, cfg.v_pad)
        self.length = 0  # positions absorbed (metadata excluded)
        # the step as one HIP graph (captured on the second step; the first
        # runs eagerly and allocates the step's workspaces)
        self.graph, self.tok_buf, self.eager_steps = None, None, 0

    def stage_tok(self, tok):
        """the step graph's token buffer (int64 [B]) holding tok; a new buffer
        (shape change) drops the captured graph"""
        if self.tok_buf is None or self.tok_buf.shape != tok.shape or self.tok_buf.device != tok.device:
            self.tok_buf = torch.empty(tok.shape, dtype=torch.int64, device=tok.device)
            self.graph = None
        if tok.data_ptr() != self.tok_buf.data_ptr():
            self.tok_buf.copy_(tok)
        return self.tok_buf


class MambaEngine:
    # decode steps replay a captured HIP graph (False: eager launches; tests / profiling)
    step_graphs = True
    # weight-gradient GEMMs of the backward on a second stream (see backward())
    overlap_dw = True

    def __init__(self, cfg: MambaConfig, flat):
        self.cfg = cfg
        self.layout = MambaLayout(cfg)
        self.act = torch.bfloat16 if cfg.precision == "bf16" else torch.float32
        self.flat = flat
        self.device = flat.device
        self.P = self.layout.views(flat.data)
        if self.act == torch.bfloat16:
            self.shadow = torch.empty(self.layout.numel, device=flat.device, dtype=torch.bfloat16)
            self.W = self.layout.views(self.shadow)
        else:
            self.shadow, self.W = None, self.P
        self._shadow_version = None
        self._acts = {}
        self.layer_grad_ready = None

    refresh_shadow = TransformerEngine.refresh_shadow
    mark_shadow_fresh = TransformerEngine.mark_shadow_fresh
    transposed_weights = TransformerEngine.transposed_weights

    def _t_names(self):
        return [f"{l}.{n}" for l in range(self.cfg.n_layers) for n in ("in_w", "out_w")] + ["lm_w"]

    def acts(self, B, T, save=True):
        key = (B, T, save)
        if key not in self._acts:
            self._acts = {k: v for k, v in self._acts.items() if k[2] != save}
            self._acts[key] = _MActs(self.cfg, B, T, self.device, self.act, save)
        return self._acts[key]

    def dlogits_buffer(self, B, T):
        return self.acts(B, T).bwd(self.cfg, self.device, self.act)["dlogits"]

    def bucket_ranges(self):
        lay, off = self.layout, self.layout.offsets
        r = {"head": (off["lnf_w"][0], lay.numel), -1: (0, off["0.in_w"][0])}
        for l in range(self.cfg.n_layers):
            r[l] = lay.layer_range(l)
        return r

    def _dims(self, A):
        c = self.cfg
        return A.B, A.L, c.d_inner, c.nheads

    def decode_cache(self, B):
        return DecodeCache(self.cfg, B, self.device, self.act)

    def forward(self, idx, meta, save=True, train=False, cache=None):
        """cache (a DecodeCache, save=False): also leave every mixer's state
        after the last position in it (the cached decode's prefill)."""
        # models/mamba/mamba.py has no dropout: train mode changes nothing
        cfg, P, W = self.cfg, self.P, self.W
        if not idx.is_cuda:
            raise RuntimeError("the MI355X engine runs on the GPU only (no CPU fallback)")
        self.refresh_shadow()
        B, T = idx.shape
        A = self.acts(B, T, save)
        A.gen += 1
        idx, meta = idx.contiguous(), meta.contiguous()
        if save:
            self._idx, self._meta = idx, meta
        d, M = cfg.d_model, A.M
        Bb, Ll, di, H = self._dims(A)
        dtc = L.BF16 if self.act == torch.bfloat16 else L.F32
        s = stream()
        x = A.x[0]
        ops.embed_fwd(x.view(B, A.L, d), P["tok_emb"], P["meta_emb"], idx, meta)
        xa = A.xa[0]
        ops.cast(xa, x)
        for l in range(cfg.n_layers):
            k = l if save else 0
            zx, xc, y, yn = A.zx[k], A.xc[k], A.y[k], A.yn[k]
            ops.gemm(xa, W[f"{l}.in_w"], out=zx)
            call("msq_mamba_conv_fwd", ptr(xc), cfg.conv_dim, ptr(zx), cfg.d_in_proj, dtc, ptr(P[f"{l}.conv_w"]),
                 ptr(P[f"{l}.conv_b"]), Bb, Ll, di, H, s)
            call("msq_mamba_ssd_fwd_state", ptr(y), di, ptr(A.states[k]), ptr(cache.ssm[l]) if cache else None,
                 ptr(xc), cfg.conv_dim, ptr(zx), cfg.d_in_proj, dtc, ptr(P[f"{l}.dt_bias"]), ptr(P[f"{l}.A_log"]),
                 ptr(P[f"{l}.D"]), Bb, Ll, di, H, s)
            if cache is not None:  # conv window: the last three pre-conv xBC rows
                cache.conv[l].copy_(zx.view(B, Ll, cfg.d_in_proj)[:, Ll - (D_CONV - 1):, di:di + cfg.conv_dim])
            call("msq_mamba_gnorm_fwd", ptr(yn), di, ptr(A.rstd[k]), ptr(y), di, ptr(zx), cfg.d_in_proj, dtc,
                 ptr(P[f"{l}.norm_w"]), M, di, float(cfg.norm_eps), s)
            if l == cfg.n_layers - 1:
                ops.gemm(yn, W[f"{l}.out_w"], out=A.xlast)
            else:
                xa = A.xa[l + 1] if save else A.xa[(l + 1) % 2]
                if xa.dtype != torch.float32 and not _keep_casts():
                    # the next layer's bf16 input straight from the GEMM's fp32
                    # accumulator: the same rounding as an fp32 row + cast
                    ops.gemm(yn, W[f"{l}.out_w"], out=xa)
                else:
                    xo = A.x[(l + 1) % 2]
                    ops.gemm(yn, W[f"{l}.out_w"], out=xo)
                    ops.cast(xa, xo)
        ops.layernorm_fwd(A.xlast, P["lnf_w"], P["lnf_b"], out=A.f, mean=A.stf[0], rstd=A.stf[1], seg=(T, N_META))
        V = cfg.vocab_size
        # full V_pad rows (pad rows of lm_w / lm_b are zero): 16-B aligned rows, 256-tile eligible
        ops.gemm(A.f, W["lm_w"], out=A.logits, epilogue=L.EPI_BIAS, bias=P["lm_b"])
        if cache is not None:
            cache.length = T
        return A.logits.view(B, T, cfg.v_pad)[:, :, :V]

    @torch.no_grad()
    def step(self, tok, cache):
        """One recurrent position for every row: tok int64 [B] (contiguous) ->
        logits [B, v_pad] (cache.logits) of that position; the cache advances.
        Equal to the last row of forward() over the grown sequence."""
        if not tok.is_cuda:
            raise RuntimeError("the MI355X engine runs on the GPU only (no CPU fallback)")
        self.refresh_shadow()
        # every launch of a step has fixed pointers and sizes (the recurrent
        # state lives in the cache): replay one captured HIP graph instead of
        # ~7 launches per layer from the host
        # (the graph reads the token from the cache's staging buffer: a fresh
        # token tensor per step costs a device copy, not a re-capture)
        # stage first: a token tensor of a new shape / device reallocates the
        # staging buffer and drops the graph that read the old one
        tb = cache.stage_tok(tok) if self.step_graphs else tok
        if self.step_graphs and cache.graph is not None:
            cache.graph.replay()
        elif self.step_graphs and cache.eager_steps >= 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step_body(tb, cache)
            cache.graph = g
            g.replay()
        else:
            self._step_body(tok, cache)
            cache.eager_steps += 1
        cache.length += 1
        return cache.logits

    def _step_body(self, tok, cache):
        cfg, P, W = self.cfg, self.P, self.W
        B, d, di, H = cache.B, cfg.d_model, cfg.d_inner, cfg.nheads
        dtc = L.BF16 if self.act == torch.bfloat16 else L.F32
        s = stream()
        call("msq_embed_fwd", ptr(cache.x), ptr(P["tok_emb"]), ptr(P["meta_emb"]), ptr(tok), None, B, 1, 0, d, s)
        ops.cast(cache.xa, cache.x)
        for l in range(cfg.n_layers):
            if dtc == L.BF16:  # in_proj with the conv step in its epilogue (one launch)
                call("msq_mamba_in_proj_conv_step", ptr(cache.zx), cfg.d_in_proj, ptr(cache.xc), cfg.conv_dim,
                     ptr(cache.conv[l]), ptr(cache.xa), d, ptr(W[f"{l}.in_w"]), d, ptr(P[f"{l}.conv_w"]),
                     ptr(P[f"{l}.conv_b"]), B, d, cfg.d_in_proj, di, H, s)
            else:
                ops.gemm(cache.xa, W[f"{l}.in_w"], out=cache.zx)
                call("msq_mamba_conv_step", ptr(cache.xc), cfg.conv_dim, ptr(cache.conv[l]), ptr(cache.zx),
                     cfg.d_in_proj, dtc, ptr(P[f"{l}.conv_w"]), ptr(P[f"{l}.conv_b"]), B, di, H, s)
            call("msq_mamba_ssd_step", ptr(cache.y), di, ptr(cache.ssm[l]), ptr(cache.xc), cfg.conv_dim, ptr(cache.zx),
                 cfg.d_in_proj, dtc, ptr(P[f"{l}.dt_bias"]), ptr(P[f"{l}.A_log"]), ptr(P[f"{l}.D"]), B, di, H, s)
            call("msq_mamba_gnorm_fwd", ptr(cache.yn), di, ptr(cache.rstd), ptr(cache.y), di, ptr(cache.zx),
                 cfg.d_in_proj, dtc, ptr(P[f"{l}.norm_w"]), B, di, float(cfg.norm_eps), s)
            if l < cfg.n_layers - 1 and cache.xa.dtype != torch.float32:
                # the next layer's bf16 input straight from the fp32 accumulator
                # (the same rounding as forward()'s fp32 row + cast)
                ops.gemm(cache.yn, W[f"{l}.out_w"], out=cache.xa)
            else:
                ops.gemm(cache.yn, W[f"{l}.out_w"], out=cache.x)
                if l < cfg.n_layers - 1:  # (the last layer's output feeds only the final LayerNorm)
                    ops.cast(cache.xa, cache.x)
        ops.layernorm_fwd(cache.x, P["lnf_w"], P["lnf_b"], out=cache.f, mean=cache.stf[0], rstd=cache.stf[1])
        ops.gemm(cache.f, W["lm_w"], out=cache.logits, epilogue=L.EPI_BIAS, bias=P["lm_b"])

    def backward(self, dlogits, grads, head_bias_done=False):
        cfg, P, W = self.cfg, self.P, self.W
        G = self.layout.views(grads)
        idx, meta = self._idx, self._meta
        B, T = idx.shape
        A = self.acts(B, T)
        Bw = A.bwd(cfg, self.device, self.act)
        Bb, Ll, di, H = self._dims(A)
        M, V = A.M, cfg.vocab_size
        dtc = L.BF16 if self.act == torch.bfloat16 else L.F32
        s = stream()
        hook = self.layer_grad_ready
        dl = dlogits[:, :V]
        # weight gradients on a second stream (ops.SideStream; the
        # Transformer's backward does the same): the out_proj / in_proj dW
        # GEMMs (MFMA-bound) overlap the HBM-bound gated-norm / SSD / conv
        # backward of the main stream. Shared buffers they read: gin (gxb in
        # bf16, else gx) and dzx, each overwritten one step later only after
        # the side launch that reads it (before_write).
        # overlap_dw = False keeps one stream.
        sd = ops.SideStream(self.device, self.overlap_dw, hook)

        def lm_w():
            ops.gemm(dlogits, A.f, ta=True, tb=True, out=G["lm_w"], epilogue=L.EPI_ACCUM)  # pad columns are 0
            if not head_bias_done:
                ops.colsum(dl, G["lm_b"][:V], accumulate=True)
        sd.run("dlogits", lm_w)
        Wt = self.transposed_weights()
        dx_gemm(dlogits, W, Wt, "lm_w", Bw["df"])
        gx, gxb = Bw["gx"], Bw["gxb"]
        gx.zero_()
        ops.layernorm_bwd(gx, Bw["df"], A.xlast, A.stf[0], A.stf[1], P["lnf_w"], G["lnf_w"], G["lnf_b"],
                          seg=(T, N_META), ordered=True)
        sd.layer_done("head")
        # per-chunk state gradients of the bf16 SSD backward (msq_mamba_ssd_bwd_workspace)
        ssd_ws = ops.workspace(L.lib().msq_mamba_ssd_bwd_workspace(Bb, Ll, H), self.device, "ssd_bwd")
        bf = self.act == torch.bfloat16
        gin = gxb if bf else gx
        if bf:
            sd.before_write("gin")
            ops.cast(gxb, gx)
        for l in reversed(range(cfg.n_layers)):

            def out_w(l=l):
                ops.gemm(gin, A.yn[l], ta=True, tb=True, out=G[f"{l}.out_w"], epilogue=L.EPI_ACCUM)
            sd.run("gin", out_w)
            dx_gemm(gin, W, Wt, f"{l}.out_w", Bw["dyn"])
            sd.before_write("dzx")
            call("msq_mamba_gnorm_bwd", ptr(Bw["dy"]), ptr(Bw["dzx"]), ptr(A.y[l]), di, ptr(A.zx[l]), cfg.d_in_proj,
                 dtc, ptr(P[f"{l}.norm_w"]), ptr(A.rstd[l]), ptr(Bw["dyn"]), di, ptr(G[f"{l}.norm_w"]), M, di, s)
            call("msq_mamba_ssd_bwd", ptr(Bw["dxc"]), cfg.conv_dim, ptr(Bw["dzx"]), ptr(Bw["dy"]), di,
                 ptr(A.states[l]), ptr(A.xc[l]), cfg.conv_dim, ptr(A.zx[l]), cfg.d_in_proj, dtc,
                 ptr(P[f"{l}.dt_bias"]), ptr(P[f"{l}.A_log"]), ptr(P[f"{l}.D"]), ptr(G[f"{l}.A_log"]), ptr(G[f"{l}.D"]),
                 ptr(G[f"{l}.dt_bias"]), Bb, Ll, di, H, ptr(ssd_ws), s)
            call("msq_mamba_conv_bwd", ptr(Bw["dzx"]), ptr(Bw["dxc"]), cfg.conv_dim, ptr(A.zx[l]), cfg.d_in_proj, dtc,
                 ptr(P[f"{l}.conv_w"]), ptr(P[f"{l}.conv_b"]), ptr(G[f"{l}.conv_w"]), ptr(G[f"{l}.conv_b"]), Bb, Ll,
                 di, H, s)

            def in_w(l=l):
                ops.gemm(Bw["dzx"], A.xa[l], ta=True, tb=True, out=G[f"{l}.in_w"], epilogue=L.EPI_ACCUM)
            sd.run("dzx", in_w)
            sd.before_write("gin")  # gin: read by this layer's out_proj dW
            # below layer 0 the next layer down reads only the bf16 copy: the dX
            # GEMM rounds its fp32 accumulator straight into it (as gx + cast would)
            direct = bf and l > 0 and not _keep_casts()
            dx_gemm(Bw["dzx"], W, Wt, f"{l}.in_w", gxb if direct else gx)
            if bf and l > 0 and not direct:
                sd.before_write("gin")
                ops.cast(gxb, gx)
            sd.layer_done(l)
        ops.embed_bwd(G["tok_emb"], G["meta_emb"], gx, idx, meta)
        sd.layer_done(-1)
        sd.finish()


class _MambaFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, idx, meta, engine):
        out = engine.forward(idx, meta)
        ctx.engine, ctx.gen, ctx.shape = engine, engine.acts(*idx.shape).gen, tuple(idx.shape)
        return out

    @staticmethod
    def backward(ctx, dlogits):
        eng = ctx.engine
        B, T = ctx.shape
        if eng.acts(B, T).gen != ctx.gen:
            raise RuntimeError("activations were overwritten by a later forward")
        cfg = eng.cfg
        buf = eng.dlogits_buffer(B, T)
        buf.view(B, T, cfg.v_pad)[:, :, :cfg.vocab_size].copy_(dlogits)
        grads = torch.zeros_like(eng.flat.data)
        eng.backward(buf, grads)
        return grads, None, None, None


class Mamba(nn.Module):
    """Mamba(d_model=1024, n_layers=10) drop-in; vocab sizes default to the
    reference's cc globals (mamba.py:12-14)."""

    def __init__(self, d_model=1024, n_layers=10, vocab_size=VOCAB_SIZE, metadata_vocab_size=METADATA_VOCAB_SIZE,
                 precision="bf16", device=None):
        super().__init__()
        self.cfg = MambaConfig(d_model=d_model, n_layers=n_layers, vocab_size=vocab_size,
                               metadata_vocab_size=metadata_vocab_size, precision=precision)
        lay = MambaLayout(self.cfg)
        self.flat = nn.Parameter(torch.zeros(lay.numel, device=device))
        self._engine = None
        self.reset_parameters()

    @property
    def layout(self):
        return MambaLayout(self.cfg)

    def reset_parameters(self, seed=0):
        """mamba_ssm-like init: A_log = log(1..H), D = 1, dt_bias = inv_softplus(dt ~ logU[1e-3, 1e-1])."""
        g = torch.Generator().manual_seed(seed)
        V = self.layout.views(self.flat.data)
        c = self.cfg
        with torch.no_grad():
            for name, (_, shape) in self.layout.offsets.items():
                t, leaf = V[name], name.split(".")[-1]
                if name in ("tok_emb", "meta_emb"):
                    t.copy_(torch.randn(shape, generator=g))
                elif leaf in ("in_w", "out_w", "lm_w"):
                    b = 1.0 / math.sqrt(shape[1])
                    t.copy_(torch.empty(shape).uniform_(-b, b, generator=g))
                elif leaf == "conv_w":
                    b = 1.0 / math.sqrt(D_CONV)
                    t.copy_(torch.empty(shape).uniform_(-b, b, generator=g))
                elif leaf in ("conv_b", "lm_b"):
                    b = 1.0 / math.sqrt(D_CONV if leaf == "conv_b" else c.d_model)
                    t.copy_(torch.empty(shape).uniform_(-b, b, generator=g))
                elif leaf == "A_log":
                    t.copy_(torch.log(torch.arange(1, shape[0] + 1, dtype=torch.float32)))
                elif leaf == "D" or leaf in ("norm_w", "lnf_w"):
                    t.fill_(1.0)
                elif leaf == "dt_bias":
                    dt = torch.exp(torch.rand(shape, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
                    dt = dt.clamp(min=1e-4)
                    t.copy_(dt + torch.log(-torch.expm1(-dt)))
                else:
                    t.zero_()
            if c.v_pad > c.vocab_size:
                V["lm_w"][c.vocab_size:].zero_()
                V["lm_b"][c.vocab_size:].zero_()
        self._engine = None

    @property
    def engine(self):
        if self._engine is None or self._engine.flat is not self.flat or self._engine.device != self.flat.device:
            self._engine = MambaEngine(self.cfg, self.flat)
        return self._engine

    def _apply(self, fn, *a, **k):
        out = super()._apply(fn, *a, **k)
        self._engine = None
        return out

    def forward(self, tokens, meta):
        if not (torch.is_grad_enabled() and self.flat.requires_grad):
            return self.engine.forward(tokens, meta, save=False)
        return _MambaFn.apply(self.flat, tokens, meta, self.engine)

    def get_name(self):
        return "Mamba"

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        V = self.layout.views(self.flat if keep_vars else self.flat.detach())
        out = OrderedDict() if destination is None else destination
        for k, (n, sel) in reference_keys(self.cfg).items():
            out[prefix + k] = _sel(V[n], sel)
        return out

    def load_state_dict(self, state_dict, strict=True, assign=False):
        V = self.layout.views(self.flat.data)
        keys = reference_keys(self.cfg)
        missing = [k for k in keys if k not in state_dict]
        unexpected = [k for k in state_dict if k not in keys]
        if strict and (missing or unexpected):
            raise RuntimeError(f"state_dict mismatch: missing {missing[:5]}, unexpected {unexpected[:5]}")
        with torch.no_grad():
            for k, (n, sel) in keys.items():
                if k in state_dict:
                    _sel(V[n], sel).copy_(state_dict[k])
        if self._engine is not None:
            self._engine.refresh_shadow(force=True)
        return torch.nn.modules.module._IncompatibleKeys(missing, unexpected)

    def grad_dict(self):
        V = self.layout.views(self.flat.grad)
        return OrderedDict((k, _sel(V[n], s)) for k, (n, s) in reference_keys(self.cfg).items())
