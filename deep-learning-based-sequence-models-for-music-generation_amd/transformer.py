"""Drop-in for models/transformer/model_transformer.py:136-168 (``Transformer``)
backed by an explicit forward/backward engine over the HIP kernels.

Layout in HBM (one allocation per kind, everything resident):
  * parameters: ONE flat fp32 buffer (the nn.Parameter the optimiser sees),
    every tensor 256-B aligned; a bf16 shadow with the same offsets feeds the
    MFMA kernels (refreshed by the fused Adam kernel or lazily on version bump);
  * gradients: ONE flat fp32 buffer with the same offsets (DDP buckets are
    contiguous slices of it, in reverse layer order);
  * the residual stream is fp32 [B*S, d]; matmul operands/activations are bf16
    (or fp32 in the exact parity mode); the per-head q/k/v projections of the
    reference are packed into one [3d, d] matrix (q heads | k heads | v heads),
    so state_dict keys map to row slices of it.
Names in state_dict() are exactly the reference's (406 keys incl. the 64
``tril`` buffers, which are emitted as views of ONE shared mask)."""
import math
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from ._lib import ptr, call, stream, dt
from .attention import relattn_fwd, relattn_bwd
from .config import N_META, VOCAB_SIZE, METADATA_VOCAB_SIZE, BLOCK_LEN, DROPOUT

# dropout sites of the counter-based keep masks (csrc/common.h; oracle/dropout.py):
# attention probabilities of layer l / batch b / head h, proj output, FFN output
DROP_ATTN, DROP_PROJ, DROP_FFN = 1 << 28, 2 << 28, 3 << 28


@dataclass
class TransformerConfig:
    n_embd: int = 1024
    n_heads: int = 8
    n_layer: int = 8
    block_len: int = BLOCK_LEN
    # configs/common/config.yaml values.dropout, merged into the Transformer's
    # params by get_transformer_dict (train_parallel.py:49-54)
    dropout: float = DROPOUT
    vocab_size: int = VOCAB_SIZE
    metadata_vocab_size: int = METADATA_VOCAB_SIZE
    precision: str = "bf16"  # "bf16" (MFMA fast path) | "fp32" (exact parity path)

    @property
    def head_size(self):
        return self.n_embd // self.n_heads

    @property
    def s_max(self):
        return self.block_len + N_META

    @property
    def v_pad(self):
        return (self.vocab_size + 7) // 8 * 8

    @classmethod
    def from_params(cls, params, **kw):
        """Accepts the reference's SimpleNamespace (train_parallel.py:49-54)."""
        return cls(n_embd=params.n_embd, n_heads=params.n_heads, n_layer=params.n_layer,
                   block_len=params.block_len, dropout=getattr(params, "dropout", DROPOUT),
                   vocab_size=params.vocab_size, metadata_vocab_size=params.metadata_vocab_size, **kw)


def _align(n, a=64):
    return (n + a - 1) // a * a


class ParamLayout:
    """Offsets of every tensor inside the flat buffer."""

    def __init__(self, cfg: TransformerConfig):
        d, H, hs = cfg.n_embd, cfg.n_heads, cfg.head_size
        entries = [("tok_emb", (cfg.vocab_size, d)), ("meta_emb", (cfg.metadata_vocab_size, d))]
        for l in range(cfg.n_layer):
            entries += [(f"{l}.ln1_w", (d,)), (f"{l}.ln1_b", (d,)), (f"{l}.wqkv", (3 * d, d)),
                        (f"{l}.R", (H, cfg.s_max, hs)), (f"{l}.wproj", (d, d)), (f"{l}.bproj", (d,)),
                        (f"{l}.ln2_w", (d,)), (f"{l}.ln2_b", (d,)), (f"{l}.w1", (4 * d, d)), (f"{l}.b1", (4 * d,)),
                        (f"{l}.w2", (d, 4 * d)), (f"{l}.b2", (d,))]
        entries += [("lnf_w", (d,)), ("lnf_b", (d,)), ("lm_w", (cfg.v_pad, d)), ("lm_b", (cfg.v_pad,))]
        self.entries, self.offsets = entries, {}
        off = 0
        for name, shape in entries:
            self.offsets[name] = (off, shape)
            off += _align(math.prod(shape))
        self.numel = off

    def layer_range(self, l):
        """[start, end) of layer l's tensors (a contiguous DDP bucket)."""
        s = self.offsets[f"{l}.ln1_w"][0]
        e = self.offsets[f"{l}.b2"][0] + _align(self.offsets[f"{l}.b2"][1][0])
        return s, e

    def views(self, flat):
        out = {}
        for name, (off, shape) in self.offsets.items():
            out[name] = flat[off:off + math.prod(shape)].view(shape)
        return out


def reference_keys(cfg: TransformerConfig):
    """Reference state_dict key -> (internal name, row slice or head index)."""
    d, hs = cfg.n_embd, cfg.head_size
    m = OrderedDict()
    m["token_embedding_table.weight"] = ("tok_emb", None)
    m["metadata_embedding_table.weight"] = ("meta_emb", None)
    for l in range(cfg.n_layer):
        for h in range(cfg.n_heads):
            p = f"blocks.{l}.sa.heads.{h}."
            m[p + "rel_pos_emb"] = (f"{l}.R", ("head", h))
            m[p + "tril"] = ("__tril__", None)
            m[p + "key.weight"] = (f"{l}.wqkv", ("rows", d + h * hs, d + (h + 1) * hs))
            m[p + "query.weight"] = (f"{l}.wqkv", ("rows", h * hs, (h + 1) * hs))
            m[p + "value.weight"] = (f"{l}.wqkv", ("rows", 2 * d + h * hs, 2 * d + (h + 1) * hs))
        p = f"blocks.{l}."
        m[p + "sa.proj.weight"] = (f"{l}.wproj", None)
        m[p + "sa.proj.bias"] = (f"{l}.bproj", None)
        m[p + "ffwd.net.0.weight"] = (f"{l}.w1", None)
        m[p + "ffwd.net.0.bias"] = (f"{l}.b1", None)
        m[p + "ffwd.net.2.weight"] = (f"{l}.w2", None)
        m[p + "ffwd.net.2.bias"] = (f"{l}.b2", None)
        m[p + "ln1.weight"] = (f"{l}.ln1_w", None)
        m[p + "ln1.bias"] = (f"{l}.ln1_b", None)
        m[p + "ln2.weight"] = (f"{l}.ln2_w", None)
        m[p + "ln2.bias"] = (f"{l}.ln2_b", None)
    m["ln_f.weight"] = ("lnf_w", None)
    m["ln_f.bias"] = ("lnf_b", None)
    m["lm_head.weight"] = ("lm_w", ("rows", 0, cfg.vocab_size))
    m["lm_head.bias"] = ("lm_b", ("rows", 0, cfg.vocab_size))
    return m


def _select(t, sel):
    if sel is None:
        return t
    if sel[0] == "head":
        return t[sel[1]]
    return t[sel[1]:sel[2]]


def tril_mask(n, device="cpu"):
    """generate_matrix(n, 1) (model_transformer.py:8-16) without the python loop."""
    i = torch.arange(n, device=device)[:, None]
    j = torch.arange(n, device=device)[None, :]
    return ((j <= i) | (j < N_META)).to(torch.float32)


class _Acts:
    """Activation + scratch buffers for one (B, T), reused across steps."""

    def __init__(self, cfg, B, T, device, act, save=True):
        d, H = cfg.n_embd, cfg.n_heads
        S = T + N_META
        M = B * S
        Lc = cfg.n_layer if save else 1  # inference: one layer's buffers, reused
        f32 = torch.float32
        e = lambda *s, dt=act: torch.empty(*s, device=device, dtype=dt)  # noqa: E731
        self.B, self.T, self.S, self.M, self.save = B, T, S, M, save
        self.x = e(Lc + 1, M, d, dt=f32)
        self.xm = e(Lc, M, d, dt=f32)
        self.a, self.c = e(Lc, M, d), e(Lc, M, d)
        self.st1, self.st2 = e(Lc, 2, M, dt=f32), e(Lc, 2, M, dt=f32)
        self.qkv = e(Lc, M, 3 * d)
        self.o = e(Lc, M, d)
        self.lse = e(Lc, B, H, S, dt=f32)
        self.h = e(Lc, M, 4 * d)
        # the FFN ReLU mask at 1 bit per element (MSQ_MASK1, written by the FFN1
        # forward beside h): the FFN2 dX epilogue reads 1/16 of the bytes of h
        self.hm = (e(Lc, M, 4 * d // 32, dt=torch.int32)
                   if save and act == torch.bfloat16 and (4 * d) % 32 == 0 else None)
        self.f = e(B * T, d)
        self.stf = e(2, B * T, dt=f32)
        self.logits = e(B * T, cfg.v_pad)
        # the lm_head epilogue's column (max, sum exp) partials per 128 rows
        # (msq_gemm_bias_colstats), valid after a forward that produced them
        self.colpart = None
        self.colpart_valid = False
        self.gen = 0
        self._bwd = None
        self.bwd_zeroed = False  # gres / gb zero-filled by the last training forward
        self.drop = None      # (seed, p) of the last training forward
        self._masks = None    # [L, 2, n] attention keep bits (row / col layouts)

    def masks(self, cfg, device):
        if self._masks is None:
            n = L.lib().msq_dropout_mask_words(self.B, cfg.n_heads, self.S)
            self._masks = torch.zeros(cfg.n_layer if self.save else 1, 2, n, device=device, dtype=torch.int32)
        return self._masks

    def bwd(self, cfg, device, act):
        if self._bwd is None:
            d = cfg.n_embd
            M = self.M
            f32 = torch.float32
            e = lambda *s, dt=act: torch.empty(*s, device=device, dtype=dt)  # noqa: E731
            need_copy = act != f32 or cfg.dropout > 0  # fp32 + dropout: masked fp32 copy
            # gb / gb2: the bf16 branch gradients of the FFN / attention halves
            # of a block (two buffers so the weight-gradient stream can still
            # read one while the main stream writes the other)
            self._bwd = dict(gres=e(M, d, dt=f32), gb=e(M, d) if need_copy else None,
                             gb2=e(M, d) if need_copy and act != f32 else None, dtmp=e(M, d),
                             dh=e(M, 4 * d), dqkv=e(M, 3 * d), df=e(self.B * self.T, d),
                             dlogits=torch.zeros(self.B * self.T, cfg.v_pad, device=device, dtype=act))
        return self._bwd


class TransformerDecodeCache:
    """State of the cached decode (generate(mode="cached"); an approximation of
    scripts/generate.py:26-31, see msq_relattn_decode and oracle/transformer.py
    CachedTransformer) for B rows and a window of ``context`` tokens:
    per layer the keys / values of the window (act dtype [L, B, H, 6 + context,
    hs], a ring: metadata in slots 0..5, sequence position p in slot
    6 + p % context), the window's logits rows (a ring [B, context, v_pad],
    empty rows -inf so they drop out of the time-axis LSE) and tokens, and the
    one-position step buffers."""

    slides = True  # keeps stepping once the window is full (the Mamba cache does not)

    def __init__(self, cfg, B, context, device, act):
        d, H, hs = cfg.n_embd, cfg.n_heads, cfg.head_size
        if context + N_META > cfg.s_max:
            raise ValueError(f"context {context} exceeds block_len {cfg.block_len}")
        f32 = torch.float32
        e = lambda *s, dt=act: torch.empty(*s, device=device, dtype=dt)  # noqa: E731
        self.B, self.ctx, self.S_ring = B, context, context + N_META
        self.k = torch.zeros(cfg.n_layer, B, H, self.S_ring, hs, device=device, dtype=act)
        self.v = torch.zeros_like(self.k)
        self.ring = torch.full((B, context, cfg.v_pad), float("-inf"), device=device, dtype=act)
        self.tokens = torch.zeros(B, context, device=device, dtype=torch.int64)
        self.lse = e(B, cfg.vocab_size, dt=f32)
        self.x, self.xm = e(B, d, dt=f32), e(B, d, dt=f32)
        self.a, self.c, self.o, self.f = e(B, d), e(B, d), e(B, d), e(B, d)
        self.qkv, self.h = e(B, 3 * d), e(B, 4 * d)
        self.st, self.stf = e(2, B, dt=f32), e(2, B, dt=f32)
        self.logits = e(B, cfg.v_pad)
        # time-axis LSE of the ring kept as per-block partials (msq_ring_lse)
        self.RB = 64
        self.nblk = (context + self.RB - 1) // self.RB
        self.part = e(B, self.nblk, cfg.vocab_size, dt=f32)
        self.part_valid = False
        # incremental state of msq_ring_step (other blocks merged, the slot
        # block's prefix and suffix table; the block id in the last 16 bytes)
        nst = L.lib().msq_ring_state_bytes(B, cfg.vocab_size, self.RB)
        self.ring_state = torch.empty(nst, device=device, dtype=torch.uint8)
        self.ring_blk = self.ring_state[nst - 16:nst - 8].view(torch.int64)
        # partials of the split decode attention (msq_relattn_decode)
        self.attn_ws = torch.empty(L.lib().msq_relattn_decode_workspace(B, H, self.S_ring), device=device,
                                   dtype=torch.uint8)
        self.length = 0  # tokens absorbed (sequence positions 0 .. length-1)
        # graph-replayed steps (TransformerEngine.step): the position of the
        # next step on the device (advanced by msq_ring_step), the logits row of
        # the step before it goes into the ring, and the captured graph
        self.pos_dev = torch.zeros(1, device=device, dtype=torch.int64)
        self.row_buf = e(B, cfg.v_pad)
        self.graph, self.graph_gen, self.tok_buf = None, None, None

    def stage_tok(self, tok):
        """the step graph's token buffer (int64 [B]) holding tok; a new buffer
        (shape change) drops the captured graph"""
        if self.tok_buf is None or self.tok_buf.shape != tok.shape or self.tok_buf.device != tok.device:
            self.tok_buf = torch.empty(tok.shape, dtype=torch.int64, device=tok.device)
            self.graph = None
        if tok.data_ptr() != self.tok_buf.data_ptr():
            self.tok_buf.copy_(tok)
        return self.tok_buf


def dx_gemm(dy, W, Wt, name, out):
    """out = dy . W[name] (the input gradient of an nn.Linear): through the
    transposed copy Wt[name] (tb = 0) when the engine keeps one (bf16), else
    W itself (tb = 1)."""
    if Wt is not None:
        return ops.gemm(dy, Wt[name], out=out, role="gemm_dX")
    return ops.gemm(dy, W[name], tb=True, out=out, role="gemm_dX")


class TransformerEngine:
    """Explicit forward / backward over the libmidiseq kernels."""

    cache_slides = True  # generate(mode="cached") keeps stepping once the window slides

    def __init__(self, cfg: TransformerConfig, flat: torch.Tensor):
        if not 0.0 <= cfg.dropout < 1.0:
            raise ValueError(f"dropout must be in [0, 1), got {cfg.dropout}")
        self.cfg = cfg
        self.layout = ParamLayout(cfg)
        self.act = torch.bfloat16 if cfg.precision == "bf16" else torch.float32
        self.bind(flat)
        self._acts = {}
        # lm_head forward emits the loss's column statistics (set by TrainStep)
        self.head_stats = False
        # weight-gradient GEMMs on a second stream in the backward (see backward())
        self.overlap_dw = True

    def bind(self, flat):
        self.flat = flat
        self.device = flat.device
        self.P = self.layout.views(flat.data)
        if self.act == torch.bfloat16:
            self.shadow = torch.empty(self.layout.numel, device=flat.device, dtype=torch.bfloat16)
            self.W = self.layout.views(self.shadow)
        else:
            self.shadow = None
            self.W = self.P
        self._shadow_version = None

    def refresh_shadow(self, force=False):
        if self.shadow is None:
            return
        v = self.flat._version
        if force or v != self._shadow_version:
            ops.cast(self.shadow, self.flat.data)
            self._shadow_version = self.flat._version
            self._wgen = getattr(self, "_wgen", 0) + 1

    def mark_shadow_fresh(self):
        self._shadow_version = self.flat._version
        self._wgen = getattr(self, "_wgen", 0) + 1

    # the dX products (dX = dY . W of every nn.Linear) read W^T: transposed
    # bf16 copies (K-contiguous, the 256 tile's tb = 0 operand: its row reads
    # run ~15-20 % faster than the transposed-quad reads of W itself,
    # tools/gemm_vs_blas.py), refreshed once per change of the bf16 shadow
    # (0.1 ms per step for all of them)
    def _t_names(self):
        return [f"{l}.{n}" for l in range(self.cfg.n_layer) for n in ("wqkv", "wproj", "w1", "w2")] + ["lm_w"]

    def transposed_weights(self):
        if self.shadow is None:
            return None
        gen = getattr(self, "_wgen", 0)
        if getattr(self, "_wt_gen", None) == gen:
            return self._wt
        W = self.W
        if getattr(self, "_wt", None) is None:
            names = self._t_names()
            total = sum(W[n].numel() for n in names)
            buf = torch.empty(total, device=self.device, dtype=torch.bfloat16)
            self._wt, off = {}, 0
            for n in names:
                r, c = W[n].shape
                self._wt[n] = buf[off:off + r * c].view(c, r)
                off += r * c
        s = stream()
        for n, t in self._wt.items():
            src = W[n]
            call("msq_transpose_bf16", ptr(t), t.stride(0), ptr(src), src.stride(0), src.shape[0], src.shape[1], s)
        self._wt_gen = gen
        return self._wt

    def acts(self, B, T, save=True):
        key = (B, T, save)
        if key not in self._acts:
            self._acts = {k: v for k, v in self._acts.items() if k[2] != save}
            self._acts[key] = _Acts(self.cfg, B, T, self.device, self.act, save)
        return self._acts[key]

    # ------------------------------------------------------------- forward
    def forward(self, idx, meta, save=True, train=False, seed=None, cache=None):
        """save=False (inference): one layer's activation buffers are reused
        and nothing is kept for a backward pass. train=True (nn.Module.train()
        mode, save=True only) applies nn.Dropout(cfg.dropout) at the reference's
        three sites (model_transformer.py:51,80,101) with keep masks drawn from
        `seed` (default: one draw of torch's CPU generator per step).
        cache (a TransformerDecodeCache, save=False): the cached decode's
        prefill — every layer's keys / values, the logits rows and the tokens
        of the window are left in it."""
        cfg, P, W = self.cfg, self.P, self.W
        if not idx.is_cuda:
            raise RuntimeError("the MI355X engine runs on the GPU only (no CPU fallback)")
        self.refresh_shadow()
        B, T = idx.shape
        if T + N_META > cfg.s_max:
            raise ValueError(f"sequence of {T} tokens exceeds block_len {cfg.block_len}")
        A = self.acts(B, T, save)
        A.gen += 1
        d, H, hs, S = cfg.n_embd, cfg.n_heads, cfg.head_size, T + N_META
        scale = d ** -0.5  # C**-0.5 with C = n_embd (model_transformer.py:65,77)
        idx = idx.contiguous()
        meta = meta.contiguous()
        if save:
            self._idx, self._meta = idx, meta
        p = float(cfg.dropout) if (train and save) else 0.0
        if p > 0:
            if seed is None:
                seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
            A.drop = (int(seed) & 0xFFFFFFFF, p)
            masks = A.masks(cfg, self.device)
        else:
            A.drop = None
        # training: every layer's attention keep words drawn up front on a side
        # stream (store-bound; they overlap the MFMA-bound forward), layer l's
        # attention waits for its own event. The words of the previous step were
        # last read by its backward, which precedes this point on the main stream.
        # The same side stream then zero-fills the backward's accumulators (the
        # residual-stream gradient and the branch-gradient copy, plus the
        # buffers a train step lists in `side_zero`, e.g. its flat gradient),
        # which the end of the forward waits for.
        mask_ev = zero_ev = None
        A.bwd_zeroed = self.side_zeroed = False
        zero = getattr(self, "side_zero", None) if (train and save) else None
        if save and ((p > 0 and cfg.n_layer > 1) or zero):
            main = torch.cuda.current_stream(self.device)
            if getattr(self, "_mask_stream", None) is None:
                self._mask_stream = torch.cuda.Stream(self.device)
            side = self._mask_stream
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if p > 0 and cfg.n_layer > 1:
                    mask_ev = []
                    for l in range(cfg.n_layer):
                        ops.dropout_attn_mask(B, H, S, seed, DROP_ATTN + l * 65536, p, self.device, out=masks[l])
                        ev = torch.cuda.Event()
                        ev.record(side)
                        mask_ev.append(ev)
                if zero:
                    Bw = A.bwd(cfg, self.device, self.act)
                    for t in [Bw["gres"], Bw["gb"]] + list(zero):
                        if t is not None:
                            t.zero_()
                    zero_ev = torch.cuda.Event()
                    zero_ev.record(side)
        ops.embed_fwd(A.x[0].view(B, S, d), P["tok_emb"], P["meta_emb"], idx, meta)
        for l in range(cfg.n_layer):
            k = l if save else 0
            x, xo = (A.x[l], A.x[l + 1]) if save else (A.x[l % 2], A.x[(l + 1) % 2])
            ops.layernorm_fwd(x, P[f"{l}.ln1_w"], P[f"{l}.ln1_b"], out=A.a[k], mean=A.st1[k, 0], rstd=A.st1[k, 1])
            ops.gemm(A.a[k], W[f"{l}.wqkv"], out=A.qkv[k])
            if cache is not None:
                kv = A.qkv[k].view(B, S, 3, H, hs)
                cache.k[l][:, :, :S].copy_(kv[:, :, 1].transpose(1, 2))
                cache.v[l][:, :, :S].copy_(kv[:, :, 2].transpose(1, 2))
            adrop = pdrop = fdrop = None
            if p > 0:
                if mask_ev is not None:
                    torch.cuda.current_stream(self.device).wait_event(mask_ev[l])
                else:
                    ops.dropout_attn_mask(B, H, S, seed, DROP_ATTN + l * 65536, p, self.device, out=masks[k])
                adrop, pdrop, fdrop = (masks[k], p), (seed, DROP_PROJ + l, p), (seed, DROP_FFN + l, p)
            relattn_fwd(A.qkv[k], W[f"{l}.R"], B, S, H, hs, scale, out=A.o[k], lse=A.lse[k], drop=adrop)
            ops.gemm(A.o[k], W[f"{l}.wproj"], out=A.xm[k], epilogue=L.EPI_BIAS_RESID, bias=P[f"{l}.bproj"], aux=x,
                     drop=pdrop)
            ops.layernorm_fwd(A.xm[k], P[f"{l}.ln2_w"], P[f"{l}.ln2_b"], out=A.c[k], mean=A.st2[k, 0],
                              rstd=A.st2[k, 1])
            ops.gemm(A.c[k], W[f"{l}.w1"], out=A.h[k], epilogue=L.EPI_BIAS_RELU, bias=P[f"{l}.b1"],
                     aux=A.hm[k] if save and A.hm is not None else None)
            ops.gemm(A.h[k], W[f"{l}.w2"], out=xo, epilogue=L.EPI_BIAS_RESID, bias=P[f"{l}.b2"], aux=A.xm[k],
                     drop=fdrop)
        x_last = A.x[cfg.n_layer] if save else A.x[cfg.n_layer % 2]
        ops.layernorm_fwd(x_last, P["lnf_w"], P["lnf_b"], out=A.f, mean=A.stf[0], rstd=A.stf[1],
                          seg=(T, N_META))
        V = cfg.vocab_size
        # full V_pad rows (pad rows of lm_w / lm_b are zero): 16-B aligned rows, 256-tile eligible.
        # head_stats (the train step's streaming loss): the time-axis column
        # statistics of filtered_logit come out of the GEMM epilogue
        A.colpart_valid = False
        if self.head_stats and cache is None and T % 256 == 0:
            if A.colpart is None:
                A.colpart = torch.empty(B * T // 128, 2, cfg.v_pad, device=self.device, dtype=torch.float32)
            A.colpart_valid = ops.gemm_bias_colstats(A.f, W["lm_w"], A.logits, P["lm_b"], A.colpart)
        if not A.colpart_valid:
            ops.gemm(A.f, W["lm_w"], out=A.logits, epilogue=L.EPI_BIAS, bias=P["lm_b"])
        if zero_ev is not None:
            torch.cuda.current_stream(self.device).wait_event(zero_ev)
            A.bwd_zeroed = self.side_zeroed = True
        if cache is not None:
            if T > cache.ctx:
                raise ValueError(f"prefill of {T} tokens exceeds the cache context {cache.ctx}")
            cache.ring.fill_(float("-inf"))
            cache.part_valid = False
            cache.ring[:, :T].copy_(A.logits.view(B, T, cfg.v_pad))
            cache.tokens[:, :T].copy_(idx)
            cache.length = T
            cache.pos_dev.fill_(T)
        return A.logits.view(B, T, cfg.v_pad)[:, :, :V]

    def decode_cache(self, B, context=None):
        return TransformerDecodeCache(self.cfg, B, context or self.cfg.block_len, self.device, self.act)

    # decode steps after the first replay one captured HIP graph
    # (False: eager launches with host-side positions; tests / profiling)
    step_graphs = True

    @torch.no_grad()
    def step(self, tok, cache):
        """One cached decode position for every row: tok int64 [B] (the token
        at sequence position cache.length) -> its logits row [B, v_pad] (the
        last row of its window, keys / values of the window from the cache).
        Leaves cache.lse = the time-axis LSE of the window's OTHER rows (what
        msq_filtered_logit_step then extends by this row) and writes the row
        into the window's logits ring.

        The first step after the prefill (every ring block's partial LSE) runs
        eagerly; every later one has the same ~60 launches with the same
        arguments once the position comes from device memory
        (msq_relattn_decode_pos, msq_ring_step), so it is captured once and
        replayed as one HIP graph."""
        if not tok.is_cuda:
            raise RuntimeError("the MI355X engine runs on the GPU only (no CPU fallback)")
        self.refresh_shadow()
        if self.step_graphs and cache.part_valid and cache.length >= 1:
            # the graph reads the token from the cache's staging buffer, so a
            # caller handing a fresh tensor every step costs a device copy,
            # not a re-capture
            tb = cache.stage_tok(tok)
            if cache.graph is None or cache.graph_gen != self._wgen_now():
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._step_dev(tb, cache)
                cache.graph, cache.graph_gen = g, self._wgen_now()
            cache.graph.replay()
            cache.length += 1
            cache.logits = cache.row_buf
            return cache.row_buf
        row = self._step_host(tok, cache)
        cache.pos_dev.fill_(cache.length)
        return row

    def _wgen_now(self):
        return getattr(self, "_wgen", 0)

    def _layers_step(self, x, cache, attn):
        """the per-layer body of a decode step; attn(l) runs the decode attention"""
        cfg, P, W = self.cfg, self.P, self.W
        L_ = cfg.n_layer
        # every LayerNorm but layer 0's ln1 comes out of the residual product before it
        # (msq_gemm_resid_ln: the split-K reduce owns whole rows and normalises them)
        ops.layernorm_fwd(x, P["0.ln1_w"], P["0.ln1_b"], out=cache.a, mean=cache.st[0], rstd=cache.st[1])
        for l in range(L_):
            ops.gemm(cache.a, W[f"{l}.wqkv"], out=cache.qkv)
            attn(l)
            ops.gemm_resid_ln(cache.o, W[f"{l}.wproj"], cache.xm, P[f"{l}.bproj"], x, P[f"{l}.ln2_w"],
                              P[f"{l}.ln2_b"], cache.c)
            ops.gemm(cache.c, W[f"{l}.w1"], out=cache.h, epilogue=L.EPI_BIAS_RELU, bias=P[f"{l}.b1"])
            nxt = (P[f"{l + 1}.ln1_w"], P[f"{l + 1}.ln1_b"], cache.a) if l + 1 < L_ else (P["lnf_w"], P["lnf_b"], cache.f)
            ops.gemm_resid_ln(cache.h, W[f"{l}.w2"], x, P[f"{l}.b2"], cache.xm, *nxt)

    def _step_dev(self, tok, cache):
        """step() with every position-dependent quantity read from cache.pos_dev"""
        cfg, P, W = self.cfg, self.P, self.W
        B, d, H, hs = cache.B, cfg.n_embd, cfg.n_heads, cfg.head_size
        s = stream()
        scale = d ** -0.5
        call("msq_embed_fwd", ptr(cache.x), ptr(P["tok_emb"]), ptr(P["meta_emb"]), ptr(tok), None, B, 1, 0, d, s)

        def attn(l):
            call("msq_relattn_decode_pos", dt(cache.qkv), ptr(cache.o), cache.o.stride(0), ptr(cache.qkv),
                 cache.qkv.stride(0), ptr(cache.k[l]), ptr(cache.v[l]), ptr(W[f"{l}.R"]), cfg.s_max, B, H, hs,
                 cache.S_ring, N_META, ptr(cache.pos_dev), float(scale), ptr(cache.attn_ws), cache.attn_ws.numel(), s)
        self._layers_step(cache.x, cache, attn)
        ops.gemm(cache.f, W["lm_w"], out=cache.row_buf, epilogue=L.EPI_BIAS, bias=P["lm_b"])
        self._ring_step(tok, cache)

    def _ring_step(self, tok, cache):
        """the new row into the logits ring, cache.lse over the window's other rows, pos_dev += 1"""
        cfg = self.cfg
        call("msq_ring_step", ptr(cache.lse), ptr(cache.part), ptr(cache.ring_state), ptr(cache.ring), dt(cache.ring),
             cfg.v_pad, cache.B, cache.ctx, cfg.vocab_size, cache.RB, ptr(cache.row_buf), cache.row_buf.stride(0),
             ptr(cache.tokens), ptr(tok), ptr(cache.pos_dev), stream())

    def _step_host(self, tok, cache):
        cfg, P, W = self.cfg, self.P, self.W
        B, d, H, hs = cache.B, cfg.n_embd, cfg.n_heads, cfg.head_size
        ctx, pos = cache.ctx, cache.length
        n_tok = min(pos + 1, ctx)
        first = pos + 1 - n_tok
        slot = pos % ctx
        s = stream()
        scale = d ** -0.5
        tok = tok.contiguous()
        call("msq_embed_fwd", ptr(cache.x), ptr(P["tok_emb"]), ptr(P["meta_emb"]), ptr(tok), None, B, 1, 0, d, s)

        def attn(l):
            call("msq_relattn_decode", dt(cache.qkv), ptr(cache.o), cache.o.stride(0), ptr(cache.qkv),
                 cache.qkv.stride(0), ptr(cache.k[l]), ptr(cache.v[l]), ptr(W[f"{l}.R"]), cfg.s_max, B, H, hs,
                 cache.S_ring, N_META, n_tok, N_META + slot, first % ctx, float(scale), ptr(cache.attn_ws),
                 cache.attn_ws.numel(), s)
        self._layers_step(cache.x, cache, attn)
        ops.gemm(cache.f, W["lm_w"], out=cache.row_buf, epilogue=L.EPI_BIAS, bias=P["lm_b"])
        if not cache.part_valid:  # first step: every block partial of the prefilled window
            call("msq_ring_lse", ptr(cache.lse), ptr(cache.part), ptr(cache.ring), dt(cache.ring), cfg.v_pad, B, ctx,
                 cfg.vocab_size, cache.RB, 0, cache.nblk, slot, -1, s)
            cache.ring_blk.fill_(-1)
            cache.part_valid = True
        cache.pos_dev.fill_(pos)
        self._ring_step(tok, cache)
        cache.length = pos + 1
        cache.logits = cache.row_buf
        return cache.row_buf

    # ------------------------------------------------------------ backward
    def backward(self, dlogits, grads, head_bias_done=False):
        """dlogits: [B*T, ld] (act dtype) whose first V columns are dL/dlogits;
        grads: flat fp32 buffer (accumulated). head_bias_done: the lm_head
        bias gradient was already accumulated (msq_filtered_ce_bias)."""
        cfg, P, W = self.cfg, self.P, self.W
        G = self.layout.views(grads)
        idx, meta = self._idx, self._meta
        B, T = idx.shape
        A = self.acts(B, T)
        Bw = A.bwd(cfg, self.device, self.act)
        d, H, hs, S, M, V = cfg.n_embd, cfg.n_heads, cfg.head_size, T + N_META, A.M, cfg.vocab_size
        scale = d ** -0.5
        dl = dlogits[:, :V]
        seed, p = A.drop if A.drop is not None else (0, 0.0)
        dsite = (lambda site: (seed, site, p)) if p > 0 else (lambda site: None)  # noqa: E731
        hook = getattr(self, "layer_grad_ready", None)
        # Weight gradients (dW GEMMs, and the bias column sums when they read a
        # bf16 branch gradient) only feed the optimizer, not the next layer's
        # backward: with overlap_dw (the default since round 3: 87.9 -> 86.8 ms
        # per step, same box; overlap_dw = False keeps one
        # stream) they run on a second stream, overlapped
        # with the dX / LayerNorm / attention chain of the main stream. Each
        # side launch waits for the main stream's producer of its inputs; the
        # main stream waits for the side stream before it overwrites a buffer
        # the side still reads (gb / gb2 / dh / dqkv, one layer of slack).
        ov = Bw["gb2"] is not None and getattr(self, "overlap_dw", False)
        sd = ops.SideStream(self.device, ov, hook)
        on_side, before_write, layer_done = sd.run, sd.before_write, sd.layer_done

        # lm_head (model_transformer.py:147,161)
        def lm_w():
            ops.gemm(dlogits, A.f, ta=True, tb=True, out=G["lm_w"], epilogue=L.EPI_ACCUM)  # pad columns are 0
            if not head_bias_done:
                ops.colsum(dl, G["lm_b"][:V], accumulate=True)
        on_side("dlogits", lm_w)
        Wt = self.transposed_weights()
        dx_gemm(dlogits, W, Wt, "lm_w", Bw["df"])
        gres = Bw["gres"]
        gb = Bw["gb"] if Bw["gb"] is not None else gres
        gb2 = Bw["gb2"] if ov else gb
        if not A.bwd_zeroed:  # else zero-filled on the forward's side stream
            gres.zero_()
            if Bw["gb"] is not None:
                gb.zero_()
        A.bwd_zeroed = False
        # dropout: gb is the gradient INTO the dropped branch (gres masked by the
        # keep mask of the site whose output was added to the residual there);
        # the bias gradients then sum gb instead of gres
        # the proj / FFN output bias gradients (column sums of the gradient into
        # each residual branch) are fused into the LayerNorm backward that
        # writes those rows (dbias): lnf / ln1 of layer l+1 -> b2 of layer l,
        # ln2 of layer l -> bproj of layer l
        ops.layernorm_bwd(gres, Bw["df"], A.x[cfg.n_layer], A.stf[0], A.stf[1], P["lnf_w"], G["lnf_w"], G["lnf_b"],
                          dx_copy=Bw["gb"], seg=(T, N_META), drop=dsite(DROP_FFN + cfg.n_layer - 1),
                          dbias=G[f"{cfg.n_layer - 1}.b2"], ordered=True)
        layer_done("head")
        for l in reversed(range(cfg.n_layer)):
            # FFN (model_transformer.py:92-105,120)
            def ffn2_w(l=l):
                ops.gemm(gb, A.h[l], ta=True, tb=True, out=G[f"{l}.w2"], epilogue=L.EPI_ACCUM)
            on_side("gb", ffn2_w)
            before_write("dh")
            # dh = ReLU-masked FFN2 dX; the FFN1 bias gradient (its column sums) in the same epilogue
            hmask = A.hm[l] if A.hm is not None else A.h[l]
            if Wt is not None:
                ops.gemm_colsum(gb, Wt[f"{l}.w2"], Bw["dh"], G[f"{l}.b1"], epilogue=L.EPI_RELU_MASK, aux=hmask,
                                accumulate=True)
            else:
                ops.gemm_colsum(gb, W[f"{l}.w2"], Bw["dh"], G[f"{l}.b1"], tb=True, epilogue=L.EPI_RELU_MASK,
                                aux=hmask, accumulate=True)

            def ffn1_w(l=l):
                ops.gemm(Bw["dh"], A.c[l], ta=True, tb=True, out=G[f"{l}.w1"], epilogue=L.EPI_ACCUM)
            on_side("dh", ffn1_w)
            dx_gemm(Bw["dh"], W, Wt, f"{l}.w1", Bw["dtmp"])
            before_write("gb2")
            ops.layernorm_bwd(gres, Bw["dtmp"], A.xm[l], A.st2[l, 0], A.st2[l, 1], P[f"{l}.ln2_w"], G[f"{l}.ln2_w"],
                              G[f"{l}.ln2_b"], dx_copy=gb2 if Bw["gb"] is not None else None,
                              drop=dsite(DROP_PROJ + l), dbias=G[f"{l}.bproj"])
            # attention (model_transformer.py:41-90,119)

            def proj_w(l=l):
                ops.gemm(gb2, A.o[l], ta=True, tb=True, out=G[f"{l}.wproj"], epilogue=L.EPI_ACCUM)
            on_side("gb2", proj_w)
            dx_gemm(gb2, W, Wt, f"{l}.wproj", Bw["dtmp"])
            before_write("dqkv")
            relattn_bwd(Bw["dtmp"], A.o[l], A.lse[l], A.qkv[l], W[f"{l}.R"], B, S, H, hs, scale, dqkv=Bw["dqkv"],
                        dR=G[f"{l}.R"], drop=(A._masks[l], p) if p > 0 else None)

            def qkv_w(l=l):
                ops.gemm(Bw["dqkv"], A.a[l], ta=True, tb=True, out=G[f"{l}.wqkv"], epilogue=L.EPI_ACCUM)
            on_side("dqkv", qkv_w)
            dx_gemm(Bw["dqkv"], W, Wt, f"{l}.wqkv", Bw["dtmp"])
            before_write("gb")
            ops.layernorm_bwd(gres, Bw["dtmp"], A.x[l], A.st1[l, 0], A.st1[l, 1], P[f"{l}.ln1_w"], G[f"{l}.ln1_w"],
                              G[f"{l}.ln1_b"], dx_copy=Bw["gb"], drop=dsite(DROP_FFN + l - 1) if l > 0 else None,
                              dbias=G[f"{l - 1}.b2"] if l > 0 else None)
            layer_done(l)
        ops.embed_bwd(G["tok_emb"], G["meta_emb"], gres, idx, meta)
        layer_done(-1)
        sd.finish()

    def bucket_ranges(self):
        from .ddp import transformer_buckets
        return transformer_buckets(self.layout)

    def dlogits_buffer(self, B, T):
        A = self.acts(B, T)
        return A.bwd(self.cfg, self.device, self.act)["dlogits"]


class _TransformerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, idx, meta, engine, train):
        logits = engine.forward(idx, meta, train=train)
        A = engine.acts(*idx.shape)
        ctx.engine, ctx.gen, ctx.shape = engine, A.gen, tuple(idx.shape)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        eng = ctx.engine
        A = eng.acts(*ctx.shape)
        if A.gen != ctx.gen:
            raise RuntimeError("activations were overwritten by a later forward; call backward before the next forward")
        B, T = ctx.shape
        cfg = eng.cfg
        # copy into the engine's zero-padded buffer: the lm_head GEMMs run over
        # all V_pad columns and rely on the pad columns being zero
        buf = eng.dlogits_buffer(B, T)
        buf.view(B, T, cfg.v_pad)[:, :, :cfg.vocab_size].copy_(dlogits)
        dl2 = buf
        grads = torch.zeros_like(eng.flat.data)
        eng.backward(dl2, grads)
        return grads, None, None, None, None


class Transformer(nn.Module):
    """Transformer(params) drop-in (model_transformer.py:136-168).

    forward(idx [B,T] int64, metadata_idx [B,6] int64) -> logits [B,T,V] (fp32
    in the exact mode, bf16 in the bf16 mode; a view into a padded buffer)."""

    def __init__(self, params, device=None, precision=None):
        super().__init__()
        cfg = params if isinstance(params, TransformerConfig) else TransformerConfig.from_params(params)
        if precision is not None:
            cfg.precision = precision
        self.cfg = cfg
        self.vocab_size = cfg.vocab_size
        self.metadata_vocab_size = cfg.metadata_vocab_size
        layout = ParamLayout(cfg)
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.flat = nn.Parameter(torch.zeros(layout.numel, device=dev))
        self._engine = None
        self.reset_parameters()

    # -- parameters --------------------------------------------------------
    def reset_parameters(self, seed=0):
        """PyTorch-default-like init (nn.Linear / nn.Embedding / randn rel_pos_emb)."""
        g = torch.Generator().manual_seed(seed)
        V = self.layout.views(self.flat.data)
        with torch.no_grad():
            for name, (_, shape) in self.layout.offsets.items():
                t = V[name]
                leaf = name.split(".")[-1]
                if leaf in ("ln1_w", "ln2_w", "lnf_w"):
                    t.fill_(1.0)
                elif leaf in ("ln1_b", "ln2_b", "lnf_b"):
                    t.zero_()
                elif name in ("tok_emb", "meta_emb") or leaf == "R":
                    t.copy_(torch.randn(shape, generator=g))
                elif leaf in ("wqkv", "wproj", "w1", "w2", "lm_w"):
                    bound = 1.0 / math.sqrt(shape[1])
                    t.copy_(torch.empty(shape).uniform_(-bound, bound, generator=g))
                else:  # biases
                    fan_in = self.cfg.n_embd if leaf != "b2" else 4 * self.cfg.n_embd
                    bound = 1.0 / math.sqrt(fan_in)
                    t.copy_(torch.empty(shape).uniform_(-bound, bound, generator=g))
            if self.cfg.v_pad > self.cfg.vocab_size:
                V["lm_w"][self.cfg.vocab_size:].zero_()
                V["lm_b"][self.cfg.vocab_size:].zero_()
        self._engine = None

    @property
    def layout(self):
        return ParamLayout(self.cfg)

    @property
    def engine(self):
        if self._engine is None or self._engine.flat is not self.flat or self._engine.device != self.flat.device:
            self._engine = TransformerEngine(self.cfg, self.flat)
        return self._engine

    def _apply(self, fn, *a, **k):
        out = super()._apply(fn, *a, **k)
        self._engine = None
        return out

    def forward(self, idx, metadata_idx, targets=None):
        if not (torch.is_grad_enabled() and self.flat.requires_grad):
            return self.engine.forward(idx, metadata_idx, save=False)
        return _TransformerFn.apply(self.flat, idx, metadata_idx, self.engine, self.training)

    def get_name(self):
        return "Transformer"

    # -- reference-compatible state_dict ------------------------------------
    def state_dict(self, *args, destination=None, prefix="", keep_vars=False, with_tril=True):
        V = self.layout.views(self.flat if keep_vars else self.flat.detach())
        out = OrderedDict() if destination is None else destination
        tril = None
        for key, (name, sel) in reference_keys(self.cfg).items():
            if name == "__tril__":
                if not with_tril:
                    continue
                if tril is None:
                    tril = tril_mask(self.cfg.s_max, self.flat.device)
                out[prefix + key] = tril
                continue
            out[prefix + key] = _select(V[name], sel)
        return out

    def load_state_dict(self, state_dict, strict=True, assign=False):
        V = self.layout.views(self.flat.data)
        keys = reference_keys(self.cfg)
        missing = [k for k, (n, _) in keys.items() if n != "__tril__" and k not in state_dict]
        unexpected = [k for k in state_dict if k not in keys]
        if strict and (missing or unexpected):
            raise RuntimeError(f"state_dict mismatch: missing {missing[:5]}, unexpected {unexpected[:5]}")
        with torch.no_grad():
            for k, (name, sel) in keys.items():
                if name == "__tril__" or k not in state_dict:
                    continue
                dst = _select(V[name], sel)
                src = state_dict[k]
                if tuple(src.shape) != tuple(dst.shape):
                    raise RuntimeError(f"{k}: shape {tuple(src.shape)} != {tuple(dst.shape)}")
                dst.copy_(src)
        if self._engine is not None:
            self._engine.refresh_shadow(force=True)
        return torch.nn.modules.module._IncompatibleKeys(missing, unexpected)

    def grad_dict(self):
        """Reference-named views of flat.grad (for parity checks)."""
        V = self.layout.views(self.flat.grad)
        return OrderedDict((k, _select(V[n], s)) for k, (n, s) in reference_keys(self.cfg).items() if n != "__tril__")
