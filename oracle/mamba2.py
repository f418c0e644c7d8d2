"""CPU oracle (test infra): the reference Mamba model (models/mamba/mamba.py:
8-35) with its ``mamba_ssm.Mamba2`` mixers (not vendored; version unknown)
restated from the published Mamba2 algorithm, defaults d_state=64, d_conv=4,
expand=2, headdim=64, ngroups=1, no bias, conv bias, rmsnorm gate with
norm_before_gate=False (eps 1e-5), dt = softplus(dt + dt_bias), A = -exp(A_log),
per-head D skip. The SSD is written as its defining sequential recurrence
    h_t = exp(dt_t A) h_{t-1} + dt_t x_t B_t^T,  y_t = h_t C_t + D x_t.
Parity of this restatement is pinned against HF transformers 5.15.0's
pure-torch Mamba2 mixer wrapped as mamba_ssm.Mamba2 under the reference's own
mamba.py (tests/golden/make_golden.py, G5); parity against mamba_ssm's Triton
kernels themselves is UNPINNED (dependency absent)."""
import torch
import torch.nn.functional as F

D_STATE, D_CONV, EXPAND, HEADDIM = 64, 4, 2, 64
META = 6


def dims(d_model):
    d_inner = EXPAND * d_model
    nheads = d_inner // HEADDIM
    conv_dim = d_inner + 2 * D_STATE
    return d_inner, nheads, conv_dim, 2 * d_inner + 2 * D_STATE + nheads


def mixer(p, pre, u, chunked=False):
    """One Mamba2 mixer. u [B, L, d_model] -> [B, L, d_model]."""
    Bsz, L, d_model = u.shape
    d_inner, H, conv_dim, _ = dims(d_model)
    zxbcdt = u @ p[pre + "in_proj.weight"].t()
    z, xBC, dt = torch.split(zxbcdt, [d_inner, conv_dim, H], dim=-1)
    w = p[pre + "conv1d.weight"]  # [conv_dim, 1, d_conv]
    xBC = F.conv1d(xBC.transpose(1, 2), w, p[pre + "conv1d.bias"], padding=D_CONV - 1, groups=conv_dim)[..., :L]
    xBC = F.silu(xBC.transpose(1, 2))
    x, Bm, Cm = torch.split(xBC, [d_inner, D_STATE, D_STATE], dim=-1)
    dt = F.softplus(dt + p[pre + "dt_bias"])             # [B, L, H]
    A = -torch.exp(p[pre + "A_log"])                      # [H]
    x = x.reshape(Bsz, L, H, HEADDIM)
    if chunked:
        y = ssd_chunked(x, dt, A, Bm, Cm) + p[pre + "D"][None, None, :, None] * x
    else:
        h = torch.zeros(Bsz, H, HEADDIM, D_STATE, dtype=u.dtype)
        ys = []
        for t in range(L):
            dA = torch.exp(dt[:, t] * A)                      # [B, H]
            h = h * dA[:, :, None, None] + (dt[:, t, :, None] * x[:, t])[..., None] * Bm[:, t, None, None, :]
            ys.append(torch.einsum("bhpn,bn->bhp", h, Cm[:, t]))
        y = torch.stack(ys, dim=1) + p[pre + "D"][None, None, :, None] * x
    y = y.reshape(Bsz, L, d_inner)
    g = y * F.silu(z)
    g = g * torch.rsqrt(g.pow(2).mean(-1, keepdim=True) + 1e-5) * p[pre + "norm.weight"]
    return g @ p[pre + "out_proj.weight"].t()


def ssd_chunked(x, dt, A, Bm, Cm, Q=256):
    """The same recurrence evaluated in chunks of Q positions (the SSD
    "chunked scan" form of the Mamba2 paper: within a chunk y = (C B^T o decay)
    (dt x), across chunks the state h carried by the recurrence at chunk
    granularity). Equal to the sequential loop up to fp32 summation order; used
    for long sequences, where autograd through 4 k single steps is slow.
    x [B,L,H,P], dt [B,L,H], A [H], Bm/Cm [B,L,N] -> y [B,L,H,P] (no D skip)."""
    Bsz, L, H, P = x.shape
    N = Bm.shape[-1]
    nc = -(-L // Q)
    pad = nc * Q - L
    if pad:  # zero tail: dt = 0 adds nothing and decays nothing
        x, dt = F.pad(x, (0, 0, 0, 0, 0, pad)), F.pad(dt, (0, 0, 0, pad))
        Bm, Cm = F.pad(Bm, (0, 0, 0, pad)), F.pad(Cm, (0, 0, 0, pad))
    x, dt = x.view(Bsz, nc, Q, H, P), dt.view(Bsz, nc, Q, H)
    Bm, Cm = Bm.view(Bsz, nc, Q, N), Cm.view(Bsz, nc, Q, N)
    acum = torch.cumsum(dt * A, dim=2)                                  # [B,c,Q,H]
    u = dt[..., None] * x                                               # [B,c,Q,H,P]
    seg = acum.transpose(2, 3)[..., :, None] - acum.transpose(2, 3)[..., None, :]  # [B,c,H,t,s]
    causal = torch.ones(Q, Q, dtype=torch.bool).tril()
    decay = torch.exp(seg.masked_fill(~causal, float("-inf")))
    cb = torch.einsum("bctn,bcsn->bcts", Cm, Bm)                        # [B,c,t,s]
    y = torch.einsum("bchts,bcshp->bcthp", cb[:, :, None] * decay, u)   # intra-chunk
    last = acum[:, :, -1:, :]                                           # [B,c,1,H]
    st = torch.einsum("bcsn,bcsh,bcshp->bchpn", Bm, torch.exp(last - acum), u)  # chunk-local end states
    h = torch.zeros(Bsz, H, P, N, dtype=x.dtype)
    prev = []
    for c in range(nc):
        prev.append(h)
        h = h * torch.exp(last[:, c, 0])[:, :, None, None] + st[:, c]
    hp = torch.stack(prev, dim=1)                                       # [B,c,H,P,N] state entering chunk c
    y = y + torch.einsum("bctn,bcth,bchpn->bcthp", Cm, torch.exp(acum), hp)
    return y.reshape(Bsz, nc * Q, H, P)[:, :L]


def forward(p, tokens, meta, n_layers, chunked=False):
    """Mamba.forward (mamba.py:27-35): NO residual, no per-layer norm."""
    x = torch.cat([p["metadata_embedding.weight"][meta], p["token_embedding.weight"][tokens]], dim=1)
    for i in range(n_layers):
        x = mixer(p, f"layers.{i}.", x, chunked)
    x = F.layer_norm(x, (x.shape[-1],), p["norm.weight"], p["norm.bias"], 1e-5)
    return (x @ p["output_layer.weight"].t() + p["output_layer.bias"])[:, META:]


def param_shapes(d_model, n_layers, vocab, meta_vocab):
    d_inner, H, conv_dim, d_in_proj = dims(d_model)
    s = {"token_embedding.weight": (vocab, d_model), "metadata_embedding.weight": (meta_vocab, d_model),
         "output_layer.weight": (vocab, d_model), "output_layer.bias": (vocab,)}
    for i in range(n_layers):
        pre = f"layers.{i}."
        s.update({pre + "dt_bias": (H,), pre + "A_log": (H,), pre + "D": (H,),
                  pre + "in_proj.weight": (d_in_proj, d_model), pre + "conv1d.weight": (conv_dim, 1, D_CONV),
                  pre + "conv1d.bias": (conv_dim,), pre + "norm.weight": (d_inner,),
                  pre + "out_proj.weight": (d_model, d_inner)})
    s["norm.weight"] = (d_model,)
    s["norm.bias"] = (d_model,)
    return s


def filled_params(shapes):
    from .fill import fill_param
    return {k: torch.from_numpy(fill_param(k, sh)) for k, sh in shapes.items()}
