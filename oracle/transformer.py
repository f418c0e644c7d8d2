"""CPU oracle (test infra): functional fp32 restatement of the reference
relative-position Transformer (models/transformer/model_transformer.py:8-165).

Parameters are a dict keyed by the reference's state_dict names; autograd
provides the backward. The golden fixtures are recorded with dropout 0
(``cc.config.values.dropout = params.dropout = 0``); ``forward(..., drop=(seed,
p))`` applies nn.Dropout(p) at the reference's three sites (attention
probabilities :80, proj output :51, FFN output :101) with the keep masks of
oracle/dropout.py (the build's counter-based stream), so the build's training
mode can be checked element for element.
"""
import math

import torch
import torch.nn.functional as F

META = 6  # metadata prefix length, hard-coded in generate_matrix (model_transformer.py:14)


def allowed_mask(S: int) -> torch.Tensor:
    """generate_matrix(n, 1) (model_transformer.py:8-16): row i sees j<=i and j<6."""
    i = torch.arange(S)[:, None]
    j = torch.arange(S)[None, :]
    return (j <= i) | (j < META)


def skew_index(S: int):
    """Index form of HeadRelPos._rel_shift (model_transformer.py:84-90).

    The reference pads a zero column in front of QR[S,S], re-views the
    [S, S+1] buffer as [S+1, S] and drops the first row. Element (i, j) of the
    result is therefore flat element f = (i+1)*S + j of the padded buffer:
    row f // (S+1), padded column f % (S+1) (column 0 is the zero pad).
    Returns (row, col, is_pad) index tensors into QR.
    """
    i = torch.arange(S)[:, None]
    j = torch.arange(S)[None, :]
    f = (i + 1) * S + j
    row = f // (S + 1)
    pc = f % (S + 1)
    return row, (pc - 1).clamp(min=0), pc == 0


def rel_head(x, wq, wk, wv, R, scale, keep=None, keep_scale=1.0):
    """One HeadRelPos (model_transformer.py:64-82): scores (q.k + skew(q.R)) * scale."""
    return rel_attention(x @ wq.t(), x @ wk.t(), x @ wv.t(), R, scale, keep, keep_scale)


def rel_attention(q, k, v, R, scale, keep=None, keep_scale=1.0):
    """Attention core of HeadRelPos given q, k, v [B,S,hs] and R [>=S, hs]."""
    S = q.shape[1]
    ac = q @ k.transpose(1, 2)
    qr = q @ R[:S].t()                       # qr[b, i, r] = q_i . R[r]
    row, col, pad = skew_index(S)
    bd = qr[:, row, col].masked_fill(pad, 0.0)
    s = (ac + bd) * scale
    s = s.masked_fill(~allowed_mask(S), float("-inf"))
    w = torch.softmax(s, dim=-1)
    if keep is not None:  # self.dropout(attn) (model_transformer.py:80)
        w = w * keep * keep_scale
    return w @ v


def forward(p: dict, idx: torch.Tensor, meta: torch.Tensor, n_layer: int, n_heads: int, drop=None) -> torch.Tensor:
    """Transformer.forward (model_transformer.py:149-165): meta rows first,
    pre-LN blocks, LN_f, lm_head, keep the last T rows. drop=(seed, p): train
    mode with nn.Dropout(p) (masks from oracle/dropout.py)."""
    from . import dropout as odrop
    B, T = idx.shape
    x = torch.cat([p["metadata_embedding_table.weight"][meta], p["token_embedding_table.weight"][idx]], dim=1)
    C = x.shape[-1]
    scale = C ** -0.5                         # n_embd^-1/2, not head_size (model_transformer.py:65,77)
    S = x.shape[1]
    if drop is not None:
        seed, pd = drop
        ks = odrop.scale(pd)

        def site(y, s):  # nn.Dropout on a [B, S, C] branch output; rows = flat b*S + i
            k = torch.from_numpy(odrop.keep(seed, s, B * S, y.shape[-1], pd)).view(B, S, -1)
            return y * k * ks
    for l in range(n_layer):
        pre = f"blocks.{l}."
        h = F.layer_norm(x, (C,), p[pre + "ln1.weight"], p[pre + "ln1.bias"], 1e-5)
        keep = torch.from_numpy(odrop.attn_keep(drop[0], l, B, n_heads, S, drop[1])) if drop is not None else None
        heads = []
        for hh in range(n_heads):
            hp = f"{pre}sa.heads.{hh}."
            heads.append(rel_head(h, p[hp + "query.weight"], p[hp + "key.weight"], p[hp + "value.weight"],
                                  p[hp + "rel_pos_emb"], scale, keep[:, hh] if keep is not None else None,
                                  odrop.scale(drop[1]) if drop is not None else 1.0))
        att = torch.cat(heads, dim=-1)
        y = F.linear(att, p[pre + "sa.proj.weight"], p[pre + "sa.proj.bias"])
        x = x + (site(y, odrop.PROJ + l) if drop is not None else y)
        h = F.layer_norm(x, (C,), p[pre + "ln2.weight"], p[pre + "ln2.bias"], 1e-5)
        h = torch.relu(F.linear(h, p[pre + "ffwd.net.0.weight"], p[pre + "ffwd.net.0.bias"]))
        y = F.linear(h, p[pre + "ffwd.net.2.weight"], p[pre + "ffwd.net.2.bias"])
        x = x + (site(y, odrop.FFN + l) if drop is not None else y)
    x = F.layer_norm(x, (C,), p["ln_f.weight"], p["ln_f.bias"], 1e-5)
    return F.linear(x, p["lm_head.weight"], p["lm_head.bias"])[:, -T:, :]


def param_shapes(n_embd, n_heads, n_layer, block_len, vocab, meta_vocab):
    """Reference state_dict keys (minus the ``tril`` buffers) and shapes."""
    hs = n_embd // n_heads
    S_max = block_len + META
    shapes = {"token_embedding_table.weight": (vocab, n_embd),
              "metadata_embedding_table.weight": (meta_vocab, n_embd)}
    for l in range(n_layer):
        pre = f"blocks.{l}."
        for h in range(n_heads):
            hp = f"{pre}sa.heads.{h}."
            shapes[hp + "rel_pos_emb"] = (S_max, hs)
            shapes[hp + "key.weight"] = (hs, n_embd)
            shapes[hp + "query.weight"] = (hs, n_embd)
            shapes[hp + "value.weight"] = (hs, n_embd)
        shapes[pre + "sa.proj.weight"] = (n_embd, n_embd)
        shapes[pre + "sa.proj.bias"] = (n_embd,)
        shapes[pre + "ffwd.net.0.weight"] = (4 * n_embd, n_embd)
        shapes[pre + "ffwd.net.0.bias"] = (4 * n_embd,)
        shapes[pre + "ffwd.net.2.weight"] = (n_embd, 4 * n_embd)
        shapes[pre + "ffwd.net.2.bias"] = (n_embd,)
        for ln in ("ln1", "ln2"):
            shapes[f"{pre}{ln}.weight"] = (n_embd,)
            shapes[f"{pre}{ln}.bias"] = (n_embd,)
    shapes["ln_f.weight"] = (n_embd,)
    shapes["ln_f.bias"] = (n_embd,)
    shapes["lm_head.weight"] = (vocab, n_embd)
    shapes["lm_head.bias"] = (vocab,)
    return shapes


def filled_params(shapes: dict) -> dict:
    from .fill import fill_param
    return {k: torch.from_numpy(fill_param(k, s)) for k, s in shapes.items()}


def n_flops_fwd_per_seq(n_embd, n_layer, S, V):
    """Algorithmic forward FLOPs per sequence (SURVEY.md §8(d) cfg 2)."""
    d = n_embd
    return n_layer * (24 * S * d * d + 3 * d * S * (S + 1)) + 2 * (S - META) * d * V


__all__ = ["forward", "param_shapes", "filled_params", "allowed_mask", "skew_index", "math"]


class CachedTransformer:
    """TEST INFRASTRUCTURE: the semantics of the build's cached Transformer
    decode (generate(mode="cached")), an APPROXIMATION of scripts/generate.py's
    full forward per token that the reference itself does not have:

    * the prompt window is prefilled by the exact forward (model_transformer.py
      :149-165); its per-layer keys / values and logits rows are kept;
    * every later token is computed ONCE, as the last row of its own window:
      for the last row i = S-1 the skew term q_i . R[S-1-i+j] is q . R[j]
      (j = the key's position in the window, metadata 0..5 first) and the row
      sees every key; its keys / values / logits row are then reused;
    * the window holds at most ``context`` tokens: the oldest token's keys /
      values / logits row leave it (metadata stays).

    Called like a model on the sampler's growing window (oracle/sampler.py
    generate): returns the cached logits rows of the window, so
    filtered_logit(window, rows)[:, -1] is the cached z."""

    def __init__(self, p, n_layer, n_heads, context):
        self.p, self.L, self.H, self.ctx = p, n_layer, n_heads, context
        self.kv = None

    def _prefill(self, idx, meta):
        p, H = self.p, self.H
        B, T = idx.shape
        x = torch.cat([p["metadata_embedding_table.weight"][meta], p["token_embedding_table.weight"][idx]], dim=1)
        C = x.shape[-1]
        scale = C ** -0.5
        self.kv = []
        for l in range(self.L):
            pre = f"blocks.{l}."
            h = F.layer_norm(x, (C,), p[pre + "ln1.weight"], p[pre + "ln1.bias"], 1e-5)
            heads, ks, vs = [], [], []
            for hh in range(H):
                hp = f"{pre}sa.heads.{hh}."
                q, k, v = h @ p[hp + "query.weight"].t(), h @ p[hp + "key.weight"].t(), h @ p[hp + "value.weight"].t()
                ks.append(k)
                vs.append(v)
                heads.append(rel_attention(q, k, v, p[hp + "rel_pos_emb"], scale))
            self.kv.append((torch.stack(ks, 1), torch.stack(vs, 1)))  # [B, H, S, hs]
            x = x + F.linear(torch.cat(heads, -1), p[pre + "sa.proj.weight"], p[pre + "sa.proj.bias"])
            h = F.layer_norm(x, (C,), p[pre + "ln2.weight"], p[pre + "ln2.bias"], 1e-5)
            h = torch.relu(F.linear(h, p[pre + "ffwd.net.0.weight"], p[pre + "ffwd.net.0.bias"]))
            x = x + F.linear(h, p[pre + "ffwd.net.2.weight"], p[pre + "ffwd.net.2.bias"])
        x = F.layer_norm(x, (C,), p["ln_f.weight"], p["ln_f.bias"], 1e-5)
        self.rows = F.linear(x, p["lm_head.weight"], p["lm_head.bias"])[:, -T:, :]
        self.meta = meta

    def _step(self, tok):
        p, H = self.p, self.H
        x = p["token_embedding_table.weight"][tok]  # [B, C]
        C = x.shape[-1]
        scale = C ** -0.5
        for l in range(self.L):
            pre = f"blocks.{l}."
            h = F.layer_norm(x, (C,), p[pre + "ln1.weight"], p[pre + "ln1.bias"], 1e-5)
            K, Vv = self.kv[l]
            nk, nv, heads = [], [], []
            for hh in range(H):
                hp = f"{pre}sa.heads.{hh}."
                q, k, v = h @ p[hp + "query.weight"].t(), h @ p[hp + "key.weight"].t(), h @ p[hp + "value.weight"].t()
                Kh = torch.cat([K[:, hh], k[:, None]], 1)      # [B, S, hs], window order
                Vh = torch.cat([Vv[:, hh], v[:, None]], 1)
                S = Kh.shape[1]
                s = (torch.einsum("bd,bjd->bj", q, Kh) + q @ p[hp + "rel_pos_emb"][:S].t()) * scale
                heads.append(torch.einsum("bj,bjd->bd", torch.softmax(s, -1), Vh))
                nk.append(k)
                nv.append(v)
            self.kv[l] = (torch.cat([K, torch.stack(nk, 1)[:, :, None]], 2), torch.cat([Vv, torch.stack(nv, 1)[:, :, None]], 2))
            x = x + F.linear(torch.cat(heads, -1), p[pre + "sa.proj.weight"], p[pre + "sa.proj.bias"])
            h = F.layer_norm(x, (C,), p[pre + "ln2.weight"], p[pre + "ln2.bias"], 1e-5)
            h = torch.relu(F.linear(h, p[pre + "ffwd.net.0.weight"], p[pre + "ffwd.net.0.bias"]))
            x = x + F.linear(h, p[pre + "ffwd.net.2.weight"], p[pre + "ffwd.net.2.bias"])
        x = F.layer_norm(x, (C,), p["ln_f.weight"], p["ln_f.bias"], 1e-5)
        self.rows = torch.cat([self.rows, F.linear(x, p["lm_head.weight"], p["lm_head.bias"])[:, None]], 1)

    def _slide(self, keep):
        """drop the oldest tokens until ``keep`` remain (metadata stays)"""
        n_meta = self.meta.shape[1]
        while self.rows.shape[1] > keep:
            self.rows = self.rows[:, 1:]
            self.kv = [(torch.cat([K[:, :, :n_meta], K[:, :, n_meta + 1:]], 2),
                        torch.cat([V[:, :, :n_meta], V[:, :, n_meta + 1:]], 2)) for K, V in self.kv]

    def __call__(self, window, meta):
        if self.kv is None:
            self._prefill(window, meta)
        else:  # the new token's window holds at most ctx tokens, itself included
            self._slide(self.ctx - 1)
            self._step(window[:, -1])
        assert self.rows.shape[1] == window.shape[1]
        return self.rows
