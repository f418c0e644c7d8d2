"""Relative-position attention launchers (HeadRelPos x n_heads,
models/transformer/model_transformer.py:41-90) over the libmidiseq C ABI."""
import torch

from . import _lib as L
from ._lib import ptr, call, stream, dt
from .ops import workspace

N_META = 6  # metadata prefix (generate_matrix, model_transformer.py:14)


def relattn_fwd(qkv, R, B, S, H, hs, scale, out=None, lse=None, n_meta=N_META, drop=None):
    """qkv [B*S, >=3*H*hs] (bf16 -> flash MFMA path, fp32 -> exact path),
    R [H, S_max, hs]. Returns (out [B*S, H*hs], lse fp32 [B, H, S]).
    drop=(masks [2, n] from ops.dropout_attn_mask, p): attention-probability dropout."""
    if out is None:
        out = torch.empty(B * S, H * hs, device=qkv.device, dtype=qkv.dtype)
    if lse is None:
        lse = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32)
    masks, p = drop if drop is not None else (None, 0.0)
    call("msq_relattn_fwd_dropout", dt(qkv), ptr(out), out.stride(0), ptr(lse), ptr(qkv), qkv.stride(0), ptr(R), B,
         S, H, hs, R.shape[1], float(scale), n_meta, ptr(masks[0]) if masks is not None else None,
         ptr(masks[1]) if masks is not None else None, float(p), stream())
    return out, lse


# workspace slot ("attn", device, stream) -> (buffer address, (dtype, B, S, H,
# n_meta)) of the backward it last served: its zero bands stay valid for the
# next backward of the same shape in the SAME buffer (msq_relattn_bwd_ws). A
# slot whose buffer was replaced (grown) has a new address and starts cold.
_ws_served = {}


def relattn_bwd(dout, out, lse, qkv, R, B, S, H, hs, scale, dqkv=None, dR=None, n_meta=N_META, drop=None):
    """Returns (dqkv [B*S, 3*H*hs] (overwritten), dR fp32 [H, S_max, hs] (accumulated))."""
    if dqkv is None:
        dqkv = torch.empty(B * S, 3 * H * hs, device=qkv.device, dtype=qkv.dtype)
    if dR is None:
        dR = torch.zeros(R.shape, device=qkv.device, dtype=torch.float32)
    nbytes = L.lib().msq_relattn_bwd_workspace(dt(qkv), B, S, H)
    ws = workspace(nbytes, qkv.device, "attn")
    masks, p = drop if drop is not None else (None, 0.0)
    key = (dt(qkv), B, S, H, n_meta)
    slot = ("attn", qkv.device, torch.cuda.current_stream(qkv.device).cuda_stream)
    ready = int(_ws_served.get(slot) == (ws.data_ptr(), key))  # the "attn" workspace serves only this op
    call("msq_relattn_bwd_ws", dt(qkv), ptr(dqkv), dqkv.stride(0), ptr(dR), ptr(dout), dout.stride(0), ptr(out),
         ptr(lse), ptr(qkv), qkv.stride(0), ptr(R), B, S, H, hs, R.shape[1], float(scale), n_meta,
         ptr(masks[0]) if masks is not None else None, ptr(masks[1]) if masks is not None else None, float(p),
         ptr(ws), ready, stream())
    _ws_served[slot] = (ws.data_ptr(), key)
    return dqkv, dR
