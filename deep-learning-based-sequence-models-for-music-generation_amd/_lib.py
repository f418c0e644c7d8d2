"""ctypes binding of libmidiseq.so (include/midiseq.h).

The product path has NO CPU fallback: if the library is missing or a call
fails, a RuntimeError is raised. torch must be imported first so that the
process-wide libamdhip64.so.7 is torch's (same SONAME, one HIP runtime).
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime before libmidiseq)

HERE = os.path.dirname(os.path.abspath(__file__))
# MSQ_LIB_PATH: an alternate build of the same library (same-box A/B tools only)
LIB_PATH = os.environ.get("MSQ_LIB_PATH") or os.path.join(HERE, "libmidiseq.so")

F32, BF16, MASK1 = 0, 1, 2
ROUTE_DEFAULT, ROUTE_TILE256, ROUTE_TILE128 = range(3)  # msq_gemm_set_route
EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_RESID, EPI_RELU_MASK, EPI_ACCUM, EPI_BIAS_DROP_RESID = range(7)

_p, _i, _i64, _f, _sz, _u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t, ctypes.c_uint32

# symbol -> (restype, argtypes); must mirror include/midiseq.h exactly
SIGNATURES = {
    "msq_last_error": (ctypes.c_char_p, []),
    "msq_version": (_i, []),
    "msq_embed_fwd": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "msq_embed_bwd": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "msq_embed_bwd_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _i64]),
    "msq_embed_bwd_sorted": (_i, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _p]),
    "msq_layernorm_fwd": (_i, [_p, _i, _p, _p, _p, _p, _p, _i64, _i64, _f, _i64, _i64, _p]),
    "msq_layernorm_bwd_workspace": (_sz, [_i64, _i64]),
    "msq_layernorm_bwd": (_i, [_p, _p, _i, _p, _p, _p, _i, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _p]),
    "msq_gemm": (_i, [_i, _i, _i, _i64, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _p, _i, _i64, _i64, _i64, _i,
                      _p, _p, _i, _i64, _i64, _p]),
    "msq_gemm_dropout": (_i, [_i, _i, _i, _i64, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _p, _i, _i64, _i64, _i64,
                              _i, _p, _p, _i, _i64, _i64, _u32, _u32, _f, _p]),
    "msq_gemm_workspace_size": (_i64, [_i, _i, _i, _i64, _i64, _i64, _i64, _i64, _i64, _i]),
    "msq_gemm_ex": (_i, [_i, _i, _i, _i64, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _p, _i, _i64, _i64, _i64,
                         _i, _p, _p, _i, _i64, _i64, _u32, _u32, _f, _p, _i64, _p]),
    "msq_layernorm_bwd_bias": (_i, [_p, _p, _i, _p, _p, _p, _p, _i, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _u32, _u32,
                                    _f, _i, _p, _p]),
    "msq_layernorm_bwd_dropout": (_i, [_p, _p, _i, _p, _p, _p, _i, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _u32, _u32,
                                       _f, _p, _p]),
    "msq_dropout_mask_ld": (_i64, [_i64]),
    "msq_dropout_mask_words": (_i64, [_i64, _i64, _i64]),
    "msq_window_gather": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _p, _i64, _i64, _i, _p, _p]),
    "msq_midi_decode": (_i, [_p, _i64, _i64, _i64, _p, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "msq_relattn_decode": (_i, [_i, _p, _i64, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                _f, _p, _sz, _p]),
    "msq_relattn_decode_workspace": (_sz, [_i64, _i64, _i64]),
    "msq_midi_encode": (_i, [_p, _p, _p, _p, _p, _p, _p, _i64, _p, _i64, _p, _p, _p, _p, _p]),
    "msq_dropout_attn_table": (_i, [_f, _p]),
    "msq_dropout_attn_mask": (_i, [_p, _p, _i64, _i64, _i64, _u32, _u32, _f, _p]),
    "msq_relattn_fwd_dropout": (_i, [_i, _p, _i64, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _f, _i64, _p, _p,
                                     _f, _p]),
    "msq_relattn_bwd_dropout": (_i, [_i, _p, _i64, _p, _p, _i64, _p, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64,
                                     _f, _i64, _p, _p, _f, _p, _p]),
    "msq_relattn_bwd_ws": (_i, [_i, _p, _i64, _p, _p, _i64, _p, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64,
                                     _f, _i64, _p, _p, _f, _p, _i, _p]),
    "msq_colsum_workspace": (_sz, [_i64, _i64]),
    "msq_gemm_colsum_workspace": (_sz, [_i64, _i64]),
    "msq_colsum": (_i, [_p, _i, _p, _i, _i64, _i64, _i64, _p, _p]),
    "msq_cast": (_i, [_p, _i, _p, _i, _i64, _p]),
    "msq_adam_step": (_i, [_p, _p, _p, _p, _p, _i64, _f, _f, _f, _f, _i64, _f, _p]),
    "msq_relattn_fwd": (_i, [_i, _p, _i64, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _f, _i64, _p]),
    "msq_filtered_workspace": (_sz, [_i64, _i64, _i64]),
    "msq_filtered_colstats": (_i, [_p, _p, _i, _i64, _i64, _i64, _i64, _p, _p]),
    "msq_gemm_colsum": (_i, [_i, _i, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64, _i, _p, _i, _i64, _p, _i, _p,
                             _i64, _p]),
    "msq_transpose_bf16": (_i, [_p, _i64, _p, _i64, _i64, _i64, _p]),
    "msq_gemm_colstats_bytes": (_sz, [_i64, _i64]),
    "msq_gemm_bias_colstats": (_i, [_i, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _p]),
    "msq_gemm_bias_colstats_applies": (_i, [_i, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p, _i64]),
    "msq_filtered_ce_bias_part": (_i, [_p, _p, _i64, _p, _p, _i, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64,
                                       _i64, _i64, _f, _p, _p, _i64, _i64, _p, _p]),
    "msq_gemm_set_route": (_i, [_i]),
    "msq_gemm_resid_ln_workspace": (_i64, [_i, _i64, _i64, _i64, _i64, _i64]),
    "msq_gemm_resid_ln": (_i, [_i, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _p, _p, _f, _p, _i,
                               _i64, _p, _i64, _p]),
    "msq_ring_step": (_i, [_p, _p, _p, _p, _i, _i64, _i64, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _p]),
    "msq_ring_state_bytes": (_sz, [_i64, _i64, _i64]),
    "msq_relattn_decode_pos": (_i, [_i, _p, _i64, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _f,
                                    _p, _sz, _p]),
    "msq_ring_lse": (_i, [_p, _p, _p, _i, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _p]),
    "msq_filtered_ce_bias": (_i, [_p, _p, _i64, _p, _p, _i, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                  _f, _p, _p, _p]),
    "msq_filtered_ce": (_i, [_p, _p, _i64, _p, _i, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _f,
                             _p, _p, _p]),
    "msq_filtered_logit": (_i, [_p, _i64, _p, _i, _i64, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _p,
                                _p, _p]),
    "msq_filtered_logit_bwd": (_i, [_p, _i64, _p, _i64, _p, _i, _i64, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64,
                                    _i64, _p, _p, _p]),
    "msq_decode_sample": (_i, [_p, _i64, _i64, _p, _i64, _i64, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "msq_mamba_states_size": (_sz, [_i64, _i64, _i64]),
    "msq_mamba_conv_fwd": (_i, [_p, _i64, _p, _i64, _i, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "msq_mamba_ssd_fwd": (_i, [_p, _i64, _p, _p, _i64, _p, _i64, _i, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "msq_mamba_gnorm_fwd": (_i, [_p, _i64, _p, _p, _i64, _p, _i64, _i, _p, _i64, _i64, _f, _p]),
    "msq_mamba_gnorm_bwd": (_i, [_p, _p, _p, _i64, _p, _i64, _i, _p, _p, _p, _i64, _p, _i64, _i64, _p]),
    "msq_mamba_ssd_bwd_workspace": (_sz, [_i64, _i64, _i64]),
    "msq_mamba_ssd_bwd": (_i, [_p, _i64, _p, _p, _i64, _p, _p, _i64, _p, _i64, _i, _p, _p, _p, _p, _p, _p, _i64,
                               _i64, _i64, _i64, _p, _p]),
    "msq_mamba_ssd_fwd_state": (_i, [_p, _i64, _p, _p, _p, _i64, _p, _i64, _i, _p, _p, _p, _i64, _i64, _i64, _i64,
                                     _p]),
    "msq_mamba_conv_step": (_i, [_p, _i64, _p, _p, _i64, _i, _p, _p, _i64, _i64, _i64, _p]),
    "msq_mamba_in_proj_conv_step": (_i, [_p, _i64, _p, _i64, _p, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _i64,
                                         _i64, _p]),
    "msq_mamba_ssd_step": (_i, [_p, _i64, _p, _p, _i64, _p, _i64, _i, _p, _p, _p, _i64, _i64, _i64, _p]),
    "msq_filtered_logit_step": (_i, [_p, _i64, _p, _p, _i, _i64, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p]),
    "msq_mamba_conv_bwd":(_i, [_p, _p, _i64, _p, _i64, _i, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "msq_relattn_bwd_workspace": (_sz, [_i, _i64, _i64, _i64]),
    "msq_relattn_bwd": (_i, [_i, _p, _i64, _p, _p, _i64, _p, _p, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _f, _i64,
                             _p, _p]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libmidiseq.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        # an A/B twin library (MSQ_LIB_PATH) of an older revision may lack newer
        # entry points; the in-tree library must export every one
        twin = "MSQ_LIB_PATH" in os.environ
        for name, (res, args) in SIGNATURES.items():
            if twin and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# optional launch observer (bench.py's per-class HIP-event timing):
# TAP(name, args, launch) must call launch() and return its result; ROLE is
# the caller's label of the launch in flight (ops.gemm(role=...)), or None
TAP = None
ROLE = None


def call(name, *args):
    if TAP is not None:
        return TAP(name, args, lambda: _call(name, args))
    return _call(name, args)


def _call(name, args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed ({rc}): {lib().msq_last_error().decode()}")
    return rc


def ptr(t):
    """device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dt(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.int32:  # a GEMM aux bitmask (MSQ_MASK1)
        return MASK1
    raise TypeError(f"unsupported dtype {t.dtype}")
