// Relative-position attention, EXACT fp32 path (parity mode, small shapes).
//
// Semantics of HeadRelPos (model_transformer.py:54-90) for one head, with
// S = T + 6 rows, scale = n_embd^-1/2 and the flat "skew" of _rel_shift:
//   score(i,j) = (q_i.k_j + BD(i,j)) * scale,  allowed iff j <= i or j < n_meta
//   BD(i,j)    = q_i.R[S-1-i+j]        j <= i
//              = 0                     j == i+1
//              = q_{i+1}.R[j-i-2]      j >= i+2   (only reachable in the meta block)
// One workgroup per query row; scores live in LDS. The backward recomputes P
// from the saved log-sum-exp and stores P / dS rows in the workspace for the
// column reductions (dK, dV, dR).
#include "attn.h"
#include <stdlib.h>

namespace {

constexpr int NTH = 256;

__device__ __forceinline__ const float* qrow(const AttnArgs& a, int64_t b, int64_t h, int64_t i, int which) {
    return (const float*)a.qkv + (b * a.S + i) * a.ldq + which * a.H * a.hs + h * a.hs;
}

__device__ __forceinline__ float dotf(const float* x, const float* y, int n) {
    float s = 0.f;
    for (int t = 0; t < n; ++t) s = fmaf(x[t], y[t], s);
    return s;
}

// raw (unscaled, unmasked) score; -inf if not allowed
__device__ float score(const AttnArgs& a, int64_t b, int64_t h, int64_t i, int64_t j) {
    if (!(j <= i || j < a.n_meta)) return -INFINITY;
    const int hs = (int)a.hs;
    const float* q = qrow(a, b, h, i, 0);
    float ac = dotf(q, qrow(a, b, h, j, 1), hs);
    float bd = 0.f;
    const float* Rh = (const float*)a.R + h * a.S_max * a.hs;
    if (j <= i) bd = dotf(q, Rh + (a.S - 1 - i + j) * a.hs, hs);
    else if (j >= i + 2) bd = dotf(qrow(a, b, h, i + 1, 0), Rh + (j - i - 2) * a.hs, hs);
    return (ac + bd) * a.scale;
}

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = is_max ? wave_max(v) : wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int k = 1; k < NTH / 64; ++k) r = is_max ? fmaxf(r, red[k]) : r + red[k];
    return r;
}

__global__ __launch_bounds__(NTH) void exact_fwd_kernel(AttnArgs a, float* out, int64_t ldo, float* lse) {
    extern __shared__ float srow[];  // S scores
    __shared__ float red[8];
    const int64_t i = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    float mx = -INFINITY;
    for (int64_t j = threadIdx.x; j < a.S; j += NTH) {
        const float s = score(a, b, h, i, j);
        srow[j] = s;
        mx = fmaxf(mx, s);
    }
    mx = block_reduce(mx, red, true);
    float sum = 0.f;
    for (int64_t j = threadIdx.x; j < a.S; j += NTH) {
        const float p = expf(srow[j] - mx);
        srow[j] = p;
        sum += p;
    }
    sum = block_reduce(sum, red, false);
    if (threadIdx.x == 0) lse[(b * a.H + h) * a.S + i] = mx + logf(sum);
    __syncthreads();
    const float inv = 1.f / sum;
    if (a.rowmask) {  // dropout: O = sum_j (p_j keep_j / (1-p)) v_j / sum
        for (int64_t j = threadIdx.x; j < a.S; j += NTH) srow[j] *= keep_bit(a, b * a.H + h, i, j);
        __syncthreads();
    }
    for (int d = threadIdx.x; d < a.hs; d += NTH) {
        float o = 0.f;
        for (int64_t j = 0; j < a.S; ++j) o = fmaf(srow[j], qrow(a, b, h, j, 2)[d], o);
        out[(b * a.S + i) * ldo + h * a.hs + d] = o * inv;
    }
}

// per query row: P, dS = P*(dP - D)*scale into the workspace; dq (AC + j<=i BD part)
__global__ __launch_bounds__(NTH) void exact_bwd_row_kernel(AttnArgs a, const float* lse, const float* dout,
                                                            int64_t ldo, float* P, float* dS, float* dqkv,
                                                            int64_t ldd) {
    extern __shared__ float sm[];
    float* sp = sm;          // P row
    float* sd = sm + a.S;    // dP row -> dS row
    __shared__ float red[8];
    const int64_t i = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const float L = lse[(b * a.H + h) * a.S + i];
    const float* dO = dout + (b * a.S + i) * ldo + h * a.hs;
    float dsum = 0.f;
    for (int64_t j = threadIdx.x; j < a.S; j += NTH) {
        const float s = score(a, b, h, i, j);
        const float p = s == -INFINITY ? 0.f : expf(s - L);
        float dp = dotf(dO, qrow(a, b, h, j, 2), (int)a.hs);
        // dropout: P' = P keep/(1-p) feeds dV; dP = dP' keep/(1-p); D = sum P' dP'
        const float kb = a.rowmask ? keep_bit(a, b * a.H + h, i, j) : 1.f;
        dp *= kb;
        sp[j] = p;
        sd[j] = dp;
        dsum += p * dp;
    }
    const float D = block_reduce(dsum, red, false);
    const int64_t rowoff = ((b * a.H + h) * a.S + i) * a.S;
    for (int64_t j = threadIdx.x; j < a.S; j += NTH) {
        const float ds = sp[j] * (sd[j] - D) * a.scale;
        sd[j] = ds;
        P[rowoff + j] = a.rowmask ? sp[j] * keep_bit(a, b * a.H + h, i, j) : sp[j];
        dS[rowoff + j] = ds;
    }
    __syncthreads();
    const float* Rh = (const float*)a.R + h * a.S_max * a.hs;
    for (int d = threadIdx.x; d < a.hs; d += NTH) {
        float g = 0.f;
        for (int64_t j = 0; j < a.S; ++j) {
            const float ds = sd[j];
            if (ds == 0.f) continue;
            float kv = qrow(a, b, h, j, 1)[d];
            if (j <= i) kv += Rh[(a.S - 1 - i + j) * a.hs + d];
            g = fmaf(ds, kv, g);
        }
        dqkv[(b * a.S + i) * ldd + h * a.hs + d] = g;
    }
}

// per key column j: dk_j = sum_i dS_ij q_i ; dv_j = sum_i P_ij dO_i
__global__ __launch_bounds__(NTH) void exact_bwd_col_kernel(AttnArgs a, const float* dout, int64_t ldo,
                                                            const float* P, const float* dS, float* dqkv,
                                                            int64_t ldd) {
    const int64_t j = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int64_t base = (b * a.H + h) * a.S * a.S;
    for (int d = threadIdx.x; d < a.hs; d += NTH) {
        float gk = 0.f, gv = 0.f;
        for (int64_t i = 0; i < a.S; ++i) {
            const float ds = dS[base + i * a.S + j], p = P[base + i * a.S + j];
            gk = fmaf(ds, qrow(a, b, h, i, 0)[d], gk);
            gv = fmaf(p, dout[(b * a.S + i) * ldo + h * a.hs + d], gv);
        }
        dqkv[(b * a.S + j) * ldd + a.H * a.hs + h * a.hs + d] = gk;
        dqkv[(b * a.S + j) * ldd + 2 * a.H * a.hs + h * a.hs + d] = gv;
    }
}

// dR[h][r] += sum_{b,i} dS[b,h,i,i-(S-1-r)] q_{b,i}  (+ meta-block terms r = j-i-2)
__global__ __launch_bounds__(NTH) void exact_bwd_dr_kernel(AttnArgs a, const float* dS, float* dR) {
    const int64_t r = blockIdx.x, h = blockIdx.y;
    const int64_t delta = a.S - 1 - r;  // i - j
    for (int d = threadIdx.x; d < a.hs; d += NTH) {
        float g = 0.f;
        for (int64_t b = 0; b < a.B; ++b) {
            const int64_t base = (b * a.H + h) * a.S * a.S;
            for (int64_t i = delta; i < a.S; ++i) g = fmaf(dS[base + i * a.S + (i - delta)], qrow(a, b, h, i, 0)[d], g);
            // meta block: j >= i+2, j < n_meta, r == j-i-2
            for (int64_t i = 0; i + 2 + r < a.n_meta && i + 1 < a.S; ++i) {
                const int64_t j = i + 2 + r;
                if (j >= a.S) break;
                g = fmaf(dS[base + i * a.S + j], qrow(a, b, h, i + 1, 0)[d], g);
            }
        }
        dR[(h * a.S_max + r) * a.hs + d] += g;
    }
}

// meta block: dq_{i+1} += dS_ij R[j-i-2] for j >= i+2, j < n_meta
__global__ void exact_bwd_meta_dq_kernel(AttnArgs a, const float* dS, float* dqkv, int64_t ldd) {
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int64_t base = (b * a.H + h) * a.S * a.S;
    const float* Rh = (const float*)a.R + h * a.S_max * a.hs;
    for (int d = threadIdx.x; d < a.hs; d += blockDim.x) {
        for (int64_t i = 0; i + 2 < a.n_meta && i + 1 < a.S; ++i) {
            float g = 0.f;
            for (int64_t j = i + 2; j < a.n_meta && j < a.S; ++j) g = fmaf(dS[base + i * a.S + j], Rh[(j - i - 2) * a.hs + d], g);
            dqkv[(b * a.S + i + 1) * ldd + h * a.hs + d] += g;
        }
    }
}

}  // namespace

size_t exact_bwd_workspace(int64_t B, int64_t S, int64_t H) { return (size_t)2 * B * H * S * S * sizeof(float); }

int exact_fwd(const AttnArgs& a, float* out, int64_t ldo, float* lse, hipStream_t s) {
    hipLaunchKernelGGL(exact_fwd_kernel, dim3((unsigned)a.S, (unsigned)a.H, (unsigned)a.B), dim3(NTH),
                       a.S * sizeof(float), s, a, out, ldo, lse);
    return 0;
}

int exact_bwd(const AttnArgs& a, const float* lse, const float* dout, int64_t ldo, float* dqkv, int64_t ldd, float* dR,
              void* ws, hipStream_t s) {
    float* P = (float*)ws;
    float* dS = P + a.B * a.H * a.S * a.S;
    const dim3 g((unsigned)a.S, (unsigned)a.H, (unsigned)a.B);
    hipLaunchKernelGGL(exact_bwd_row_kernel, g, dim3(NTH), 2 * a.S * sizeof(float), s, a, lse, dout, ldo, P, dS, dqkv, ldd);
    hipLaunchKernelGGL(exact_bwd_col_kernel, g, dim3(NTH), 0, s, a, dout, ldo, P, dS, dqkv, ldd);
    hipLaunchKernelGGL(exact_bwd_dr_kernel, dim3((unsigned)a.S, (unsigned)a.H), dim3(NTH), 0, s, a, dS, dR);
    hipLaunchKernelGGL(exact_bwd_meta_dq_kernel, dim3(1, (unsigned)a.H, (unsigned)a.B), dim3(128), 0, s, a, dS, dqkv, ldd);
    return 0;
}

// ---------------------------------------------------------------- C entry points
static AttnArgs mk(int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max, int64_t n_meta, float scale,
                   const void* qkv, int64_t ldq, const void* R) {
    AttnArgs a;
    a.B = B; a.S = S; a.H = H; a.hs = hs; a.S_max = S_max; a.n_meta = n_meta; a.scale = scale;
    a.qkv = qkv; a.ldq = ldq; a.R = R;
    a.xcd = 1;  // XCD-aware block order (xcd_blk3)
    return a;
}

static void set_drop(AttnArgs& a, const uint32_t* rowmask, const uint32_t* colmask, float p) {
    a.rowmask = rowmask;
    a.colmask = colmask;
    a.mask_ld = msq_dropout_mask_ld(a.S);
    a.keep_scale = 1.f / (1.f - p);
}

extern "C" size_t msq_relattn_bwd_workspace(int dtype, int64_t B, int64_t S, int64_t H) {
    return dtype == MSQ_F32 ? exact_bwd_workspace(B, S, H) : flash_bwd_workspace(B, S, H);
}

static int relattn_fwd(int dtype, void* out, int64_t ld_out, float* lse, const AttnArgs& a, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_F32) {
        exact_fwd(a, (float*)out, ld_out, lse, s);
    } else {
        MSQ_CHECK_ARG(a.hs == 128 && a.ldq % 8 == 0 && ld_out % 4 == 0, "msq_relattn_fwd: bf16 path needs hs == 128");
        if (flash_fwd3(a, (bf16*)out, ld_out, lse, s))
            return msq_set_error(MSQ_ERR_UNSUPPORTED,
                                 "msq_relattn_fwd: shape outside the flash kernel (n_meta > 8 or a > 4 GB operand)");
    }
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_relattn_fwd(int dtype, void* out, int64_t ld_out, float* lse, const void* qkv, int64_t ld_qkv,
                               const void* R, int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale,
                               int64_t n_meta, void* stream) {
    return msq_relattn_fwd_dropout(dtype, out, ld_out, lse, qkv, ld_qkv, R, B, S, H, hs, S_max, scale, n_meta,
                                   nullptr, nullptr, 0.f, stream);
}

extern "C" int msq_relattn_fwd_dropout(int dtype, void* out, int64_t ld_out, float* lse, const void* qkv,
                                       int64_t ld_qkv, const void* R, int64_t B, int64_t S, int64_t H, int64_t hs,
                                       int64_t S_max, float scale, int64_t n_meta, const uint32_t* rowmask,
                                       const uint32_t* colmask, float p, void* stream) {
    MSQ_CHECK_ARG(B > 0 && S > 0 && H > 0 && hs > 0 && S <= S_max, "msq_relattn_fwd: bad sizes (S <= S_max)");
    MSQ_CHECK_ARG(ld_qkv >= 3 * H * hs && ld_out >= H * hs, "msq_relattn_fwd: leading dims too small");
    MSQ_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || (rowmask && colmask)), "msq_relattn_fwd: dropout needs masks");
    AttnArgs a = mk(B, S, H, hs, S_max, n_meta, scale, qkv, ld_qkv, R);
    if (p > 0.f) set_drop(a, rowmask, colmask, p);
    return relattn_fwd(dtype, out, ld_out, lse, a, stream);
}

static int relattn_bwd(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout, int64_t ld_dout,
                       const void* out, const float* lse, const AttnArgs& a, void* workspace, int ws_ready,
                       void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_F32) {
        exact_bwd(a, lse, (const float*)dout, ld_dout, (float*)dqkv, ld_dqkv, dR, workspace, s);
    } else {
        MSQ_CHECK_ARG(a.hs == 128 && a.ldq % 8 == 0 && ld_dout % 8 == 0 && ld_dqkv % 8 == 0,
                      "msq_relattn_bwd: bf16 path needs hs == 128, ld %% 8 == 0");
        int rc = flash_bwd(a, lse, (const bf16*)dout, ld_dout, (const bf16*)out, (bf16*)dqkv, ld_dqkv, dR, workspace,
                           ws_ready != 0, s);
        if (rc) return rc;
    }
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_relattn_bwd(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout, int64_t ld_dout,
                               const void* out, const float* lse, const void* qkv, int64_t ld_qkv, const void* R,
                               int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale, int64_t n_meta,
                               void* workspace, void* stream) {
    return msq_relattn_bwd_dropout(dtype, dqkv, ld_dqkv, dR, dout, ld_dout, out, lse, qkv, ld_qkv, R, B, S, H, hs,
                                   S_max, scale, n_meta, nullptr, nullptr, 0.f, workspace, stream);
}

extern "C" int msq_relattn_bwd_dropout(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout,
                                       int64_t ld_dout, const void* out, const float* lse, const void* qkv,
                                       int64_t ld_qkv, const void* R, int64_t B, int64_t S, int64_t H, int64_t hs,
                                       int64_t S_max, float scale, int64_t n_meta, const uint32_t* rowmask,
                                       const uint32_t* colmask, float p, void* workspace, void* stream) {
    return msq_relattn_bwd_ws(dtype, dqkv, ld_dqkv, dR, dout, ld_dout, out, lse, qkv, ld_qkv, R, B, S, H, hs, S_max,
                              scale, n_meta, rowmask, colmask, p, workspace, 0, stream);
}

extern "C" int msq_relattn_bwd_ws(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout,
                                  int64_t ld_dout, const void* out, const float* lse, const void* qkv, int64_t ld_qkv,
                                  const void* R, int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max,
                                  float scale, int64_t n_meta, const uint32_t* rowmask, const uint32_t* colmask,
                                  float p, void* workspace, int ws_ready, void* stream) {
    MSQ_CHECK_ARG(B > 0 && S > 0 && H > 0 && hs > 0 && S <= S_max && workspace && n_meta <= 8,
                  "msq_relattn_bwd: bad args");
    MSQ_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || (rowmask && colmask)), "msq_relattn_bwd: dropout needs masks");
    AttnArgs a = mk(B, S, H, hs, S_max, n_meta, scale, qkv, ld_qkv, R);
    if (p > 0.f) set_drop(a, rowmask, colmask, p);
    return relattn_bwd(dtype, dqkv, ld_dqkv, dR, dout, ld_dout, out, lse, a, workspace, ws_ready, stream);
}
