// Recurrent (one token per call) Mamba2 mixer step and the running filtered
// logit of the cached decode (the intent of the
// reference's test_inference.ipynb cells 3-5, applied to scripts/generate.py:
// 14-95 with a Mamba model).
//
// While the decode window still holds the whole history (prompt + new tokens
// <= context_len) the reference's per-step full forward is causal in every
// Mamba2 mixer, so the logits of the new last position equal one recurrent
// step of each mixer from the states after the previous position:
//   conv : xBC_t = silu(b + w0 s0 + w1 s1 + w2 s2 + w3 in_t),  (s0, s1, s2) <- (s1, s2, in_t)
//   ssd  : h = exp(dt A) h + dt x_t B_t^T ;  y_t = h C_t + D x_t   (dt = softplus(dt_raw + dt_bias))
// and the filtered logit's log-softmax over the time axis (train.py:133-138)
// only needs a running per-vocabulary LSE over the positions seen so far.
//
// State layouts (fp32, owned by the caller):
//   conv state [B][3][conv_dim]  (the last three pre-conv xBC rows, oldest first)
//   ssm state  [B][H][P][N]      (P = N = 64)
//   col_lse    [B][V]
#include "common.h"

namespace {

constexpr int P = 64, N = 64, KW = 4;

// as mamba.hip's silu (v_exp_f32 + v_rcp_f32), so the step matches the forward
__device__ __forceinline__ float silu(float x) {
    return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// one thread per (b, channel c) of xBC
template <typename T>
__global__ __launch_bounds__(256) void conv_step_kernel(T* __restrict__ xc, int64_t ldxc, const T* __restrict__ zx,
                                                        int64_t ldz, int64_t d_inner, int64_t conv_dim,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        float* __restrict__ st) {
    const int64_t c = blockIdx.x * 256LL + threadIdx.x, b = blockIdx.y;
    if (c >= conv_dim) return;
    const float in = (float)zx[b * ldz + d_inner + c];
    float* s = st + b * 3 * conv_dim + c;
    const float s0 = s[0], s1 = s[conv_dim], s2 = s[2 * conv_dim];
    const float* wc = w + c * KW;
    float acc = bias[c];
    acc += wc[0] * s0;
    acc += wc[1] * s1;
    acc += wc[2] * s2;
    acc += wc[3] * in;
    xc[b * ldxc + c] = (T)silu(acc);
    s[0] = s1;
    s[conv_dim] = s2;
    s[2 * conv_dim] = in;
}

// one workgroup per (b, h); the 64 x 64 fp32 state is swept in 4 passes of 16
// rows: thread t owns columns 4 (t % 16) .. +3 of row 16 u + t / 16, so one
// wave instruction moves 1 KiB of contiguous state (4 whole rows) and every
// state byte is read and written once (the step's HBM bound: 32 KiB per (b, h));
// 15.6 us per layer at B = 64, H = 32 (4.3 TB/s) against 19.0 us for the
// previous row-per-4-threads mapping (rocprofv3, same box)
template <typename T>
__global__ __launch_bounds__(256) void ssd_step_kernel(T* __restrict__ y, int64_t ldy, float* __restrict__ state,
                                                       const T* __restrict__ xc, int64_t ldxc, const T* __restrict__ zx,
                                                       int64_t ldz, int64_t d_inner, int64_t conv_dim, int64_t H,
                                                       const float* __restrict__ dt_bias,
                                                       const float* __restrict__ A_log, const float* __restrict__ Dp) {
    const int64_t bh = blockIdx.x, b = bh / H, h = bh % H;
    const int t = threadIdx.x, c4 = t & 15, r0 = t >> 4;
    const T* xr = xc + b * ldxc;
    float* sp = state + bh * P * N + (int64_t)r0 * N + 4 * c4;
    f32x4 hv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) hv[u] = *(const f32x4*)(sp + u * 16 * N);  // all four rows in flight
    const float dt = softplus((float)zx[b * ldz + d_inner + conv_dim + h] + dt_bias[h]);
    const float dA = expf(dt * -expf(A_log[h]));
    float Bn[4], Cn[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        Bn[i] = (float)xr[d_inner + 4 * c4 + i];
        Cn[i] = (float)xr[d_inner + N + 4 * c4 + i];
    }
    const float Dh = Dp[h];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int p = 16 * u + r0;
        const float x = (float)xr[h * P + p];
        const float dx = dt * x;
        float ys = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            hv[u][i] = hv[u][i] * dA + dx * Bn[i];
            ys += hv[u][i] * Cn[i];
        }
        *(f32x4*)(sp + u * 16 * N) = hv[u];
        ys += __shfl_xor(ys, 1, 64);
        ys += __shfl_xor(ys, 2, 64);
        ys += __shfl_xor(ys, 4, 64);
        ys += __shfl_xor(ys, 8, 64);
        if (c4 == 0) y[b * ldy + h * P + p] = (T)(ys + Dh * x);
    }
}

// running column LSE over the positions seen so far, then z of the new position:
// lse[b,v] = logaddexp(lse[b,v], o[b,v]); z[b,v] = -(o - lse) * wtab[bucket(tok[b])][v]
template <typename T>
__global__ __launch_bounds__(256) void filtered_step_kernel(float* __restrict__ z, int64_t ldz, float* __restrict__ lse,
                                                            const T* __restrict__ o, int64_t ld,
                                                            const int64_t* __restrict__ tok,
                                                            const float* __restrict__ wtab, int64_t b0, int64_t b1,
                                                            int64_t b2, int64_t b3, int64_t V) {
    const int64_t v = blockIdx.x * 256LL + threadIdx.x, b = blockIdx.y;
    if (v >= V) return;
    const float ov = (float)o[b * ld + v];
    const float l = lse[b * V + v];
    const float m = fmaxf(l, ov);
    const float nl = m + logf(expf(l - m) + expf(ov - m));
    lse[b * V + v] = nl;
    const int64_t tk = tok[b];
    const int bk = (tk > b0) + (tk > b1) + (tk > b2) + (tk > b3);
    z[b * ldz + v] = -(ov - nl) * wtab[bk * V + v];
}

}  // namespace

extern "C" int msq_mamba_conv_step(void* xc, int64_t ldxc, float* conv_state, const void* zxbcdt, int64_t ldz,
                                   int dtype, const float* conv_w, const float* conv_b, int64_t B, int64_t d_inner,
                                   int64_t nheads, void* stream) {
    MSQ_CHECK_ARG(xc && conv_state && zxbcdt && conv_w && conv_b && B > 0 && nheads > 0 && d_inner == nheads * P &&
                      (dtype == MSQ_BF16 || dtype == MSQ_F32),
                  "msq_mamba_conv_step: bad args");
    const int64_t cd = d_inner + 2 * N;
    const dim3 grid((unsigned)((cd + 255) / 256), (unsigned)B);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_BF16)
        hipLaunchKernelGGL(conv_step_kernel<bf16>, grid, dim3(256), 0, s, (bf16*)xc, ldxc, (const bf16*)zxbcdt, ldz,
                           d_inner, cd, conv_w, conv_b, conv_state);
    else
        hipLaunchKernelGGL(conv_step_kernel<float>, grid, dim3(256), 0, s, (float*)xc, ldxc, (const float*)zxbcdt,
                           ldz, d_inner, cd, conv_w, conv_b, conv_state);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_ssd_step(void* y, int64_t ldy, float* ssm_state, const void* xc, int64_t ldxc,
                                  const void* zxbcdt, int64_t ldz, int dtype, const float* dt_bias,
                                  const float* A_log, const float* D, int64_t B, int64_t d_inner, int64_t nheads,
                                  void* stream) {
    MSQ_CHECK_ARG(y && ssm_state && xc && zxbcdt && dt_bias && A_log && D && B > 0 && nheads > 0 &&
                      d_inner == nheads * P && (dtype == MSQ_BF16 || dtype == MSQ_F32),
                  "msq_mamba_ssd_step: bad args");
    const int64_t cd = d_inner + 2 * N;
    const dim3 grid((unsigned)(B * nheads));
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_BF16)
        hipLaunchKernelGGL(ssd_step_kernel<bf16>, grid, dim3(256), 0, s, (bf16*)y, ldy, ssm_state, (const bf16*)xc, ldxc,
                           (const bf16*)zxbcdt, ldz, d_inner, cd, nheads, dt_bias, A_log, D);
    else
        hipLaunchKernelGGL(ssd_step_kernel<float>, grid, dim3(256), 0, s, (float*)y, ldy, ssm_state, (const float*)xc, ldxc,
                           (const float*)zxbcdt, ldz, d_inner, cd, nheads, dt_bias, A_log, D);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_filtered_logit_step(float* z, int64_t ldz, float* col_lse, const void* logits, int dtype,
                                       int64_t ld, const int64_t* tok, const float* wtab, int64_t b0, int64_t b1,
                                       int64_t b2, int64_t b3, int64_t B, int64_t V, void* stream) {
    MSQ_CHECK_ARG(z && col_lse && logits && tok && wtab && B > 0 && V > 0 && ld >= V && ldz >= V &&
                      (dtype == MSQ_BF16 || dtype == MSQ_F32),
                  "msq_filtered_logit_step: bad args");
    const dim3 grid((unsigned)((V + 255) / 256), (unsigned)B);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_BF16)
        hipLaunchKernelGGL(filtered_step_kernel<bf16>, grid, dim3(256), 0, s, z, ldz, col_lse, (const bf16*)logits, ld,
                           tok, wtab, b0, b1, b2, b3, V);
    else
        hipLaunchKernelGGL(filtered_step_kernel<float>, grid, dim3(256), 0, s, z, ldz, col_lse, (const float*)logits,
                           ld, tok, wtab, b0, b1, b2, b3, V);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
