// Mamba2 mixer kernels (mamba_ssm.Mamba2 as used by models/mamba/mamba.py:
// d_state 64, d_conv 4, expand 2, headdim 64, ngroups 1, rmsnorm gate with
// norm_before_gate=False). The GEMMs (in_proj / out_proj) use msq_gemm.
//
//   conv : xBC = silu(causal depthwise conv1d_k4(zxbcdt[:, d_inner : d_inner+conv_dim]) + bias)
//   ssd  : h_t = exp(dt_t A) h_{t-1} + dt_t x_t B_t^T ; y_t = h_t C_t + D x_t,
//          dt = softplus(dt_raw + dt_bias), A = -exp(A_log)   (per head, P = N = 64)
//          evaluated in chunks of 64 steps (the SSD block form): one workgroup
//          per (batch, head) walks its chunks; inside a chunk the four 64^3
//          products (C B^T, masked-decay . dt x, C H^T, decayed x^T B) run
//          from LDS in fp32; chunk-entry states are kept for the backward.
//   gate : y * silu(z) -> RMSNorm(eps) * w
// Backward kernels mirror these (chunked SSD backward, reverse over chunks).
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int Q = 64;   // chunk length
constexpr int P = 64;   // head dim
constexpr int N = 64;   // state dim
constexpr int LD = 68;  // LDS row stride (floats) for 64x64 tiles

struct MambaArgs {
    int64_t B, L, d_inner, nheads, conv_dim, ldz;  // ldz: row stride of zxbcdt
    int64_t ldxc;                                  // row stride of the conv output (xBC)
};

__device__ __forceinline__ float silu(float x) { return x / (1.f + expf(-x)); }
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// ------------------------------------------------------------------ conv
// out[b,t,c] = silu(bias[c] + sum_k w[c,k] * in[b, t-3+k, c]), in = zxbcdt[:, off + c]
template <typename T, typename TO>
__global__ void conv_fwd_kernel(MambaArgs a, const T* __restrict__ zx, const float* __restrict__ w,
                                const float* __restrict__ bias, TO* __restrict__ out) {
    const int64_t total = a.B * a.L * a.conv_dim;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e % a.conv_dim, bt = e / a.conv_dim;
        const int64_t t = bt % a.L;
        const T* src = zx + bt * a.ldz + a.d_inner + c;
        float acc = bias[c];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t tt = t - 3 + k;
            if (tt >= 0) acc += w[c * 4 + k] * (float)src[(k - 3) * a.ldz];
        }
        out[bt * a.ldxc + c] = (TO)silu(acc);
    }
}

// dpre = dout * silu'(pre); dzx_in[t] = sum_k w[k] dpre[t+3-k]; dw, dbias via per-block partials (atomics)
template <typename T, typename TD>
__global__ void conv_bwd_kernel(MambaArgs a, const T* __restrict__ zx, const float* __restrict__ w,
                                const float* __restrict__ bias, const float* __restrict__ dout, int64_t ldd,
                                TD* __restrict__ dzx, float* __restrict__ dw, float* __restrict__ dbias) {
    // block: 64 channels x 4 time-slices; grid (conv_dim/64, B, tchunks)
    const int lane = threadIdx.x & 63, ws = threadIdx.x >> 6;
    const int64_t c = blockIdx.x * 64 + lane;
    const int64_t b = blockIdx.y;
    const int64_t per = (a.L + gridDim.z - 1) / gridDim.z;
    const int64_t t0 = blockIdx.z * per, t1 = min(a.L, t0 + per);
    if (c >= a.conv_dim) return;
    const T* src = zx + b * a.L * a.ldz + a.d_inner + c;
    const float* dsrc = dout + b * a.L * ldd + c;
    float wk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) wk[k] = w[c * 4 + k];
    const float bc = bias[c];
    auto pre_at = [&](int64_t t) {
        float acc = bc;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t tt = t - 3 + k;
            if (tt >= 0) acc += wk[k] * (float)src[tt * a.ldz];
        }
        return acc;
    };
    auto dpre_at = [&](int64_t t) {
        if (t >= a.L) return 0.f;
        const float p = pre_at(t);
        const float s = sigm(p);
        return dsrc[t * ldd] * s * (1.f + p * (1.f - s));
    };
    float gw[4] = {0.f, 0.f, 0.f, 0.f}, gb = 0.f;
    for (int64_t t = t0 + ws; t < t1; t += 4) {
        // d input at time t: sum_k w[k] * dpre[t + 3 - k]
        float di = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) di += wk[k] * dpre_at(t + 3 - k);
        dzx[(b * a.L + t) * a.ldz + a.d_inner + c] = (TD)di;
        const float dp = dpre_at(t);
        gb += dp;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t tt = t - 3 + k;
            if (tt >= 0) gw[k] += dp * (float)src[tt * a.ldz];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(dw + c * 4 + k, gw[k]);
    atomicAdd(dbias + c, gb);
}

// ------------------------------------------------------------------ 64^3 tile product helper
// acc[i][j] (+)= sum_k Aop[r0+i][k] * Bop[k][c0+j], 4x4 per thread (r0=(tid>>4)*4, c0=(tid&15)*4)
// Aop[r][k] = AT ? A[k*LD + r] : A[r*LD + k] ; Bop[k][c] = BT ? Bm[c*LD + k] : Bm[k*LD + c]
template <bool AT, bool BT>
__device__ __forceinline__ void mm64(float (&acc)[4][4], const float* A, const float* Bm, int tid) {
    const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll 4
    for (int k = 0; k < 64; ++k) {
        float av[4], bv[4];
        if (AT) {
            const f32x4 t = *(const f32x4*)(A + k * LD + r0);
            av[0] = t[0]; av[1] = t[1]; av[2] = t[2]; av[3] = t[3];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) av[i] = A[(r0 + i) * LD + k];
        }
        if (!BT) {
            const f32x4 t = *(const f32x4*)(Bm + k * LD + c0);
            bv[0] = t[0]; bv[1] = t[1]; bv[2] = t[2]; bv[3] = t[3];
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = Bm[(c0 + j) * LD + k];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
}

__device__ __forceinline__ void zero44(float (&a)[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) a[i][j] = 0.f;
}

__device__ __forceinline__ void store44(float* dst, const float (&a)[4][4], int tid) {
    const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) *(f32x4*)(dst + (r0 + i) * LD + c0) = (f32x4){a[i][0], a[i][1], a[i][2], a[i][3]};
}

// load a [64 t][64 col] tile (rows t0.. of a row-major [L, ld] source, cols c0..c0+63) into LDS as fp32
template <typename T>
__device__ __forceinline__ void load_tile(float* dst, const T* src, int64_t ld, int64_t t0, int64_t L, int tid) {
    for (int e = tid; e < 64 * 16; e += NT) {
        const int r = e >> 4, c4 = (e & 15) * 4;
        f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (t0 + r < L) v = load4(src + (t0 + r) * ld + c4);
        *(f32x4*)(dst + r * LD + c4) = v;
    }
}

// ------------------------------------------------------------------ SSD forward
template <typename T>
__global__ __launch_bounds__(NT) void ssd_fwd_kernel(MambaArgs a, const T* __restrict__ xc,
                                                     const T* __restrict__ zx, const float* __restrict__ dt_bias,
                                                     const float* __restrict__ A_log, const float* __restrict__ Dp,
                                                     float* __restrict__ y, int64_t ldy, float* __restrict__ states) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* sX = sm;              // dt*x  [t][p]
    float* sB = sX + 64 * LD;    // B     [t][n]
    float* sC = sB + 64 * LD;    // C     [t][n]
    float* sM = sC + 64 * LD;    // masked decay . C B^T [t][s]
    float* sH = sM + 64 * LD;    // state [p][n]
    float* sx = sH + 64 * LD;    // raw x [t][p]
    float* sdt = sx + 64 * LD;   // dt [64]
    float* scum = sdt + 64;      // cumsum(dt*A) [64]
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x / a.nheads, h = blockIdx.x % a.nheads;
    const float A = -expf(A_log[h]);
    const float Dh = Dp[h];
    const int nch = (int)((a.L + Q - 1) / Q);
    const T* xb = xc + b * a.L * a.ldxc;
    for (int e = tid; e < 64 * 64; e += NT) sH[(e >> 6) * LD + (e & 63)] = 0.f;
    for (int ch = 0; ch < nch; ++ch) {
        const int64_t t0 = (int64_t)ch * Q;
        __syncthreads();
        // chunk-entry state for the backward
        float* st = states + ((b * a.nheads + h) * nch + ch) * (int64_t)(P * N);
        for (int e = tid; e < P * N; e += NT) st[e] = sH[(e >> 6) * LD + (e & 63)];
        load_tile(sx, xb + h * P, a.ldxc, t0, a.L, tid);
        load_tile(sB, xb + a.d_inner, a.ldxc, t0, a.L, tid);
        load_tile(sC, xb + a.d_inner + N, a.ldxc, t0, a.L, tid);
        if (tid < 64) {
            const int64_t t = t0 + tid;
            float d = 0.f;
            if (t < a.L) d = softplus((float)zx[(b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + h] + dt_bias[h]);
            sdt[tid] = d;
            // inclusive scan of d*A over the chunk (wave-level)
            float v = d * A;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float u = __shfl_up(v, o, 64);
                if (tid >= o) v += u;
            }
            scum[tid] = v;
        }
        __syncthreads();
        for (int e = tid; e < 64 * 64; e += NT) {
            const int r = e >> 6, c = e & 63;
            sX[r * LD + c] = sx[r * LD + c] * sdt[r];
        }
        // G = C B^T, masked decay
        float acc[4][4];
        zero44(acc);
        mm64<false, true>(acc, sC, sB, tid);
        {
            const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = r0 + i, s = c0 + j;
                    acc[i][j] = s <= t ? acc[i][j] * expf(scum[t] - scum[s]) : 0.f;
                }
        }
        __syncthreads();
        store44(sM, acc, tid);
        __syncthreads();
        // Y = M XS + e^{cum_t} C H^T + D x
        float yo[4][4];
        zero44(yo);
        mm64<false, true>(yo, sC, sH, tid);  // [t][p] = sum_n C[t][n] H[p][n]
        zero44(acc);
        mm64<false, false>(acc, sM, sX, tid);
        {
            const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int t = r0 + i;
                if (t0 + t >= a.L) continue;
                const float et = expf(scum[t]);
                f32x4 o;
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = acc[i][j] + et * yo[i][j] + Dh * sx[t * LD + c0 + j];
                *(f32x4*)(y + (b * a.L + t0 + t) * ldy + h * P + c0) = o;
            }
        }
        // H' = e^{cum_last} H + sum_s e^{cum_last - cum_s} xs_s B_s^T   ([p][n])
        const int nval = (int)min<int64_t>(Q, a.L - t0);
        const float clast = scum[nval - 1];
        __syncthreads();
        for (int e = tid; e < 64 * 64; e += NT) {
            const int r = e >> 6, c = e & 63;
            const float wgt = r < nval ? expf(clast - scum[r]) : 0.f;
            sX[r * LD + c] *= wgt;
        }
        __syncthreads();
        zero44(acc);
        mm64<true, false>(acc, sX, sB, tid);  // [p][n] = sum_s XSw[s][p] B[s][n]
        {
            const float ec = expf(clast);
            const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += ec * sH[(r0 + i) * LD + c0 + j];
        }
        __syncthreads();
        store44(sH, acc, tid);
    }
}

// ------------------------------------------------------------------ SSD backward
// dY fp32 [B*L, ldy] (grad of y), states from the forward. Outputs:
//   dxc fp32 [B*L, ldxc]: dx (head columns, written), dB / dC (atomics over heads)
//   ddt_raw -> dzx[:, d_inner + conv_dim + h] (TD), dA_log / dD / ddt_bias (atomics)
template <typename T, typename TD>
__global__ __launch_bounds__(NT) void ssd_bwd_kernel(MambaArgs a, const T* __restrict__ xc, const T* __restrict__ zx,
                                                     const float* __restrict__ dt_bias, const float* __restrict__ A_log,
                                                     const float* __restrict__ Dp, const float* __restrict__ dY,
                                                     int64_t ldy, const float* __restrict__ states,
                                                     float* __restrict__ dxc, TD* __restrict__ dzx,
                                                     float* __restrict__ gA_log, float* __restrict__ gD,
                                                     float* __restrict__ gdt_bias) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* sx = sm;              // x [t][p]
    float* sXS = sx + 64 * LD;   // dt*x [t][p]
    float* sB = sXS + 64 * LD;   // B [t][n]
    float* sC = sB + 64 * LD;    // C [t][n]
    float* sH = sC + 64 * LD;    // chunk-entry state [p][n]
    float* sdH = sH + 64 * LD;   // grad wrt chunk-exit state [p][n]
    float* sdY = sdH + 64 * LD;  // dY [t][p]
    float* sM = sdY + 64 * LD;   // M [t][s], later dG
    float* sT = sM + 64 * LD;    // scratch 64x64
    float* sdt = sT + 64 * LD;   // dt [64]
    float* scum = sdt + 64;      // cum [64]
    float* sdcum = scum + 64;    // d cum [64]
    float* sred = sdcum + 64;    // reductions [64]
    const int tid = threadIdx.x;
    const int r0 = (tid >> 4) * 4, c0 = (tid & 15) * 4;
    const int64_t b = blockIdx.x / a.nheads, h = blockIdx.x % a.nheads;
    const float A = -expf(A_log[h]);
    const float Dh = Dp[h];
    const int nch = (int)((a.L + Q - 1) / Q);
    const T* xb = xc + b * a.L * a.ldxc;
    float gAacc = 0.f, gDacc = 0.f, gdtb = 0.f;
    for (int e = tid; e < 64 * 64; e += NT) sdH[(e >> 6) * LD + (e & 63)] = 0.f;
    for (int ch = nch - 1; ch >= 0; --ch) {
        const int64_t t0 = (int64_t)ch * Q;
        const int nval = (int)min<int64_t>(Q, a.L - t0);
        __syncthreads();
        const float* st = states + ((b * a.nheads + h) * nch + ch) * (int64_t)(P * N);
        for (int e = tid; e < P * N; e += NT) sH[(e >> 6) * LD + (e & 63)] = st[e];
        load_tile(sx, xb + h * P, a.ldxc, t0, a.L, tid);
        load_tile(sB, xb + a.d_inner, a.ldxc, t0, a.L, tid);
        load_tile(sC, xb + a.d_inner + N, a.ldxc, t0, a.L, tid);
        load_tile(sdY, dY + b * a.L * ldy + h * P, ldy, t0, a.L, tid);
        if (tid < 64) {
            const int64_t t = t0 + tid;
            float d = 0.f;
            if (t < a.L) d = softplus((float)zx[(b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + h] + dt_bias[h]);
            sdt[tid] = d;
            float v = d * A;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float u = __shfl_up(v, o, 64);
                if (tid >= o) v += u;
            }
            scum[tid] = v;
            sdcum[tid] = 0.f;
        }
        __syncthreads();
        for (int e = tid; e < 64 * 64; e += NT) {
            const int r = e >> 6, c = e & 63;
            sXS[r * LD + c] = sx[r * LD + c] * sdt[r];
        }
        const float clast = scum[nval - 1];
        // M = (C B^T) o Lmat
        float acc[4][4];
        zero44(acc);
        mm64<false, true>(acc, sC, sB, tid);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = r0 + i, s = c0 + j;
                acc[i][j] = s <= t ? acc[i][j] * expf(scum[t] - scum[s]) : 0.f;
            }
        __syncthreads();
        store44(sM, acc, tid);
        __syncthreads();
        // dM = dY XS^T (s <= t), dcum from the decay mask: dcum_t += sum_s dM M ; dcum_s -= sum_t dM M
        float dm[4][4];
        zero44(dm);
        mm64<false, true>(dm, sdY, sXS, tid);
        float rowc[4] = {0.f, 0.f, 0.f, 0.f}, colc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = r0 + i, s = c0 + j;
                if (s > t) dm[i][j] = 0.f;
                const float mm = sM[t * LD + s];
                const float q = dm[i][j] * mm;
                rowc[i] += q;
                colc[j] += q;
                // dG = dM o Lmat
                dm[i][j] = s <= t ? dm[i][j] * expf(scum[t] - scum[s]) : 0.f;
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(&sdcum[r0 + i], rowc[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(&sdcum[c0 + j], -colc[j]);
        // dXS = M^T dY  [s][p]
        zero44(acc);
        mm64<true, false>(acc, sM, sdY, tid);
        __syncthreads();
        store44(sM, dm, tid);  // sM := dG
        store44(sT, acc, tid); // sT := dXS (diag part)
        __syncthreads();
        // dC = dG B + e^{cum_t} dY H   ;  dB = dG^T C
        float dC[4][4], dBm[4][4];
        zero44(dC);
        mm64<false, false>(dC, sM, sB, tid);
        float dyh[4][4];
        zero44(dyh);
        mm64<false, false>(dyh, sdY, sH, tid);  // [t][n] = sum_p dY[t][p] H[p][n]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float et = expf(scum[r0 + i]);
#pragma unroll
            for (int j = 0; j < 4; ++j) dC[i][j] += et * dyh[i][j];
        }
        zero44(dBm);
        mm64<true, false>(dBm, sM, sC, tid);  // [s][n] = sum_t dG[t][s] C[t][n]
        // dcum_t += sum_p dY[t][p] Yoff[t][p], Yoff = e^{cum_t} C H^T -> = e^{cum_t} sum_n C[t][n] dyh[t][n]
        {
            float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float et = expf(scum[r0 + i]);
#pragma unroll
                for (int j = 0; j < 4; ++j) rs[i] += et * sC[(r0 + i) * LD + c0 + j] * dyh[i][j];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(&sdcum[r0 + i], rs[i]);
        }
        // state carry: w_s = e^{clast - cum_s}; T1[s][p] = sum_n B[s][n] dH[p][n]
        float t1[4][4];
        zero44(t1);
        mm64<false, true>(t1, sB, sdH, tid);
        float dxs_state[4][4];
        {
            float dws[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int s = r0 + i;
                const float wgt = s < nval ? expf(clast - scum[s]) : 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    dxs_state[i][j] = wgt * t1[i][j];
                    dws[i] += sXS[s * LD + c0 + j] * t1[i][j] * wgt;
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(&sdcum[r0 + i], -dws[i]);
            float tot = dws[0] + dws[1] + dws[2] + dws[3];
            tot = wave_sum(tot);
            if ((tid & 63) == 0) atomicAdd(&sdcum[nval - 1], tot);
        }
        // dB_state[s][n] = w_s sum_p xs[s][p] dH[p][n]
        float tb[4][4];
        zero44(tb);
        mm64<false, false>(tb, sXS, sdH, tid);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = r0 + i;
            const float wgt = s < nval ? expf(clast - scum[s]) : 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) dBm[i][j] += wgt * tb[i][j];
        }
        // dcum_last += sum dH o e^{clast} H
        {
            float q = 0.f;
            const float ec = expf(clast);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) q += sdH[(r0 + i) * LD + c0 + j] * ec * sH[(r0 + i) * LD + c0 + j];
            q = wave_sum(q);
            if ((tid & 63) == 0) atomicAdd(&sdcum[nval - 1], q);
        }
        // dH_in = e^{clast} dH + sum_t e^{cum_t} dY[t][p] C[t][n]   ([p][n])
        float dhin[4][4];
        zero44(dhin);
        // scale dY rows by e^{cum_t} into the scratch (sT holds dXS; use sx slots after x is consumed below)
        __syncthreads();
        // dx / ddt need x; compute them now (dXS total = diag part + state part)
        float ddt_part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = r0 + i;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float dxs = sT[s * LD + c0 + j] + dxs_state[i][j];
                const float xv = sx[s * LD + c0 + j];
                const float dyv = sdY[s * LD + c0 + j];
                ddt_part[i] += dxs * xv;
                gDacc += dyv * xv;
                if (t0 + s < a.L) dxc[(b * a.L + t0 + s) * a.ldxc + h * P + c0 + j] = dxs * sdt[s] + Dh * dyv;
            }
        }
        __syncthreads();
        // sT := e^{cum_t} dY
        for (int e = tid; e < 64 * 64; e += NT) {
            const int r = e >> 6, c = e & 63;
            sT[r * LD + c] = sdY[r * LD + c] * expf(scum[r]);
        }
        __syncthreads();
        mm64<true, false>(dhin, sT, sC, tid);  // [p][n] = sum_t sT[t][p] C[t][n]
        {
            const float ec = expf(clast);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) dhin[i][j] += ec * sdH[(r0 + i) * LD + c0 + j];
        }
        // dB, dC rows -> global (atomics over heads)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = r0 + i;
            if (t0 + t >= a.L) continue;
            float* row = dxc + (b * a.L + t0 + t) * a.ldxc + a.d_inner;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                atomicAdd(row + c0 + j, dBm[i][j]);
                atomicAdd(row + N + c0 + j, dC[i][j]);
            }
        }
        // row-sum of ddt_part over the 16 threads sharing r0
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float v = ddt_part[i];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
            ddt_part[i] = v;
        }
        __syncthreads();
        store44(sdH, dhin, tid);
        // finish per-step scalars: da_t = sum_{tau >= t} dcum_tau ; ddt = A da + sum_p dXS x
        if (tid < 64) sred[tid] = 0.f;
        __syncthreads();
        if ((tid & 15) == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) sred[r0 + i] = ddt_part[i];
        }
        __syncthreads();
        if (tid < 64) {
            // reverse inclusive scan of dcum over the valid steps
            float v = tid < nval ? sdcum[tid] : 0.f;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float u = __shfl_down(v, o, 64);
                if (tid + o < 64) v += u;
            }
            const float da = v;
            const int64_t t = t0 + tid;
            if (tid < nval) {
                const float d = sdt[tid];
                const float ddt = A * da + sred[tid];
                gAacc += d * da;
                const float raw = (float)zx[(b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + h] + dt_bias[h];
                const float draw = ddt * sigm(raw);
                dzx[(b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + h] = (TD)draw;
                gdtb += draw;
            }
        }
    }
    // per-head parameter grads
    gAacc = wave_sum(gAacc);
    gdtb = wave_sum(gdtb);
    gDacc = wave_sum(gDacc);
    if (tid == 0) {
        atomicAdd(gA_log + h, gAacc * A);  // A = -exp(A_log) -> dA/dA_log = A
        atomicAdd(gdt_bias + h, gdtb);
    }
    if ((tid & 63) == 0) atomicAdd(gD + h, gDacc);
}

// ------------------------------------------------------------------ gated RMSNorm
// out = (y * silu(z)) * rstd * w ; one wave per row (d_inner <= 4096)
template <typename TZ, typename TO>
__global__ __launch_bounds__(256) void gnorm_fwd_kernel(const float* __restrict__ y, int64_t ldy,
                                                        const TZ* __restrict__ z, int64_t ldz,
                                                        const float* __restrict__ w, TO* __restrict__ out,
                                                        int64_t ldo, float* __restrict__ rstd, int64_t rows, int dn,
                                                        float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    if (row >= rows) return;
    float ss = 0.f;
    for (int c = lane * 4; c < dn; c += 256) {
        const f32x4 yv = *(const f32x4*)(y + row * ldy + c);
        const f32x4 zv = load4(z + row * ldz + c);
#pragma unroll
        for (int t = 0; t < 4; ++t) { const float g = yv[t] * silu(zv[t]); ss += g * g; }
    }
    const float r = rsqrtf(wave_sum(ss) / dn + eps);
    if (lane == 0) rstd[row] = r;
    for (int c = lane * 4; c < dn; c += 256) {
        const f32x4 yv = *(const f32x4*)(y + row * ldy + c);
        const f32x4 zv = load4(z + row * ldz + c);
        const f32x4 wv = *(const f32x4*)(w + c);
        f32x4 o;
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] = yv[t] * silu(zv[t]) * r * wv[t];
        store4(out + row * ldo + c, o);
    }
}

// dn = dout*w ; dg = r (dn - n mean(dn n)) ; dy = dg silu(z) ; dz = dg y silu'(z) ; dw += dout n
template <typename TZ, typename TD>
__global__ __launch_bounds__(256) void gnorm_bwd_kernel(const float* __restrict__ y, int64_t ldy,
                                                        const TZ* __restrict__ z, int64_t ldz,
                                                        const float* __restrict__ w, const float* __restrict__ rstd,
                                                        const float* __restrict__ dout, int64_t ldd,
                                                        float* __restrict__ dy, TD* __restrict__ dz,
                                                        float* __restrict__ dw, int64_t rows, int dn) {
    const int lane = threadIdx.x & 63;
    // per-thread column partials for dw: block handles a stride of rows
    float pw[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) pw[i] = 0.f;
    for (int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6); row < rows; row += (int64_t)gridDim.x * 4) {
        const float r = rstd[row];
        float s = 0.f;
        for (int c = lane * 4; c < dn; c += 256) {
            const f32x4 yv = *(const f32x4*)(y + row * ldy + c);
            const f32x4 zv = load4(z + row * ldz + c);
            const f32x4 dv = *(const f32x4*)(dout + row * ldd + c);
            const f32x4 wv = *(const f32x4*)(w + c);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float n = yv[t] * silu(zv[t]) * r;
                s += dv[t] * wv[t] * n;
            }
        }
        const float mdn = wave_sum(s) / dn;
        int k = 0;
        for (int c = lane * 4; c < dn; c += 256, ++k) {
            const f32x4 yv = *(const f32x4*)(y + row * ldy + c);
            const f32x4 zv = load4(z + row * ldz + c);
            const f32x4 dv = *(const f32x4*)(dout + row * ldd + c);
            const f32x4 wv = *(const f32x4*)(w + c);
            f32x4 o;
            float zo[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float sg = sigm(zv[t]);
                const float sl = zv[t] * sg;
                const float n = yv[t] * sl * r;
                const float dg = r * (dv[t] * wv[t] - n * mdn);
                o[t] = dg * sl;
                zo[t] = dg * yv[t] * sg * (1.f + zv[t] * (1.f - sg));
                if (k < 16) pw[k * 4 + t] += dv[t] * n;
            }
            *(f32x4*)(dy + row * ldy + c) = o;
            store4(dz + row * ldz + c, (f32x4){zo[0], zo[1], zo[2], zo[3]});
        }
    }
    int k = 0;
    for (int c = lane * 4; c < dn && k < 16; c += 256, ++k)
#pragma unroll
        for (int t = 0; t < 4; ++t) atomicAdd(dw + c + t, pw[k * 4 + t]);
}

MambaArgs mk(int64_t B, int64_t L, int64_t d_inner, int64_t nheads, int64_t ldz, int64_t ldxc) {
    MambaArgs a;
    a.B = B; a.L = L; a.d_inner = d_inner; a.nheads = nheads; a.conv_dim = d_inner + 2 * N; a.ldz = ldz;
    a.ldxc = ldxc;
    return a;
}

constexpr size_t FWD_LDS = (6 * 64 * LD + 128) * sizeof(float);
constexpr size_t BWD_LDS = (9 * 64 * LD + 256) * sizeof(float);

template <typename K>
void allow_lds(K kernel, size_t bytes) {
    hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" size_t msq_mamba_states_size(int64_t B, int64_t L, int64_t nheads) {
    return (size_t)B * nheads * ((L + Q - 1) / Q) * P * N * sizeof(float);
}

#define MAMBA_CHECK()                                                                                         \
    MSQ_CHECK_ARG(B > 0 && L > 0 && nheads > 0 && d_inner == nheads * P && ldz % 4 == 0 && ldxc % 4 == 0,     \
                  "mamba: bad sizes (headdim 64, d_state 64, ld %% 4 == 0)")

extern "C" int msq_mamba_conv_fwd(void* xc, int64_t ldxc, const void* zxbcdt, int64_t ldz, int dtype,
                                  const float* conv_w, const float* conv_b, int64_t B, int64_t L, int64_t d_inner,
                                  int64_t nheads, void* stream) {
    MAMBA_CHECK();
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ldxc);
    const int64_t total = B * L * a.conv_dim;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((conv_fwd_kernel<bf16, bf16>), dim3(grid), dim3(256), 0, s, a, (const bf16*)zxbcdt, conv_w, conv_b, (bf16*)xc);
    else hipLaunchKernelGGL((conv_fwd_kernel<float, float>), dim3(grid), dim3(256), 0, s, a, (const float*)zxbcdt, conv_w, conv_b, (float*)xc);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_ssd_fwd(float* y, int64_t ldy, float* states, const void* xc, int64_t ldxc,
                                 const void* zxbcdt, int64_t ldz, int dtype, const float* dt_bias,
                                 const float* A_log, const float* D, int64_t B, int64_t L, int64_t d_inner,
                                 int64_t nheads, void* stream) {
    MAMBA_CHECK();
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ldxc);
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)(B * nheads));
    allow_lds(ssd_fwd_kernel<bf16>, FWD_LDS);
    allow_lds(ssd_fwd_kernel<float>, FWD_LDS);
    if (dtype == MSQ_BF16) hipLaunchKernelGGL(ssd_fwd_kernel<bf16>, grid, dim3(NT), FWD_LDS, s, a, (const bf16*)xc, (const bf16*)zxbcdt, dt_bias, A_log, D, y, ldy, states);
    else hipLaunchKernelGGL(ssd_fwd_kernel<float>, grid, dim3(NT), FWD_LDS, s, a, (const float*)xc, (const float*)zxbcdt, dt_bias, A_log, D, y, ldy, states);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_gnorm_fwd(void* out, int64_t ldo, float* rstd, const float* y, int64_t ldy,
                                   const void* zxbcdt, int64_t ldz, int dtype, const float* w, int64_t rows,
                                   int64_t d_inner, float eps, void* stream) {
    MSQ_CHECK_ARG(rows > 0 && d_inner % 4 == 0 && d_inner <= 4096, "mamba gnorm: bad sizes");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((gnorm_fwd_kernel<bf16, bf16>), grid, dim3(256), 0, s, y, ldy, (const bf16*)zxbcdt, ldz, w, (bf16*)out, ldo, rstd, rows, (int)d_inner, eps);
    else hipLaunchKernelGGL((gnorm_fwd_kernel<float, float>), grid, dim3(256), 0, s, y, ldy, (const float*)zxbcdt, ldz, w, (float*)out, ldo, rstd, rows, (int)d_inner, eps);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_gnorm_bwd(float* dy, void* dzxbcdt, const float* y, int64_t ldy, const void* zxbcdt,
                                   int64_t ldz, int dtype, const float* w, const float* rstd, const float* dout,
                                   int64_t ldd, float* dw, int64_t rows, int64_t d_inner, void* stream) {
    MSQ_CHECK_ARG(rows > 0 && d_inner % 4 == 0 && d_inner <= 4096, "mamba gnorm bwd: bad sizes");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(1024);
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((gnorm_bwd_kernel<bf16, bf16>), grid, dim3(256), 0, s, y, ldy, (const bf16*)zxbcdt, ldz, w, rstd, dout, ldd, dy, (bf16*)dzxbcdt, dw, rows, (int)d_inner);
    else hipLaunchKernelGGL((gnorm_bwd_kernel<float, float>), grid, dim3(256), 0, s, y, ldy, (const float*)zxbcdt, ldz, w, rstd, dout, ldd, dy, (float*)dzxbcdt, dw, rows, (int)d_inner);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_ssd_bwd(float* dxc, int64_t ld_dxc, void* dzxbcdt, const float* dY, int64_t ldy,
                                 const float* states, const void* xc, int64_t ldxc, const void* zxbcdt, int64_t ldz,
                                 int dtype, const float* dt_bias, const float* A_log, const float* D, float* gA_log,
                                 float* gD, float* gdt_bias, int64_t B, int64_t L, int64_t d_inner, int64_t nheads,
                                 void* stream) {
    MAMBA_CHECK();
    MSQ_CHECK_ARG(ld_dxc == ldxc, "msq_mamba_ssd_bwd: dxc must share the xBC row stride");
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ldxc);
    hipStream_t s = (hipStream_t)stream;
    // dB / dC columns are accumulated with atomics across heads
    hipMemset2DAsync(dxc + d_inner, ldxc * sizeof(float), 0, 2 * N * sizeof(float), B * L, s);
    const dim3 grid((unsigned)(B * nheads));
    allow_lds(ssd_bwd_kernel<bf16, bf16>, BWD_LDS);
    allow_lds(ssd_bwd_kernel<float, float>, BWD_LDS);
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((ssd_bwd_kernel<bf16, bf16>), grid, dim3(NT), BWD_LDS, s, a, (const bf16*)xc, (const bf16*)zxbcdt, dt_bias, A_log, D, dY, ldy, states, dxc, (bf16*)dzxbcdt, gA_log, gD, gdt_bias);
    else hipLaunchKernelGGL((ssd_bwd_kernel<float, float>), grid, dim3(NT), BWD_LDS, s, a, (const float*)xc, (const float*)zxbcdt, dt_bias, A_log, D, dY, ldy, states, dxc, (float*)dzxbcdt, gA_log, gD, gdt_bias);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_conv_bwd(void* dzxbcdt, const float* dxc, int64_t ld_dxc, const void* zxbcdt, int64_t ldz,
                                  int dtype, const float* conv_w, const float* conv_b, float* g_conv_w,
                                  float* g_conv_b, int64_t B, int64_t L, int64_t d_inner, int64_t nheads,
                                  void* stream) {
    MSQ_CHECK_ARG(B > 0 && L > 0 && d_inner == nheads * P && ldz % 4 == 0, "mamba conv bwd: bad sizes");
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ld_dxc);
    hipStream_t s = (hipStream_t)stream;
    const unsigned tch = (unsigned)std::max<int64_t>(1, std::min<int64_t>(64, L / 64));
    const dim3 grid((unsigned)((a.conv_dim + 63) / 64), (unsigned)B, tch);
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((conv_bwd_kernel<bf16, bf16>), grid, dim3(256), 0, s, a, (const bf16*)zxbcdt, conv_w, conv_b, dxc, ld_dxc, (bf16*)dzxbcdt, g_conv_w, g_conv_b);
    else hipLaunchKernelGGL((conv_bwd_kernel<float, float>), grid, dim3(256), 0, s, a, (const float*)zxbcdt, conv_w, conv_b, dxc, ld_dxc, (float*)dzxbcdt, g_conv_w, g_conv_b);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
