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
#include "attn_tiles.h"
#include <type_traits>

namespace {

constexpr int NT = 256;
constexpr int Q = 64;   // chunk length
constexpr int P = 64;   // head dim
constexpr int N = 64;   // state dim
constexpr int LD = 68;  // LDS row stride (floats) for 64x64 tiles

struct MambaArgs {
    int64_t B, L, d_inner, nheads, conv_dim, ldz;  // ldz: row stride of zxbcdt
    int64_t ldxc;                                  // row stride of the conv output (xBC)
    // chunk kernels: XCD-aware block order, the heads of one (b, chunk) on one
    // XCD (they share the chunk's B / C rows)
    int xcd;
};

// sigmoid by one v_exp_f32 and one v_rcp_f32 (~1 ulp each; the library expf
// and the IEEE division cost ~25 VALU per element); mamba_step.hip's silu is
// the same expression, so the cached decode step matches the forward
__device__ __forceinline__ float sigm(float x) {
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float silu(float x) { return x * sigm(x); }
__device__ __forceinline__ float softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }
// e^x of a log-decay (cum / segment sums, x <= 0 wherever the value is used) as
// one v_exp_f32 of x log2(e): the library expf's range reduction and
// over/underflow selects cost ~14 VALU per value in the chunk-pair loops
constexpr float LOG2E_F = 1.4426950408889634f;
__device__ __forceinline__ float exp_decay(float x) { return __builtin_amdgcn_exp2f(x * LOG2E_F); }
// cross-lane sums and scans in VALU (DPP / permlane) instead of ds_bpermute
// round trips (__shfl_xor / __shfl_up: an LDS-latency wait per step)
template <int CTRL, int ROWS = 0xF, bool BOUND = true>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROWS, 0xF, BOUND));
}
// sum over the 16 lanes of a row, in every lane: quad xor 1, xor 2, half-row
// mirror (quad q with its neighbour), row mirror (half with half)
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    return v;
}
// sum over the lanes l, l ^ 16, l ^ 32, l ^ 48
__device__ __forceinline__ float cross4_sum(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float wave_sum_dpp(float v) { return cross4_sum(row16_sum(v)); }
// inclusive prefix sum over the 64 lanes: row_shr 1 / 2 / 4 / 8 within the
// 16-lane rows (lanes without a source add 0), then row_bcast:15 (each row's
// last lane into rows 1 and 3) and row_bcast:31 (lane 31 into rows 2 and 3)
__device__ __forceinline__ float wave_scan_dpp(float v) {
    v += dpp_f<0x111>(v);
    v += dpp_f<0x112>(v);
    v += dpp_f<0x114>(v);
    v += dpp_f<0x118>(v);
    v += dpp_f<0x142, 0xA, false>(v);
    v += dpp_f<0x143, 0xC, false>(v);
    return v;
}

// ------------------------------------------------------------------ conv
// out[b,t,c] = silu(bias[c] + sum_k w[c,k] * in[b, t-3+k, c]), in = zxbcdt[:, off + c]
// block: 64 lanes x 2 channels each (4-B bf16 / 8-B fp32 loads and stores: a wave
// instruction moves 128 channels of one time step) x 4 waves, each wave a
// contiguous segment of CONV_SEG steps with a sliding 4-tap window (one load per
// input element). Per channel the arithmetic is the scalar form's, in its order.
// Measured per step (cfg 3, same box): 1 channel per lane, 64 steps 2.71 ms;
// 2 channels, 32 steps 2.47 (64 steps: the same); 4 channels (222 VGPRs in the
// backward) 3.38.
constexpr int CONV_SEG = 32;
constexpr int CONV_U = 8;
constexpr int CONV_CV = 2;  // channels per lane
typedef float f32x2c __attribute__((ext_vector_type(2)));
typedef f32x2c conv_vec;
template <typename T>
using conv_raw_t = typename std::conditional<sizeof(T) == 2, uint32_t, f32x2c>::type;
template <typename T>
__device__ __forceinline__ conv_raw_t<T> conv_ld(const T* p) {
    return *(const conv_raw_t<T>*)p;
}
__device__ __forceinline__ conv_vec conv_widen(uint32_t v) {
    return (conv_vec){__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
}
__device__ __forceinline__ conv_vec conv_widen(f32x2c v) { return v; }
__device__ __forceinline__ void conv_st(bf16* p, conv_vec v) {
    union { uint32_t u; bf16 e[2]; } h;
    h.e[0] = (bf16)v[0];
    h.e[1] = (bf16)v[1];
    *(uint32_t*)p = h.u;
}
__device__ __forceinline__ void conv_st(float* p, conv_vec v) { *(f32x2c*)p = v; }

template <typename T, typename TO>
__global__ __launch_bounds__(256) void conv_fwd_kernel(MambaArgs a, const T* __restrict__ zx, const float* __restrict__ w,
                                                       const float* __restrict__ bias, TO* __restrict__ out) {
    const int lane = threadIdx.x & 63, ws = threadIdx.x >> 6;
    const int64_t c = (blockIdx.x * 64 + lane) * CONV_CV;
    const int64_t b = blockIdx.y;
    const int64_t t0 = ((int64_t)blockIdx.z * 4 + ws) * CONV_SEG, t1 = min(a.L, t0 + CONV_SEG);
    if (c >= a.conv_dim || t0 >= a.L) return;
    const T* src = zx + b * a.L * a.ldz + a.d_inner + c;
    TO* dst = out + b * a.L * a.ldxc + c;
    conv_vec wk[4], win[4], bc;
#pragma unroll
    for (int v = 0; v < CONV_CV; ++v) {
#pragma unroll
        for (int k = 0; k < 4; ++k) wk[k][v] = w[(c + v) * 4 + k];
        bc[v] = bias[c + v];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t tt = t0 - 3 + k;
        win[k + 1] = tt >= 0 ? conv_widen(conv_ld(src + tt * a.ldz)) : (conv_vec){0.f, 0.f};
    }
    // CONV_U steps per batch: their loads are issued together (clamped to the
    // segment, so no branch skips one), then the sliding window runs over them
    for (int64_t tb = t0; tb < t1; tb += CONV_U) {
        conv_raw_t<T> xin[CONV_U];
#pragma unroll
        for (int u = 0; u < CONV_U; ++u) xin[u] = conv_ld(src + min(tb + u, t1 - 1) * a.ldz);
#pragma unroll
        for (int u = 0; u < CONV_U; ++u) {
#pragma unroll
            for (int k = 0; k < 3; ++k) win[k] = win[k + 1];
            win[3] = conv_widen(xin[u]);
            conv_vec o;
#pragma unroll
            for (int v = 0; v < CONV_CV; ++v) {
                float acc = bc[v];
#pragma unroll
                for (int k = 0; k < 4; ++k) acc += wk[k][v] * win[k][v];
                o[v] = silu(acc);
            }
            if (tb + u < t1) conv_st(dst + (tb + u) * a.ldxc, o);
        }
    }
}

// dpre = dout * silu'(pre); dzx_in[t] = sum_k w[k] dpre[t+3-k]; dw, dbias via per-block partials (atomics)
// block: 64 lanes x 4 channels x 4 waves; wave ws walks the contiguous time
// segment [t0, t1) of CONV_SEG steps with a sliding window: each input and each
// dout is loaded once (plus a 3-step halo), pre / dpre computed once per step.
template <typename T, typename TD>
__global__ __launch_bounds__(256) void conv_bwd_kernel(MambaArgs a, const T* __restrict__ zx, const float* __restrict__ w,
                                                       const float* __restrict__ bias, const float* __restrict__ dout,
                                                       int64_t ldd, TD* __restrict__ dzx, float* __restrict__ dw,
                                                       float* __restrict__ dbias) {
    __shared__ conv_vec red[4][5][64];
    const int lane = threadIdx.x & 63, ws = threadIdx.x >> 6;
    const int64_t c = (blockIdx.x * 64 + lane) * CONV_CV;
    const int64_t b = blockIdx.y;
    const int64_t t0 = ((int64_t)blockIdx.z * 4 + ws) * CONV_SEG, t1 = min(a.L, t0 + CONV_SEG);
    const conv_vec z4 = (conv_vec){0.f, 0.f};
    conv_vec gw[4] = {z4, z4, z4, z4}, gb = z4;
    if (c < a.conv_dim && t0 < a.L) {
        const T* src = zx + b * a.L * a.ldz + a.d_inner + c;
        const float* dsrc = dout + b * a.L * ldd + c;
        conv_vec wk[4], bc;
#pragma unroll
        for (int v = 0; v < CONV_CV; ++v) {
#pragma unroll
            for (int k = 0; k < 4; ++k) wk[k][v] = w[(c + v) * 4 + k];
            bc[v] = bias[c + v];
        }
        // input window in[tau-3 .. tau], dpre ring of tau-3 .. tau
        conv_vec win[4], dp[4] = {z4, z4, z4, z4};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int64_t tt = t0 - 3 + k;
            win[k + 1] = tt >= 0 ? conv_widen(conv_ld(src + tt * a.ldz)) : z4;
        }
        const int64_t tend = min(a.L, t1 + 3);
        // CONV_U steps per batch, their input / dout loads issued together
        // (clamped to tend - 1: no branch skips a load)
        for (int64_t tb = t0; tb < t1 + 3; tb += CONV_U) {
            conv_raw_t<T> xin[CONV_U];
            conv_vec dyin[CONV_U];
#pragma unroll
            for (int u = 0; u < CONV_U; ++u) {
                const int64_t tl = min(tb + u, tend - 1);
                xin[u] = conv_ld(src + tl * a.ldz);
                dyin[u] = *(const conv_vec*)(dsrc + tl * ldd);
            }
#pragma unroll
            for (int u = 0; u < CONV_U; ++u) {
                const int64_t tau = tb + u;
                if (tau >= t1 + 3) break;
#pragma unroll
                for (int k = 0; k < 3; ++k) win[k] = win[k + 1], dp[k] = dp[k + 1];
                conv_vec d = z4;
                if (tau < tend) {
                    win[3] = conv_widen(xin[u]);
#pragma unroll
                    for (int v = 0; v < CONV_CV; ++v) {
                        float pre = bc[v];
#pragma unroll
                        for (int k = 0; k < 4; ++k) pre += wk[k][v] * win[k][v];
                        const float sg = sigm(pre);
                        d[v] = dyin[u][v] * sg * (1.f + pre * (1.f - sg));
                    }
                    if (tau < t1) {
                        gb += d;
#pragma unroll
                        for (int k = 0; k < 4; ++k) gw[k] += d * win[k];
                    }
                } else {
                    win[3] = z4;
                }
                dp[3] = d;
                // dzx_in[tau - 3] = sum_k w[k] dpre[tau - k]
                const int64_t t = tau - 3;
                if (t >= t0 && t < t1) {
                    conv_vec di = z4;
#pragma unroll
                    for (int k = 0; k < 4; ++k) di += wk[k] * dp[3 - k];
                    conv_st(dzx + (b * a.L + t) * a.ldz + a.d_inner + c, di);
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[ws][k][lane] = gw[k];
    red[ws][4][lane] = gb;
    __syncthreads();
    if (ws == 0 && c < a.conv_dim) {
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const conv_vec v = red[0][k][lane] + red[1][k][lane] + red[2][k][lane] + red[3][k][lane];
#pragma unroll
            for (int e = 0; e < CONV_CV; ++e) {
                if (k < 4) atomicAdd(dw + (c + e) * 4 + k, v[e]);
                else atomicAdd(dbias + c + e, v[e]);
            }
        }
    }
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
                                                     float* __restrict__ y, int64_t ldy, float* __restrict__ states,
                                                     float* __restrict__ fin) {
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
    if (fin) {  // state after the last position (cached decode)
        __syncthreads();
        float* f = fin + (b * a.nheads + h) * (int64_t)(P * N);
        for (int e = tid; e < P * N; e += NT) f[e] = sH[(e >> 6) * LD + (e & 63)];
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
// out = (y * silu(z)) * rstd * w ; one wave per row (d_inner <= 4096); y is in
// the compute dtype, like z (bf16 in the bf16 path, as mamba_ssm stores it)
template <typename TZ, typename TO>
__global__ __launch_bounds__(256) void gnorm_fwd_kernel(const TZ* __restrict__ y, int64_t ldy,
                                                        const TZ* __restrict__ z, int64_t ldz,
                                                        const float* __restrict__ w, TO* __restrict__ out,
                                                        int64_t ldo, float* __restrict__ rstd, int64_t rows, int dn,
                                                        float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    if (row >= rows) return;
    float ss = 0.f;
    for (int c = lane * 4; c < dn; c += 256) {
        const f32x4 yv = load4(y + row * ldy + c);
        const f32x4 zv = load4(z + row * ldz + c);
#pragma unroll
        for (int t = 0; t < 4; ++t) { const float g = yv[t] * silu(zv[t]); ss += g * g; }
    }
    const float r = rsqrtf(wave_sum(ss) / dn + eps);
    if (lane == 0) rstd[row] = r;
    for (int c = lane * 4; c < dn; c += 256) {
        const f32x4 yv = load4(y + row * ldy + c);
        const f32x4 zv = load4(z + row * ldz + c);
        const f32x4 wv = *(const f32x4*)(w + c);
        f32x4 o;
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] = yv[t] * silu(zv[t]) * r * wv[t];
        store4(out + row * ldo + c, o);
    }
}

// decode rows (few rows): one 256-thread block per row, the row in registers
// (NK = ceil(dn / 1024) <= 4 float4 per thread), one block reduction
template <typename TZ, typename TO, int NK>
__global__ __launch_bounds__(256) void gnorm_fwd_row_kernel(const TZ* __restrict__ y, int64_t ldy,
                                                            const TZ* __restrict__ z, int64_t ldz,
                                                            const float* __restrict__ w, TO* __restrict__ out,
                                                            int64_t ldo, float* __restrict__ rstd, int dn, float eps) {
    __shared__ float red[4];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    f32x4 gv[NK];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const int c = tid * 4 + k * 1024;
        if (c < dn) {
            const f32x4 yv = load4(y + row * ldy + c);
            const f32x4 zv = load4(z + row * ldz + c);
#pragma unroll
            for (int t = 0; t < 4; ++t) { gv[k][t] = yv[t] * silu(zv[t]); ss += gv[k][t] * gv[k][t]; }
        }
    }
    ss = wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    const float r = rsqrtf(((red[0] + red[1]) + (red[2] + red[3])) / dn + eps);
    if (tid == 0) rstd[row] = r;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const int c = tid * 4 + k * 1024;
        if (c < dn) {
            const f32x4 wv = *(const f32x4*)(w + c);
            f32x4 o;
#pragma unroll
            for (int t = 0; t < 4; ++t) o[t] = gv[k][t] * r * wv[t];
            store4(out + row * ldo + c, o);
        }
    }
}

// dn = dout*w ; dg = r (dn - n mean(dn n)) ; dy = dg silu(z) ; dz = dg y silu'(z) ; dw += dout n
// One wave per row, the row's y / z / dout held in registers (one HBM pass):
// lane owns columns 4 lane + 256 k, k < NK (NK = ceil(d_inner / 256), compile time).
constexpr int GN_K = 16;
template <typename TZ, typename TD, int NK>
__global__ __launch_bounds__(256, (NK >= 8 ? 2 : 1)) void gnorm_bwd_kernel(
    const TZ* __restrict__ y, int64_t ldy, const TZ* __restrict__ z, int64_t ldz, const float* __restrict__ w,
    const float* __restrict__ rstd, const float* __restrict__ dout, int64_t ldd, TZ* __restrict__ dy,
    TD* __restrict__ dz, float* __restrict__ dw, int64_t rows, int dn) {
    // bf16 y / z are held as their raw bits (8 B per 4 columns) and widened at
    // each use, so every load of a row is issued in one burst before the row's
    // reduction and none after it; the dw partials live in each wave's LDS slice
    // (lane-owned columns). At d_inner > 1024 that is 2 waves per SIMD without
    // spills (measured 0.27 ms per step faster than 3 waves with 22 spilled
    // VGPRs, and 0.42 ms faster than re-reading z after the reduction). ZRE
    // (fp32 z): z is read again in the second pass instead of held.
    constexpr bool RAW = sizeof(TZ) == 2;
    constexpr bool ZRE = NK >= 8 && !RAW;
    typedef typename std::conditional<RAW, uint2, f32x4>::type raw4;
    auto ld_raw = [](const TZ* p) -> raw4 {
        if constexpr (RAW) return *(const uint2*)p;
        else return *(const f32x4*)p;
    };
    auto widen = [](raw4 v) -> f32x4 {
        if constexpr (RAW)
            return (f32x4){__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                           __uint_as_float(v.y & 0xffff0000u)};
        else return v;
    };
    const int lane = threadIdx.x & 63, ws = threadIdx.x >> 6;
    __shared__ f32x4 red[4][64 * NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) red[ws][lane + 64 * k] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int64_t row = blockIdx.x * 4LL + ws; row < rows; row += (int64_t)gridDim.x * 4) {
        const float r = rstd[row];
        raw4 yv[NK], zv[ZRE ? 1 : NK];
        f32x4 dv[NK];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int c = lane * 4 + 256 * k;
            yv[k] = raw4{};
            dv[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (!ZRE) zv[k] = raw4{};
            if (c < dn) {
                yv[k] = ld_raw(y + row * ldy + c);
                dv[k] = *(const f32x4*)(dout + row * ldd + c);
                if (!ZRE) zv[k] = ld_raw(z + row * ldz + c);
            }
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int c = lane * 4 + 256 * k;
            if (c >= dn) continue;
            const f32x4 wv = *(const f32x4*)(w + c);
            const f32x4 zk = ZRE ? load4(z + row * ldz + c) : widen(zv[ZRE ? 0 : k]);
            const f32x4 yk = widen(yv[k]);
#pragma unroll
            for (int t = 0; t < 4; ++t) s += dv[k][t] * wv[t] * yk[t] * silu(zk[t]) * r;
        }
        const float mdn = wave_sum(s) / dn;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int c = lane * 4 + 256 * k;
            if (c >= dn) continue;
            const f32x4 wv = *(const f32x4*)(w + c);
            const f32x4 zk = ZRE ? load4(z + row * ldz + c) : widen(zv[ZRE ? 0 : k]);
            const f32x4 yk = widen(yv[k]);
            f32x4 o, zo, pw = red[ws][lane + 64 * k];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float sg = sigm(zk[t]);
                const float sl = zk[t] * sg;
                const float n = yk[t] * sl * r;
                const float dg = r * (dv[k][t] * wv[t] - n * mdn);
                o[t] = dg * sl;
                zo[t] = dg * yk[t] * sg * (1.f + zk[t] * (1.f - sg));
                pw[t] += dv[k][t] * n;
            }
            red[ws][lane + 64 * k] = pw;
            store4(dy + row * ldy + c, o);
            store4(dz + row * ldz + c, zo);
        }
    }
    // dw: the 4 waves' column partials summed, then one atomic per column per block
    __syncthreads();
    const float* rf = (const float*)red;
    for (int c = threadIdx.x; c < dn; c += 256) {
        const int i = ((c % 256) / 4 + 64 * (c / 256)) * 4 + c % 4;  // column c: red[w][l + 64 k][t]
        atomicAdd(dw + c, rf[i] + rf[64 * NK * 4 + i] + rf[2 * 64 * NK * 4 + i] + rf[3 * 64 * NK * 4 + i]);
    }
}

// The same backward with each row split over a pair of waves (bf16 y / z, dn in
// (256 (NKH - 1) * 2, 512 NKH]): wave h of pair q owns columns 4 lane + 256 (h NKH
// + k), k < NKH, so a lane holds half the row (114 VGPRs at NKH = 4: 4 waves per
// SIMD instead of 2). The row's sum is the two waves' sums through LDS (double
// buffered by iteration, one barrier per row pair); every wave runs the same
// number of iterations (rows past the end skip their loads and stores).
template <typename TD, int NKH>
__global__ __launch_bounds__(256, 3) void gnorm_bwd2_kernel(
    const bf16* __restrict__ y, int64_t ldy, const bf16* __restrict__ z, int64_t ldz, const float* __restrict__ w,
    const float* __restrict__ rstd, const float* __restrict__ dout, int64_t ldd, bf16* __restrict__ dy,
    TD* __restrict__ dz, float* __restrict__ dw, int64_t rows, int dn) {
    auto widen = [](uint2 v) -> f32x4 {
        return (f32x4){__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                       __uint_as_float(v.y & 0xffff0000u)};
    };
    const int lane = threadIdx.x & 63, ws = threadIdx.x >> 6, q = ws >> 1, h = ws & 1;
    __shared__ f32x4 red[4][64 * NKH];
    __shared__ f32x4 sw[2 * 64 * NKH];  // w, read from LDS in the loop (a global load there
                                        // would wait, in order, for the prefetched rows)
    __shared__ float sred[2][2][2];  // [iteration parity][pair][half]
#pragma unroll
    for (int k = 0; k < NKH; ++k) red[ws][lane + 64 * k] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int e = threadIdx.x; e < 2 * 64 * NKH; e += 256)
        sw[e] = 4 * e < dn ? *(const f32x4*)(w + 4 * e) : (f32x4){0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    // the next row pair's y / z / dout / rstd are loaded while this pair is
    // reduced and written (one pair at a time it waited on every load: the
    // LayerNorm backward's fix, round 6)
    uint2 nyv[NKH], nzv[NKH];
    f32x4 ndv[NKH];
    float nr = 0.f;
    // (unconditional loads from a clamped row / column: exec-masked loads made
    // the compiler wait vmcnt(0) for the prefetch at every use; rows past the
    // end are skipped below, columns past dn are never stored)
    auto fetch = [&](int64_t row) {
        const int64_t rr = row < rows ? row : rows - 1;
        nr = rstd[rr];
#pragma unroll
        for (int k = 0; k < NKH; ++k) {
            const int c = min(lane * 4 + 256 * (h * NKH + k), dn - 4);
            nyv[k] = *(const uint2*)(y + rr * ldy + c);
            ndv[k] = *(const f32x4*)(dout + rr * ldd + c);
            nzv[k] = *(const uint2*)(z + rr * ldz + c);
        }
    };
    const int64_t stride = (int64_t)gridDim.x * 2;
    int it = 0;
    fetch(blockIdx.x * 2LL + q);
    for (int64_t base = blockIdx.x * 2LL; base < rows; base += stride, ++it) {
        const int64_t row = base + q;
        const bool ok = row < rows;
        const float r = nr;
        uint2 yv[NKH], zv[NKH];
        f32x4 dv[NKH];
#pragma unroll
        for (int k = 0; k < NKH; ++k) {
            yv[k] = nyv[k];
            zv[k] = nzv[k];
            dv[k] = ndv[k];
        }
        fetch(row + stride);
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NKH; ++k) {
            const int c = lane * 4 + 256 * (h * NKH + k);
            if (c >= dn) continue;
            const f32x4 wv = sw[c / 4];
            const f32x4 zk = widen(zv[k]), yk = widen(yv[k]);
#pragma unroll
            for (int t = 0; t < 4; ++t) s += dv[k][t] * wv[t] * yk[t] * silu(zk[t]) * r;
        }
        s = wave_sum(s);
        if (lane == 0) sred[it & 1][q][h] = s;
        // (a raw barrier: the fence of __syncthreads would wait for the next
        // pair's loads, vmcnt(0))
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const float mdn = (sred[it & 1][q][0] + sred[it & 1][q][1]) / dn;
        if (!ok) continue;
#pragma unroll
        for (int k = 0; k < NKH; ++k) {
            const int c = lane * 4 + 256 * (h * NKH + k);
            if (c >= dn) continue;
            const f32x4 wv = sw[c / 4];
            const f32x4 zk = widen(zv[k]), yk = widen(yv[k]);
            f32x4 o, zo, pw = red[ws][lane + 64 * k];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float sg = sigm(zk[t]);
                const float sl = zk[t] * sg;
                const float n = yk[t] * sl * r;
                const float dg = r * (dv[k][t] * wv[t] - n * mdn);
                o[t] = dg * sl;
                zo[t] = dg * yk[t] * sg * (1.f + zk[t] * (1.f - sg));
                pw[t] += dv[k][t] * n;
            }
            red[ws][lane + 64 * k] = pw;
            store4(dy + row * ldy + c, o);
            store4(dz + row * ldz + c, zo);
        }
    }
    // dw: column c's partials sit with wave h = (c / 256) / NKH of both pairs
    __syncthreads();
    const float* rf = (const float*)red;
    for (int c = threadIdx.x; c < dn; c += 256) {
        const int kk = c / 256, hh = kk / NKH, k = kk % NKH;
        const int i = ((c % 256) / 4 + 64 * k) * 4 + c % 4;
        atomicAdd(dw + c, rf[hh * 64 * NKH * 4 + i] + rf[(2 + hh) * 64 * NKH * 4 + i]);
    }
}

template <typename TZ, typename TD>
void gnorm_bwd_launch(dim3 grid, hipStream_t s, const TZ* y, int64_t ldy, const TZ* z, int64_t ldz, const float* w,
                      const float* rstd, const float* dout, int64_t ldd, TZ* dy, TD* dz, float* dw, int64_t rows,
                      int dn) {
    const int need = (dn + 255) / 256;
#define GN(K) hipLaunchKernelGGL((gnorm_bwd_kernel<TZ, TD, K>), grid, dim3(256), 0, s, y, ldy, z, ldz, w, rstd, dout, \
                                 ldd, dy, dz, dw, rows, dn)
    if (need <= 1) GN(1);
    else if (need <= 2) GN(2);
    else if (need <= 4) GN(4);
    else if (need <= 8) GN(8);
    else GN(16);
#undef GN
}

MambaArgs mk(int64_t B, int64_t L, int64_t d_inner, int64_t nheads, int64_t ldz, int64_t ldxc) {
    MambaArgs a;
    a.B = B; a.L = L; a.d_inner = d_inner; a.nheads = nheads; a.conv_dim = d_inner + 2 * N; a.ldz = ldz;
    a.ldxc = ldxc;
    a.xcd = 1;  // the chunk kernels walk one (b, chunk)'s heads on one XCD (chunk_of)
    return a;
}

constexpr size_t FWD_LDS = (6 * 64 * LD + 128) * sizeof(float);
constexpr size_t BWD_LDS = (9 * 64 * LD + 256) * sizeof(float);

template <typename K>
void allow_lds(K kernel, size_t bytes) {
    hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}


// ================================================================== SSD, bf16 MFMA chunk-parallel path
// The sequential walk over chunks above keeps one workgroup per (batch, head)
// busy for the whole sequence with fp32 FMA products read from LDS. The bf16
// path splits the same SSD block form (mamba_ssm's chunk_state / state_passing
// / chunk_scan) into three launches:
//   state : per (b, h, chunk)  S_c = sum_s e^{cum_last - cum_s} dt_s x_s B_s^T    [p][n]
//   pass  : per (b, h, p, n)   H_c = entry state: H_0 = 0, H_{c+1} = e^{cum_last_c} H_c + S_c
//                              (in place over S; the entry states are what the backward reads)
//   out   : per (b, h, chunk)  y = (C B^T o L) (dt x) + e^{cum_t} C H_c^T + D x
// with every 64x64x64 product on v_mfma_f32_16x16x32_bf16 (bf16 operands -- x, B, C
// are the bf16 conv output; dt x, the decay-masked C B^T and H are rounded to bf16 as
// mamba_ssm's Triton kernels do -- fp32 accumulation). Tiles live in LDS as 64-row
// images with 256-B rows in the dual swizzle of cdna_hip_programming.md T10 (b), read
// either as K-contiguous rows (ds_read_b128) or transposed (ds_read_b64_tr_b16).
namespace ssd2 {
using attn::cat8;
using attn::tr_read;
constexpr int IMG = 64 * 256;  // bytes of one tile image

__device__ __forceinline__ int offd(int row, int ch) {
    return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}
// An image holds two 64-column tiles side by side: half 0 in chunks 0-7, half 1
// in chunks 8-15 (offd is a bijection on (row, chunk), so they never collide).
// K-contiguous fragment: image rows rb .. rb+15, k = 32 ks + 8 g .. +7 of tile half hf
__device__ __forceinline__ bf16x8 fk(const char* s, int rb, int ks, int lane, int hf) {
    return *(const bf16x8*)(s + offd(rb + (lane & 15), 8 * hf + ks * 4 + (lane >> 4)));
}
// transposed fragment: image rows are k (32 ks + 8 g + 0..3 / 4..7), columns cb + (lane & 15)
// of tile half hf
__device__ __forceinline__ bf16x8 fm(const char* s, int cb, int ks, int lane, int hf) {
    const int i = lane & 15, q = i >> 2, pp = i & 3, g = lane >> 4;
    const int kA = ks * 32 + 8 * g + q, ch = 8 * hf + (cb >> 3) + (pp >> 1), sub = (pp & 1) * 8;
    return cat8(tr_read(s, offd(kA, ch) + sub), tr_read(s, offd(kA + 4, ch) + sub));
}
// acc[i][j] (lane (il, g), element r) = sum_k A[rb + 16 i + il][k] Bt[cb + 16 j + 4 g + r][k]
// over k < 64; A rows from image sa (K-contiguous, or transposed when AT), Bt rows likewise
template <bool AT, bool BT, int NJ = 2>
__device__ __forceinline__ void mm(f32x4 (&acc)[2][NJ], const char* sa, int ha, const char* sb, int hb, int rb, int cb,
                                   int lane) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        bf16x8 av[2], bv[NJ];
#pragma unroll
        for (int i = 0; i < 2; ++i)
            av[i] = AT ? fm(sa, rb + 16 * i, ks, lane, ha) : fk(sa, rb + 16 * i, ks, lane, ha);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            bv[j] = BT ? fm(sb, cb + 16 * j, ks, lane, hb) : fk(sb, cb + 16 * j, ks, lane, hb);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[i][j] = attn::mfma(bv[j], av[i], acc[i][j]);
    }
}
__device__ __forceinline__ void zero22(f32x4 (&a)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) a[i][j] = attn::zero4();
}
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
    union { u32x4 u; bf16 e[8]; } r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.e[k] = (bf16)v[k];
    return r.u;
}
__device__ __forceinline__ uint64_t pack4(f32x4 v) {
    union { uint64_t u; bf16 e[4]; } r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r.e[k] = (bf16)v[k];
    return r.u;
}
__device__ __forceinline__ void unpack8(u32x4 u, float (&v)[8]) {
    union { u32x4 u; bf16 e[8]; } r;
    r.u = u;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (float)r.e[k];
}

// chunk geometry + dt / cumulative decay of one (b, h, chunk); threads 0..63 (wave 0)
struct Chunk {
    int64_t b, h, c, t0;
    int nval;
};
// hg > 1: one workgroup per group of hg heads (k.h = the group's first head)
__device__ __forceinline__ Chunk chunk_of(const MambaArgs& a, int nch, int hg = 1) {
    Chunk k;
    // 32-bit quotients (grid ids are 32-bit; the 64-bit forms expand to a
    // long scalar division sequence per workgroup)
    const uint32_t ng = (uint32_t)(a.nheads / hg), nc = (uint32_t)nch;
    if (a.xcd) {  // logical id (h fastest, then chunk, then b), contiguous per XCD
        const uint32_t id = __builtin_amdgcn_readfirstlane(xcd_remap((int)blockIdx.x, (int)gridDim.x));
        k.h = (int64_t)(id % ng) * hg;
        const uint32_t r = id / ng;
        k.c = r % nc;
        k.b = r / nc;
    } else {
        const uint32_t bh = blockIdx.x / nc;
        k.c = blockIdx.x % nc;
        k.b = bh / ng;
        k.h = (int64_t)(bh % ng) * hg;
    }
    k.t0 = k.c * Q;
    k.nval = (int)min<int64_t>(Q, a.L - k.t0);
    return k;
}
__device__ __forceinline__ void dt_cum(const MambaArgs& a, const Chunk& k, const bf16* zx, const float* dt_bias,
                                       float A, float* sdt, float* scum, int tid) {
    if (tid < 64) {
        const int64_t t = k.t0 + tid;
        float d = 0.f;
        if (tid < k.nval) d = softplus((float)zx[(k.b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + k.h] + dt_bias[k.h]);
        sdt[tid] = d;
        scum[tid] = wave_scan_dpp(d * A);
    }
}
// 16-B chunk e (row e >> 3, chunk e & 7) of a 64-column bf16 tile starting at column col0 of xc rows
__device__ __forceinline__ u32x4 ld_chunk(const MambaArgs& a, const Chunk& k, const bf16* xc, int64_t col0, int e) {
    const int row = e >> 3, ch = e & 7;
    if (row >= k.nval) return (u32x4){0u, 0u, 0u, 0u};
    return *(const u32x4*)(xc + (k.b * a.L + k.t0 + row) * a.ldxc + col0 + ch * 8);
}

// state: S_c [p][n] into the chunk's slot of `states`, e^{cum_last} factor into clast
__global__ __launch_bounds__(256) void state_kernel(MambaArgs a, const bf16* __restrict__ xc,
                                                    const bf16* __restrict__ zx, const float* __restrict__ dt_bias,
                                                    const float* __restrict__ A_log, float* __restrict__ states,
                                                    float* __restrict__ clast, int nch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sXB = smem;  // half 0: dt x e^{cum_last - cum_s} [s][p]; half 1: B [s][n]
    float* sdt = (float*)(smem + IMG);
    float* scum = sdt + 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const Chunk k = chunk_of(a, nch);
    const float A = -expf(A_log[k.h]);
    u32x4 xr[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u;
        xr[u] = ld_chunk(a, k, xc, k.h * P, e);
        *(u32x4*)(sXB + offd(e >> 3, 8 + (e & 7))) = ld_chunk(a, k, xc, a.d_inner, e);
    }
    dt_cum(a, k, zx, dt_bias, A, sdt, scum, tid);
    __syncthreads();
    const float cl = scum[k.nval - 1];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, row = e >> 3;
        const float f = row < k.nval ? sdt[row] * expf(cl - scum[row]) : 0.f;
        float v[8];
        unpack8(xr[u], v);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] *= f;
        *(u32x4*)(sXB + offd(row, e & 7)) = pack8(v);
    }
    __syncthreads();
    f32x4 acc[2][2];
    zero22(acc);
    const int rb = 32 * (w >> 1), cb = 32 * (w & 1);
    mm<true, true>(acc, sXB, 0, sXB, 1, rb, cb, lane);  // [p][n] = sum_s X[s][p] B[s][n]
    float* st = states + ((k.b * a.nheads + k.h) * nch + k.c) * (int64_t)(P * N);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            *(f32x4*)(st + (rb + 16 * i + (lane & 15)) * N + cb + 16 * j + 4 * (lane >> 4)) = acc[i][j];
    if (tid == 0) clast[(k.b * a.nheads + k.h) * nch + k.c] = cl;
}

// pass: in place over the per-chunk S, H_0 = 0, H_{c+1} = e^{cum_last_c} H_c + S_c
__global__ __launch_bounds__(256) void pass_kernel(float* __restrict__ states, const float* __restrict__ clast,
                                                   int64_t nbh, int nch, float* __restrict__ fin) {
    const int64_t e = blockIdx.x * 256LL + threadIdx.x;  // (bh, p, n)
    if (e >= nbh * P * N) return;
    const int64_t bh = e / (P * N), pn = e % (P * N);
    float* st = states + bh * nch * (int64_t)(P * N) + pn;
    const float* cl = clast + bh * nch;
    float hcur = 0.f;
    for (int c = 0; c < nch; ++c) {
        const float sc = st[(int64_t)c * P * N];
        st[(int64_t)c * P * N] = hcur;
        hcur = expf(cl[c]) * hcur + sc;
    }
    if (fin) fin[e] = hcur;  // state after the last position (cached decode)
}

// out: y = (C B^T o L) (dt x) + e^{cum_t} C H_c^T + D x
// One workgroup per (b, chunk, group of hg heads): the chunk's B / C rows and
// C B^T (head-independent: only the decay mask L is per head) are staged /
// computed once and serve the group's heads in turn.
// 8 consecutive state values as bf16 (fp32 storage: rounded here; optionally unpacked)
template <bool SB>
__device__ __forceinline__ u32x4 ld_state(const void* base, int64_t e) {
    if constexpr (SB) return *(const u32x4*)((const bf16*)base + e);
    const float* f = (const float*)base + e;
    const f32x4 h0 = *(const f32x4*)f, h1 = *(const f32x4*)(f + 4);
    const float hv[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    return pack8(hv);
}
// SB: the entry states are bf16 (the fused scan's form) or fp32 (the three-kernel
// path's); either way the product reads them as bf16 (the same RNE rounding)
template <bool SB>
__global__ __launch_bounds__(512) void out_kernel(MambaArgs a, const bf16* __restrict__ xc,
                                                  const bf16* __restrict__ zx, const float* __restrict__ dt_bias,
                                                  const float* __restrict__ A_log, const float* __restrict__ Dp,
                                                  bf16* __restrict__ y, int64_t ldy, const void* __restrict__ states,
                                                  int nch, float* __restrict__ clast, int hg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sCB = smem;           // half 0: C [t][n];     half 1: B [s][n]
    char* sXH = smem + IMG;     // half 0: dt x [s][p];  half 1: H [p][n]
    char* sM = smem + 2 * IMG;  // half 0: (C B^T) o L [t][s]
    float* sdt = (float*)(smem + 3 * IMG);
    float* scum = sdt + 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, il = lane & 15, g = lane >> 4;
    const Chunk kg = chunk_of(a, nch, hg);
    // 8 waves: wave w computes output rows 32 (w >> 2) .. +31, columns 16 (w & 3) .. +15
    const int rb = 32 * (w >> 2), cb = 16 * (w & 3);
    {
        const int row = tid >> 3, ch = tid & 7;
        *(u32x4*)(sCB + offd(row, 8 + ch)) = ld_chunk(a, kg, xc, a.d_inner, tid);
        *(u32x4*)(sCB + offd(row, ch)) = ld_chunk(a, kg, xc, a.d_inner + N, tid);
    }
    __syncthreads();
    f32x4 gm[2][1];  // C B^T [t][s], shared by the group's heads
    gm[0][0] = gm[1][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
    mm<false, false, 1>(gm, sCB, 0, sCB, 1, rb, cb, lane);  // [t][s] = sum_n C[t][n] B[s][n]
    for (int hh = 0; hh < hg; ++hh) {
        if (hh) __syncthreads();  // the previous head's reads of sXH / sM / scum are done
        Chunk k = kg;
        k.h = kg.h + hh;
        const float A = -expf(A_log[k.h]), Dh = Dp[k.h];
        u32x4 xr;
        const int64_t slot = ((k.b * a.nheads + k.h) * nch + k.c) * (int64_t)(P * N);
        {
            const int row = tid >> 3, ch = tid & 7;
            xr = ld_chunk(a, k, xc, k.h * P, tid);
            *(u32x4*)(sXH + offd(row, 8 + ch)) = ld_state<SB>(states, slot + row * N + ch * 8);
        }
        dt_cum(a, k, zx, dt_bias, A, sdt, scum, tid);
        __syncthreads();
        if (tid == 0) clast[(k.b * a.nheads + k.h) * nch + k.c] = scum[k.nval - 1];  // for rpass
        {
            const int row = tid >> 3;
            float v[8];
            unpack8(xr, v);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] *= sdt[row];
            *(u32x4*)(sXH + offd(row, tid & 7)) = pack8(v);
        }
        f32x4 y2[2][1];
        y2[0][0] = y2[1][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
        mm<false, false, 1>(y2, sCB, 0, sXH, 1, rb, cb, lane);  // [t][p] = sum_n C[t][n] H[p][n]
        // cum of this lane's rows t / columns s read once, log2 units (as grad_kernel)
        float ct[2], cs[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) ct[i] = scum[rb + 16 * i + il] * LOG2E_F;
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[r] = scum[cb + 4 * g + r] * LOG2E_F;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 1; ++j) {
                const int t = rb + 16 * i + il, s0 = cb + 16 * j + 4 * g;
                union { uint64_t u; bf16 e[4]; } mv;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int s = s0 + r;
                    const float e = __builtin_amdgcn_exp2f(ct[i] - cs[r]);
                    mv.e[r] = (bf16)(s <= t ? gm[i][j][r] * e : 0.f);
                }
                *(uint64_t*)(sM + offd(t, s0 >> 3) + (s0 & 7) * 2) = mv.u;
            }
        __syncthreads();
        f32x4 y1[2][1];
        y1[0][0] = y1[1][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
        mm<false, true, 1>(y1, sM, 0, sXH, 0, rb, cb, lane);  // [t][p] = sum_s M[t][s] X[s][p]
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = rb + 16 * i + il;
            if (t >= k.nval) continue;
            const float et = exp_decay(scum[t]);
            const int64_t row = k.b * a.L + k.t0 + t;
#pragma unroll
            for (int j = 0; j < 1; ++j) {
                const int pcol = cb + 16 * j + 4 * g;
                const f32x4 xv = load4(xc + row * a.ldxc + k.h * P + pcol);
                store4(y + row * ldy + k.h * P + pcol, y1[i][j] + et * y2[i][j] + Dh * xv);
            }
        }
    }
}

// ---------------------------------------------------------------- SSD backward, bf16 MFMA path
// dH_c = gradient of the chunk-EXIT state (= entry of chunk c+1) satisfies the
// reverse recurrence dH_{c-1} = e^{cum_last_c} dH_c + U_c, U_c = sum_t e^{cum_t} dY_t^T C_t:
//   uterm : per (b, h, chunk)  U_c   [p][n]            (into the workspace)
//   rpass : per (b, h, p, n)   in place U -> dH (exit gradient of every chunk)
//   grad  : per (b, h, chunk)  everything else from (H_c entry, dH_c exit): the eight
//           64^3 products of the chunk backward on MFMA, dx / dB / dC / ddt and the
//           per-head parameter gradients (the same algebra as ssd_bwd_kernel above).
__global__ __launch_bounds__(256) void uterm_kernel(MambaArgs a, const bf16* __restrict__ xc,
                                                    const bf16* __restrict__ zx, const float* __restrict__ dt_bias,
                                                    const float* __restrict__ A_log, const bf16* __restrict__ dY,
                                                    int64_t ldy, float* __restrict__ U, int nch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sYC = smem;  // half 0: e^{cum_t} dY [t][p]; half 1: C [t][n]
    float* sdt = (float*)(smem + IMG);
    float* scum = sdt + 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const Chunk k = chunk_of(a, nch);
    const float A = -expf(A_log[k.h]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u;
        *(u32x4*)(sYC + offd(e >> 3, 8 + (e & 7))) = ld_chunk(a, k, xc, a.d_inner + N, e);
    }
    dt_cum(a, k, zx, dt_bias, A, sdt, scum, tid);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, row = e >> 3, ch = e & 7;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (row < k.nval) {
            unpack8(*(const u32x4*)(dY + (k.b * a.L + k.t0 + row) * ldy + k.h * P + ch * 8), v);
            const float et = expf(scum[row]);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] *= et;
        }
        *(u32x4*)(sYC + offd(row, ch)) = pack8(v);
    }
    __syncthreads();
    f32x4 acc[2][2];
    zero22(acc);
    const int rb = 32 * (w >> 1), cb = 32 * (w & 1);
    mm<true, true>(acc, sYC, 0, sYC, 1, rb, cb, lane);  // [p][n] = sum_t Ys[t][p] C[t][n]
    float* dst = U + ((k.b * a.nheads + k.h) * nch + k.c) * (int64_t)(P * N);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            *(f32x4*)(dst + (rb + 16 * i + (lane & 15)) * N + cb + 16 * j + 4 * (lane >> 4)) = acc[i][j];
}

// in place: dH = 0; for c = last .. 0: out[c] = dH; dH = e^{cum_last_c} dH + U_c
__global__ __launch_bounds__(256) void rpass_kernel(float* __restrict__ U, const float* __restrict__ clast,
                                                    int64_t nbh, int nch) {
    const int64_t e = blockIdx.x * 256LL + threadIdx.x;
    if (e >= nbh * P * N) return;
    const int64_t bh = e / (P * N), pn = e % (P * N);
    float* u = U + bh * nch * (int64_t)(P * N) + pn;
    const float* cl = clast + bh * nch;
    float d = 0.f;
    for (int c = nch - 1; c >= 0; --c) {
        const float uc = u[(int64_t)c * P * N];
        u[(int64_t)c * P * N] = d;
        d = expf(cl[c]) * d + uc;
    }
}

// ---------------------------------------------------------------- fused chunk scans
// state + pass (forward) and uterm + rpass (backward) as one launch each: one
// workgroup per (b, h) walks its chunks in order and keeps the running state (or
// the running exit gradient) in the MFMA accumulator registers, so the per-chunk
// S_c / U_c never go to HBM -- the only state traffic is the one fp32 store of
// every chunk's entry state H_c (exit gradient dH_c) that `out` / `grad` read.
// The next chunk's x / B (dY / C) and dt rows are loaded into registers while the
// current chunk's product runs. Same arithmetic as state -> pass (uterm -> rpass):
// H_{c+1} = e^{cum_last_c} H_c + S_c with S_c from the same MFMA sequence.
__device__ __forceinline__ Chunk chunk_at(const MambaArgs& a, int64_t bh, int c) {
    Chunk k;
    k.b = bh / a.nheads;
    k.h = bh % a.nheads;
    k.c = c;
    k.t0 = (int64_t)c * Q;
    k.nval = (int)min<int64_t>(Q, a.L - k.t0);
    return k;
}
// raw dt bits (bf16 in the low half): converted only where dt_cum_raw uses them, so
// the prefetch does not wait for its own load (a conversion right after the load does)
__device__ __forceinline__ unsigned dt_raw(const MambaArgs& a, const Chunk& k, const bf16* zx, int tid) {
    const unsigned short* zu = (const unsigned short*)zx;
    return tid < k.nval ? (unsigned)zu[(k.b * a.L + k.t0 + tid) * a.ldz + a.d_inner + a.conv_dim + k.h] : 0u;
}
// unmasked forms for the scan kernels: rows past nval read the chunk's last valid
// row (finite data; the consumer zeroes its weight), so no branch skips a load
__device__ __forceinline__ u32x4 ld_clamped(const MambaArgs& a, const Chunk& k, const bf16* xc, int64_t col0, int e) {
    const int row = min(e >> 3, k.nval - 1), ch = e & 7;
    return *(const u32x4*)(xc + (k.b * a.L + k.t0 + row) * a.ldxc + col0 + ch * 8);
}
__device__ __forceinline__ unsigned dt_raw_clamped(const MambaArgs& a, const Chunk& k, const bf16* zx, int tid) {
    const unsigned short* zu = (const unsigned short*)zx;
    const int row = min(tid & 63, k.nval - 1);
    return (unsigned)zu[(k.b * a.L + k.t0 + row) * a.ldz + a.d_inner + a.conv_dim + k.h];
}
// wave 0: dt = softplus(raw + bias) (0 past nval), inclusive scan of dt A
__device__ __forceinline__ void dt_cum_raw(const Chunk& k, unsigned raw, float bias, float A, float* sdt,
                                           float* scum, int tid) {
    if (tid < 64) {
        const float d = tid < k.nval ? softplus(__uint_as_float(raw << 16) + bias) : 0.f;
        sdt[tid] = d;
        scum[tid] = wave_scan_dpp(d * A);  // (the same scan as dt_cum: identical cum values)
    }
}

// Two chunks' rows are in flight ahead of the one being multiplied (register sets
// alternate with the chunk parity), and the LDS image / dt / cum rows are double
// buffered, so one iteration has two barriers and no load on its critical path.
constexpr size_t SCAN_LDS = 2 * (IMG + 512);
__global__ __launch_bounds__(512) void scan_fwd_kernel(MambaArgs a, const bf16* __restrict__ xc,
                                                       const bf16* __restrict__ zx, const float* __restrict__ dt_bias,
                                                       const float* __restrict__ A_log, bf16* __restrict__ states,
                                                       float* __restrict__ clast, int nch, float* __restrict__ fin) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t bh = blockIdx.x;
    const int64_t h = bh % a.nheads;
    const float A = -expf(A_log[h]), bias = dt_bias[h];
    // 8 waves: wave w owns state rows 32 (w >> 2) .. +31, columns 16 (w & 3) .. +15
    const int rb = 32 * (w >> 2), cb = 16 * (w & 3);
    f32x4 H[2][1];
    H[0][0] = H[1][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
    u32x4 x0[1], b0[1], x1[1], b1[1];
    unsigned r0 = 0u, r1 = 0u;
    // entry states in bf16 (what out / grad multiply with); the final state in fp32
    auto store_state = [&](bf16* st) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            *(uint64_t*)(st + (rb + 16 * i + (lane & 15)) * N + cb + 4 * (lane >> 4)) = pack4(H[i][0]);
        }
    };
    auto store_fin = [&](float* st) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
            *(f32x4*)(st + (rb + 16 * i + (lane & 15)) * N + cb + 4 * (lane >> 4)) = H[i][0];
    };
    auto load = [&](int c, u32x4 (&xr)[1], u32x4 (&br)[1], unsigned& raw) {
        const Chunk k = chunk_at(a, bh, c);
        xr[0] = ld_clamped(a, k, xc, h * P, tid);
        br[0] = ld_clamped(a, k, xc, a.d_inner, tid);
        raw = dt_raw_clamped(a, k, zx, tid);
    };
    // chunk c from its register set; then that set takes chunk c + 2
    // c == nch (the odd tail of the unrolled pair) repeats chunk nch - 1 without
    // updating H: every trip runs both bodies, so no branch skips a load or store
    auto body = [&](int c0, u32x4 (&xr)[1], u32x4 (&br)[1], unsigned& raw) {
        const bool valid = c0 < nch;
        const int c = min(c0, nch - 1);
        const Chunk k = chunk_at(a, bh, c);
        char* sXB = smem + (c & 1) * (IMG + 512);  // half 0: dt x e^{cum_last - cum_s} [s][p]; half 1: B [s][n]
        float* sdt = (float*)(sXB + IMG);
        float* scum = sdt + 64;
        *(u32x4*)(sXB + offd(tid >> 3, 8 + (tid & 7))) = br[0];
        dt_cum_raw(k, raw, bias, A, sdt, scum, tid);
        __syncthreads();
        const float cl = scum[k.nval - 1];
        {
            const int row = tid >> 3;
            const float f = row < k.nval ? sdt[row] * exp_decay(cl - scum[row]) : 0.f;
            float v[8];
            unpack8(xr[0], v);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] *= f;
            *(u32x4*)(sXB + offd(row, tid & 7)) = pack8(v);
        }
        load(min(c + 2, nch - 1), xr, br, raw);  // unconditional: the wait counts stay static
        __syncthreads();
        f32x4 acc[2][1];
        acc[0][0] = acc[1][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
        mm<true, true, 1>(acc, sXB, 0, sXB, 1, rb, cb, lane);  // [p][n] = sum_s X[s][p] B[s][n]
        const float ecl = exp_decay(cl);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) H[i][0][r] = valid ? ecl * H[i][0][r] + acc[i][0][r] : H[i][0][r];
        // the entry state of chunk c + 1 (or the final state) is stored right after
        // the update: H is next overwritten one chunk later, so the wait the store's
        // source registers need does not also wait for the next loads
        if (c + 1 < nch) store_state(states + (bh * nch + c + 1) * (int64_t)(P * N));
        else store_fin(fin + bh * (int64_t)(P * N));
        // no trailing barrier: chunk c + 1 writes the other buffer, and chunk c + 2
        // writes this one only after every wave has passed chunk c + 1's first barrier
    };
    store_state(states + bh * nch * (int64_t)(P * N));  // H_0 = 0
    load(0, x0, b0, r0);
    load(min(1, nch - 1), x1, b1, r1);
    for (int c = 0; c < nch; c += 2) {
        body(c, x0, b0, r0);
        body(c + 1, x1, b1, r1);
    }
}

// reverse: dH = 0; for c = last .. 0: U[c] = dH (exit gradient); dH = e^{cum_last_c} dH + U_c
__global__ __launch_bounds__(256) void scan_bwd_kernel(MambaArgs a, const bf16* __restrict__ xc,
                                                       const bf16* __restrict__ zx, const float* __restrict__ dt_bias,
                                                       const float* __restrict__ A_log, const bf16* __restrict__ dY,
                                                       int64_t ldy, bf16* __restrict__ U, int nch,
                                                       bf16* __restrict__ dh0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t bh = blockIdx.x;
    const int64_t h = bh % a.nheads;
    const float A = -expf(A_log[h]), bias = dt_bias[h];
    const int rb = 32 * (w >> 1), cb = 32 * (w & 1);
    f32x4 D[2][2];
    zero22(D);
    u32x4 c0[2], c1[2];
    u32x4 y0[2], y1[2];  // raw bf16 dY rows
    unsigned r0 = 0u, r1 = 0u;
    auto store_d = [&](bf16* dst) {  // bf16, as grad multiplies with it
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                *(uint64_t*)(dst + (rb + 16 * i + (lane & 15)) * N + cb + 16 * j + 4 * (lane >> 4)) = pack4(D[i][j]);
    };
    auto load = [&](int c, u32x4 (&cr)[2], u32x4 (&yr)[2], unsigned& raw) {
        const Chunk k = chunk_at(a, bh, c);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + 256 * u, row = e >> 3, ch = e & 7;
            cr[u] = ld_clamped(a, k, xc, a.d_inner + N, e);
            // rows past nval: zeroed where used
            yr[u] = *(const u32x4*)(dY + (k.b * a.L + k.t0 + min(row, k.nval - 1)) * ldy + h * P + ch * 8);
        }
        raw = dt_raw_clamped(a, k, zx, tid);
    };
    auto body = [&](int c0, u32x4 (&cr)[2], u32x4 (&yr)[2], unsigned& raw) {
        const bool valid = c0 >= 0;  // c0 == -1: the odd tail, chunk 0 again without an update
        const int c = max(c0, 0);
        const Chunk k = chunk_at(a, bh, c);
        char* sYC = smem + (c & 1) * (IMG + 512);  // half 0: e^{cum_t} dY [t][p]; half 1: C [t][n]
        float* sdt = (float*)(sYC + IMG);
        float* scum = sdt + 64;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + 256 * u;
            *(u32x4*)(sYC + offd(e >> 3, 8 + (e & 7))) = cr[u];
        }
        dt_cum_raw(k, raw, bias, A, sdt, scum, tid);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + 256 * u, row = e >> 3, ch = e & 7;
            const float et = row < k.nval ? exp_decay(scum[row]) : 0.f;
            float v[8];
            unpack8(yr[u], v);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] *= et;
            *(u32x4*)(sYC + offd(row, ch)) = pack8(v);
        }
        const float cl = scum[k.nval - 1];
        load(max(c - 2, 0), cr, yr, raw);  // unconditional: the wait counts stay static
        __syncthreads();
        f32x4 acc[2][2];
        zero22(acc);
        mm<true, true>(acc, sYC, 0, sYC, 1, rb, cb, lane);  // [p][n] = sum_t Ys[t][p] C[t][n]
        const float ecl = exp_decay(cl);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) D[i][j][r] = valid ? ecl * D[i][j][r] + acc[i][j][r] : D[i][j][r];
        // exit gradient of chunk c - 1 (chunk 0's entry gradient goes to the scratch dh0)
        store_d(c > 0 ? U + (bh * nch + c - 1) * (int64_t)(P * N) : dh0 + bh * (int64_t)(P * N));
    };
    // chunks walk down from nch - 1; the parity of (nch - 1 - c) picks the register set
    store_d(U + (bh * nch + nch - 1) * (int64_t)(P * N));  // the last chunk's exit gradient is 0
    load(nch - 1, c0, y0, r0);
    load(max(nch - 2, 0), c1, y1, r1);
    for (int c = nch - 1; c >= 0; c -= 2) {
        body(c, c0, y0, r0);
        body(c - 1, c1, y1, r1);
    }
}

template <typename TD, bool SB>
__global__ __launch_bounds__(256, 2) void grad_kernel(MambaArgs a, const bf16* __restrict__ xc,
                                                      const bf16* __restrict__ zx, const float* __restrict__ dt_bias,
                                                      const float* __restrict__ A_log, const float* __restrict__ Dp,
                                                      const bf16* __restrict__ dY, int64_t ldy,
                                                      const void* __restrict__ states, const void* __restrict__ dHx,
                                                      float* __restrict__ dxc, float* __restrict__ dbc,
                                                      TD* __restrict__ dzx,
                                                      float* __restrict__ gA_log, float* __restrict__ gD,
                                                      float* __restrict__ gdt_bias, int nch, int hg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sCB = smem;            // C [t][n]   | B [s][n]
    char* sXY = smem + IMG;      // dt x [s][p] | dY [t][p]
    char* sHD = smem + 2 * IMG;  // H [p][n]   | dH [p][n]
    char* sMG = smem + 3 * IMG;  // M [t][s]   | dG [t][s]
    float* sdt = (float*)(smem + 4 * IMG);
    float* scum = sdt + 64;
    float* sdcum = scum + 64;
    float* sddt = sdcum + 64;
    float* sred = sddt + 64;  // 8 block-reduction slots
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, il = lane & 15, g = lane >> 4;
    const Chunk kg = chunk_of(a, nch, hg);
    const int nv = kg.nval;
    const int rb = 32 * (w >> 1), cb = 32 * (w & 1);
    // the chunk's B / C rows, shared by the group's heads
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, row = e >> 3, ch = e & 7;
        *(u32x4*)(sCB + offd(row, 8 + ch)) = ld_chunk(a, kg, xc, a.d_inner, e);
        *(u32x4*)(sCB + offd(row, ch)) = ld_chunk(a, kg, xc, a.d_inner + N, e);
    }
    // dC [t][n] / dB [s][n] of the chunk summed over the group's heads (fp32, in
    // registers); dbc_reduce_kernel adds the nheads / hg group rows
    f32x4 dcs[2][2], dbs[2][2];
    zero22(dcs);
    zero22(dbs);
    // a head's x / H / dH / dY chunks are loaded during the previous head's
    // products (each head waited on its own loads: 68 % of wave cycles in
    // SQ_WAIT_ANY at two waves per SIMD); unconditional loads from clamped rows
    // (rows past nval are zeroed where they are used or written)
    u32x4 pxr[2], phb[2], pdb[2], pdy[2];
    auto prefetch = [&](int h2) {
        const int64_t hd = kg.h + h2;
        const int64_t slot2 = ((kg.b * a.nheads + hd) * nch + kg.c) * (int64_t)(P * N);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + 256 * u, row = e >> 3, ch = e & 7, rr = min(row, nv - 1);
            const int64_t grow = kg.b * a.L + kg.t0 + rr;
            pxr[u] = *(const u32x4*)(xc + grow * a.ldxc + hd * P + ch * 8);
            phb[u] = ld_state<SB>(states, slot2 + row * N + ch * 8);
            pdb[u] = ld_state<SB>(dHx, slot2 + row * N + ch * 8);
            pdy[u] = *(const u32x4*)(dY + grow * ldy + hd * P + ch * 8);
        }
    };
    prefetch(0);
    for (int hh = 0; hh < hg; ++hh) {
    if (hh) __syncthreads();  // the previous head's last LDS reads are done
    Chunk k = kg;
    k.h = kg.h + hh;
    const float A = -expf(A_log[k.h]), Dh = Dp[k.h];
    u32x4 xr[2];
    float hdh = 0.f;  // sum dH o H (the cum_last term)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, row = e >> 3, ch = e & 7;
        xr[u] = row < k.nval ? pxr[u] : (u32x4){0u, 0u, 0u, 0u};
        // H / dH as bf16 (the MFMA operands); the cum_last term from the same values
        const u32x4 hb = phb[u], db = pdb[u];
        {
            float hv[8], dv[8];
            unpack8(hb, hv);
            unpack8(db, dv);
#pragma unroll
            for (int q = 0; q < 8; ++q) hdh += hv[q] * dv[q];
        }
        *(u32x4*)(sHD + offd(row, ch)) = hb;
        *(u32x4*)(sHD + offd(row, 8 + ch)) = db;
        // dY rows are bf16 already: copied into the image as they are (zero past nval)
        *(u32x4*)(sXY + offd(row, 8 + ch)) = row < k.nval ? pdy[u] : (u32x4){0u, 0u, 0u, 0u};
    }
    dt_cum(a, k, zx, dt_bias, A, sdt, scum, tid);
    if (tid < 64) sdcum[tid] = sddt[tid] = 0.f;
    hdh = wave_sum_dpp(hdh);
    if (lane == 0) sred[w] = hdh;
    __syncthreads();
    const float cl = scum[nv - 1];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, row = e >> 3;
        float v[8];
        unpack8(xr[u], v);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] *= sdt[row];
        *(u32x4*)(sXY + offd(row, e & 7)) = pack8(v);
    }
    if (hh + 1 < hg) prefetch(hh + 1);
    // M = (C B^T) o L ; dM = dY XS^T (s <= t)
    f32x4 mt[2][2], dm[2][2];
    zero22(mt);
    mm<false, false>(mt, sCB, 0, sCB, 1, rb, cb, lane);  // [t][s]
    __syncthreads();  // XS written
    zero22(dm);
    mm<false, false>(dm, sXY, 1, sXY, 0, rb, cb, lane);  // [t][s] = sum_p dY[t][p] XS[s][p]
    float rowq[2] = {0.f, 0.f}, colq[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) colq[q] = 0.f;
    // this lane's 2 rows t and 8 columns s of cum, read once (log2 units):
    // L = 2^(ct - cs), computed for every pair and selected (no branch, no
    // LDS round trip per pair)
    float ct[2], cs[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) ct[i] = scum[rb + 16 * i + il] * LOG2E_F;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[j][r] = scum[cb + 16 * j + 4 * g + r] * LOG2E_F;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int t = rb + 16 * i + il, s0 = cb + 16 * j + 4 * g;
            union { uint64_t u; bf16 e[4]; } mv, gv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int s = s0 + r;
                const float e = __builtin_amdgcn_exp2f(ct[i] - cs[j][r]);
                const float L_ = s <= t ? e : 0.f;
                const float m = mt[i][j][r] * L_;
                const float d = s <= t ? dm[i][j][r] : 0.f;
                const float q = d * m;
                rowq[i] += q;
                colq[j * 4 + r] += q;
                mv.e[r] = (bf16)m;
                gv.e[r] = (bf16)(d * L_);
            }
            *(uint64_t*)(sMG + offd(t, s0 >> 3) + (s0 & 7) * 2) = mv.u;
            *(uint64_t*)(sMG + offd(t, 8 + (s0 >> 3)) + (s0 & 7) * 2) = gv.u;
        }
    // dcum_t += sum_s dM M ; dcum_s -= sum_t dM M
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float v = cross4_sum(rowq[i]);
        if (g == 0) atomicAdd(&sdcum[rb + 16 * i + il], v);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float v = row16_sum(colq[q]);
        if (il == 0) atomicAdd(&sdcum[cb + 16 * (q >> 2) + 4 * g + (q & 3)], -v);
    }
    __syncthreads();  // M, dG images
    // dXS = M^T dY + w_s (B dH^T) ; dx = dXS dt + D dY ; ddt_s += sum_p dXS x ; dcum_s -= w_s sum_p XS t1
    f32x4 dxs[2][2], t1[2][2];
    zero22(dxs);
    zero22(t1);
    mm<true, true>(dxs, sMG, 0, sXY, 1, rb, cb, lane);   // [s][p] = sum_t M[t][s] dY[t][p]
    mm<false, false>(t1, sCB, 1, sHD, 1, rb, cb, lane);  // [s][p] = sum_n B[s][n] dH[p][n]
    float gd = 0.f, dws_tot = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int s = rb + 16 * i + il;
        const float ws = s < nv ? exp_decay(cl - scum[s]) : 0.f;
        float ddt_p = 0.f, dws = 0.f;
        const int64_t row = k.b * a.L + k.t0 + s;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int pc = cb + 16 * j + 4 * g;
            f32x4 xv = (f32x4){0.f, 0.f, 0.f, 0.f}, yv = xv;
            if (s < nv) {
                xv = load4(xc + row * a.ldxc + k.h * P + pc);
                yv = load4(dY + row * ldy + k.h * P + pc);
            }
            f32x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float tot = dxs[i][j][r] + ws * t1[i][j][r];
                ddt_p += tot * xv[r];
                dws += xv[r] * sdt[s] * t1[i][j][r] * ws;
                gd += yv[r] * xv[r];
                o[r] = tot * sdt[s] + Dh * yv[r];
            }
            if (s < nv) *(f32x4*)(dxc + row * a.ldxc + k.h * P + pc) = o;
        }
        ddt_p = cross4_sum(ddt_p);
        dws = cross4_sum(dws);
        if (g == 0) {
            atomicAdd(&sddt[s], ddt_p);
            atomicAdd(&sdcum[s], -dws);
        }
        dws_tot += dws;  // every g holds the same row sum: counted once below
    }
    // dC = dG B + e^{cum_t} dY H ; dcum_t += e^{cum_t} sum_n C dyh
    {
        f32x4 dyh[2][2];
        zero22(dyh);
        mm<false, true>(dcs, sMG, 1, sCB, 1, rb, cb, lane);  // [t][n] += sum_s dG[t][s] B[s][n]
        mm<false, true>(dyh, sXY, 1, sHD, 0, rb, cb, lane);  // [t][n] = sum_p dY[t][p] H[p][n]
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int t = rb + 16 * i + il;
            const float et = exp_decay(scum[t]);
            float rs = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n0 = cb + 16 * j + 4 * g;
                union { uint64_t u; bf16 e[4]; } cv;
                cv.u = *(const uint64_t*)(sCB + offd(t, n0 >> 3) + (n0 & 7) * 2);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    rs += et * (float)cv.e[r] * dyh[i][j][r];
                    dcs[i][j][r] += et * dyh[i][j][r];
                }
            }
            rs = cross4_sum(rs);
            if (g == 0) atomicAdd(&sdcum[t], rs);
        }
    }
    // dB = dG^T C + w_s (XS dH)
    {
        f32x4 tb[2][2];
        zero22(tb);
        mm<true, true>(dbs, sMG, 1, sCB, 0, rb, cb, lane);   // [s][n] += sum_t dG[t][s] C[t][n]
        mm<false, true>(tb, sXY, 0, sHD, 1, rb, cb, lane);   // [s][n] = sum_p XS[s][p] dH[p][n]
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int s = rb + 16 * i + il;
            const float ws = exp_decay(cl - scum[s]);  // rows s >= nv are never stored
#pragma unroll
            for (int j = 0; j < 2; ++j) dbs[i][j] += ws * tb[i][j];
        }
    }
    // dcum_last += sum_s dws_s + e^{cum_last} sum dH o H
    dws_tot = wave_sum_dpp(dws_tot) * 0.25f;  // each row sum was held by its 4 g-lanes
    gd = wave_sum_dpp(gd);
    if (lane == 0) {
        atomicAdd(&sdcum[nv - 1], dws_tot);
        sred[4 + w] = gd;
    }
    __syncthreads();
    if (tid == 0) sdcum[nv - 1] += exp_decay(cl) * (sred[0] + sred[1] + sred[2] + sred[3]);
    __syncthreads();
    if (tid < 64) {
        // da_t = sum_{tau >= t} dcum_tau ; ddt = A da + sum_p dXS x ; d dt_raw = ddt sigmoid(raw)
        // (suffix sum = prefix scan over the reversed lanes, back through the
        // same LDS row: one wave, its LDS operations in issue order)
        const float rv = 63 - tid < nv ? sdcum[63 - tid] : 0.f;
        sdcum[63 - tid] = wave_scan_dpp(rv);
        const float v = sdcum[tid];
        float gA = 0.f, gdb = 0.f;
        if (tid < nv) {
            const int64_t t = k.t0 + tid;
            const float ddt = A * v + sddt[tid];
            gA = sdt[tid] * v;
            const float raw = (float)zx[(k.b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + k.h] + dt_bias[k.h];
            const float draw = ddt * sigm(raw);
            dzx[(k.b * a.L + t) * a.ldz + a.d_inner + a.conv_dim + k.h] = (TD)draw;
            gdb = draw;
        }
        gA = wave_sum_dpp(gA);
        gdb = wave_sum_dpp(gdb);
        if (tid == 0) {
            atomicAdd(gA_log + k.h, gA * A);  // A = -exp(A_log) -> dA/dA_log = A
            atomicAdd(gdt_bias + k.h, gdb);
            atomicAdd(gD + k.h, sred[4] + sred[5] + sred[6] + sred[7]);
        }
    }
    }  // heads of the group
    const int64_t ng = a.nheads / hg, grp = kg.h / hg;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int t = rb + 16 * i + il;
        if (t >= nv) continue;
        float* rowp = dbc + ((kg.b * a.L + kg.t0 + t) * ng + grp) * (2 * N);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n0 = cb + 16 * j + 4 * g;
            *(f32x4*)(rowp + n0) = dbs[i][j];
            *(f32x4*)(rowp + N + n0) = dcs[i][j];
        }
    }
}

// dxc[bt][d_inner + c] = sum_g dbc[bt][g][c]   (dB | dC, c < 2N; g < nheads / hg head groups)
__global__ __launch_bounds__(256) void dbc_reduce_kernel(const float* __restrict__ dbc, float* __restrict__ dxc,
                                                         int64_t rows, int64_t nheads, int64_t ldxc, int64_t d_inner) {
    const int64_t e = blockIdx.x * 256LL + threadIdx.x;  // (row, 4-column group)
    if (e >= rows * (2 * N / 4)) return;
    const int64_t row = e / (2 * N / 4), c = (e % (2 * N / 4)) * 4;
    const float* p = dbc + row * nheads * (2 * N) + c;
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int64_t h = 0; h < nheads; ++h) acc += *(const f32x4*)(p + h * (2 * N));
    *(f32x4*)(dxc + row * ldxc + d_inner + c) = acc;
}

constexpr size_t UTERM_LDS = IMG + 512, GRAD_LDS = 4 * IMG + 2048;  // + sdt, scum, sdcum, sddt, sred

constexpr size_t STATE_LDS = IMG + 512, OUT_LDS = 3 * IMG + 512;
}  // namespace ssd2
}  // namespace

extern "C" size_t msq_mamba_states_size(int64_t B, int64_t L, int64_t nheads) {
    // chunk-entry states [B][H][nch][P][N] + per-chunk decay sums cum_last [B][H][nch]
    // + [B][H][P][N] final state written when the caller passes none
    const int64_t nch = (L + Q - 1) / Q;
    return (size_t)B * nheads * (nch * (P * N + 1) + P * N) * sizeof(float);
}

#define MAMBA_CHECK()                                                                                         \
    MSQ_CHECK_ARG(B > 0 && L > 0 && nheads > 0 && d_inner == nheads * P && ldz % 4 == 0 && ldxc % 4 == 0,     \
                  "mamba: bad sizes (headdim 64, d_state 64, ld %% 4 == 0)")

extern "C" int msq_mamba_conv_fwd(void* xc, int64_t ldxc, const void* zxbcdt, int64_t ldz, int dtype,
                                  const float* conv_w, const float* conv_b, int64_t B, int64_t L, int64_t d_inner,
                                  int64_t nheads, void* stream) {
    MAMBA_CHECK();
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ldxc);
    MSQ_CHECK_ARG((uintptr_t)zxbcdt % 16 == 0 && (uintptr_t)xc % 16 == 0, "msq_mamba_conv_fwd: 16-B aligned buffers");
    const dim3 grid((unsigned)((a.conv_dim + 64 * CONV_CV - 1) / (64 * CONV_CV)), (unsigned)B,
                    (unsigned)((L + 4 * CONV_SEG - 1) / (4 * CONV_SEG)));
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((conv_fwd_kernel<bf16, bf16>), grid, dim3(256), 0, s, a, (const bf16*)zxbcdt, conv_w, conv_b, (bf16*)xc);
    else hipLaunchKernelGGL((conv_fwd_kernel<float, float>), grid, dim3(256), 0, s, a, (const float*)zxbcdt, conv_w, conv_b, (float*)xc);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_ssd_fwd_state(void* y, int64_t ldy, float* states, float* final_state, const void* xc,
                                       int64_t ldxc, const void* zxbcdt, int64_t ldz, int dtype,
                                       const float* dt_bias, const float* A_log, const float* D, int64_t B,
                                       int64_t L, int64_t d_inner, int64_t nheads, void* stream) {
    MAMBA_CHECK();
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ldxc);
    hipStream_t s = (hipStream_t)stream;
    const int nch = (int)((L + Q - 1) / Q);
    if (dtype == MSQ_BF16) {
        float* clast = states + B * nheads * nch * (int64_t)(P * N);
        const dim3 gch((unsigned)(B * nheads * nch));
        const bool k3 = getenv("MSQ_MAMBA_SSD_3K") != nullptr;
        if (k3) allow_lds(ssd2::out_kernel<false>, ssd2::OUT_LDS);
        else allow_lds(ssd2::out_kernel<true>, ssd2::OUT_LDS);
        if (k3) {  // per-chunk state kernel + separate pass (round-2 form)
            allow_lds(ssd2::state_kernel, ssd2::STATE_LDS);
            hipLaunchKernelGGL(ssd2::state_kernel, gch, dim3(256), ssd2::STATE_LDS, s, a, (const bf16*)xc,
                               (const bf16*)zxbcdt, dt_bias, A_log, states, clast, nch);
            hipLaunchKernelGGL(ssd2::pass_kernel, dim3((unsigned)((B * nheads * P * N + 255) / 256)), dim3(256), 0,
                               s, states, clast, B * nheads, nch, final_state);
        } else {
            allow_lds(ssd2::scan_fwd_kernel, ssd2::SCAN_LDS);
            if (!final_state) final_state = clast + B * nheads * nch;  // scratch past cum_last
            hipLaunchKernelGGL(ssd2::scan_fwd_kernel, dim3((unsigned)(B * nheads)), dim3(512), ssd2::SCAN_LDS, s, a,
                               (const bf16*)xc, (const bf16*)zxbcdt, dt_bias, A_log, (bf16*)states, clast, nch,
                               final_state);
        }
        // out: one workgroup per (b, chunk, group of hg heads), as grad
        const int hg = nheads % 4 == 0 ? 4 : nheads % 2 == 0 ? 2 : 1;
        const dim3 go((unsigned)(B * (nheads / hg) * nch));
        if (k3) hipLaunchKernelGGL(ssd2::out_kernel<false>, go, dim3(512), ssd2::OUT_LDS, s, a, (const bf16*)xc,
                                   (const bf16*)zxbcdt, dt_bias, A_log, D, (bf16*)y, ldy, states, nch, clast, hg);
        else hipLaunchKernelGGL(ssd2::out_kernel<true>, go, dim3(512), ssd2::OUT_LDS, s, a, (const bf16*)xc,
                                (const bf16*)zxbcdt, dt_bias, A_log, D, (bf16*)y, ldy, states, nch, clast, hg);
        MSQ_LAUNCH_CHECK();
        return MSQ_OK;
    }
    const dim3 grid((unsigned)(B * nheads));
    allow_lds(ssd_fwd_kernel<float>, FWD_LDS);
    hipLaunchKernelGGL(ssd_fwd_kernel<float>, grid, dim3(NT), FWD_LDS, s, a, (const float*)xc, (const float*)zxbcdt,
                       dt_bias, A_log, D, (float*)y, ldy, states, final_state);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_ssd_fwd(void* y, int64_t ldy, float* states, const void* xc, int64_t ldxc,
                                 const void* zxbcdt, int64_t ldz, int dtype, const float* dt_bias,
                                 const float* A_log, const float* D, int64_t B, int64_t L, int64_t d_inner,
                                 int64_t nheads, void* stream) {
    return msq_mamba_ssd_fwd_state(y, ldy, states, nullptr, xc, ldxc, zxbcdt, ldz, dtype, dt_bias, A_log, D, B, L,
                                   d_inner, nheads, stream);
}

extern "C" int msq_mamba_gnorm_fwd(void* out, int64_t ldo, float* rstd, const void* y, int64_t ldy,
                                   const void* zxbcdt, int64_t ldz, int dtype, const float* w, int64_t rows,
                                   int64_t d_inner, float eps, void* stream) {
    MSQ_CHECK_ARG(rows > 0 && d_inner % 4 == 0 && d_inner <= 4096, "mamba gnorm: bad sizes");
    hipStream_t s = (hipStream_t)stream;
    if (rows <= 1024) {  // decode steps: a block per row
        const int nk = (int)((d_inner + 1023) / 1024);
#define GN_ROW(NK)                                                                                                     \
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((gnorm_fwd_row_kernel<bf16, bf16, NK>), dim3((unsigned)rows), dim3(256), 0, s, (const bf16*)y, ldy, (const bf16*)zxbcdt, ldz, w, (bf16*)out, ldo, rstd, (int)d_inner, eps); \
    else hipLaunchKernelGGL((gnorm_fwd_row_kernel<float, float, NK>), dim3((unsigned)rows), dim3(256), 0, s, (const float*)y, ldy, (const float*)zxbcdt, ldz, w, (float*)out, ldo, rstd, (int)d_inner, eps);
        if (nk == 1) { GN_ROW(1) } else if (nk == 2) { GN_ROW(2) } else if (nk == 3) { GN_ROW(3) } else { GN_ROW(4) }
#undef GN_ROW
        MSQ_LAUNCH_CHECK();
        return MSQ_OK;
    }
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((gnorm_fwd_kernel<bf16, bf16>), grid, dim3(256), 0, s, (const bf16*)y, ldy, (const bf16*)zxbcdt, ldz, w, (bf16*)out, ldo, rstd, rows, (int)d_inner, eps);
    else hipLaunchKernelGGL((gnorm_fwd_kernel<float, float>), grid, dim3(256), 0, s, (const float*)y, ldy, (const float*)zxbcdt, ldz, w, (float*)out, ldo, rstd, rows, (int)d_inner, eps);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_gnorm_bwd(void* dy, void* dzxbcdt, const void* y, int64_t ldy, const void* zxbcdt,
                                   int64_t ldz, int dtype, const float* w, const float* rstd, const float* dout,
                                   int64_t ldd, float* dw, int64_t rows, int64_t d_inner, void* stream) {
    MSQ_CHECK_ARG(rows > 0 && d_inner % 4 == 0 && d_inner <= 256 * GN_K, "mamba gnorm bwd: bad sizes");
    hipStream_t s = (hipStream_t)stream;
    // persistent: 3 workgroups per CU (the wide-row kernel's occupancy); each
    // reduces its dw partials in LDS first
    const dim3 grid(768);
    if (dtype == MSQ_BF16 && d_inner > 1024 && d_inner <= 2048) {
        // the row over a wave pair, the next pair's loads in flight (3 waves per
        // SIMD: 3 workgroups per CU)
        hipLaunchKernelGGL((gnorm_bwd2_kernel<bf16, 4>), dim3(768), dim3(256), 0, s, (const bf16*)y, ldy,
                           (const bf16*)zxbcdt, ldz, w, rstd, dout, ldd, (bf16*)dy, (bf16*)dzxbcdt, dw, rows,
                           (int)d_inner);
        MSQ_LAUNCH_CHECK();
        return MSQ_OK;
    }
    if (dtype == MSQ_BF16)
        gnorm_bwd_launch<bf16, bf16>(grid, s, (const bf16*)y, ldy, (const bf16*)zxbcdt, ldz, w, rstd, dout, ldd, (bf16*)dy, (bf16*)dzxbcdt,
                                     dw, rows, (int)d_inner);
    else
        gnorm_bwd_launch<float, float>(grid, s, (const float*)y, ldy, (const float*)zxbcdt, ldz, w, rstd, dout, ldd, (float*)dy,
                                       (float*)dzxbcdt, dw, rows, (int)d_inner);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" size_t msq_mamba_ssd_bwd_workspace(int64_t B, int64_t L, int64_t nheads) {
    // per-chunk state gradients [B][H][nch][P][N] | per-head dB, dC rows [B*L][H][2N]
    // + [B][H][P][N] scratch for the scan's gradient of the initial state
    return (size_t)B * nheads * ((L + Q - 1) / Q) * P * N * sizeof(float) + (size_t)B * L * nheads * 2 * N * sizeof(float) +
           (size_t)B * nheads * P * N * sizeof(float);
}

extern "C" int msq_mamba_ssd_bwd(float* dxc, int64_t ld_dxc, void* dzxbcdt, const void* dY, int64_t ldy,
                                 const float* states, const void* xc, int64_t ldxc, const void* zxbcdt, int64_t ldz,
                                 int dtype, const float* dt_bias, const float* A_log, const float* D, float* gA_log,
                                 float* gD, float* gdt_bias, int64_t B, int64_t L, int64_t d_inner, int64_t nheads,
                                 void* workspace, void* stream) {
    MAMBA_CHECK();
    MSQ_CHECK_ARG(ld_dxc == ldxc, "msq_mamba_ssd_bwd: dxc must share the xBC row stride");
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ldxc);
    hipStream_t s = (hipStream_t)stream;
    // bf16 path: grad writes one dB / dC row per (token, head group) into dbc and
    // dbc_reduce_kernel sums the groups' rows in a fixed order (no atomics); the
    // fp32 path below accumulates the columns with atomics across heads
    if (dtype == MSQ_BF16) {
        MSQ_CHECK_ARG(workspace, "msq_mamba_ssd_bwd: the bf16 path needs msq_mamba_ssd_bwd_workspace() bytes");
        const int nch = (int)((L + Q - 1) / Q);
        const float* clast = states + B * nheads * nch * (int64_t)(P * N);
        float* U = (float*)workspace;
        float* dbc = U + B * nheads * nch * (int64_t)(P * N);
        const dim3 gch((unsigned)(B * nheads * nch));
        // grad: one workgroup per (b, chunk, group of hg heads); the group's B / C
        // tile is staged once and its dB / dC rows summed in registers
        const int hg = nheads % 4 == 0 ? 4 : nheads % 2 == 0 ? 2 : 1;
        const bool k3 = getenv("MSQ_MAMBA_SSD_3K") != nullptr;
        if (k3) allow_lds(ssd2::grad_kernel<bf16, false>, ssd2::GRAD_LDS);
        else allow_lds(ssd2::grad_kernel<bf16, true>, ssd2::GRAD_LDS);
        if (k3) {
            allow_lds(ssd2::uterm_kernel, ssd2::UTERM_LDS);
            hipLaunchKernelGGL(ssd2::uterm_kernel, gch, dim3(256), ssd2::UTERM_LDS, s, a, (const bf16*)xc,
                               (const bf16*)zxbcdt, dt_bias, A_log, (const bf16*)dY, ldy, U, nch);
            hipLaunchKernelGGL(ssd2::rpass_kernel, dim3((unsigned)((B * nheads * P * N + 255) / 256)), dim3(256), 0,
                               s, U, clast, B * nheads, nch);
        } else {
            allow_lds(ssd2::scan_bwd_kernel, ssd2::SCAN_LDS);
            hipLaunchKernelGGL(ssd2::scan_bwd_kernel, dim3((unsigned)(B * nheads)), dim3(256), ssd2::SCAN_LDS, s, a,
                               (const bf16*)xc, (const bf16*)zxbcdt, dt_bias, A_log, (const bf16*)dY, ldy, (bf16*)U,
                               nch, (bf16*)(dbc + B * L * nheads * 2 * N));
        }
        const dim3 gg((unsigned)(B * (nheads / hg) * nch));
        if (k3) hipLaunchKernelGGL((ssd2::grad_kernel<bf16, false>), gg, dim3(256), ssd2::GRAD_LDS, s, a, (const bf16*)xc,
                                   (const bf16*)zxbcdt, dt_bias, A_log, D, (const bf16*)dY, ldy, states, U, dxc, dbc,
                                   (bf16*)dzxbcdt, gA_log, gD, gdt_bias, nch, hg);
        else hipLaunchKernelGGL((ssd2::grad_kernel<bf16, true>), gg, dim3(256), ssd2::GRAD_LDS, s, a, (const bf16*)xc,
                                (const bf16*)zxbcdt, dt_bias, A_log, D, (const bf16*)dY, ldy, states, U, dxc, dbc,
                                (bf16*)dzxbcdt, gA_log, gD, gdt_bias, nch, hg);
        hipLaunchKernelGGL(ssd2::dbc_reduce_kernel, dim3((unsigned)((B * L * (2 * N / 4) + 255) / 256)), dim3(256), 0,
                           s, dbc, dxc, B * L, nheads / hg, ldxc, d_inner);
        MSQ_LAUNCH_CHECK();
        return MSQ_OK;
    }
    hipMemset2DAsync(dxc + d_inner, ldxc * sizeof(float), 0, 2 * N * sizeof(float), B * L, s);
    const dim3 grid((unsigned)(B * nheads));
    allow_lds(ssd_bwd_kernel<float, float>, BWD_LDS);
    hipLaunchKernelGGL((ssd_bwd_kernel<float, float>), grid, dim3(NT), BWD_LDS, s, a, (const float*)xc, (const float*)zxbcdt, dt_bias, A_log, D, (const float*)dY, ldy, states, dxc, (float*)dzxbcdt, gA_log, gD, gdt_bias);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_mamba_conv_bwd(void* dzxbcdt, const float* dxc, int64_t ld_dxc, const void* zxbcdt, int64_t ldz,
                                  int dtype, const float* conv_w, const float* conv_b, float* g_conv_w,
                                  float* g_conv_b, int64_t B, int64_t L, int64_t d_inner, int64_t nheads,
                                  void* stream) {
    MSQ_CHECK_ARG(B > 0 && L > 0 && d_inner == nheads * P && ldz % 4 == 0 && ld_dxc % 4 == 0,
                  "mamba conv bwd: bad sizes");
    MSQ_CHECK_ARG((uintptr_t)zxbcdt % 16 == 0 && (uintptr_t)dzxbcdt % 16 == 0 && (uintptr_t)dxc % 16 == 0,
                  "msq_mamba_conv_bwd: 16-B aligned buffers");
    const MambaArgs a = mk(B, L, d_inner, nheads, ldz, ld_dxc);
    hipStream_t s = (hipStream_t)stream;
    const unsigned tch = (unsigned)((L + 4 * CONV_SEG - 1) / (4 * CONV_SEG));
    const dim3 grid((unsigned)((a.conv_dim + 64 * CONV_CV - 1) / (64 * CONV_CV)), (unsigned)B, tch);
    if (dtype == MSQ_BF16) hipLaunchKernelGGL((conv_bwd_kernel<bf16, bf16>), grid, dim3(256), 0, s, a, (const bf16*)zxbcdt, conv_w, conv_b, dxc, ld_dxc, (bf16*)dzxbcdt, g_conv_w, g_conv_b);
    else hipLaunchKernelGGL((conv_bwd_kernel<float, float>), grid, dim3(256), 0, s, a, (const float*)zxbcdt, conv_w, conv_b, dxc, ld_dxc, (float*)dzxbcdt, g_conv_w, g_conv_b);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
