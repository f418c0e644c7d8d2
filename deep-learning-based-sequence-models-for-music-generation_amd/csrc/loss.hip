// Grammar-weighted "filtered" loss (train.py:79-138, train_parallel.py:83-141,
// CrossEntropyLoss at :156,179) without materialising any [B,T,V] weights:
//   W[b,t,:]  = wtab[bucket(src[b,t])]          (5 x V table, L2 resident)
//   lse_t     = logsumexp over the TIME axis of logits[b,:,v]   (colstats)
//   Z[b,t,v]  = -(o[b,t,v] - lse_t[b,v]) * W[b,t,v]             (filtered_logit)
//   loss      = mean_{b,t} ( logsumexp_v Z[b,t,:] - Z[b,t,y] )
// Backward for an upstream dZ (CE: dZ = (softmax_v Z - onehot y) * gs):
//   dO = -W*dZ + softmax_t(o) * colsum_t(W*dZ)
// Kernels: colstats (online max/sum over t, split over t), a row kernel (one
// workgroup per 32 rows of one sequence; a row of V values stays in
// registers; the column sums of W*dZ are accumulated in registers over the 32
// rows and flushed with one atomic per column), and an elementwise finisher.
#include "common.h"
#include <type_traits>
#include <stdlib.h>

namespace {

constexpr int NT = 256;
constexpr int VPT = 4;             // values per thread per chunk (vector width)
constexpr int CHUNK = NT * VPT;    // 1024 columns per chunk
constexpr int MAXCH = 18;          // V <= 18432
constexpr int ROWS = 32;           // rows per workgroup in the row kernel
constexpr int TSPLIT = 16;         // time splits in colstats

struct LossArgs {
    const void* o; int64_t ld;
    const int64_t* src; const int64_t* trg;
    const float* wtab;
    int64_t b0, b1, b2, b3;  // bucket boundaries (dyn-1, length-1, time-1, tempo-1)
    int64_t B, T, V;
};

__device__ __forceinline__ int bucket_of(const LossArgs& a, int64_t tok) {
    return (tok > a.b0) + (tok > a.b1) + (tok > a.b2) + (tok > a.b3);
}

template <typename T>
__device__ __forceinline__ f32x4 ld4(const T* p, int64_t v, int64_t V) {
    if (v + 4 <= V) return load4(p + v);
    f32x4 x = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < 4 && v + i < V; ++i) x[i] = (float)p[v + i];
    return x;
}

__device__ __forceinline__ float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- colstats: partial (max, sumexp) over a time split, then merge
template <typename T>
__global__ __launch_bounds__(NT) void colstats_part_kernel(LossArgs a, float* __restrict__ part) {
    const int64_t v = ((int64_t)blockIdx.x * NT + threadIdx.x) * VPT;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (a.T + TSPLIT - 1) / TSPLIT;
    const int64_t t0 = ts * per, t1 = min(a.T, t0 + per);
    if (v >= a.V) return;
    const T* o = (const T*)a.o + b * a.T * a.ld;
    f32x4 m = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY}, s = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int64_t t = t0; t < t1; ++t) {
        const f32x4 x = ld4(o + t * a.ld, v, a.V);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // -inf rows (the cached decode's empty / leaving ring slots) add
            // nothing; skipping them also keeps -inf - -inf out of the sum
            const float mn = fmaxf(m[i], x[i]);
            if (mn != -INFINITY) {
                s[i] = s[i] * expf(m[i] - mn) + expf(x[i] - mn);
                m[i] = mn;
            }
        }
    }
    float* pm = part + ((b * TSPLIT + ts) * 2) * a.V;
    for (int i = 0; i < 4 && v + i < a.V; ++i) {
        pm[v + i] = m[i];
        pm[a.V + v + i] = s[i];
    }
}

__global__ void colstats_merge_kernel(LossArgs a, const float* __restrict__ part, float* __restrict__ col_lse) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.B * a.V) return;
    const int64_t b = e / a.V, v = e % a.V;
    float m = -INFINITY;
    for (int ts = 0; ts < TSPLIT; ++ts) m = fmaxf(m, part[((b * TSPLIT + ts) * 2) * a.V + v]);
    float s = 0.f;
    for (int ts = 0; ts < TSPLIT; ++ts) {
        const float pm = part[((b * TSPLIT + ts) * 2) * a.V + v];
        if (pm != -INFINITY) s += part[((b * TSPLIT + ts) * 2 + 1) * a.V + v] * expf(pm - m);
    }
    col_lse[e] = m + logf(s);
}

// ---- row kernel. MODE 0: loss only; 1: CE train (loss + dO partial);
// 2: given dZ (autograd of filtered_logit); 3: write Z (filtered_logit fwd)
template <int MODE, typename T, typename TD>
__global__ __launch_bounds__(NT) void row_kernel(LossArgs a, const float* __restrict__ col_lse,
                                                 float* __restrict__ loss_rows, TD* __restrict__ dout, int64_t ldd,
                                                 const float* __restrict__ dz, int64_t ldz,
                                                 float* __restrict__ colsum, float gs, int64_t t_begin) {
    __shared__ float red[4];
    const int64_t nrows = a.T - t_begin;
    const int64_t blocks_per_b = (nrows + ROWS - 1) / ROWS;
    const int64_t b = blockIdx.x / blocks_per_b;
    const int64_t r0 = t_begin + (blockIdx.x % blocks_per_b) * ROWS;
    const int64_t r1 = min(a.T, r0 + ROWS);
    const int tid = threadIdx.x;
    const int nch = (int)((a.V + CHUNK - 1) / CHUNK);
    const float* cl = col_lse + b * a.V;
    f32x4 csum[MAXCH];
#pragma unroll
    for (int c = 0; c < MAXCH; ++c) csum[c] = (f32x4){0.f, 0.f, 0.f, 0.f};

    for (int64_t t = r0; t < r1; ++t) {
        const int64_t row = b * a.T + t;
        const T* o = (const T*)a.o + row * a.ld;
        const float* w = a.wtab + bucket_of(a, a.src[row]) * a.V;
        f32x4 z[MAXCH];
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < MAXCH; ++c) {
            const int64_t v = (int64_t)c * CHUNK + tid * VPT;
            z[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (c < nch && v < a.V) {
                const f32x4 ov = ld4(o, v, a.V), cv = ld4(cl, v, a.V), wv = ld4(w, v, a.V);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    z[c][i] = -(ov[i] - cv[i]) * wv[i];
                    if (v + i < a.V) mx = fmaxf(mx, z[c][i]);
                }
            }
        }
        if (MODE == 3) {  // Z output
            TD* zp = dout + (b * nrows + (t - t_begin)) * ldd;  // z rows [B, T - t_begin, V]
#pragma unroll
            for (int c = 0; c < MAXCH; ++c) {
                const int64_t v = (int64_t)c * CHUNK + tid * VPT;
                if (c < nch && v < a.V) {
                    if (v + 4 <= a.V) store4(zp + v, z[c]);
                    else for (int i = 0; v + i < a.V; ++i) zp[v + i] = (TD)z[c][i];
                }
            }
            continue;
        }
        float lse = 0.f;
        if (MODE == 0 || MODE == 1) {
            mx = block_max(mx, red);
            float se = 0.f;
#pragma unroll
            for (int c = 0; c < MAXCH; ++c) {
                const int64_t v = (int64_t)c * CHUNK + tid * VPT;
                if (c < nch && v < a.V) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (v + i < a.V) se += expf(z[c][i] - mx);
                }
            }
            lse = mx + logf(block_sum(se, red));
            if (tid == 0) {
                const int64_t y = a.trg[row];
                const float zy = -((float)((const T*)a.o)[row * a.ld + y] - cl[y]) * w[y];
                loss_rows[row] = lse - zy;
            }
        }
        if (MODE == 0) continue;
        // dZ -> wg = W*dZ ; dO = -wg ; colsum += wg
        const int64_t y = MODE == 1 ? a.trg[row] : -1;
        TD* dp = dout + row * ldd;
#pragma unroll
        for (int c = 0; c < MAXCH; ++c) {
            const int64_t v = (int64_t)c * CHUNK + tid * VPT;
            if (c < nch && v < a.V) {
                const f32x4 wv = ld4(w, v, a.V);
                f32x4 g;
                if (MODE == 1) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) g[i] = (expf(z[c][i] - lse) - (v + i == y ? 1.f : 0.f)) * gs;
                } else {
                    g = ld4(dz + (b * a.T + t) * ldz, v, a.V);
                    g *= gs;
                }
                const f32x4 wg = wv * g;
                csum[c] += wg;
                if (v + 4 <= a.V) store4(dp + v, -wg);
                else for (int i = 0; v + i < a.V; ++i) dp[v + i] = (TD)(-wg[i]);
            }
        }
    }
    if (MODE == 1 || MODE == 2) {
#pragma unroll
        for (int c = 0; c < MAXCH; ++c) {
            const int64_t v = (int64_t)c * CHUNK + tid * VPT;
            if (c < nch && v < a.V) {
                for (int i = 0; i < 4 && v + i < a.V; ++i) atomicAdd(colsum + b * a.V + v + i, csum[c][i]);
            }
        }
    }
}

// dO[b,t,v] += exp(o[b,t,v] - lse_t[b,v]) * colsum[b,v]
template <typename T, typename TD>
__global__ void finish_kernel(LossArgs a, const float* __restrict__ col_lse, const float* __restrict__ colsum,
                              TD* __restrict__ dout, int64_t ldd) {
    const int64_t V4 = (a.V + 3) / 4;
    const int64_t total = a.B * a.T * V4;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = e / V4, v = (e % V4) * 4;
        const int64_t b = row / a.T;
        const f32x4 ov = ld4((const T*)a.o + row * a.ld, v, a.V);
        const f32x4 cl = ld4(col_lse + b * a.V, v, a.V);
        const f32x4 cs = ld4(colsum + b * a.V, v, a.V);
        TD* dp = dout + row * ldd;
        f32x4 d = ld4(dp, v, a.V);
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] += expf(ov[i] - cl[i]) * cs[i];
        if (v + 4 <= a.V) store4(dp + v, d);
        else for (int i = 0; v + i < a.V; ++i) dp[v + i] = (TD)d[i];
    }
}

// mean of n floats, one 1024-thread workgroup, fixed summation order: 16-B
// loads, 4 running sums per thread, unrolled so several loads are in flight
// (the 256-thread scalar loop took 100 us for the 65 536 rows of cfg 2)
__global__ __launch_bounds__(1024) void mean_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
    __shared__ float red[16];
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    const int64_t n4 = ((uintptr_t)x % 16) == 0 ? n / 4 : 0;
#pragma unroll 8
    for (int64_t q = threadIdx.x; q < n4; q += 1024) {
        const f32x4 v = ((const f32x4*)x)[q];
        s0 += v[0];
        s1 += v[1];
        s2 += v[2];
        s3 += v[3];
    }
    for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += 1024) s0 += x[i];
    float s = wave_sum((s0 + s1) + (s2 + s3));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < 16; ++w) t += red[w];
        *out = t / (float)n;
    }
}

// ---- streaming CE path (train step): three passes over the logits, each
// one coalesced 16-B-per-lane read (+ one write in pass 3):
//   colstats2  per (b, v) online max / sum over a time split       (read o)
//   rowstats2  per row: logsumexp_v Z, loss, and colsum_t(W dZ)     (read o)
//   finish2    dO = -W dZ + softmax_t(o) colsum_t(W dZ)             (read o, write dO)
// W rows come from the L2-resident 5 x V table; col_lse and colsum of a
// thread's columns stay in registers across rows. VEC columns per thread
// (8 bf16 / 4 fp32 = 16 B).
template <typename T> struct VecOf { static constexpr int N = 16 / sizeof(T); };

// 16-B aligned vector load / store of N = 16/sizeof(T) elements (callers keep
// every access inside a padded row)
template <typename T, int N>
__device__ __forceinline__ void ldv(const T* p, float (&x)[N]) {
    if constexpr (sizeof(T) == 2) {
        const bf16x8 u = *(const bf16x8*)p;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = (float)u[i];
    } else {
        const f32x4 u = *(const f32x4*)p;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = u[i];
    }
}
template <int N>
__device__ __forceinline__ void ldf(const float* p, float (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
        const f32x4 u = *(const f32x4*)(p + i);
        x[i] = u[0], x[i + 1] = u[1], x[i + 2] = u[2], x[i + 3] = u[3];
    }
}
template <typename T, int N>
__device__ __forceinline__ void stv(T* p, const float (&x)[N]) {
    if constexpr (sizeof(T) == 2) {
        bf16x8 u;
#pragma unroll
        for (int i = 0; i < N; ++i) u[i] = (bf16)x[i];
        *(bf16x8*)p = u;
    } else {
        *(f32x4*)p = (f32x4){x[0], x[1], x[2], x[3]};
    }
}
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

constexpr int TS2 = 32;    // time splits of colstats2 / finish2

// Padded layouts (Vp = V rounded up to 16): col_lse copy, colsum and the 5-row
// weight table live in the workspace with zero pads, so every 16-B access is
// in bounds and unconditional; only the last column chunk masks v >= V.
__global__ void pad_table_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t rows, int64_t V,
                                 int64_t Vp) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * Vp) return;
    const int64_t r = e / Vp, v = e % Vp;
    dst[e] = v < V ? src[r * V + v] : 0.f;
}

template <typename T>
__global__ __launch_bounds__(NT) void colstats2_kernel(LossArgs a, float* __restrict__ part) {
    constexpr int N = VecOf<T>::N;
    const int v = (blockIdx.x * NT + threadIdx.x) * N;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (a.T + TS2 - 1) / TS2;
    const int64_t t0 = ts * per, t1 = min(a.T, t0 + per);
    if (v >= a.V) return;
    const T* o = (const T*)a.o + b * a.T * a.ld + v;
    constexpr float L2E = 1.4426950408889634f;
    float m[N], s[N];
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = -INFINITY, s[i] = 0.f;
    // 4 rows per online-softmax update: 5 exponentials per 4 elements, 4 loads in flight
    constexpr int U = 4;
    int64_t t = t0;
    for (; t + U <= t1; t += U) {
        float x[U][N];
#pragma unroll
        for (int u = 0; u < U; ++u) ldv<T, N>(o + (t + u) * a.ld, x[u]);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float mn = fmaxf(fmaxf(m[i], fmaxf(x[0][i], x[1][i])), fmaxf(x[2][i], x[3][i]));
            const float ml = mn * L2E;
            float e = s[i] * __builtin_amdgcn_exp2f(__builtin_fmaf(m[i], L2E, -ml));
#pragma unroll
            for (int u = 0; u < U; ++u) e += __builtin_amdgcn_exp2f(__builtin_fmaf(x[u][i], L2E, -ml));
            s[i] = e;
            m[i] = mn;
        }
    }
    for (; t < t1; ++t) {
        float x[N];
        ldv<T, N>(o + t * a.ld, x);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float mn = fmaxf(m[i], x[i]);
            s[i] = s[i] * fexp(m[i] - mn) + fexp(x[i] - mn);
            m[i] = mn;
        }
    }
    float* pm = part + ((b * TS2 + ts) * 2) * a.V;
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (v + i < a.V) {
            pm[v + i] = m[i];
            pm[a.V + v + i] = s[i];
        }
}

// nts partials per sequence, (max, sum) rows of stride pst: part[((b nts + ts) 2) pst + v]
// (colstats2: nts = TS2, pst = V; the lm_head GEMM epilogue: nts = T / 128, pst = its ld)
__global__ void colstats2_merge_kernel(LossArgs a, const float* __restrict__ part, float* __restrict__ col_lse,
                                       float* __restrict__ clp, int64_t Vp, int nts, int64_t pst) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.B * Vp) return;
    const int64_t b = e / Vp, v = e % Vp;
    if (v >= a.V) {
        clp[e] = 0.f;
        return;
    }
    float m = -INFINITY;
    for (int ts = 0; ts < nts; ++ts) m = fmaxf(m, part[((b * nts + ts) * 2) * pst + v]);
    float s = 0.f;
    for (int ts = 0; ts < nts; ++ts) {
        const float pm = part[((b * nts + ts) * 2) * pst + v];
        if (pm != -INFINITY) s += part[((b * nts + ts) * 2 + 1) * pst + v] * expf(pm - m);
    }
    const float l = m + logf(s);
    col_lse[b * a.V + v] = l;
    clp[e] = l;
}

__device__ __forceinline__ float block8_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) r = fmaxf(r, red[i]);
    return r;
}
__device__ __forceinline__ float block8_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
}

// nonzero column range [lo, hi) of every weight-table row (lo = hi = 0 for an
// all-zero row): rowstats2 reads only the logits of those columns, since
// Z = -(o - col_lse) W is exactly 0 wherever W is 0
__global__ void wrange_kernel(const float* __restrict__ wtp, int64_t Vp, int64_t V, int* __restrict__ range) {
    __shared__ int red[2][4];
    const int k = blockIdx.x, tid = threadIdx.x;
    int lo = INT32_MAX, hi = -1;
    for (int64_t v = tid; v < V; v += 256)
        if (wtp[k * Vp + v] != 0.f) lo = min(lo, (int)v), hi = max(hi, (int)v);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lo = min(lo, __shfl_xor(lo, o, 64)), hi = max(hi, __shfl_xor(hi, o, 64));
    if ((tid & 63) == 0) red[0][tid >> 6] = lo, red[1][tid >> 6] = hi;
    __syncthreads();
    if (tid == 0) {
        lo = min(min(red[0][0], red[0][1]), min(red[0][2], red[0][3]));
        hi = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
        range[2 * k] = hi < 0 ? 0 : lo;
        range[2 * k + 1] = hi + 1;
    }
}

// Per row, one wave (log2 domain, z = Z log2 e = (cl - o) W log2 e):
//   row_lse = logsumexp_v Z,  loss_row = row_lse - Z[y]
// Only the bucket's nonzero weight range [lo, hi) is read; the V - (hi - lo)
// columns outside it have Z = 0 exactly and enter the sum analytically.
template <typename T>
__global__ __launch_bounds__(256) void rowlse_kernel(LossArgs a, const float* __restrict__ clp,
                                                     const float* __restrict__ wtp, int Vp,
                                                     const int* __restrict__ wrange, float* __restrict__ loss_rows,
                                                     float* __restrict__ row_lse) {
    constexpr int N = VecOf<T>::N;
    constexpr float L2E = 1.4426950408889634f;
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    if (row >= a.B * a.T) return;  // whole waves; no block-level sync below
    const int64_t b = row / a.T;
    const int bk = bucket_of(a, a.src[row]);
    const int lo = wrange[2 * bk], hi = wrange[2 * bk + 1];
    const T* o = (const T*)a.o + row * a.ld;
    const float* cl = clp + b * Vp;
    const float* w = wtp + (int64_t)bk * Vp;
    float m = -INFINITY, s = 0.f;
    for (int v = (lo & ~(N - 1)) + lane * N; v < hi; v += 64 * N) {
        float x[N], c[N], ww[N], z[N];
        ldv<T, N>(o + v, x);
        ldf<N>(cl + v, c);
        ldf<N>(w + v, ww);
        float mm = m;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            z[i] = (v + i >= lo && v + i < hi) ? (c[i] - x[i]) * ww[i] * L2E : -INFINITY;
            mm = fmaxf(mm, z[i]);
        }
        if (mm != -INFINITY) {
            float e = m == -INFINITY ? 0.f : s * __builtin_amdgcn_exp2f(m - mm);
#pragma unroll
            for (int i = 0; i < N; ++i) e += __builtin_amdgcn_exp2f(z[i] - mm);
            s = e;
            m = mm;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
        const float mn = fmaxf(m, m2);
        s = (mn == -INFINITY) ? 0.f
                              : (m == -INFINITY ? 0.f : s * __builtin_amdgcn_exp2f(m - mn)) +
                                    (m2 == -INFINITY ? 0.f : s2 * __builtin_amdgcn_exp2f(m2 - mn));
        m = mn;
    }
    if (lane == 0) {
        const int inact = (int)a.V - (hi - lo);  // columns with Z = 0 outside the range
        if (inact > 0) {
            const float mn = fmaxf(m, 0.f);
            s = (m == -INFINITY ? 0.f : s * __builtin_amdgcn_exp2f(m - mn)) + (float)inact * __builtin_amdgcn_exp2f(-mn);
            m = mn;
        }
        const float lse2 = m + __builtin_log2f(s);
        const int y = (int)a.trg[row];
        const float zy = (y >= lo && y < hi) ? (cl[y] - (float)o[y]) * w[y] * L2E : 0.f;
        loss_rows[row] = (lse2 - zy) / L2E;
        row_lse[row] = lse2 / L2E;
    }
}

// colsum_t(W dZ) partials per (batch, time split): thread-owned columns as in
// finish2, W dZ = W gs (softmax_v Z - onehot y); rows whose bucket has zero
// weight on the thread's columns contribute 0 and are not read.
template <typename T>
__global__ __launch_bounds__(NT) void cspart_kernel(LossArgs a, const float* __restrict__ clp,
                                                    const float* __restrict__ wtp, int Vp,
                                                    const float* __restrict__ row_lse, float gs,
                                                    float* __restrict__ part) {
    constexpr int N = VecOf<T>::N;
    constexpr float L2E = 1.4426950408889634f;
    __shared__ f32x4 wl[5][NT * N / 4];
    const int tid = threadIdx.x;
    const int v = (blockIdx.x * NT + tid) * N;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (a.T + TS2 - 1) / TS2;
    const int64_t t0 = ts * per, t1 = min(a.T, t0 + per);
    if (v >= a.V) return;  // only this thread's own LDS slots are read
    float cl2[N], cs[N];
    ldf<N>(clp + b * Vp + v, cl2);
#pragma unroll
    for (int i = 0; i < N; ++i) cl2[i] *= L2E, cs[i] = 0.f;
    unsigned nzb = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        float w[N];
        ldf<N>(wtp + (int64_t)k * Vp + v, w);
        bool nz = false;
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            wl[k][tid * (N / 4) + i / 4] = (f32x4){w[i], w[i + 1], w[i + 2], w[i + 3]};
            nz |= (w[i] != 0.f) | (w[i + 1] != 0.f) | (w[i + 2] != 0.f) | (w[i + 3] != 0.f);
        }
        nzb |= (unsigned)nz << k;
    }
    auto one = [&](const float (&ov)[N], int bk, int y, float lse) {
        float w[N];
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            const f32x4 u = wl[bk][tid * (N / 4) + i / 4];
            w[i] = u[0], w[i + 1] = u[1], w[i + 2] = u[2], w[i + 3] = u[3];
        }
        const float l2 = lse * L2E;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float av = __builtin_fmaf(ov[i], L2E, -cl2[i]);
            const float sv = __builtin_amdgcn_exp2f(__builtin_fmaf(-av, w[i], -l2));
            cs[i] = __builtin_fmaf(w[i] * gs, sv, cs[i]);
        }
        if ((unsigned)(y - v) < (unsigned)N) {
#pragma unroll
            for (int i = 0; i < N; ++i)
                if (v + i == y) cs[i] -= w[i] * gs;
        }
    };
    constexpr int U = 4;
    int64_t t = t0;
    for (; t + U <= t1; t += U) {
        float ov[U][N];
        int bk[U], y[U];
        float lse[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = b * a.T + t + u;
            bk[u] = bucket_of(a, a.src[row]);
            y[u] = (int)a.trg[row];
            lse[u] = row_lse[row];
            if ((nzb >> bk[u]) & 1) ldv<T, N>((const T*)a.o + row * a.ld + v, ov[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if ((nzb >> bk[u]) & 1) one(ov[u], bk[u], y[u], lse[u]);
    }
    for (; t < t1; ++t) {
        const int64_t row = b * a.T + t;
        const int bk = bucket_of(a, a.src[row]);
        if ((nzb >> bk) & 1) {
            float ov[N];
            ldv<T, N>((const T*)a.o + row * a.ld + v, ov);
            one(ov, bk, (int)a.trg[row], row_lse[row]);
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) part[(b * TS2 + ts) * Vp + v + i] = v + i < a.V ? cs[i] : 0.f;
}

// colsum[b][v] = sum over the TS2 partials in a fixed order (pads -> 0)
__global__ void cs_reduce_kernel(const float* __restrict__ part, int64_t B, int64_t V, int64_t Vp,
                                 float* __restrict__ colsum) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= B * Vp) return;
    const int64_t b = e / Vp, v = e % Vp;
    float s = 0.f;
    if (v < V) {
        const float* p = part + b * TS2 * Vp + v;
#pragma unroll 8
        for (int ts = 0; ts < TS2; ++ts) s += p[ts * Vp];
    }
    colsum[e] = s;
}

// dO[t,v] = -W[v] dZ[t,v] + softmax_t(o)[t,v] colsum_t(W dZ)[v], in the log2
// domain (a = (o - col_lse) log2 e):
//   softmax_t(o) = 2^a,  softmax_v(Z) = 2^(-a W - row_lse log2 e)
// A thread's 5 weight rows sit in LDS (indexed by the row's bucket, no
// register select chains); a bucket whose weights are all 0 on the thread's
// columns (most columns of the sparse grammar rows) skips the dZ term.
template <typename T, typename TD>
__global__ __launch_bounds__(NT) void finish2_kernel(LossArgs a, const float* __restrict__ clp,
                                                     const float* __restrict__ wtp, int Vp,
                                                     const float* __restrict__ row_lse,
                                                     const float* __restrict__ colsum, TD* __restrict__ dout,
                                                     int64_t ldd, float gs, float* __restrict__ dbias) {
    constexpr int N = VecOf<T>::N;
    constexpr float L2E = 1.4426950408889634f;
    __shared__ f32x4 wl[5][NT * N / 4];
    const int tid = threadIdx.x;
    const int v = (blockIdx.x * NT + tid) * N;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (a.T + TS2 - 1) / TS2;
    const int64_t t0 = ts * per, t1 = min(a.T, t0 + per);
    if (v >= a.V) return;  // only this thread's own LDS slots are ever read: no barrier needed
    float cl2[N], cs[N];
    ldf<N>(clp + b * Vp + v, cl2);
    ldf<N>(colsum + b * Vp + v, cs);
#pragma unroll
    for (int i = 0; i < N; ++i) cl2[i] *= L2E;
    unsigned nzb = 0;  // bit k: bucket k has a nonzero weight on this thread's columns
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        float w[N];
        ldf<N>(wtp + (int64_t)k * Vp + v, w);
        bool nz = false;
#pragma unroll
        for (int i = 0; i < N; i += 4) {
            wl[k][tid * (N / 4) + i / 4] = (f32x4){w[i], w[i + 1], w[i + 2], w[i + 3]};
            nz |= (w[i] != 0.f) | (w[i + 1] != 0.f) | (w[i + 2] != 0.f) | (w[i + 3] != 0.f);
        }
        nzb |= (unsigned)nz << k;
    }
    const bool edge = v + N > a.V;  // the one thread holding pad columns
    float bs[N];
#pragma unroll
    for (int i = 0; i < N; ++i) bs[i] = 0.f;
    auto one = [&](int64_t row, const float (&ov)[N], int bk, int y, float lse) {
        float d[N], ea[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float av = __builtin_fmaf(ov[i], L2E, -cl2[i]);
            ea[i] = __builtin_amdgcn_exp2f(av);
            d[i] = av;
        }
        if ((nzb >> bk) & 1) {
            float w[N];
#pragma unroll
            for (int i = 0; i < N; i += 4) {
                const f32x4 u = wl[bk][tid * (N / 4) + i / 4];
                w[i] = u[0], w[i + 1] = u[1], w[i + 2] = u[2], w[i + 3] = u[3];
            }
            const float l2 = lse * L2E;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const float sv = __builtin_amdgcn_exp2f(__builtin_fmaf(-d[i], w[i], -l2));  // softmax_v Z
                d[i] = __builtin_fmaf(ea[i], cs[i], -w[i] * sv * gs);
            }
            if ((unsigned)(y - v) < (unsigned)N) {
#pragma unroll
                for (int i = 0; i < N; ++i)
                    if (v + i == y) d[i] += w[i] * gs;
            }
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) d[i] = ea[i] * cs[i];
        }
        if (edge) {
#pragma unroll
            for (int i = 0; i < N; ++i)
                if (v + i >= a.V) d[i] = 0.f;  // pad columns stay 0
        }
#pragma unroll
        for (int i = 0; i < N; ++i) bs[i] += d[i];
        stv<TD, N>(dout + row * ldd + v, d);
    };
    // 4 rows per step: their loads are all in flight before the first use
    constexpr int U = 4;
    int64_t t = t0;
    for (; t + U <= t1; t += U) {
        float ov[U][N];
        int bk[U], y[U];
        float lse[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = b * a.T + t + u;
            ldv<T, N>((const T*)a.o + row * a.ld + v, ov[u]);
            bk[u] = bucket_of(a, a.src[row]);
            y[u] = (int)a.trg[row];
            lse[u] = row_lse[row];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) one(b * a.T + t + u, ov[u], bk[u], y[u], lse[u]);
    }
    for (; t < t1; ++t) {
        const int64_t row = b * a.T + t;
        float ov[N];
        ldv<T, N>((const T*)a.o + row * a.ld + v, ov);
        one(row, ov, bucket_of(a, a.src[row]), (int)a.trg[row], row_lse[row]);
    }
    // dbias partials: column sums of this thread's dlogits rows (the output bias
    // gradient), written per (batch, time split) and reduced in a fixed order by
    // dbias_reduce_kernel, so the bias gradient is bitwise reproducible
    if (dbias) {
#pragma unroll
        for (int i = 0; i < N; ++i) dbias[(b * TS2 + ts) * Vp + v + i] = bs[i];
    }
}

// 1024 threads = 64 columns x 16 partial groups (partials g, g+16, ...), the
// 16 group sums added in a fixed order through LDS: deterministic, and 16
// waves per CU keep enough loads in flight for the [B*TS2][Vp] partials
__global__ __launch_bounds__(1024) void dbias_reduce_kernel(const float* __restrict__ part, int64_t nparts, int Vp,
                                                            int64_t V, float* __restrict__ dbias) {
    __shared__ float red[16][64];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t v = (int64_t)blockIdx.x * 64 + c;
    float s = 0.f;
    if (v < V) {
        int64_t p = g;
        for (; p + 48 < nparts; p += 64) {
            const float x0 = part[p * Vp + v], x1 = part[(p + 16) * Vp + v];
            const float x2 = part[(p + 32) * Vp + v], x3 = part[(p + 48) * Vp + v];
            s += x0; s += x1; s += x2; s += x3;
        }
        for (; p < nparts; p += 16) s += part[p * Vp + v];
    }
    red[g][c] = s;
    __syncthreads();
    if (g == 0 && v < V) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) t += red[k][c];
        dbias[v] += t;
    }
}

// fallback for dbias where finish2 does not run: column sums of dlogits rows
template <typename TD>
__global__ void dlogit_colsum_kernel(const TD* __restrict__ d, int64_t ldd, int64_t rows, int64_t V,
                                     float* __restrict__ dbias) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    float s = 0.f;
    for (int64_t r = 0; r < rows; ++r) s += (float)d[r * ldd + v];
    dbias[v] += s;
}

LossArgs mk(const void* o, int64_t ld, const int64_t* src, const int64_t* trg, const float* wtab, int64_t b0,
            int64_t b1, int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V) {
    LossArgs a;
    a.o = o; a.ld = ld; a.src = src; a.trg = trg; a.wtab = wtab;
    a.b0 = b0; a.b1 = b1; a.b2 = b2; a.b3 = b3;
    a.B = B; a.T = T; a.V = V;
    return a;
}

template <typename T>
void colstats_launch(const LossArgs& a, float* col_lse, float* part, hipStream_t s) {
    dim3 grid((unsigned)((a.V + CHUNK - 1) / CHUNK), (unsigned)a.B, TSPLIT);
    hipLaunchKernelGGL(colstats_part_kernel<T>, grid, dim3(NT), 0, s, a, part);
    hipLaunchKernelGGL(colstats_merge_kernel, dim3((unsigned)((a.B * a.V + 255) / 256)), dim3(256), 0, s, a, part,
                       col_lse);
}

// ---- cached decode (TransformerEngine.step): time-axis LSE over a ring of
// logits rows [B][ctx][ld], kept as per-block partials lse_blk[b][blk][v] over
// RB-row blocks, so a step re-reads one or two blocks instead of the window.
// partial LSE of ring rows [blk*rb, blk*rb + rb) except row `skip` for this
// thread's N columns v..v+N-1 of row set b
template <typename T>
__device__ __forceinline__ void ring_block_lse(const T* __restrict__ ring, int64_t ld, int64_t ctx, int64_t V,
                                               int64_t rb, int64_t b, int64_t blk, int64_t skip, int64_t v,
                                               float* __restrict__ part, int64_t nblk) {
    constexpr int N = VecOf<T>::N;
    constexpr float L2E = 1.4426950408889634f;
    const int64_t t0 = blk * rb, t1 = min(ctx, t0 + rb);
    float m[N], sm[N];
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = -INFINITY, sm[i] = 0.f;
    for (int64_t t = t0; t < t1; ++t) {
        if (t == skip) continue;
        float x[N];
        ldv<T, N>(ring + (b * ctx + t) * ld + v, x);
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (x[i] == -INFINITY) continue;  // empty ring rows
            const float mn = fmaxf(m[i], x[i]);
            sm[i] = (m[i] == -INFINITY ? 0.f : sm[i] * __builtin_amdgcn_exp2f((m[i] - mn) * L2E)) +
                    __builtin_amdgcn_exp2f((x[i] - mn) * L2E);
            m[i] = mn;
        }
    }
    float* pp = part + (b * nblk + blk) * V;
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (v + i < V) pp[v + i] = m[i] == -INFINITY ? -INFINITY : m[i] + logf(sm[i]);
}

template <typename T>
__global__ __launch_bounds__(NT) void ring_block_lse_kernel(const T* __restrict__ ring, int64_t ld, int64_t ctx,
                                                            int64_t V, int64_t rb, int64_t blk0, int64_t skip,
                                                            float* __restrict__ part, int64_t nblk) {
    const int64_t v = ((int64_t)blockIdx.x * NT + threadIdx.x) * VecOf<T>::N;
    if (v >= V) return;
    ring_block_lse<T>(ring, ld, ctx, V, rb, blockIdx.y, blk0 + blockIdx.z, skip, v, part, nblk);
}

// Graph-replayed decode step (msq_ring_step), position from *pos, slot j =
// pos % ctx in block c (row jj of it). The LSE of the window's other rows is
//   lae(O_c, P, Q_c[jj]):  O_c = the blocks other than c (their partials),
//   P = the rows of block c before j (this ring cycle's new rows, kept as a
//   running prefix), Q_c[jj] = the rows of block c after j (last cycle's rows,
//   a suffix table built when the step enters block c).
// Blocks other than c do not change while the slot walks through c, so a
// step reads ~22 B per (b, v) instead of re-reading a 64-row block and
// merging every block partial (~2.3 KB at ctx 2048). A step entering a block
// (slot jj = 0, or cur_blk != c: also the first step, cur_blk = -1 after
// msq_ring_lse filled every partial) stores the finished prefix as the left
// block's partial, merges O_c and scans block c's rows once for the suffix
// table and the prefix.
__device__ __forceinline__ void lse_acc(float& m, float& sm, float x) {  // running (max, scaled sum)
    if (x == -INFINITY) return;
    if (x > m) {
        sm = (m == -INFINITY ? 0.f : sm * expf(m - x)) + 1.f;
        m = x;
    } else {
        sm += expf(x - m);
    }
}
__device__ __forceinline__ float lse_val(float m, float sm) { return m == -INFINITY ? -INFINITY : m + logf(sm); }

template <typename T>
__global__ __launch_bounds__(NT) void ring_inc_kernel(const T* __restrict__ ring, int64_t ld, int64_t ctx, int64_t V,
                                                      int64_t rb, int64_t nblk, const int64_t* __restrict__ posp,
                                                      float* __restrict__ part, float* __restrict__ others,
                                                      float* __restrict__ pre, float* __restrict__ suf,
                                                      const int64_t* __restrict__ cur_blk,
                                                      float* __restrict__ col_lse) {
    constexpr int N = VecOf<T>::N;
    const int64_t v = ((int64_t)blockIdx.x * NT + threadIdx.x) * N, b = blockIdx.y;
    if (v >= V) return;
    const int nv = (int)min<int64_t>(N, V - v);
    const int64_t j = *posp % ctx, c = j / rb, jj = j - c * rb, t_end = min(ctx, c * rb + rb);
    const int64_t cb = *cur_blk;
    const T* rb_ = ring + b * ctx * ld + v;
    float* pp = pre + b * V + v;
    float* op = others + b * V + v;
    float* sp = suf + b * rb * V + v;
    float P[N], O[N], Q[N];
    if (cb != c || jj == 0) {  // entering block c (also: the ring wrapped onto the same block)
        float m[N], sm[N], x[N];
        for (int i = 0; i < nv; ++i) P[i] = pp[i];
        if (cb >= 0)  // the block just left: its finished prefix is its partial
            for (int i = 0; i < nv; ++i) part[(b * nblk + cb) * V + v + i] = P[i];
        for (int i = 0; i < N; ++i) m[i] = -INFINITY, sm[i] = 0.f;
        for (int64_t k = 0; k < nblk; ++k) {
            if (k == c) continue;
            for (int i = 0; i < nv; ++i) lse_acc(m[i], sm[i], k == cb ? P[i] : part[(b * nblk + k) * V + v + i]);
        }
        for (int i = 0; i < nv; ++i) op[i] = O[i] = lse_val(m[i], sm[i]);
        // suffix table: Q[i'] = rows c*rb + i' + 1 .. t_end - 1, for i' = t_end-1-c*rb down to jj
        for (int i = 0; i < N; ++i) m[i] = -INFINITY, sm[i] = 0.f;
        for (int64_t t = t_end - 1; t >= j; --t) {
            for (int i = 0; i < nv; ++i) sp[(t - c * rb) * V + i] = lse_val(m[i], sm[i]);
            if (t == j) break;
            ldv<T, N>(rb_ + t * ld, x);
            for (int i = 0; i < nv; ++i) lse_acc(m[i], sm[i], x[i]);
        }
        for (int i = 0; i < nv; ++i) Q[i] = lse_val(m[i], sm[i]);
        // prefix: rows c*rb .. j-1
        for (int i = 0; i < N; ++i) m[i] = -INFINITY, sm[i] = 0.f;
        for (int64_t t = c * rb; t < j; ++t) {
            ldv<T, N>(rb_ + t * ld, x);
            for (int i = 0; i < nv; ++i) lse_acc(m[i], sm[i], x[i]);
        }
        for (int i = 0; i < nv; ++i) P[i] = lse_val(m[i], sm[i]);
    } else {
        for (int i = 0; i < nv; ++i) P[i] = pp[i], O[i] = op[i], Q[i] = sp[jj * V + i];
    }
    float x[N];
    ldv<T, N>(rb_ + j * ld, x);  // the new row (ring_put_kernel ran before)
    for (int i = 0; i < nv; ++i) {
        float m = -INFINITY, sm = 0.f;
        lse_acc(m, sm, O[i]);
        lse_acc(m, sm, P[i]);
        lse_acc(m, sm, Q[i]);
        col_lse[b * V + v + i] = lse_val(m, sm);
        m = -INFINITY, sm = 0.f;  // the prefix of the next step takes the new row
        lse_acc(m, sm, P[i]);
        lse_acc(m, sm, x[i]);
        pp[i] = lse_val(m, sm);
    }
}

// after the step's last reader of *pos: the block the tables now describe, and the next position
__global__ void ring_advance_kernel(int64_t* __restrict__ pos, int64_t* __restrict__ cur_blk, int64_t ctx, int64_t rb) {
    if (threadIdx.x == 0) {
        *cur_blk = (*pos % ctx) / rb;
        *pos += 1;
    }
}

// the new logits row into its ring slot and its token into the token ring
template <typename T>
__global__ __launch_bounds__(NT) void ring_put_kernel(T* __restrict__ ring, int64_t ld, int64_t ctx,
                                                      const T* __restrict__ row, int64_t ldrow,
                                                      int64_t* __restrict__ tokens, const int64_t* __restrict__ tok,
                                                      const int64_t* __restrict__ posp) {
    constexpr int N = VecOf<T>::N;
    const int64_t b = blockIdx.y, v = ((int64_t)blockIdx.x * NT + threadIdx.x) * N;
    const int64_t slot = *posp % ctx;
    if (v + N <= ld) *(u32x4*)(ring + (b * ctx + slot) * ld + v) = *(const u32x4*)(row + b * ldrow + v);
    if (blockIdx.x == 0 && threadIdx.x == 0) tokens[b * ctx + slot] = tok[b];
}

__global__ void ring_lse_merge_kernel(const float* __restrict__ part, int64_t B, int64_t nblk, int64_t V,
                                      float* __restrict__ col_lse) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= B * V) return;
    const int64_t b = e / V, v = e % V;
    const float* p = part + b * nblk * V + v;
    float m = -INFINITY;
    for (int64_t k = 0; k < nblk; ++k) m = fmaxf(m, p[k * V]);
    float sm = 0.f;
    if (m != -INFINITY)
        for (int64_t k = 0; k < nblk; ++k) {
            const float x = p[k * V];
            if (x != -INFINITY) sm += expf(x - m);
        }
    col_lse[e] = m == -INFINITY ? -INFINITY : m + logf(sm);
}

}  // namespace

extern "C" size_t msq_filtered_workspace(int64_t B, int64_t T, int64_t V) {
    // colstats partials | colsum [B,V] | loss rows [B*T]
    (void)T;
    // | row_lse [B*T] | colstats2 partials [B][TS2][2][V] | clp, colsum [B][Vp] | wtab [5][Vp]
    const size_t Vp = (V + 15) / 16 * 16;
    return (size_t)B * TSPLIT * 2 * V * 4 + (size_t)B * V * 4 + (size_t)B * T * 4 * 2 + 256 +
           (size_t)B * 32 * 2 * V * 4 + (2 * (size_t)B + 5) * Vp * 4 + 64 + 256;
}

#define LOSS_CHECK()                                                                                  \
    MSQ_CHECK_ARG(B > 0 && T > 0 && V > 0 && V <= (int64_t)MAXCH * CHUNK && ld >= V && ld % 4 == 0,    \
                  "filtered loss: bad sizes (V <= %d, ld %% 4 == 0)", MAXCH * CHUNK)

extern "C" int msq_filtered_colstats(float* col_lse, const void* logits, int dtype, int64_t ld, int64_t B, int64_t T,
                                     int64_t V, void* workspace, void* stream) {
    LOSS_CHECK();
    const LossArgs a = mk(logits, ld, nullptr, nullptr, nullptr, 0, 0, 0, 0, B, T, V);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == MSQ_BF16) colstats_launch<bf16>(a, col_lse, (float*)workspace, s);
    else colstats_launch<float>(a, col_lse, (float*)workspace, s);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_filtered_ce(float* loss, void* dlogits, int64_t ldd, const void* logits, int dtype, int64_t ld,
                               const int64_t* src, const int64_t* trg, const float* wtab, int64_t b0, int64_t b1,
                               int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V, float grad_scale,
                               float* col_lse, void* workspace, void* stream) {
    return msq_filtered_ce_bias(loss, dlogits, ldd, nullptr, logits, dtype, ld, src, trg, wtab, b0, b1, b2, b3, B, T, V,
                                grad_scale, col_lse, workspace, stream);
}

static int filtered_ce_impl(float* loss, void* dlogits, int64_t ldd, float* dbias, const void* logits, int dtype,
                            int64_t ld, const int64_t* src, const int64_t* trg, const float* wtab, int64_t b0,
                            int64_t b1, int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V, float grad_scale,
                            float* col_lse, void* workspace, void* stream, const float* colpart, int64_t nts,
                            int64_t pld) {
    MSQ_CHECK_ARG(!dbias || dlogits, "msq_filtered_ce_bias: dbias needs dlogits");
    MSQ_CHECK_ARG(!dlogits || ldd % 4 == 0, "msq_filtered_ce: ldd %% 4 != 0");
    const LossArgs a = mk(logits, ld, src, trg, wtab, b0, b1, b2, b3, B, T, V);
    hipStream_t s = (hipStream_t)stream;
    char* ws = (char*)workspace;
    float* part = (float*)ws;
    float* colsum = (float*)(ws + (size_t)B * TSPLIT * 2 * V * 4);
    float* rows = colsum + B * V;
    float* part2 = (float*)(ws + (size_t)B * TSPLIT * 2 * V * 4 + (size_t)B * V * 4 + (size_t)B * T * 4 * 2 + 256);
    const bool bfl = dtype == MSQ_BF16;
    const bool stream2 = dlogits && ld % 8 == 0 && ldd % 8 == 0 && ((uintptr_t)logits % 16) == 0 &&
                         ((uintptr_t)dlogits % 16) == 0;
    if (!stream2) {
        if (bfl) colstats_launch<bf16>(a, col_lse, part, s);
        else colstats_launch<float>(a, col_lse, part, s);
    }
    const unsigned nblk = (unsigned)(B * ((T + ROWS - 1) / ROWS));
    if (!dlogits) {
        if (bfl) hipLaunchKernelGGL((row_kernel<0, bf16, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, rows, (float*)nullptr, 0, nullptr, 0, nullptr, 0.f, 0);
        else hipLaunchKernelGGL((row_kernel<0, float, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, rows, (float*)nullptr, 0, nullptr, 0, nullptr, 0.f, 0);
    } else if (stream2) {
        // streaming path: colstats2 -> rowlse -> cspart -> finish2 on zero-padded copies
        const int64_t Vp = (V + 15) / 16 * 16;
        float* clp = part2 + (size_t)B * TS2 * 2 * V;
        float* csp = clp + B * Vp;
        float* wtp = csp + B * Vp;
        float* row_lse = rows + B * T;
        hipLaunchKernelGGL(pad_table_kernel, dim3((unsigned)((5 * Vp + 255) / 256)), dim3(256), 0, s, wtab, wtp,
                           (int64_t)5, V, Vp);
        const int N = bfl ? 8 : 4;
        const dim3 gc((unsigned)((V + NT * N - 1) / (NT * N)), (unsigned)B, TS2);
        const dim3 gm((unsigned)((B * Vp + 255) / 256));
        const dim3 gr((unsigned)((B * T + 3) / 4));
        int* wrange = (int*)(wtp + 5 * Vp);
        hipLaunchKernelGGL(wrange_kernel, dim3(5), dim3(256), 0, s, wtp, Vp, V, wrange);
        // part2 carries, in turn: colstats2 partials, colsum partials, dbias partials
        if (colpart) {  // column (max, sum) partials from the lm_head GEMM epilogue
            hipLaunchKernelGGL(colstats2_merge_kernel, gm, dim3(256), 0, s, a, colpart, col_lse, clp, Vp, (int)nts, pld);
        } else if (bfl) {
            hipLaunchKernelGGL(colstats2_kernel<bf16>, gc, dim3(NT), 0, s, a, part2);
            hipLaunchKernelGGL(colstats2_merge_kernel, gm, dim3(256), 0, s, a, part2, col_lse, clp, Vp, TS2, V);
        } else {
            hipLaunchKernelGGL(colstats2_kernel<float>, gc, dim3(NT), 0, s, a, part2);
            hipLaunchKernelGGL(colstats2_merge_kernel, gm, dim3(256), 0, s, a, part2, col_lse, clp, Vp, TS2, V);
        }
        if (bfl) {
            hipLaunchKernelGGL(rowlse_kernel<bf16>, gr, dim3(256), 0, s, a, clp, wtp, (int)Vp, wrange, rows, row_lse);
            hipLaunchKernelGGL(cspart_kernel<bf16>, gc, dim3(NT), 0, s, a, clp, wtp, (int)Vp, row_lse, grad_scale, part2);
            hipLaunchKernelGGL(cs_reduce_kernel, gm, dim3(256), 0, s, part2, B, V, Vp, csp);
            hipLaunchKernelGGL((finish2_kernel<bf16, bf16>), gc, dim3(NT), 0, s, a, clp, wtp, (int)Vp, row_lse, csp, (bf16*)dlogits, ldd, grad_scale, dbias ? part2 : nullptr);
        } else {
            hipLaunchKernelGGL(rowlse_kernel<float>, gr, dim3(256), 0, s, a, clp, wtp, (int)Vp, wrange, rows, row_lse);
            hipLaunchKernelGGL(cspart_kernel<float>, gc, dim3(NT), 0, s, a, clp, wtp, (int)Vp, row_lse, grad_scale, part2);
            hipLaunchKernelGGL(cs_reduce_kernel, gm, dim3(256), 0, s, part2, B, V, Vp, csp);
            hipLaunchKernelGGL((finish2_kernel<float, float>), gc, dim3(NT), 0, s, a, clp, wtp, (int)Vp, row_lse, csp, (float*)dlogits, ldd, grad_scale, dbias ? part2 : nullptr);
        }
        if (dbias)  // part2 is free after colstats2_merge: finish2 left [B*TS2][Vp] partials in it
            hipLaunchKernelGGL(dbias_reduce_kernel, dim3((unsigned)((V + 63) / 64)), dim3(1024), 0, s, part2,
                               B * TS2, (int)Vp, V, dbias);
    } else {
        hipMemsetAsync(colsum, 0, (size_t)B * V * 4, s);
        const unsigned gf = (unsigned)std::min<int64_t>(B * T * ((V + 3) / 4) / 256 + 1, 16384);
        if (bfl) {
            hipLaunchKernelGGL((row_kernel<1, bf16, bf16>), dim3(nblk), dim3(NT), 0, s, a, col_lse, rows, (bf16*)dlogits, ldd, nullptr, 0, colsum, grad_scale, 0);
            hipLaunchKernelGGL((finish_kernel<bf16, bf16>), dim3(gf), dim3(256), 0, s, a, col_lse, colsum, (bf16*)dlogits, ldd);
        } else {
            hipLaunchKernelGGL((row_kernel<1, float, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, rows, (float*)dlogits, ldd, nullptr, 0, colsum, grad_scale, 0);
            hipLaunchKernelGGL((finish_kernel<float, float>), dim3(gf), dim3(256), 0, s, a, col_lse, colsum, (float*)dlogits, ldd);
        }
        if (dbias) {
            const dim3 gb((unsigned)((V + 255) / 256));
            if (bfl) hipLaunchKernelGGL(dlogit_colsum_kernel<bf16>, gb, dim3(256), 0, s, (const bf16*)dlogits, ldd, B * T, V, dbias);
            else hipLaunchKernelGGL(dlogit_colsum_kernel<float>, gb, dim3(256), 0, s, (const float*)dlogits, ldd, B * T, V, dbias);
        }
    }
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, s, rows, B * T, loss);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_filtered_ce_bias(float* loss, void* dlogits, int64_t ldd, float* dbias, const void* logits,
                                    int dtype, int64_t ld, const int64_t* src, const int64_t* trg, const float* wtab,
                                    int64_t b0, int64_t b1, int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V,
                                    float grad_scale, float* col_lse, void* workspace, void* stream) {
    LOSS_CHECK();
    return filtered_ce_impl(loss, dlogits, ldd, dbias, logits, dtype, ld, src, trg, wtab, b0, b1, b2, b3, B, T, V,
                            grad_scale, col_lse, workspace, stream, nullptr, 0, 0);
}

extern "C" int msq_filtered_ce_bias_part(float* loss, void* dlogits, int64_t ldd, float* dbias, const void* logits,
                                         int dtype, int64_t ld, const int64_t* src, const int64_t* trg,
                                         const float* wtab, int64_t b0, int64_t b1, int64_t b2, int64_t b3, int64_t B,
                                         int64_t T, int64_t V, float grad_scale, float* col_lse, const float* colpart,
                                         int64_t nts, int64_t pld, void* workspace, void* stream) {
    LOSS_CHECK();
    MSQ_CHECK_ARG(colpart && nts > 0 && pld >= V, "msq_filtered_ce_bias_part: colpart / nts / pld");
    MSQ_CHECK_ARG(dlogits && ld % 8 == 0 && ldd % 8 == 0 && ((uintptr_t)logits % 16) == 0 &&
                      ((uintptr_t)dlogits % 16) == 0,
                  "msq_filtered_ce_bias_part: needs the streaming path (dlogits, ld / ldd %% 8, 16-B aligned)");
    return filtered_ce_impl(loss, dlogits, ldd, dbias, logits, dtype, ld, src, trg, wtab, b0, b1, b2, b3, B, T, V,
                            grad_scale, col_lse, workspace, stream, colpart, nts, pld);
}

extern "C" int msq_filtered_logit(float* z, int64_t ldz, const void* logits, int dtype, int64_t ld,
                                  const int64_t* src, const float* wtab, int64_t b0, int64_t b1, int64_t b2,
                                  int64_t b3, int64_t B, int64_t T, int64_t V, int64_t t_begin, float* col_lse,
                                  void* workspace, void* stream) {
    LOSS_CHECK();
    MSQ_CHECK_ARG(t_begin >= 0 && t_begin < T && ldz % 4 == 0, "msq_filtered_logit: bad t_begin / ldz");
    const LossArgs a = mk(logits, ld, src, nullptr, wtab, b0, b1, b2, b3, B, T, V);
    hipStream_t s = (hipStream_t)stream;
    const unsigned nblk = (unsigned)(B * ((T - t_begin + ROWS - 1) / ROWS));
    if (dtype == MSQ_BF16) {
        colstats_launch<bf16>(a, col_lse, (float*)workspace, s);
        hipLaunchKernelGGL((row_kernel<3, bf16, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, nullptr, z, ldz, nullptr, 0, nullptr, 0.f, t_begin);
    } else {
        colstats_launch<float>(a, col_lse, (float*)workspace, s);
        hipLaunchKernelGGL((row_kernel<3, float, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, nullptr, z, ldz, nullptr, 0, nullptr, 0.f, t_begin);
    }
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_filtered_logit_bwd(void* dlogits, int64_t ldd, const float* dz, int64_t ldz, const void* logits,
                                      int dtype, int64_t ld, const int64_t* src, const float* wtab, int64_t b0,
                                      int64_t b1, int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V,
                                      const float* col_lse, void* workspace, void* stream) {
    LOSS_CHECK();
    const LossArgs a = mk(logits, ld, src, nullptr, wtab, b0, b1, b2, b3, B, T, V);
    hipStream_t s = (hipStream_t)stream;
    float* colsum = (float*)((char*)workspace + (size_t)B * TSPLIT * 2 * V * 4);
    hipMemsetAsync(colsum, 0, (size_t)B * V * 4, s);
    const unsigned nblk = (unsigned)(B * ((T + ROWS - 1) / ROWS));
    const unsigned gf = (unsigned)std::min<int64_t>(B * T * ((V + 3) / 4) / 256 + 1, 16384);
    if (dtype == MSQ_BF16) {
        hipLaunchKernelGGL((row_kernel<2, bf16, bf16>), dim3(nblk), dim3(NT), 0, s, a, col_lse, nullptr, (bf16*)dlogits, ldd, dz, ldz, colsum, 1.f, 0);
        hipLaunchKernelGGL((finish_kernel<bf16, bf16>), dim3(gf), dim3(256), 0, s, a, col_lse, colsum, (bf16*)dlogits, ldd);
    } else {
        hipLaunchKernelGGL((row_kernel<2, float, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, nullptr, (float*)dlogits, ldd, dz, ldz, colsum, 1.f, 0);
        hipLaunchKernelGGL((finish_kernel<float, float>), dim3(gf), dim3(256), 0, s, a, col_lse, colsum, (float*)dlogits, ldd);
    }
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_ring_lse(float* col_lse, float* part, const void* ring, int dtype, int64_t ld, int64_t B,
                            int64_t ctx, int64_t V, int64_t rows_per_block, int64_t blk_lo, int64_t blk_hi,
                            int64_t skip_row, int64_t blk_extra, void* stream) {
    const int64_t nblk = rows_per_block > 0 ? (ctx + rows_per_block - 1) / rows_per_block : 0;
    MSQ_CHECK_ARG(B > 0 && ctx > 0 && V > 0 && ld >= V && ld % 8 == 0 && rows_per_block > 0 && ((uintptr_t)ring % 16) == 0,
                  "msq_ring_lse: bad sizes (ld %% 8 == 0, 16-B aligned ring)");
    MSQ_CHECK_ARG(0 <= blk_lo && blk_lo <= blk_hi && blk_hi <= nblk && blk_extra < nblk, "msq_ring_lse: bad block range");
    hipStream_t s = (hipStream_t)stream;
    const bool bfl = dtype == MSQ_BF16;
    const int N = bfl ? 8 : 4;
    const unsigned gx = (unsigned)((V + NT * N - 1) / (NT * N));
    auto blocks = [&](int64_t lo, int64_t n, int64_t skip) {
        if (n <= 0) return;
        const dim3 g(gx, (unsigned)B, (unsigned)n);
        if (bfl) hipLaunchKernelGGL(ring_block_lse_kernel<bf16>, g, dim3(NT), 0, s, (const bf16*)ring, ld, ctx, V, rows_per_block, lo, skip, part, nblk);
        else hipLaunchKernelGGL(ring_block_lse_kernel<float>, g, dim3(NT), 0, s, (const float*)ring, ld, ctx, V, rows_per_block, lo, skip, part, nblk);
    };
    blocks(blk_lo, blk_hi - blk_lo, skip_row);
    if (blk_extra >= 0 && (blk_extra < blk_lo || blk_extra >= blk_hi)) blocks(blk_extra, 1, -1);
    hipLaunchKernelGGL(ring_lse_merge_kernel, dim3((unsigned)((B * V + 255) / 256)), dim3(256), 0, s, part, B, nblk, V,
                       col_lse);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" size_t msq_ring_state_bytes(int64_t B, int64_t V, int64_t rows_per_block) {
    // others | pre | suf (fp32) | 16-B aligned int64 block id in the last 16 bytes
    return ((size_t)B * V * (2 + rows_per_block) * 4 + 15) / 16 * 16 + 16;
}

extern "C" int msq_ring_step(float* col_lse, float* part, void* state, void* ring, int dtype, int64_t ld, int64_t B,
                             int64_t ctx, int64_t V, int64_t rows_per_block, const void* row, int64_t ld_row,
                             int64_t* tokens, const int64_t* tok, int64_t* pos, void* stream) {
    const int64_t nblk = rows_per_block > 0 ? (ctx + rows_per_block - 1) / rows_per_block : 0;
    MSQ_CHECK_ARG(col_lse && part && state && ring && row && tokens && tok && pos, "msq_ring_step: null pointer");
    MSQ_CHECK_ARG(B > 0 && ctx > 0 && V > 0 && ld >= V && ld % 8 == 0 && ld_row >= ld && ld_row % 8 == 0 &&
                      rows_per_block > 0 && ((uintptr_t)ring % 16) == 0 && ((uintptr_t)row % 16) == 0 &&
                      ((uintptr_t)state % 16) == 0,
                  "msq_ring_step: bad sizes (ld %% 8 == 0, 16-B aligned ring / row / state)");
    MSQ_CHECK_ARG(dtype == MSQ_BF16 || dtype == MSQ_F32, "msq_ring_step: dtype %d", dtype);
    hipStream_t s = (hipStream_t)stream;
    const bool bfl = dtype == MSQ_BF16;
    const int N = bfl ? 8 : 4;
    float* others = (float*)state;
    float* pre = others + B * V;
    float* suf = pre + B * V;
    int64_t* cur_blk = (int64_t*)((char*)state + msq_ring_state_bytes(B, V, rows_per_block) - 16);
    const dim3 gp((unsigned)((ld + NT * N - 1) / (NT * N)), (unsigned)B);
    const dim3 gl((unsigned)((V + NT * N - 1) / (NT * N)), (unsigned)B);
    if (bfl) {
        hipLaunchKernelGGL(ring_put_kernel<bf16>, gp, dim3(NT), 0, s, (bf16*)ring, ld, ctx, (const bf16*)row, ld_row,
                           tokens, tok, pos);
        hipLaunchKernelGGL(ring_inc_kernel<bf16>, gl, dim3(NT), 0, s, (const bf16*)ring, ld, ctx, V, rows_per_block,
                           nblk, pos, part, others, pre, suf, cur_blk, col_lse);
    } else {
        hipLaunchKernelGGL(ring_put_kernel<float>, gp, dim3(NT), 0, s, (float*)ring, ld, ctx, (const float*)row,
                           ld_row, tokens, tok, pos);
        hipLaunchKernelGGL(ring_inc_kernel<float>, gl, dim3(NT), 0, s, (const float*)ring, ld, ctx, V,
                           rows_per_block, nblk, pos, part, others, pre, suf, cur_blk, col_lse);
    }
    hipLaunchKernelGGL(ring_advance_kernel, dim3(1), dim3(64), 0, s, pos, cur_blk, ctx, rows_per_block);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
