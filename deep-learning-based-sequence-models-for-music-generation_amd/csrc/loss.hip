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

__global__ void mean_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += NT) s += x[i];
    s = block_sum(s, red);
    if (threadIdx.x == 0) *out = s / (float)n;
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
constexpr int ROWS2 = 64;  // rows per workgroup of rowstats2
constexpr int NT2 = 512;   // rowstats2: 8 waves, a whole row of V columns in registers

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
    float m[N], s[N];
#pragma unroll
    for (int i = 0; i < N; ++i) m[i] = -INFINITY, s[i] = 0.f;
    for (int64_t t = t0; t < t1; ++t) {
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

__global__ void colstats2_merge_kernel(LossArgs a, const float* __restrict__ part, float* __restrict__ col_lse,
                                       float* __restrict__ clp, int64_t Vp) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.B * Vp) return;
    const int64_t b = e / Vp, v = e % Vp;
    if (v >= a.V) {
        clp[e] = 0.f;
        return;
    }
    float m = -INFINITY;
    for (int ts = 0; ts < TS2; ++ts) m = fmaxf(m, part[((b * TS2 + ts) * 2) * a.V + v]);
    float s = 0.f;
    for (int ts = 0; ts < TS2; ++ts) {
        const float pm = part[((b * TS2 + ts) * 2) * a.V + v];
        if (pm != -INFINITY) s += part[((b * TS2 + ts) * 2 + 1) * a.V + v] * expf(pm - m);
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

// NC = column chunks of NT2*N: chunks 0..NC-2 are full for every thread
template <typename T, int NC>
__global__ __launch_bounds__(NT2) void rowstats2_kernel(LossArgs a, const float* __restrict__ clp,
                                                        const float* __restrict__ wtp, int Vp,
                                                        float* __restrict__ loss_rows, float* __restrict__ row_lse,
                                                        float* __restrict__ colsum, float gs) {
    constexpr int N = VecOf<T>::N, CH = NT2 * N;
    __shared__ float red[8];
    const int blocks_per_b = (int)((a.T + ROWS2 - 1) / ROWS2);
    const int b = blockIdx.x / blocks_per_b;
    const int r0 = (blockIdx.x % blocks_per_b) * ROWS2, r1 = min((int)a.T, r0 + ROWS2);
    const int tid = threadIdx.x, V = (int)a.V;
    const int v0 = tid * N;
    const bool last_ok = v0 + (NC - 1) * CH < V;  // this thread's part of the last chunk
    float cl[NC][N], cs[NC][N];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int i = 0; i < N; ++i) cs[c][i] = 0.f, cl[c][i] = 0.f;
        if (c < NC - 1 || last_ok) ldf<N>(clp + (int64_t)b * Vp + v0 + c * CH, cl[c]);
    }
    for (int t = r0; t < r1; ++t) {
        const int64_t row = (int64_t)b * a.T + t;
        const T* o = (const T*)a.o + row * a.ld + v0;
        const float* w = wtp + (int64_t)bucket_of(a, a.src[row]) * Vp + v0;
        const int y = (int)a.trg[row];
        float z[NC][N];
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < NC - 1 || last_ok) {
                float ov[N], wv[N];
                ldv<T, N>(o + c * CH, ov);
                ldf<N>(w + c * CH, wv);
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const bool in = c < NC - 1 || v0 + c * CH + i < V;
                    z[c][i] = in ? -(ov[i] - cl[c][i]) * wv[i] : -INFINITY;
                    mx = fmaxf(mx, z[c][i]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < N; ++i) z[c][i] = -INFINITY;
            }
        }
        mx = block8_max(mx, red);
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < N; ++i) se += fexp(z[c][i] - mx);
        const float lse = mx + logf(block8_sum(se, red));
        if (tid == 0) {
            const float zy = -((float)((const T*)a.o)[row * a.ld + y] - clp[(int64_t)b * Vp + y]) *
                             wtp[(int64_t)bucket_of(a, a.src[row]) * Vp + y];
            loss_rows[row] = lse - zy;
            row_lse[row] = lse;
        }
        // colsum_t(W dZ), dZ = (softmax_v Z - onehot y) gs   (pads: W = 0)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < NC - 1 || last_ok) {
                float wv[N];
                ldf<N>(w + c * CH, wv);
                const int vb = v0 + c * CH;
#pragma unroll
                for (int i = 0; i < N; ++i) cs[c][i] += wv[i] * (fexp(z[c][i] - lse) - (vb + i == y ? 1.f : 0.f)) * gs;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int vb = v0 + c * CH;
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (vb + i < V) atomicAdd(colsum + (int64_t)b * Vp + vb + i, cs[c][i]);
    }
}

template <typename T, typename TD>
__global__ __launch_bounds__(NT) void finish2_kernel(LossArgs a, const float* __restrict__ clp,
                                                     const float* __restrict__ wtp, int Vp,
                                                     const float* __restrict__ row_lse,
                                                     const float* __restrict__ colsum, TD* __restrict__ dout,
                                                     int64_t ldd, float gs) {
    constexpr int N = VecOf<T>::N;
    const int v = (blockIdx.x * NT + threadIdx.x) * N;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (a.T + TS2 - 1) / TS2;
    const int64_t t0 = ts * per, t1 = min(a.T, t0 + per);
    if (v >= a.V) return;
    float cl[N], cs[N], wt[5][N];
    ldf<N>(clp + b * Vp + v, cl);
    ldf<N>(colsum + b * Vp + v, cs);
#pragma unroll
    for (int k = 0; k < 5; ++k) ldf<N>(wtp + (int64_t)k * Vp + v, wt[k]);
    auto one = [&](int64_t row, const float (&ov)[N], int bk, int y, float lse) {
        float d[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float wv = bk == 0 ? wt[0][i] : bk == 1 ? wt[1][i] : bk == 2 ? wt[2][i] : bk == 3 ? wt[3][i] : wt[4][i];
            const float oc = ov[i] - cl[i];
            const float dz = (fexp(-oc * wv - lse) - (v + i == y ? 1.f : 0.f)) * gs;
            d[i] = (v + i < a.V) ? -wv * dz + fexp(oc) * cs[i] : 0.f;  // pad columns stay 0
        }
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

}  // namespace

extern "C" size_t msq_filtered_workspace(int64_t B, int64_t T, int64_t V) {
    // colstats partials | colsum [B,V] | loss rows [B*T]
    (void)T;
    // | row_lse [B*T] | colstats2 partials [B][TS2][2][V] | clp, colsum [B][Vp] | wtab [5][Vp]
    const size_t Vp = (V + 15) / 16 * 16;
    return (size_t)B * TSPLIT * 2 * V * 4 + (size_t)B * V * 4 + (size_t)B * T * 4 * 2 + 256 +
           (size_t)B * 32 * 2 * V * 4 + (2 * (size_t)B + 5) * Vp * 4 + 256;
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
    LOSS_CHECK();
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
                         ((uintptr_t)dlogits % 16) == 0 &&
                         (V + (bfl ? 4095 : 2047)) / (bfl ? 4096 : 2048) <= (bfl ? 5 : 9) && !getenv("MSQ_CE_V1");
    if (!stream2) {
        if (bfl) colstats_launch<bf16>(a, col_lse, part, s);
        else colstats_launch<float>(a, col_lse, part, s);
    }
    const unsigned nblk = (unsigned)(B * ((T + ROWS - 1) / ROWS));
    if (!dlogits) {
        if (bfl) hipLaunchKernelGGL((row_kernel<0, bf16, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, rows, (float*)nullptr, 0, nullptr, 0, nullptr, 0.f, 0);
        else hipLaunchKernelGGL((row_kernel<0, float, float>), dim3(nblk), dim3(NT), 0, s, a, col_lse, rows, (float*)nullptr, 0, nullptr, 0, nullptr, 0.f, 0);
    } else if (stream2) {
        // streaming path: colstats2 -> rowstats2 -> finish2 on zero-padded copies
        const int64_t Vp = (V + 15) / 16 * 16;
        float* clp = part2 + (size_t)B * TS2 * 2 * V;
        float* csp = clp + B * Vp;
        float* wtp = csp + B * Vp;
        float* row_lse = rows + B * T;
        hipMemsetAsync(csp, 0, (size_t)B * Vp * 4, s);
        hipLaunchKernelGGL(pad_table_kernel, dim3((unsigned)((5 * Vp + 255) / 256)), dim3(256), 0, s, wtab, wtp,
                           (int64_t)5, V, Vp);
        const int N = bfl ? 8 : 4;
        const dim3 gc((unsigned)((V + NT * N - 1) / (NT * N)), (unsigned)B, TS2);
        const unsigned nb2 = (unsigned)(B * ((T + ROWS2 - 1) / ROWS2));
        const int nc = (int)((V + NT2 * N - 1) / (NT2 * N));
        const dim3 gm((unsigned)((B * Vp + 255) / 256));
#define ROWSTATS(TT, NCV) hipLaunchKernelGGL((rowstats2_kernel<TT, NCV>), dim3(nb2), dim3(NT2), 0, s, a, clp, wtp, (int)Vp, rows, row_lse, csp, grad_scale)
        if (bfl) {
            hipLaunchKernelGGL(colstats2_kernel<bf16>, gc, dim3(NT), 0, s, a, part2);
            hipLaunchKernelGGL(colstats2_merge_kernel, gm, dim3(256), 0, s, a, part2, col_lse, clp, Vp);
            switch (nc) {
                case 1: ROWSTATS(bf16, 1); break;
                case 2: ROWSTATS(bf16, 2); break;
                case 3: ROWSTATS(bf16, 3); break;
                case 4: ROWSTATS(bf16, 4); break;
                default: ROWSTATS(bf16, 5); break;
            }
            hipLaunchKernelGGL((finish2_kernel<bf16, bf16>), gc, dim3(NT), 0, s, a, clp, wtp, (int)Vp, row_lse, csp, (bf16*)dlogits, ldd, grad_scale);
        } else {
            hipLaunchKernelGGL(colstats2_kernel<float>, gc, dim3(NT), 0, s, a, part2);
            hipLaunchKernelGGL(colstats2_merge_kernel, gm, dim3(256), 0, s, a, part2, col_lse, clp, Vp);
            switch (nc) {
                case 1: ROWSTATS(float, 1); break;
                case 2: ROWSTATS(float, 2); break;
                case 3: ROWSTATS(float, 3); break;
                case 4: ROWSTATS(float, 4); break;
                case 5: ROWSTATS(float, 5); break;
                case 6: ROWSTATS(float, 6); break;
                case 7: ROWSTATS(float, 7); break;
                case 8: ROWSTATS(float, 8); break;
                default: ROWSTATS(float, 9); break;
            }
            hipLaunchKernelGGL((finish2_kernel<float, float>), gc, dim3(NT), 0, s, a, clp, wtp, (int)Vp, row_lse, csp, (float*)dlogits, ldd, grad_scale);
        }
#undef ROWSTATS
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
    }
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(NT), 0, s, rows, B * T, loss);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
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
