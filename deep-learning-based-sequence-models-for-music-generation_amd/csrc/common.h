// Shared device/host helpers for libmidiseq (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <math.h>

#include "../../include/midiseq.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64
#define LDS_PTR(T) T __attribute__((address_space(3)))*

// ---- host-side error plumbing (capi.cpp owns the thread-local message) ----
int msq_set_error(int code, const char* fmt, ...);

#define MSQ_CHECK_ARG(cond, ...)                                   \
    do {                                                           \
        if (!(cond)) return msq_set_error(MSQ_ERR_ARG, __VA_ARGS__); \
    } while (0)

#define MSQ_LAUNCH_CHECK()                                                           \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess)                                                        \
            return msq_set_error(MSQ_ERR_HIP, "%s: %s", __func__, hipGetErrorString(e_)); \
    } while (0)

// ---- device helpers ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

template <typename T>
__device__ __forceinline__ float to_f(T v) { return (float)v; }

template <typename T>
__device__ __forceinline__ T from_f(float v) { return (T)v; }

// load/store 4 consecutive elements as float4 (T = float or bf16)
__device__ __forceinline__ f32x4 load4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 load4(const bf16* p) {
    bf16x4 v = *(const bf16x4*)p;
    return (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ void store4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void store4(bf16* p, f32x4 v) {
    *(bf16x4*)p = (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5, T1)
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = bid % 8, loc = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}
// the same for a 3-D grid: the hardware hands workgroups to the 8 XCDs round
// robin in x-fastest dispatch order; logical ids are contiguous per XCD and
// decoded x fastest, so the x-blocks of one (y, z) run on one XCD and meet its
// L2 (the attention kernels: the key / query blocks of one (b, h) re-read the
// same Q, dO, K, V, R rows). remap = false: the plain (blockIdx.x, .y, .z).
struct Blk3 {
    int x, y, z;
};
__device__ __forceinline__ Blk3 xcd_blk3(bool remap) {
    Blk3 r;
    if (!remap) {
        r.x = blockIdx.x; r.y = blockIdx.y; r.z = blockIdx.z;
        return r;
    }
    const int nx = gridDim.x, ny = gridDim.y;
    const int lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    const int L = __builtin_amdgcn_readfirstlane(xcd_remap(lin, nx * ny * (int)gridDim.z));
    r.x = L % nx;
    r.y = (L / nx) % ny;
    r.z = L / (nx * ny);
    return r;
}

// the same with the x blocks outermost inside each XCD's contiguous range of
// logical ids (when the range holds whole (y, z) pairs): for grids whose x
// block 0 is the heaviest (the attention forward's last query block), every
// XCD runs its pairs' heavy blocks first and the light ones last, so its CUs
// finish together (longest first). The key/value pass keeps xcd_blk3: its
// blocks of one (b, h) share the query rows they stream, which the
// interleaved order keeps in L2 together (heavy-first measured slower there
// in the step)
__device__ __forceinline__ Blk3 xcd_blk3_heavy_first(bool remap) {
    if (!remap) return xcd_blk3(false);
    const int nx = gridDim.x, ny = gridDim.y, n = nx * ny * (int)gridDim.z;
    const int lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    int L = __builtin_amdgcn_readfirstlane(xcd_remap(lin, n));
    if (n % 8 == 0 && (n / 8) % nx == 0) {
        const int q = n / 8, start = L / q * q, j = L - start, P = q / nx;
        L = start + (j % P) * nx + j / P;
    }
    Blk3 r;
    r.x = L % nx;
    r.y = (L / nx) % ny;
    r.z = L / (nx * ny);
    return r;
}

// ---- dropout (nn.Dropout, model_transformer.py:51,80,101) ----
// Counter-based keep mask: element (row, col) of dropout site `site` under the
// step seed `seed` is kept iff drop_bits(drop_row(drop_base(seed, site), row),
// col) >= thr, thr = round(p * 2^32); kept values are scaled by 1/(1-p).
// oracle/dropout.py restates these four functions bit-exactly.
// one multiply (v_mul_lo_u32 is a quarter-rate op; the mask kernel and the
// dropout epilogues are bound by this hash's VALU issue)
__host__ __device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    return x;
}
__host__ __device__ __forceinline__ uint32_t drop_base(uint32_t seed, uint32_t site) {
    return drop_mix(seed ^ drop_mix(site + 0x9e3779b9u));
}
__host__ __device__ __forceinline__ uint32_t drop_row(uint32_t base, uint32_t row) {
    return drop_mix(base + row * 0x9e3779b9u);
}
__host__ __device__ __forceinline__ uint32_t drop_bits(uint32_t rowkey, uint32_t col) {
    return drop_mix(rowkey ^ (col * 0x85ebca6bu));
}
// host: keep threshold for drop probability p
static inline uint32_t drop_threshold(float p) {
    const double t = (double)p * 4294967296.0;
    return t <= 0.0 ? 0u : (t >= 4294967295.0 ? 0xffffffffu : (uint32_t)(t + 0.5));
}

// Attention-probability dropout (model_transformer.py:80) draws one 64-bit keep
// word per (query row i, 64-key block jb) instead of one hash per element:
//   key = drop_mix(drop_row(base, i) ^ ((jb + 1) * 0xc2b2ae35))
//   k   = #{t < 64 : key >= T[t]},  T[t] = round(2^32 P(K <= t)), K ~ Binomial(64, p)
//   k dropped keys, distinct and uniform: for s = 0 .. k-1 the n-th (from bit 0)
//   still-kept bit is cleared, n = mulhi(drop_mix(key + (s + 1) * 0x9e3779b9), 64 - s).
// Every element is then kept with probability 1 - p, independently (up to the
// 2^-32 quantisation of T and of the n draws), as in nn.Dropout; a row word
// costs 1 + k hashes (k = 0.64 on average at p = 0.01) instead of 64.
// oracle/dropout.py (attn_keep) restates this bit-exactly.
__host__ __device__ __forceinline__ uint32_t attn_word_key(uint32_t rowkey, uint32_t jb) {
    return drop_mix(rowkey ^ ((jb + 1u) * 0xc2b2ae35u));
}
__host__ __device__ __forceinline__ uint32_t attn_drop_draw(uint32_t key, uint32_t s) {
    return drop_mix(key + (s + 1u) * 0x9e3779b9u);
}
// bit index of the n-th (0-based, from bit 0) set bit of w (n < popcount(w))
__host__ __device__ __forceinline__ int nth_set_bit(uint64_t w, uint32_t n) {
    int pos = 0;
    for (int sh = 32; sh >= 1; sh >>= 1) {
        const uint32_t c = (uint32_t)__builtin_popcountll(w & ((1ull << sh) - 1));
        if (n >= c) {
            n -= c;
            w >>= sh;
            pos += sh;
        }
    }
    return pos;
}
// host: T of attn_word_key's Binomial(64, p) draw (double recurrence, no
// contraction, so that oracle/dropout.py's float64 numpy reproduces it exactly)
static inline void attn_drop_table(float p, uint32_t* T) {
#pragma clang fp contract(off)
    const double q = (double)p;
    const double r = q / (1.0 - q);
    double pmf = 1.0 - q;  // (1 - q)^64 by six squarings
    for (int i = 0; i < 6; ++i) pmf = pmf * pmf;
    double cdf = 0.0;
    for (int t = 0; t < 64; ++t) {
        cdf = cdf + pmf;
        const double sc = cdf * 4294967296.0;
        const double rd = sc + 0.5;
        T[t] = q <= 0.0 || rd >= 4294967295.0 ? 0xffffffffu : (uint32_t)rd;
        pmf = pmf * (double)(64 - t);
        pmf = pmf / (double)(t + 1);
        pmf = pmf * r;
    }
}
