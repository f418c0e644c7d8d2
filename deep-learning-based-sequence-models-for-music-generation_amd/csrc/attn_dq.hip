// Relative-position attention backward, query gradient (model_transformer.py:72-80
// differentiated w.r.t. q):
//   dq_i = sum_j dS_ij k_j  +  sum_j dS_ij R[S-1-i+j]
//        = sum_j dQR[i][S-1-i+j] K[j]  +  sum_r dQR[i][r] R[r]    (r = S-1-i+j)
// The key/value pass (attn_bwd4.hip) writes dS once, r-indexed (dQR; zero for
// j > i, in the row padding r >= S). Both products are contractions over one K
// axis, so one kernel runs them back to back into the same accumulators: a
// 128-query x 128-dim output tile per (b, h), K range j in [0, i0+128) then r
// in [S-1-i_last rounded down to 64, S) (rows below S-1-i are zero: the band
// the dQR writer zeroes). In the first range row i's A chunk j..j+7 is the
// dQR run starting at r = S-1-i+j: a 2-byte aligned 16-B buffer load (the
// same unaligned access as the writer's 16-B stores; the descriptor covers the
// (b, h) slab exactly, and every run stays inside its own row: r <= S + 133 <
// ldr). The metadata entries j > i are added afterwards by flash_bwd_meta_kernel.
//
// Tile: 256 threads = 4 waves (2x2), each 64x64 from v_mfma_f32_16x16x32_bf16;
// operands staged global -> registers -> LDS (double buffered, one barrier per
// 64-deep K step). A (dSj / dQR rows, K-contiguous) is read with ds_read_b128
// from a (row>>1)&7 chunk-swizzled image; B (K / R rows = [k][d], d contiguous)
// with ds_read_b64_tr_b16 from a 2*g(k) chunk-swizzled image (T10).
#include "attn.h"
#include <cstdlib>

namespace {

constexpr int BM = 128, NT = 256, HSZ = 128;

// A rows of BK bf16: 8 chunks (BK 64, chunk ^= (row >> 1) & 7) or 4 chunks
// (BK 32, chunk ^= (row >> 2) & 3); either way 16 rows at one chunk are conflict-free
template <int BK>
__device__ __forceinline__ int swz_k(int row, int chunk) {
    return BK == 64 ? chunk ^ ((row >> 1) & 7) : chunk ^ ((row >> 2) & 3);
}
__device__ __forceinline__ int swz_mn(int k, int chunk) { return chunk ^ ((((k & 3) | ((k >> 1) & 4))) << 1); }

__device__ __forceinline__ u32x4 load_chunk(const bf16* p, int valid) {
    if (valid >= 8) return *(const u32x4*)p;
    union { u32x4 v; bf16 e[8]; } u;
    u.v = (u32x4){0u, 0u, 0u, 0u};
    for (int i = 0; i < valid; ++i) u.e[i] = p[i];
    return u.v;
}

template <int BK>
__device__ __forceinline__ bf16x8 frag_k(const char* s, int rb, int ks, int lane) {
    const int row = rb + (lane & 15), ch = ks * 4 + (lane >> 4);
    return *(const bf16x8*)(s + row * (BK * 2) + swz_k<BK>(row, ch) * 16);
}
__device__ __forceinline__ bf16x8 frag_mn(const char* s, int rb, int ks, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int kA = ks * 32 + 8 * g + q, kB = kA + 4;
    const int ch = (rb >> 3) + (p >> 1);
    typedef __attribute__((address_space(3))) char lc;
    const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (i16x4 __attribute__((address_space(3)))*)((lc*)s + kA * 256 + swz_mn(kA, ch) * 16 + (p & 1) * 8));
    const i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (i16x4 __attribute__((address_space(3)))*)((lc*)s + kB * 256 + swz_mn(kB, ch) * 16 + (p & 1) * 8));
    union { i16x4 h[2]; bf16x8 v; } u;
    u.h[0] = a;
    u.h[1] = b;
    return u.v;
}

// 8 bf16 starting sh elements into the 16 bf16 lo | hi (sh wave-uniform: a
// scalar branch picks the words, odd shifts funnel two words by 2 bytes)
__device__ __forceinline__ u32x4 shift_bf16(u32x4 lo, u32x4 hi, int sh) {
    const uint32_t w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#define MSQ_W4(q) (u32x4){w[q], w[q + 1], w[q + 2], w[q + 3]}
#define MSQ_F4(q)                                                                                                 \
    (u32x4){__builtin_amdgcn_alignbyte(w[q + 1], w[q], 2), __builtin_amdgcn_alignbyte(w[q + 2], w[q + 1], 2),    \
            __builtin_amdgcn_alignbyte(w[q + 3], w[q + 2], 2), __builtin_amdgcn_alignbyte(w[q + 4], w[q + 3], 2)}
    switch (sh) {
        case 0: return lo;
        case 1: return MSQ_F4(0);
        case 2: return MSQ_W4(1);
        case 3: return MSQ_F4(1);
        case 4: return MSQ_W4(2);
        case 5: return MSQ_F4(2);
        case 6: return MSQ_W4(3);
        default: return MSQ_F4(3);
    }
#undef MSQ_W4
#undef MSQ_F4
}

// 64 KB of LDS (BK 64), two workgroups per CU
constexpr int BK = 64;
__global__ __launch_bounds__(NT, 2) void flash_bwd_dq_kernel(AttnArgs a, const bf16* __restrict__ dqr, int64_t ldr,
                                                             bf16* __restrict__ dqkv, int64_t ldd) {
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BK * HSZ * 2, STAGE = A_BYTES + B_BYTES;
    constexpr int NU = BK / 16;  // 16-B chunks per thread per operand and stage
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t S = a.S, H = a.H, ldq = a.ldq;
    const int nqt = (int)((S + BM - 1) / BM);
    const int qt = nqt - 1 - (int)blockIdx.x;  // the longest K ranges first
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int64_t i0 = (int64_t)qt * BM, ilast = min<int64_t>(S - 1, i0 + BM - 1);
    const int64_t rows = ((h * a.B + b) * S) * ldr;
    // the (b, h) slab of dQR: S rows of ldr (S * ldr * 2 < 4 GB, checked by the caller)
    const uint64_t abase = (uint64_t)(dqr + rows);
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(abase >> 32)) << 32) |
                __builtin_amdgcn_readfirstlane((uint32_t)abase)),
        (short)0, (int)__builtin_amdgcn_readfirstlane((uint32_t)(S * ldr * 2)), 0x00020000);
    const bf16* B0 = (const bf16*)a.qkv + b * S * ldq + (H + h) * HSZ;
    const bf16* B1 = (const bf16*)a.R + h * a.S_max * HSZ;
    const int64_t ke0 = min<int64_t>(S, i0 + BM);        // j range [0, ke0)
    const int64_t kb1 = (S - 1 - ilast) / BK * BK;       // r range [kb1, S)
    const int n0 = (int)((ke0 + BK - 1) / BK), n1 = (int)((S - kb1 + BK - 1) / BK), nt = n0 + n1;
    // the two ranges are walked interleaved, K-step t of each back to back: at
    // equal t they read nearly the same dQR runs (row i's j-view run at j0 is
    // its r run at S-1-i+j0), so the second read of a run is an L2 hit and the
    // kernel reads dQR from memory about once instead of twice
    const int nmin = min(n0, n1);
    // A chunk u of a thread: tile row 8 (8 (u >> 1) + lane / 8) + 2 wid + (u & 1),
    // 16-B chunk lane & 7. Each (wave, u) holds the rows of ONE residue mod 8,
    // so the j-view's misalignment (S-1-i) & 7 is wave-uniform: two aligned
    // 16-B loads and a scalar-branch shift (unaligned 16-B loads are not used)
    auto a_row = [&](int u) { return 8 * (8 * (u >> 1) + (lane >> 3)) + 2 * wid + (u & 1); };
    int shv[2];
#pragma unroll
    for (int p = 0; p < 2; ++p)
        shv[p] = __builtin_amdgcn_readfirstlane((int)((((S - 1 - i0 - 2 * wid - p) % 8) + 8) % 8));

    u32x4 ra[NU], rb[NU];
    auto load = [&](int t) {
        bool s1;
        int idx;
        if (t < 2 * nmin) {
            s1 = t & 1;
            idx = t >> 1;
        } else {
            s1 = n1 > n0;
            idx = nmin + (t - 2 * nmin);
        }
        const int64_t k0 = s1 ? kb1 + (int64_t)idx * BK : (int64_t)idx * BK;
        const int64_t kend = s1 ? S : ke0;
        const bf16* B = s1 ? B1 : B0;
        const int64_t ldb = s1 ? HSZ : ldq;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            {  // A [128 rows][BK k]: dQR run at r = gk (second range) or S-1-i+gk (first)
                const int row = a_row(u), ch = lane & 7;
                const int64_t gi = i0 + row, gk = k0 + ch * 8;
                if (s1) {
                    const uint32_t off = gi < S ? (uint32_t)((gi * ldr + gk) * 2) : 0xFFFF0000u;
                    ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rA, off, 0, 0);
                } else {
                    const int sh = shv[u & 1];
                    const int64_t e = gi * ldr + (S - 1 - gi) + gk - sh;  // 8-element aligned
                    const bool ok = gi < S && gk < kend;
                    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rA, ok ? (uint32_t)(e * 2) : 0xFFFF0000u, 0, 0);
                    const u32x4 hi =
                        __builtin_amdgcn_raw_buffer_load_b128(rA, ok ? (uint32_t)((e + 8) * 2) : 0xFFFF0000u, 0, 0);
                    ra[u] = shift_bf16(lo, hi, sh);
                }
            }
            {  // B [BK k][128 d]
                const int c = tid + NT * u;
                const int kr = c >> 4, ch = c & 15;
                const int64_t gk = k0 + kr;
                rb[u] = load_chunk(B + gk * ldb + ch * 8, gk < kend ? 8 : 0);
            }
        }
    };
    auto store = [&](int buf) {
        char* sa = smem + buf * STAGE;
        char* sb = sa + A_BYTES;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int row = a_row(u), ch = lane & 7;
            *(u32x4*)(sa + row * (BK * 2) + swz_k<BK>(row, ch) * 16) = ra[u];
            const int c = tid + NT * u;
            const int kr = c >> 4, chb = c & 15;
            *(u32x4*)(sb + kr * 256 + swz_mn(kr, chb) * 16) = rb[u];
        }
    };

    const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    load(0);
    store(0);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        const int cur = t & 1;
        const char* sa = smem + cur * STAGE;
        const char* sb = sa + A_BYTES;
        const bool more = t + 1 < nt;
        if (more) load(t + 1);
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
            bf16x8 af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = frag_k<BK>(sa, wm + i * 16, ks, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = frag_mn(sb, wn + j * 16, ks, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
        if (more) store(cur ^ 1);
        __syncthreads();
    }

    // lane holds dq[i = row][d .. d+3]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t m = i0 + wm + i * 16 + (lane & 15);
        if (m >= S) continue;
        bf16* p = dqkv + (b * S + m) * ldd + h * HSZ;
#pragma unroll
        for (int j = 0; j < 4; ++j) store4(p + wn + j * 16 + 4 * (lane >> 4), acc[i][j]);
    }
}

}  // namespace

void flash_bwd_dq(const AttnArgs& a, const bf16* dqr, int64_t ldr, bf16* dqkv, int64_t ldd, hipStream_t s) {
    const dim3 grid((unsigned)((a.S + BM - 1) / BM), (unsigned)a.H, (unsigned)a.B);
    hipLaunchKernelGGL(flash_bwd_dq_kernel, grid, dim3(NT), 0, s, a, dqr, ldr, dqkv, ldd);
}
