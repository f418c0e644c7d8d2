// Relative-position attention backward, query gradient (model_transformer.py:72-80
// differentiated w.r.t. q):
//   dq_i = sum_j dS_ij k_j  +  sum_j dS_ij R[S-1-i+j]
//        = sum_j dQR[i][S-1-i+j] K[j]  +  sum_r dQR[i][r] R[r]     (r = S-1-i+j)
// The key/value pass (attn_bwd5.hip) writes dS once, r-indexed (dQR, zero for
// j > i inside the tiles it visits); the K term reads its j-view, i.e. the same
// memory with row pitch ldr - 1 from element S - 1 (unaligned 16-B loads: row i
// starts S-1-i elements into its r-row). Both products are plain
// contractions over one K axis, so one kernel runs them back to back into the
// same accumulators: a 128-query x 128-dim output tile per (b, h), K range
// j in [0, i0+128) then r in [S-1-i_last rounded down to 64, S) (rows below
// S-1-i are zero: the band the dQR writer zeroes). The metadata entries j > i
// are added afterwards by flash_bwd_meta5_kernel.
//
// Tile: 256 threads = 4 waves (2x2), each 64x64 from v_mfma_f32_16x16x32_bf16;
// operands staged global -> registers -> LDS (double buffered, one barrier per
// 64-deep K step). A (dSj / dQR rows, K-contiguous) is read with ds_read_b128
// from a (row>>1)&7 chunk-swizzled image; B (K / R rows = [k][d], d contiguous)
// with ds_read_b64_tr_b16 from a 2*g(k) chunk-swizzled image (T10).
#include "attn.h"

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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dq_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// 64 KB of LDS, two workgroups per CU.
__global__ __launch_bounds__(NT, 2) void flash_bwd_dq_kernel(AttnArgs a, const bf16* __restrict__ dqr, int64_t ldr,
                                                             bf16* __restrict__ dqkv, int64_t ldd) {
    constexpr int BK = 64;
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BK * HSZ * 2, STAGE = A_BYTES + B_BYTES;
    constexpr int NU = BK / 16;  // 16-B chunks per thread per operand and stage
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t S = a.S, H = a.H, ldq = a.ldq;
    const int nqt = (int)((S + BM - 1) / BM);
    const Blk3 blk = xcd_blk3(a.xcd);
    const int qt = nqt - 1 - blk.x;  // the longest K ranges first
    const int64_t h = blk.y, b = blk.z;
    const int64_t i0 = (int64_t)qt * BM, ilast = min<int64_t>(S - 1, i0 + BM - 1);
    const int64_t rows = ((h * a.B + b) * S) * ldr;
    const uint32_t slab = (uint32_t)(S * ldr * 2);
    const __amdgpu_buffer_rsrc_t rR = dq_rsrc(dqr + rows, slab);
    const bf16* B0 = (const bf16*)a.qkv + b * S * ldq + (H + h) * HSZ;
    const bf16* B1 = (const bf16*)a.R + h * a.S_max * HSZ;
    const int64_t ke0 = min<int64_t>(S, i0 + BM);        // j range [0, ke0)
    const int64_t kb1 = (S - 1 - ilast) / BK * BK;       // r range [kb1, S)
    const int n0 = (int)((ke0 + BK - 1) / BK), nt = n0 + (int)((S - kb1 + BK - 1) / BK);
    // A-operand load u of this wave: rows 64 rb + r8 + 8 m (m = lane / 8), chunk lane % 8
    const int m8 = lane >> 3, ch8 = lane & 7;
    int arow[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int cls = wid * NU + u, r8 = cls & 7, rb = cls >> 3;
        arow[u] = 64 * rb + r8 + 8 * m8;
    }

    u32x4 ra[NU], rb[NU];
    auto load = [&](int t) {
        const bool s1 = t >= n0;
        const int64_t k0 = s1 ? kb1 + (int64_t)(t - n0) * BK : (int64_t)t * BK;
        const int64_t kend = s1 ? S : ke0;
        const bf16* B = s1 ? B1 : B0;
        const int64_t ldb = s1 ? HSZ : ldq;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            {  // A [128 rows][BK k]
                const int64_t gi = i0 + arow[u];
                // K term: element j of row gi's j-view = r = S-1-gi+j of its r-row
                const int64_t c0 = s1 ? k0 : S - 1 - gi + k0;
                const uint32_t off = gi < S ? (uint32_t)((gi * ldr + c0 + 8 * ch8) * 2) : 0xFFFF0000u;
                ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rR, off, 0, 0);
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
            const int row = arow[u];
            *(u32x4*)(sa + row * (BK * 2) + swz_k<BK>(row, ch8) * 16) = ra[u];
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
            for (int i = 0; i < 4; ++i) af[i] = frag_k<64>(sa, wm + i * 16, ks, lane);
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
