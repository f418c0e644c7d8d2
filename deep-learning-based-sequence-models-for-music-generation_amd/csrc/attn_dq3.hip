// Relative-position attention backward, query gradient, v3
// (model_transformer.py:72-80 differentiated w.r.t. q):
//   dq_i = sum_j dSj[i][j] K[j]  +  sum_r dQR[i][r] R[r]          (r = S-1-i+j)
// both dS images written by the key/value pass (attn_bwd5.hip). One workgroup =
// 256 query rows of one (b, h) x all 128 dims, 8 waves (2 per SIMD); wave w
// owns rows 64 (w >> 1) .. +63 and dims 64 (w & 1) .. +63 as 2 x 2 blocks of
// v_mfma_f32_32x32x16_bf16, computing dq^T[d][i] = K^T[d][k] . dS^T[k][i] so
// the key-row operand is read transposed (ds_read_b64_tr_b16, the chunk-major
// image of attn_bwd5.hip) and the dS operand as plain 16-B row reads.
//
// K loop: 32-deep stages, first j in [0, i_end) (dSj, B = K rows), then r in
// [kb1, S) (dQR, B = R rows); each stage (16 KB of dS + 8 KB of K / R rows)
// arrives by LDS-DMA NS-1 stages ahead (96 KB in flight per CU: the kernel is
// bound by the 2 x 1.08 GB dS read). Waves skip the stages outside their own
// rows' ranges (the band below a row's r-range is zero in dQR, the entries
// past the diagonal in the visited key blocks are zero in dSj); rows and keys
// past the sequence end read as zeros through the buffer descriptors. The
// metadata entries j > i are added afterwards by flash_bwd_meta5_kernel.
#include "attn_tiles.h"

namespace {
using namespace attn;

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 512, BM = 256, BK = 32, NS = 5;
constexpr int A_BYTES = BM * BK * 2;        // 16 KB: row r at 64 r, chunk c at 16 (c ^ ((r >> 2) & 3))
constexpr int B_BYTES = BK * HS * 2;        // 8 KB: chunk-major (attn_bwd5.hip), rows bit-2/3 swapped
constexpr int STAGE = A_BYTES + B_BYTES;
constexpr int LDS_BYTES = NS * STAGE;
constexpr uint32_t OOB = 0xFFFF0000u;
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* dst_wave, uint32_t vo) {
    lds_dma16(rs, dst_wave, vo);
}

__global__ __launch_bounds__(NT, 1) void flash_bwd_dq3_kernel(AttnArgs a, const bf16* __restrict__ dsj,
                                                              const bf16* __restrict__ dqr, int64_t ldr,
                                                              bf16* __restrict__ dqkv, int64_t ldd) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, c32 = lane & 31;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = (int)a.S, H = (int)a.H;
    const int nqt = (S + BM - 1) / BM;
    const Blk3 blk = xcd_blk3(a.xcd);
    const int qt = nqt - 1 - blk.x;  // the longest K ranges first
    const int h = blk.y, b = blk.z;
    const int i0 = qt * BM, iend = min(S, i0 + BM), ilast = iend - 1;
    // K stages: j in [0, 32 nj) then r in [kb1, kb1 + 32 nr)
    const int nj = (iend + BK - 1) / BK;
    const int kb1 = (S - 1 - ilast) / BK * BK;
    const int nr = (S - kb1 + BK - 1) / BK, nt = nj + nr;
    // this wave's rows [iw0, iw1]: j stages t < tj1, r stages from tr0
    const int rg = w >> 1, cg = w & 1;
    const int iw0 = i0 + 64 * rg, iw1 = min(S - 1, iw0 + 63);
    const bool rows_live = iw0 < S;
    const int tj1 = (iw1 + 1 + BK - 1) / BK;
    const int tr0 = nj + max(0, (S - 1 - iw1) - kb1) / BK;

    const int64_t slab_rows = ((int64_t)h * a.B + b) * S;
    const uint32_t ds_bytes = (uint32_t)((int64_t)S * ldr * 2);
    const __amdgpu_buffer_rsrc_t rJ = rsrc(dsj + slab_rows * ldr, ds_bytes);
    const __amdgpu_buffer_rsrc_t rR = rsrc(dqr + slab_rows * ldr, ds_bytes);
    const int64_t ldq = a.ldq;
    const __amdgpu_buffer_rsrc_t rK =
        rsrc((const bf16*)a.qkv + (int64_t)b * S * ldq + (int64_t)(H + h) * HS, (uint32_t)((int64_t)S * ldq * 2));
    const __amdgpu_buffer_rsrc_t rP = rsrc((const bf16*)a.R + (int64_t)h * a.S_max * HS, (uint32_t)(S * HS * 2));

    // A (dS) DMA: wave-instruction q = 2 w + k fills rows 16 q .. +15; lane l
    // lands in slot l & 3 of row 16 q + (l >> 2) and loads its chunk
    // (l & 3) ^ ((row >> 2) & 3)
    uint32_t offA[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int row = 16 * (2 * w + k) + (lane >> 2);
        const int ch = (lane & 3) ^ ((row >> 2) & 3);
        offA[k] = (i0 + row < S) ? (uint32_t)(((int64_t)(i0 + row) * ldr + 8 * ch) * 2) : OOB;
    }
    // B (K / R rows) DMA, chunk-major image of attn_bwd5.hip (16-B chunk ch of
    // image row r at ch*512 + (16 r ^ 64 (ch & 3))): wave w fills chunk
    // 4 (w >> 1) + 2 (w & 1) + hh, lane c32 lands in slot c32 = image row
    // c32 ^ 4 (2 (w & 1) + hh); image row rho holds K-row swap23(rho) (bits 2
    // and 3 exchanged) so that the transposed fragments' k order, (e & 3) +
    // 8 (e >> 2) + 4 hh, meets the dS rows' natural 8 hh + e
    int brow;
    uint32_t bcol;
    {
        const int k = w & 1, ch = 4 * (w >> 1) + 2 * k + hh;
        const int rho = c32 ^ ((2 * k + hh) << 2);
        brow = (rho & 0x13) | ((rho & 4) << 1) | ((rho & 8) >> 1);
        bcol = (uint32_t)(ch * 16);
    }
    auto issue = [&](int t) {
        char* st = smem + (t % NS) * STAGE;
        const bool live = t < nt;
        const bool sj = t < nj;
        const int k0 = sj ? BK * t : kb1 + BK * (t - nj);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t o = (live && offA[k] != OOB) ? offA[k] + (uint32_t)(k0 * 2) : OOB;
            if (sj) dma16(rJ, st + (2 * w + k) * 1024, o);
            else dma16(rR, st + (2 * w + k) * 1024, o);
        }
        const int kr = k0 + brow;
        char* bd = st + A_BYTES + (w >> 1) * 2048 + (w & 1) * 1024;
        if (sj) dma16(rK, bd, (live && kr < S) ? (uint32_t)((int64_t)kr * ldq * 2) + bcol : OOB);
        else dma16(rP, bd, (live && kr < S) ? (uint32_t)(kr * HS * 2) + bcol : OOB);
    };

    // transposed fragment offsets (attn_bwd5.hip tr_frag): rows 16 s + 8 u +
    // 4 (G >> 1) + q, columns 32 db + 16 (G & 1) + 4 p
    int tb[2];
    {
        const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, x = 2 * (G & 1) + (p >> 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) tb[u] = x * 512 + ((128 * u + 64 * (G >> 1) + 16 * q) ^ (x << 6)) + (p & 1) * 8;
    }
    // dS fragment of row block rb, k-step s: row 64 rg + 32 rb + c32, chunk 2 s + hh
    int aof[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int row = 64 * rg + 32 * rb + c32, ch = 2 * s + hh;
            aof[rb][s] = row * 64 + ((ch ^ ((row >> 2) & 3)) << 4);
        }

    f32x16 acc[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[rb][db][e] = 0.f;

#pragma unroll
    for (int t = 0; t < NS - 1; ++t) issue(t);
    for (int t = 0; t < nt; ++t) {
        // stage t landed (3 DMA per thread and stage; NS - 2 stages stay in flight)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (NS - 2)) : "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // every wave is past stage t-1: its buffer takes stage t + NS - 1
        issue(t + NS - 1);
        const bool need = rows_live && (t < nj ? t < tj1 : t >= tr0);
        if (need) {
            const char* st = smem + (t % NS) * STAGE;
            const char* bi = st + A_BYTES;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 kf[2], sf[2];
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const int d = 2 * cg + db;
                    kf[db] = cat8(tr_read(bi, tb[0] + 2048 * d + 256 * s), tr_read(bi, tb[1] + 2048 * d + 256 * s));
                }
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) sf[rb] = *(const bf16x8*)(st + aof[rb][s]);
#pragma unroll
                for (int rb = 0; rb < 2; ++rb)
#pragma unroll
                    for (int db = 0; db < 2; ++db)
                        acc[rb][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[db], sf[rb], acc[rb][db], 0, 0, 0);
            }
        }
    }
    // the DMA issued past the end lands before the workgroup gives its LDS back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // lane holds dq^T[d = 64 cg + 32 db + (e & 3) + 8 (e >> 2) + 4 hh][i = 64 rg + 32 rb + c32]
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
        const int i = iw0 + 32 * rb + c32;
        if (i >= S) continue;
        bf16* p = dqkv + ((int64_t)b * S + i) * ldd + (int64_t)h * HS + 64 * cg;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
                const f32x16& v = acc[rb][db];
                store4(p + 32 * db + 8 * e4 + 4 * hh, (f32x4){v[4 * e4], v[4 * e4 + 1], v[4 * e4 + 2], v[4 * e4 + 3]});
            }
    }
}

}  // namespace

int flash_bwd_dq3(const AttnArgs& a, const bf16* dsj, const bf16* dqr, int64_t ldr, bf16* dqkv, int64_t ldd,
                  hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_bwd_dq3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        attr = true;
    }
    if (a.S * ldr * 2 >= (int64_t)OOB || a.S * a.ldq * 2 >= (int64_t)OOB || ldr % 8 || a.ldq % 8) return -1;
    const dim3 grid((unsigned)((a.S + BM - 1) / BM), (unsigned)a.H, (unsigned)a.B);
    hipLaunchKernelGGL(flash_bwd_dq3_kernel, grid, dim3(NT), LDS_BYTES, s, a, dsj, dqr, ldr, dqkv, ldd);
    return 0;
}
