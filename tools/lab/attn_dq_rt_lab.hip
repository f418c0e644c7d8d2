// LAB (not built): the query pass with every stream two iterations ahead and
// the R term's operand read from a transposed R^T copy straight into
// registers (needs AttnArgs.Rt / ldt and flash_bwd's R^T workspace +
// transpose kernel, removed with it). Outputs bitwise equal to the shipped
// attn_dq.hip; measured 20-60 us per launch SLOWER.
// Relative-position attention backward, query gradient (model_transformer.py:72-80
// differentiated w.r.t. q):
//   dq_i = sum_j dS_ij k_j  +  sum_j dS_ij R[S-1-i+j]
//        = sum_j dQR[i][S-1-i+j] K[j]  +  sum_r dQR[i][r] R[r]     (r = S-1-i+j)
// The key/value pass (attn_bwd5.hip) writes dS once, r-indexed (dQR). Both
// terms contract the SAME entries of row i, r in [S-1-i, S): the R term as
// stored, the K term skewed (column S-1-i+j of row i pairs with key j). This
// pass reads each dQR entry from HBM once: a 128-query tile's r-window is
// streamed through an LDS ring, and the K term takes its skewed fragments from
// the same ring (three 8-B reads + a per-lane funnel shift; the shift is
// (S-1-i) mod 4, a lane constant). The metadata entries j > i are added
// afterwards by flash_bwd_meta5_kernel.
//
// Tile: 128 queries x 128 dims of one (b, h); tiles are aligned to the END of
// the sequence (tile 0 = the last 128 queries, the heaviest; the ragged tile
// holds the first rows), so the r-window starts at R0 = S-1-i_last = 128 qb, a
// multiple of the 32-wide r-block, and tile row ro (query i0 + ro) reads its
// K term at ring column x = (127 - ro) + j.
// Workgroup: 4 waves, two workgroups per CU. Wave 0 / 1 run the K term of
// query half wr = 0 / 1 (64 queries x 128 dims), waves 2 / 3 the R term of
// dims half 0 / 1 (128 queries x 64 dims; v_mfma_f32_16x16x32_bf16); the
// partial sums meet in LDS at the end.
// Iteration t (one barrier): the R term contracts r-block t (32 columns)
// against R rows [R0 + 32 t, +32); the K term of half wr contracts key block
// u = t - 4 + 2 wr, whose skewed columns lie in r-blocks t-2 .. t for both
// halves. LDS (80 KB): a ring of 5 r-blocks (128 x 32) and 5 key blocks
// (32 x 128), staged by LDS-DMA two iterations ahead (every wave a quarter
// of each block). The R term's operand comes straight from R^T (flash_bwd's
// transposed copy, k-contiguous 16-B fragments, L2-resident) into registers,
// also two iterations ahead: that freed the R blocks' LDS for the second
// stage of the other two streams.
#include "attn_tiles.h"

#include <type_traits>

namespace {
using namespace attn;

constexpr int NT = 256, BM = 128, BK = 32;
constexpr int SLOT = BM * BK * 2;  // 8 KB: a ring block (128 x 32) or a key / R block (32 x 128)
constexpr int NRING = 5, NKS = 5;
constexpr int O_RING = 0, O_K = NRING * SLOT;
constexpr int LDS_BYTES = O_K + NKS * SLOT;
constexpr uint32_t OOB = 0xFFFF0000u;
static_assert(LDS_BYTES <= 80 * 1024, "two workgroups per CU");
static_assert(2 * 32 * 64 * 16 <= LDS_BYTES, "epilogue scratch");
static_assert(O_RING == 0, "the ring slot arithmetic");

// ring image: row ro (64 B) at ro * 64, 16-B chunk k at k ^ f(ro),
// f = {0, 2, 3, 1}[(ro >> 2) & 3]: the R term's aligned fragment reads are
// conflict-free (each ds_read_b128 lane group meets 16 distinct 16-B slots)
__device__ __forceinline__ int ring_f(int ro) { return (0x78 >> (2 * ((ro >> 2) & 3))) & 3; }
// key / R image: row k (256 B) chunk c at c ^ 2 g(k) (transposed reads, T10)
__device__ __forceinline__ int kr_pos(int k, int c) { return c ^ ((((k & 3) | ((k >> 1) & 4))) << 1); }

// B fragment (key / R rows [k][d], d contiguous) by ds_read_b64_tr_b16: lane
// (n = lane & 15 of column block cb, k-group g) gets k = 8 g + 0..7
__device__ __forceinline__ bf16x8 frag_b(const char* s, int cb, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int kA = 8 * g + q, kB = kA + 4;
    const int ch = (cb >> 3) + (p >> 1);
    return cat8(tr_read(s, kA * 256 + kr_pos(kA, ch) * 16 + (p & 1) * 8),
                tr_read(s, kB * 256 + kr_pos(kB, ch) * 16 + (p & 1) * 8));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dq_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(NT, 2) void flash_bwd_dq_kernel(AttnArgs a, const bf16* __restrict__ dqr, int64_t ldr,
                                                             bf16* __restrict__ dqkv, int64_t ldd) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = (int)a.S, H = (int)a.H;
    const int64_t ldq = a.ldq;
    const Blk3 blk = xcd_blk3(a.xcd);
    const int qb = blk.x;  // 0 = the last 128 queries (the longest key range)
    const int h = blk.y, b = blk.z;
    const int ihi = S - BM * qb, i0 = ihi - BM;  // tile rows i0 + ro, ro in [0, 128) (i0 < 0: ragged)
    const int R0 = BM * qb;                      // S - 1 - (i0 + 127)
    const int nk = (ihi + BK - 1) / BK;          // key blocks; also the R term's r-blocks
    const int T = nk + 4;

    const bool kterm = w < 2;
    const int wr = w & 1;  // query half
    const int rho = lane & 15, g = lane >> 4;

    // ---- staging: every wave moves a quarter of each block by LDS-DMA (lane-
    // linear 1 KB pieces, the images' swizzles applied to the source addresses)
    // into the slots the previous barrier released, two iterations ahead:
    // iteration t fills key block t and ring block t+2. Per lane: ring rows 32 w + 16 n + lane / 4, source chunk
    // (lane % 4) ^ f(row); key rows 8 w + 4 n + lane / 16, source chunk
    // kr_pos(row, lane % 16) (n = 0, 1: the wave's two pieces per block)
    const __amdgpu_buffer_rsrc_t rQ =
        dq_rsrc(dqr + ((int64_t)h * a.B + b) * S * ldr, (uint32_t)((int64_t)S * ldr * 2));
    const __amdgpu_buffer_rsrc_t rK = dq_rsrc((const bf16*)a.qkv + (int64_t)b * S * ldq, (uint32_t)((int64_t)S * ldq * 2));
    uint32_t q_off[2], k_off[2];  // global byte offsets at block 0
    int q_lim[2];                 // ring block bi valid while 32 bi < q_lim
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int ro = 32 * w + 16 * n + (lane >> 2), k = (lane & 3) ^ ring_f(ro), i = i0 + ro;
        const bool ok = i >= 0 && i < S;
        q_off[n] = (uint32_t)(((int64_t)(ok ? i : 0) * ldr + R0 + 8 * k) * 2);
        q_lim[n] = ok ? S - (R0 + 8 * k) : 0;
        const int kr = 8 * w + 4 * n + (lane >> 4), ch = kr_pos(kr, lane & 15);
        k_off[n] = (uint32_t)(((int64_t)kr * ldq + (int64_t)(H + h) * HS + ch * 8) * 2);
    }
    // BI: the builtin (the compiler counts it; the R-term waves, whose own
    // register loads the compiler waits for) or lds_dma16 (the K-term waves:
    // the builtin would make their transposed reads wait for vmcnt(0))
    auto dma = [&](auto bi_tag, __amdgpu_buffer_rsrc_t rs, int off, uint32_t voff) {
        if constexpr (decltype(bi_tag)::value)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_char*)(smem + off), 16, voff, 0, 0, 0);
        else lds_dma16(rs, smem + off, voff);
    };
    auto dma_k = [&](auto bi_tag, int u, int slot) {
#pragma unroll
        for (int n = 0; n < 2; ++n)
            dma(bi_tag, rK, O_K + slot * SLOT + (2 * w + n) * 1024,
                u >= 0 && u < nk ? k_off[n] + (uint32_t)((int64_t)BK * u * ldq * 2) : OOB);
    };
    auto dma_ring = [&](auto bi_tag, int bi, int slot) {
#pragma unroll
        for (int n = 0; n < 2; ++n)
            dma(bi_tag, rQ, O_RING + slot * SLOT + (2 * w + n) * 1024,
                BK * bi < q_lim[n] ? q_off[n] + (uint32_t)(BK * bi * 2) : OOB);
    };
    // R term operand, r-block t: R-term wave dh (= wr) covers dims 64 dh ..
    // +63 of all 128 rows; lane (m = d = 64 dh + 16 jj + rho, k-group g) holds
    // R^T[d][R0 + 32 t + 8 g .. +7] (the 16x16x32 A layout), one 16-B load per jj
    const __amdgpu_buffer_rsrc_t rT =
        dq_rsrc((const bf16*)a.Rt + (int64_t)h * HS * a.ldt, (uint32_t)(HS * a.ldt * 2));
    const uint32_t t_off = (uint32_t)(((64 * wr + rho) * a.ldt + R0 + 8 * g) * 2);
    const int t_row = (int)(16 * a.ldt * 2);  // bytes per jj
    // (kept as u32x4 until the MFMA: bf16x8 registers were copied through
    // v_bfi merges at the loop's back edge, each waiting for its load)
    auto load_rt = [&](u32x4 (&f)[4], int t) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
            f[jj] = __builtin_amdgcn_raw_buffer_load_b128(rT, t_off + (uint32_t)(64 * t), jj * t_row, 0);
    };

    // ---- fragment addressing (ring rows 64 wr + 16 rf + rho; f(row) depends on rho only)
    const int fr = ring_f(rho);
    // K term, fragment rf of iteration t: ring element E = (127 - ro) + 32 u + 8 g with
    // u = t - 4 + 2 wr, i.e. E = 32 t + 8 c + e, c = g - 1 - 2 rf - rho / 8, e = 7 - rho % 8:
    // chunks c0 = 4 t + c and c0 + 1 (block t + floor(c / 4), the next one when c % 4 == 3).
    // Three 8-B pieces from element 4 floor(E / 4) — e < 4: (c0, lo) (c0, hi) (c1, lo);
    // e >= 4: (c0, hi) (c1, lo) (c1, hi) — then elements [e % 4, +8) of the 12:
    // dword select by bit 1 of e (64-bit shift by 0 / 32), 16-bit funnel shift by bit 0.
    const int e = 7 - (rho & 7);
    const bool hi4 = (e & 4) != 0;
    const uint32_t s64 = (e & 2) ? 32u : 0u;
    const uint32_t sh = (uint32_t)(e & 1) * 16u;
    int kb_hi[4], kp0[4], kp1[4];
    bool c1wrap[4];
#pragma unroll
    for (int rf = 0; rf < 4; ++rf) {
        const int ro = 64 * wr + 16 * rf + rho;
        const int c = g - 1 - 2 * rf - (rho >> 3);  // c0 - 4 t (may be negative)
        kb_hi[rf] = c >> 2;                       // floor
        c1wrap[rf] = (c & 3) == 3;
        kp0[rf] = ro * 64 + (((c & 3) ^ fr) << 4) + (hi4 ? 8 : 0);
        kp1[rf] = ro * 64 + ((((c + 1) & 3) ^ fr) << 4);
    }
    // R term, fragment rf8: row 16 rf8 + rho, chunk g
    const int ra = rho * 64 + ((g ^ fr) << 4);

    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = zero4();

    // one iteration's MFMAs (t: the R term's r-block / the K term's key block
    // u; ts = t mod 5, the ring slot of r-block t; rf8: the R operand of t)
    auto compute = [&](int t, int ts, const u32x4 (&rop)[4]) {
        const int u = t - 4 + 2 * wr;
        const bool active = kterm ? (u >= 0 && u < nk) : (t < nk);
        if (!active) return;
        if (kterm) {
            bf16x8 af[4];
#pragma unroll
            for (int rf = 0; rf < 4; ++rf) {
                // ring slots of blocks t + kb_hi and the next (kb_hi in -2 .. 0)
                int s0 = ts + kb_hi[rf];
                s0 = s0 < 0 ? s0 + NRING : s0;
                int s1 = s0 + 1 == NRING ? 0 : s0 + 1;
                s1 = c1wrap[rf] ? s1 : s0;
                const char* p0 = smem + O_RING + s0 * SLOT + kp0[rf];
                const char* p1 = smem + O_RING + s1 * SLOT + kp1[rf];
                const uint2 d0 = *(const uint2*)p0;
                const uint2 d1 = *(const uint2*)(hi4 ? p1 : p0 + 8);
                const uint2 d2 = *(const uint2*)(p1 + (hi4 ? 8 : 0));
                const uint32_t W[6] = {d0.x, d0.y, d1.x, d1.y, d2.x, d2.y};
                // (the dword select as a 64-bit shift by 0 / 32: written as a ternary
                // the compiler turned it into a dynamically indexed scratch array)
                uint32_t X[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) X[k] = (uint32_t)(((((uint64_t)W[k + 1]) << 32) | W[k]) >> s64);
                const u32x4 o = {__builtin_amdgcn_alignbit(X[1], X[0], sh), __builtin_amdgcn_alignbit(X[2], X[1], sh),
                                 __builtin_amdgcn_alignbit(X[3], X[2], sh), __builtin_amdgcn_alignbit(X[4], X[3], sh)};
                af[rf] = __builtin_bit_cast(bf16x8, o);
            }
            const char* sb = smem + O_K + (u % NKS) * SLOT;  // (u >= 0 here)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bf16x8 bfr = frag_b(sb, 16 * j, lane);
#pragma unroll
                for (int rf = 0; rf < 4; ++rf) acc[rf][j] = mfma(bfr, af[rf], acc[rf][j]);
            }
        } else {
            // acc[rf8 / 2][4 (rf8 % 2) + jj]: rows 16 rf8 + rho, dims 64 dh + 16 jj
            bf16x8 af[8];
            const char* sq = smem + O_RING + ts * SLOT + ra;
#pragma unroll
            for (int rf8 = 0; rf8 < 8; ++rf8) af[rf8] = *(const bf16x8*)(sq + rf8 * 16 * 64);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int rf8 = 0; rf8 < 8; ++rf8)
                    acc[rf8 >> 1][(rf8 & 1) * 4 + jj] =
                        mfma(__builtin_bit_cast(bf16x8, rop[jj]), af[rf8], acc[rf8 >> 1][(rf8 & 1) * 4 + jj]);
        }
    };
    // iteration t: key block t and ring block t+2 by DMA, the MFMAs of t,
    // then the R operand of t+2 (R-term waves, into the registers t just
    // used); the barrier's wait leaves this iteration's transfers in flight
    // and retires the previous one's (a wave's vector-memory operations retire
    // in issue order): vmcnt(4) / vmcnt(8) (R-term waves)
    // The two roles run separate loops (same iterations and barriers), so the
    // R operand's 64 registers are not live in the K-term waves.
    auto next_slot = [](int ts) { return ts + 1 == NRING ? 0 : ts + 1; };
    auto ring_slot2 = [](int ts) { return ts + 2 >= NRING ? ts + 2 - NRING : ts + 2; };
    const std::false_type ASM{};
    const std::true_type BUILTIN{};
    if (kterm) {
        const u32x4 none[4] = {};
        dma_ring(ASM, 0, 0);
        dma_ring(ASM, 1, 1);
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        bar();
        int ts = 0;
        for (int t = 0; t < T; ++t) {
            dma_k(ASM, t, ts);  // (t mod 5 == ts)
            dma_ring(ASM, t + 2, ring_slot2(ts));
            compute(t, ts, none);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            bar();
            ts = next_slot(ts);
        }
    } else {
        // prologue: ring blocks 0 and 1, the R operand of r-blocks 0 and 1
        // (key blocks below 0 read as zeros)
        // in the order of a loop step's transfers (key block -1 is an
        // out-of-range fill of a slot no one reads): the compiler's wait
        // analysis then sees the same load ages on both paths into the loop
        u32x4 rA[4], rB[4];
        dma_ring(BUILTIN, 0, 0);
        load_rt(rA, 0);
        asm volatile("" ::: "memory");
        dma_k(BUILTIN, -1, NKS - 1);
        dma_ring(BUILTIN, 1, 1);
        load_rt(rB, 1);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        bar();
        auto step = [&](int t, int ts, u32x4 (&cur)[4]) {
            dma_k(BUILTIN, t, ts);
            dma_ring(BUILTIN, t + 2, ring_slot2(ts));
            compute(t, ts, cur);
            load_rt(cur, t + 2);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            bar();
        };
        // (pairs of steps, then the odd one: the compiler's wait analysis then
        // sees the same load order on every path into the loop)
        int ts = 0, t = 0;
        for (; t + 1 < T; t += 2) {
            step(t, ts, rA);
            ts = next_slot(ts);
            step(t + 1, ts, rB);
            ts = next_slot(ts);
        }
        if (t < T) step(t, ts, rA);
    }
    // the last iterations' DMA (zero-filled, out of range) before LDS reuse
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // the R-term waves hand their sums to the K-term waves: entry (row
    // fragment rf8, dim fragment 4 dh + jj) at scr[rf8 * 8 + 4 dh + jj]
    f32x4* scr = (f32x4*)smem;
    if (!kterm) {
#pragma unroll
        for (int rf8 = 0; rf8 < 8; ++rf8)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                scr[(rf8 * 8 + 4 * wr + jj) * 64 + lane] = acc[rf8 >> 1][(rf8 & 1) * 4 + jj];
    }
    bar();
    if (!kterm) return;
    // lane holds dq[i = row][d .. d+3]
#pragma unroll
    for (int rf = 0; rf < 4; ++rf) {
        const int m = i0 + 64 * wr + 16 * rf + rho;
        if (m < 0 || m >= S) continue;
        bf16* p = dqkv + ((int64_t)b * S + m) * ldd + (int64_t)h * HS + 4 * g;
#pragma unroll
        for (int j = 0; j < 8; ++j) store4(p + 16 * j, acc[rf][j] + scr[((4 * wr + rf) * 8 + j) * 64 + lane]);
    }
}

}  // namespace

int flash_bwd_dq(const AttnArgs& a, const bf16* dqr, int64_t ldr, bf16* dqkv, int64_t ldd, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_bwd_dq_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        attr = true;
    }
    // 32-bit buffer offsets (rows past S of the key / R blocks included)
    if ((a.S + BK) * ldr * 2 >= (int64_t)OOB || (a.S + BK) * a.ldq * 2 >= (int64_t)OOB || ldr < a.S + 8) return -1;
    const dim3 grid((unsigned)((a.S + BM - 1) / BM), (unsigned)a.H, (unsigned)a.B);
    hipLaunchKernelGGL(flash_bwd_dq_kernel, grid, dim3(NT), LDS_BYTES, s, a, dqr, ldr, dqkv, ldd);
    return 0;
}
