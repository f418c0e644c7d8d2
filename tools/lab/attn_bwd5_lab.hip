// Relative-position flash attention backward, key/value-major pass, v5
// (model_transformer.py:54-90 differentiated; P recomputed from the forward's
// row log-sum-exp):
//   P_ij  = exp(scale (q_i.k_j + q_i.R[S-1-i+j]) - lse_i)
//   dS_ij = P_ij (dO_i.v_j m_ij ks - D_i) scale,   D_i = dO_i.O_i
//   dV_j  = ks sum_i P_ij m_ij dO_i,  dK_j = sum_i dS_ij q_i   (accumulated here)
//   (m_ij the dropout keep bit, ks = 1/(1-p); m = 1, ks = 1 without dropout)
//   dS written r-indexed, dQR[h][b][i][r = S-1-i+j] (the dq kernel reads its
//   j-view, the dR product its r-view), and j-indexed (dSj, dq's K term).
//   The metadata-block entries j > i (i < j < n_meta: keys every query sees)
//   are masked here like the rest of the upper triangle; flash_bwd_meta_kernel
//   adds their dK / dV / dq / dR terms.
//
// Geometry as v4 (round 3, replaced by this pass): one workgroup = 4 waves, one per SIMD, =
// 128 keys of one (b, h); a wave owns 32 keys on the lanes of
// v_mfma_f32_32x32x16; K / V rows stay in AGPRs as the B operands of S = Q.K^T
// and dP = dO.V^T, whose accumulators (key on the lane) are the B operands of
// dV^T += dO^T.P and dK^T += Q^T.dS; the relative term is a 64-row R window
// per wave and 32-query tile, skewed onto the keys by one ds_bpermute per
// register; Q / dO / R arrive by LDS-DMA in chunk-major images.
//
// What is new: a one-wave-per-SIMD kernel has nothing to hide its VALU behind
// but its own MFMAs, and v4 ran the score products, the skew + softmax and the
// dV / dK products one after the other (~5,400 cycles per wave-tile against
// 1,536 of MFMA). v5 software-pipelines the query tiles. Iteration t:
//   * barrier (tile t+1 landed; tile t-1's buffers free), then the 32 MFMAs
//     of A(t+1) = S / QR / dP of tile t+1, with the skew + softmax of tile t
//     (whose accumulators A(t) finished one iteration earlier) cut into 32
//     snippets, one per MFMA gap, and the staging DMA of tile t+1+DEPTH and
//     the row stores of dS(t-1) in the first gaps;
//   * the 16 MFMAs of C(t) = dV / dK of tile t beside the dS(t) staging writes.
// Two accumulator sets ping-pong (the loop is unrolled twice so their
// registers are fixed); each (MFMA, snippet) pair is fenced by a sched_barrier.
#include <type_traits>
#include <utility>

#include "attn_tiles.h"

namespace {
using namespace attn;

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256;
constexpr int DEPTH = 2;          // tiles in flight beyond the one A(t+1) reads
constexpr int NB = DEPTH + 2;     // Q / dO / row-constant buffers
constexpr int KB = 128, QT = 32;  // keys per workgroup, queries per tile
constexpr int NCH = 5 + DEPTH;    // R ring (32-row chunks)
constexpr int TILE = QT * 256;    // 32 rows x 128 bf16
constexpr int O_Q = 0, O_O = NB * TILE, O_R = 2 * NB * TILE;
constexpr int O_L = O_R + NCH * TILE;       // lse log2(e), D scale: NB tiles x 2 x 64 floats
constexpr int O_D = O_L + NB * 2 * 64 * 4;  // dropout keep words of the 128 keys, NB tiles
constexpr int T_PITCH = 272, T_BYTES = QT * T_PITCH;  // dS staging: 32 rows x 128 keys bf16
constexpr int O_T = O_D + NB * KB * 4;
constexpr int LDS_BYTES = O_T + 2 * T_BYTES;
// vector memory ops per wave and iteration: NDMA staging pieces (Q 2, dO 2,
// one 4-byte piece: lse / D on waves 0-1, keep words or a dummy on waves 2-3,
// R 2), then the dS row stores (2, or 4 with the j-indexed copy)
constexpr int NDMA = 7;
constexpr uint32_t OOB = 0xFFFF0000u;
#ifndef KV_STORE_AUX
// cache policy of the dS row stores: nt (2.16 GB per layer streamed through
// L2 evicted the staging reads' lines): kv 1578 -> 1498 us, and the dq pass
// that reads them back 795 -> 763 us (same box)
#define KV_STORE_AUX 2
#endif
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* dst_wave, uint32_t vo) {
    lds_dma16(rs, dst_wave, vo);
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, char* dst_wave, uint32_t vo) {
    lds_dma4(rs, dst_wave, vo);
}
__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
#ifndef KV5_NOSB
#define SB() __builtin_amdgcn_sched_barrier(0)
#else
#define SB() ((void)0)
#endif

// MFMAs as asm statements so the register classes stay fixed (AGPRs: dK^T /
// dV^T and the K / V operands; VGPRs: the per-tile S, dP, QR accumulators that
// the softmax reads). Hazards hipcc does not pad inside asm
// (cdna_hip_programming.md §5.7 item 2): an operand may be a fresh VALU result
// (s_nop 1 first); a D register is read by VALU only a whole pipeline stage
// (>= 16 MFMAs) after its last MFMA, or after drain4.
__device__ __forceinline__ void mfma_acc_a(f32x16& acc, bf16x8 a, bf16x8 b) {  // D = C in AGPRs
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_first_va(f32x16& acc, bf16x8 a, const bf16x8& b) {  // D = A.B (B in AGPRs)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma_acc_va(f32x16& acc, bf16x8 a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma_first_vv(f32x16& acc, bf16x8 a, bf16x8 b) {
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc_vv(f32x16& acc, bf16x8 a, bf16x8 b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void drain4(f32x16& a, f32x16& b, f32x16& c, f32x16& d) {
    asm volatile("s_nop 15\n\ts_nop 7" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void drain_a(f32x16 (&x)[4], f32x16 (&y)[4]) {
    asm volatile("s_nop 15\n\ts_nop 7" : "+a"(x[0]), "+a"(x[1]), "+a"(x[2]), "+a"(x[3]), "+a"(y[0]), "+a"(y[1]),
                 "+a"(y[2]), "+a"(y[3]));
}
// query row of accumulator register e in lane half hh (32x32 C/D map)
__device__ __forceinline__ int acc_row(int e, int hh) { return (e & 3) + 8 * (e >> 2) + 4 * hh; }
__device__ __forceinline__ float and_f(float x, int m) { return __int_as_float(__float_as_int(x) & m); }
// D = A.B + C with C a separate register tuple (the row constants)
__device__ __forceinline__ void mfma_init_va(f32x16& acc, bf16x8 a, const bf16x8& b, const f32x16& c) {
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(acc) : "v"(a), "a"(b), "v"(c));
}
// IR-level pin: a value passed through an empty volatile asm is (re)defined
// at that point of the side-effect-ordered instruction stream, so arithmetic
// on it cannot be hoisted into an earlier MFMA gap, and a pinned result exists
// before the next gap's sched_barrier. Without them the IR passes gathered
// the softmax of 16 gaps into 3 (one gap carried 71 VALU and 8 v_exp).
template <typename T>
__device__ __forceinline__ void pin(T& x) {
#ifndef KV_NOPIN
    asm volatile("" : "+v"(x));
#endif
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    const bf16x2 v = (bf16x2){(bf16)a, (bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ bf16x8 words8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return __builtin_bit_cast(bf16x8, (u32x4){a, b, c, d});
}
__device__ __forceinline__ f32x16 cat16(const f32x4 (&v)[4]) {
    f32x16 r;
#pragma unroll
    for (int e = 0; e < 16; ++e) r[e] = v[e >> 2][e & 3];
    return r;
}

struct Acc {
    f32x16 s, dp, q0, q1;  // S = Q.K^T, dP = dO.V^T, QR window blocks 0 / 1 (query rows x keys)
};

// nls = -lse / scale, ndk = -D / ks (per query row, flash_bwd_pre_vec_kernel):
// the initial accumulators of the S and dP chains, so that (c2 = scale log2 e)
//   S' = q.k - lse/scale,  P ks scale = exp2(c2 (S' + q.R) + log2(ks scale)),
//   dP' = dO.v - D/ks,     dS = (P ks scale) (m ? dP' : -D/ks)
// (dV, accumulated from the same P ks scale, is divided by scale at the end)
template <bool DROP>
__global__ __launch_bounds__(NT, 1) void flash_bwd_kv5_kernel(AttnArgs a, const float* __restrict__ nls,
                                                              const float* __restrict__ ndk,
                                                              const bf16* __restrict__ dout, int64_t ldo,
                                                              bf16* __restrict__ dqkv, int64_t ldd,
                                                              bf16* __restrict__ dqr, int64_t ldr) {
#ifndef KV_ABL_NOSTORE
    constexpr int NST = 2;  // dS row stores per wave and iteration (r-indexed; the dq pass reads the j-view)
#else
    constexpr int NST = 0;  // (ablation build: no dS stores)
#endif
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sR = smem + O_R;
    const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, c32 = lane & 31;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = (int)a.S, H = (int)a.H;
    const int64_t ldq = a.ldq;
    const Blk3 blk = xcd_blk3(a.xcd);
    const int kb = blk.x;  // 0 = keys 0..127 (the heaviest block)
    const int h = blk.y, b = blk.z;
    const int j0 = kb * KB, jw0 = j0 + 32 * w, jk = jw0 + c32;  // this lane's key
    const bf16* qkv_b = (const bf16*)a.qkv + (int64_t)b * S * ldq;
    const bf16* dout_b = dout + (int64_t)b * S * ldo;
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv_b, (uint32_t)((int64_t)S * ldq * 2));
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(dout_b, (uint32_t)((int64_t)S * ldo * 2));
    const __amdgpu_buffer_rsrc_t rr = make_rsrc((const bf16*)a.R + (int64_t)h * a.S_max * HS, (uint32_t)(S * HS * 2));
    const float* Lp = nls + ((int64_t)b * H + h) * S;
    const float* Dp = ndk + ((int64_t)b * H + h) * S;
    const __amdgpu_buffer_rsrc_t rl = make_rsrc(Lp, (uint32_t)(S * 4));
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(Dp, (uint32_t)(S * 4));
    bf16* qr_rows = dqr + ((int64_t)h * a.B + b) * S * ldr;
    const float c2 = a.scale * LOG2E;
    // P ks scale = exp2(c2 x + lks): the dS factor ks scale rides in P
    const float ks_scale = (DROP ? a.keep_scale : 1.f) * a.scale;
    const float lks = __builtin_log2f(ks_scale);

    // key-side B operands: lane (key c32, half hh) holds K[key][16 ks + 8 hh + 0..7]
    bf16x8 kf[8], vf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        if (jk < S) {
            kf[ks] = *(const bf16x8*)(qkv_b + (int64_t)jk * ldq + (H + h) * HS + ks * 16 + hh * 8);
            vf[ks] = *(const bf16x8*)(qkv_b + (int64_t)jk * ldq + (2 * H + h) * HS + ks * 16 + hh * 8);
        } else {
            kf[ks] = vf[ks] = (bf16x8){};
        }
        // pinned to AGPRs for the whole kernel (else the allocator keeps them in
        // VGPRs and copies them into AGPRs at every use)
        asm volatile("" : "+a"(kf[ks]), "+a"(vf[ks]));
    }
    f32x16 dk[4], dv[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) dk[n][e] = dv[n][e] = 0.f;

    // mutable copies of the lane constants the loop uses (made opaque per iteration)
    int ltid = tid, lhh = hh, lc32 = c32, ljk = jk;
    // query tiles i0 = j0 + 32 t (causal: i >= j0; block 0 also the metadata rows)
    const int it0 = j0;
    const int nqt = (S - it0 + QT - 1) / QT;
    // R window: chunk c = rows S + 96 - 32 c + [0, 32); wave w of tile T reads
    // chunks T + 4 - w (window block 0) and T + 3 - w (block 1)
    const int rw0 = S - QT;

    // DMA: wave-instruction k (0, 1) of wave w fills chunks 4w + 2k + hh (a
    // 1-KB run of the chunk-major image: 16-B chunk ch of row r at
    // ch*512 + (16 r ^ 64 (ch & 3))); lane c32 of half hh lands in slot c32,
    // which holds row c32 ^ 4 (2k + hh)
    int lrow[2];
    uint32_t offQ[2], offO[2], offR[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int ch = 4 * w + 2 * k + hh;
        lrow[k] = c32 ^ ((2 * k + hh) << 2);
        offQ[k] = (uint32_t)((lrow[k] * ldq + (int64_t)h * HS + ch * 8) * 2);
        offO[k] = (uint32_t)((lrow[k] * ldo + (int64_t)h * HS + ch * 8) * 2);
        offR[k] = (uint32_t)((lrow[k] * HS + ch * 8) * 2);
    }
    const int64_t mld = a.mask_ld;
    const __amdgpu_buffer_rsrc_t rm =
        make_rsrc(DROP ? (const void*)(a.colmask + (int64_t)(b * H + h) * (mask_bh_bytes(mld) / 4)) : (const void*)a.R,
                  DROP ? (uint32_t)mask_bh_bytes(mld) : 0u);
    // the row-constant / keep-word piece: its descriptor and lane part (the
    // keep word of key j against queries c.. is mask_word(mld, j, c) = lane
    // part (key) + query part (c), computed per tile in scalars)
    const __amdgpu_buffer_rsrc_t rpc = w == 0 ? rl : (w == 1 ? rd : rm);
    const uint32_t pc_lane = [&] {
        const int ln = lane;
        if (w < 2) return (uint32_t)(ln * 4);
        const int64_t key = j0 + 64 * (w - 2) + ln;
        return (uint32_t)((((key >> 6) * (mld >> 1)) * 128 + (key & 63) * 2) * 4);
    }();
    // staging piece p (0..6) of query tile T (R chunk T + 4): Q 0-1, dO 2-3,
    // row constants 4 (nls / ndk on waves 0-1, keep words colmask[b,h,j][i0/32]
    // of the block's keys on waves 2-3, a zero-filling dummy without dropout),
    // R 5-6. Every piece is issued by every wave (out-of-range rows: dropped
    // offset), so the per-iteration vmcnt arithmetic is exact.
    // Out-of-range rows need no select: every descriptor's num_records ends at
    // the sequence end, so rows past it (and the R rows before 0, whose offsets
    // wrap to just below 2^32) read as zeros (launch check: S + 128 rows < 4 GB).
    auto dma_piece = [&](int p, int T) {
        const int i0 = it0 + QT * T, buf = T % NB;
        if (p < 4) {
            const int k = p & 1;
            if (p < 2) dma16(rq, smem + O_Q + buf * TILE + w * 2048 + k * 1024, offQ[k] + (uint32_t)i0 * (uint32_t)(ldq * 2));
            else dma16(ro, smem + O_O + buf * TILE + w * 2048 + k * 1024, offO[k] + (uint32_t)i0 * (uint32_t)(ldo * 2));
        } else if (p == 4) {
            // one dword per lane, branch-free: waves 0 / 1 the row constants of
            // rows i0 + lane, waves 2 / 3 the keep words of keys j0 + 64 (w-2) + lane
            const uint32_t sc = w < 2 ? (uint32_t)(i0 * 4) : (uint32_t)(((i0 >> 6) * 128 + ((i0 >> 5) & 1)) * 4);
            const bool ok = w < 2 || (DROP && i0 < S);
            dma4(rpc, smem + (w < 2 ? O_L + (buf * 2 + w) * 256 : O_D + buf * KB * 4 + (w - 2) * 256),
                 ok ? pc_lane + sc : OOB);
        } else {
            const int k = p - 5, c = T + 4, r0 = rw0 + 128 - 32 * c;
            dma16(rr, sR + (c % NCH) * TILE + w * 2048 + k * 1024, offR[k] + (uint32_t)(r0 * HS * 2));
        }
    };

    // row reads (Q / dO A operands, R B operands): chunk 2 ks + hh of row c32 =
    // rof[ks & 1] + 1024 ks
    int rof[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) rof[k] = hh * 512 + ((c32 * 16) ^ ((2 * k + hh) << 6));
    // transposed quads (dV^T / dK^T A operands): lane 4q+p of 16-lane group G
    // reads rows 16 s + 8 u + 4 (G>>1) + q, columns 32 db + 16 (G&1) + 4p .. +3,
    // i.e. tb[u] + 2048 db + 256 s
    int tb[2];
    {
        const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, x = 2 * (G & 1) + (p >> 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) tb[u] = x * 512 + ((128 * u + 64 * (G >> 1) + 16 * q) ^ (x << 6)) + (p & 1) * 8;
    }
    auto tr_frag = [&](const char* img, int s2, int db) {
        return cat8(tr_read(img, tb[0] + 2048 * db + 256 * s2), tr_read(img, tb[1] + 2048 * db + 256 * s2));
    };

    // dS row stores of the staged tile ip (NST / 2 per row half): thread t
    // stores 8 keys of query rows t/16 and 16 + t/16, r-indexed at
    // r = S-1-i+j (2-byte aligned rows, unaligned 16-B stores; entries j > i
    // land at r >= S, in the row padding) and j-indexed. Rows past the
    // sequence end and the slot before tile 0 use the dropped offset, so every
    // wave issues exactly NST stores per iteration.
    const uint32_t ds_bytes = (uint32_t)min<int64_t>((int64_t)S * ldr * 2, OOB - 1);
    const int ldr2 = (int)(ldr * 2);
    // per-lane part of the two pieces' offsets (row = t/16 + 16 k, 8 keys
    // from j0 + 8 (t & 15)); i = ip + row adds ip (ldr2 - 2)
    uint32_t st_r[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int row = (tid >> 4) + 16 * k, j = j0 + 8 * (tid & 15);
        st_r[k] = (uint32_t)(row * (ldr2 - 2) + 2 * (S - 1 + j));
    }
    auto store_read = [&](int k, int sbuf) {
        const int row = (ltid >> 4) + 16 * k, ch = ltid & 15;
        return *(const u32x4*)(smem + O_T + sbuf * T_BYTES + row * T_PITCH + ch * 16);
    };
    auto store_piece = [&](int k, const u32x4& v, int ip, bool valid) {
        // descriptor rebuilt per use from readfirstlane'd halves (kept live
        // across the loop it would sit in VGPRs: a waterfall loop per store)
        // 32-bit offsets (S * ldr * 2 < 4 GB, checked at launch); rows past the
        // sequence end fall past num_records. Unaligned 16-B stores: row i's
        // keys j0.. start at r = S-1-i+j0
        const __amdgpu_buffer_rsrc_t rqr = make_rsrc(qr_rows, ds_bytes);
        __builtin_amdgcn_raw_buffer_store_b128(v, rqr, valid ? st_r[k] + (uint32_t)ip * (uint32_t)(ldr2 - 2) : OOB, 0,
                                               KV_STORE_AUX);
    };

    // skew: register e of lane c32 takes the window value from lane
    // (c32 - row(e) - 1) mod 32 of the same half; the source selects block 0
    // when c32 + row(e) >= 31 (z = c32 + 4 hh against 31 - (e&3) - 8 (e>>2)).
    // Both are lane constants per e: the select mask and the bpermute address
    // are computed once (32 VGPRs; per tile they cost 3 VALU per register)
    uint32_t skm[16];
    int ska[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int k = (e & 3) + 8 * (e >> 2);
        skm[e] = (c32 + 4 * hh >= 31 - k) ? 0xffffffffu : 0u;
        ska[e] = ((((c32 - 4 * hh - 1) * 4) - 4 * k) & 124) | (hh << 7);
        // opaque: known 0 / -1 lane masks the compiler keeps as 16 SGPR pairs
        // for v_cndmask, and the SGPR file then spills into VGPR lanes
        pin(skm[e]);
    }

    // pipeline state carried between iterations: one set of accumulators
    // (VGPRs; the AGPRs hold dK^T / dV^T and K / V) and the skewed relative
    // term bp of the tile the next iteration's softmax reads
    Acc acc;
    float bp[16];               // raw window values (the causal mask applies in stage a)
    f32x4 Dr[4];                // -D/ks of the carried tile's rows (the dropped entries' dP')
    uint32_t vm = 0u, mk = 0u;  // its causal mask (tiles 0..3) and dropout keep word

    // ---- per-tile constants of tile T for the NEXT iteration's softmax
    // (nothing here is read before that iteration's barrier, whose lgkmcnt(0)
    // retires these LDS reads; the bpermute is an asm statement so the
    // compiler places no wait behind it)
    auto skew_setup = [&](int T) {
        const int i0 = it0 + QT * T, buf = T % NB;
        // rows k + 4hh valid: jk <= i0 + k + 4hh. Only the first four tiles
        // meet the diagonal (t >= 4: every key of the block is below i0); rows
        // past the sequence end need no mask (their Q, dO and row constants read
        // as zeros, so P ks scale = ks scale and dP' = 0: no dV, dK or dS);
        // the metadata tile's j > i entries are left to flash_bwd_meta5_kernel
        const int lo = ljk - i0 - 4 * lhh;
        vm = lo <= 0 ? 0xffffffffu : (lo >= 32 ? 0u : (0xffffffffu << lo));
        if (DROP) {
            const float* cL = (const float*)(smem + O_L + buf * 512);
#pragma unroll
            for (int g = 0; g < 4; ++g) Dr[g] = *(const f32x4*)(cL + 64 + 8 * g + 4 * lhh);
            // keep word of this lane's key over the tile's 32 queries; bit k of
            // mk = query row k + 4 hh
            mk = ((const uint32_t*)(smem + O_D + buf * KB * 4))[32 * w + lc32] >> (4 * lhh);
        }
    };
    auto skew = [&](auto E) {
        constexpr int e = decltype(E)::value;
        float x0 = acc.q0[e], x1 = acc.q1[e];
        pin(x0);
        pin(x1);
        const float sel = __uint_as_float((__float_as_uint(x0) & skm[e]) | (__float_as_uint(x1) & ~skm[e]));
        float r;
#ifndef KV_ABL_NOSKEW
        asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(r) : "v"(ska[e]), "v"(sel));
#else
        r = sel;
#endif
        bp[e] = r;
    };
    // row constants of tile T as the initial accumulators (register e = row
    // acc_row(e, hh))
    auto row_consts = [&](int T, int which) {
        const float* cL = (const float*)(smem + O_L + (T % NB) * 512) + 64 * which;
        f32x4 v[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) v[g] = *(const f32x4*)(cL + 8 * g + 4 * lhh);
        return cat16(v);
    };

    // ---- one iteration (t): with DO_A, A(t+1) runs beside it; MASK: tile t
    // is one of the first four (the causal diagonal crosses it).
    //  phase 1 (16 MFMAs: QR window of t+1 into q0 / q1) | softmax stage a of
    //           tile t (p from s' + bp), the staging DMA of tile t+1+DEPTH,
    //           the dS(t-1) row stores, tile t+1's -lse/scale
    //  phase 2 (16 MFMAs: S' of t+1 from -lse/scale, then dP' of t+1 from
    //           -D/ks, into the registers tile t's s / dp just left) | softmax
    //           stage b (dS from dp'), dS(t) staging writes
    //  phase 3 (16 MFMAs: C(t) = dV / dK of tile t) | skew of tile t+1
    auto iter = [&](auto DOA, auto MSK, int t) {
        constexpr bool DO_A = decltype(DOA)::value;
        constexpr bool MASK = decltype(MSK)::value;
        const int i0 = it0 + QT * t, buf = t % NB, sb = t & 1, T = t + 1;
        // the lane constants are re-declared opaque every iteration: the
        // unrolled gaps derive dozens of per-lane addresses from them, and
        // hoisted out of the loop those pinned (and spilled) ~100 VGPRs
        asm volatile("" : "+v"(lrow[0]), "+v"(lrow[1]), "+v"(offQ[0]), "+v"(offQ[1]), "+v"(offO[0]), "+v"(offO[1]),
                     "+v"(offR[0]), "+v"(offR[1]));
        asm volatile("" : "+v"(rof[0]), "+v"(rof[1]), "+v"(tb[0]), "+v"(tb[1]), "+v"(ltid), "+v"(ljk), "+v"(lhh),
                     "+v"(lc32));
        // tile t+1's data: issued DEPTH iterations ago
#ifndef KV_ABL_NODMA
        if (t >= DEPTH) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST + (NDMA + NST) * (DEPTH - 1)) : "memory");
#endif
#ifndef KV_ABL_NOBAR
        bar();  // tile t+1 landed everywhere; tile t-1's buffers and dS(t-1) staging published
#else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        float pv[16], dsv[16];
        uint32_t pw[8], dw[8];  // bf16 pairs (rows e, e+1 of the lane's key) of P and dS
        // stage a: P ks scale = exp2(c2 (s' + bp) + lks), -inf where masked;
        // the dropped P for dV in bf16 pairs
        auto stage_a = [&](auto E) {
            constexpr int e = decltype(E)::value, k = (e & 3) + 8 * (e >> 2);
            float sv = acc.s[e], bv = bp[e];
            pin(sv);
            pin(bv);
            float x = sv + bv;
            if (MASK) {
                const int m = __builtin_amdgcn_sbfe((int)vm, k, 1);
                x = __int_as_float((__float_as_int(x) & m) | ((int)0xff800000 & ~m));
            }
            float p = __builtin_amdgcn_exp2f(fmaf(x, c2, lks));
            pin(p);
            pv[e] = p;
            if constexpr ((e & 1) == 1) {
                float p0 = pv[e - 1], p1 = p;
                if (DROP) {
                    p0 = and_f(p0, __builtin_amdgcn_sbfe((int)mk, k - 1, 1));
                    p1 = and_f(p1, __builtin_amdgcn_sbfe((int)mk, k, 1));
                }
                uint32_t wv = pack2(p0, p1);
                pin(wv);
                pw[e >> 1] = wv;
            }
        };
        // stage b: dS = (P ks scale) (m ? dP' : -D/ks), bf16 pairs
        auto stage_b = [&](auto E) {
            constexpr int e = decltype(E)::value, k = (e & 3) + 8 * (e >> 2);
            float dpv = acc.dp[e];
            pin(dpv);
            if (DROP) {
                const int m = __builtin_amdgcn_sbfe((int)mk, k, 1);
                dpv = __int_as_float((__float_as_int(dpv) & m) | (__float_as_int(Dr[e >> 2][e & 3]) & ~m));
            }
            float ds = pv[e] * dpv;
            pin(ds);
            dsv[e] = ds;
            if constexpr ((e & 1) == 1) {
                uint32_t wv = pack2(dsv[e - 1], ds);
                pin(wv);
                dw[e >> 1] = wv;
            }
        };
        const char* cQn = smem + O_Q + (T % NB) * TILE;
        const char* cOn = smem + O_O + (T % NB) * TILE;
        const char* rb0 = sR + ((T + 4 - w) % NCH) * TILE;
        const char* rb1 = sR + ((T + 3 - w) % NCH) * TILE;
        bf16x8 fq[3], fx[3], fy[3];  // two k-steps ahead
        auto ldqr = [&](int ks, int n) {
            const int off = rof[ks & 1] + 1024 * ks;
            fq[n] = *(const bf16x8*)(cQn + off);
            fx[n] = *(const bf16x8*)(rb0 + off);
            fy[n] = *(const bf16x8*)(rb1 + off);
        };
        // phase 2's fragments, three ahead (the first three from phase 1's end)
        bf16x8 fa[4];
        auto lds1 = [&](int g) {
            const int ks = g & 7, off = rof[ks & 1] + 1024 * ks;
            fa[g & 3] = *(const bf16x8*)((g < 8 ? cQn : cOn) + off);
        };
        f32x16 Lrow, Drow;
        u32x4 stv[2];  // dS(t-1) staging rows for the row stores
        // ---- phase 1
        if (DO_A) {
            ldqr(0, 0);
            ldqr(1, 1);
        }
        static_for<16>([&](auto G) {
            constexpr int g = decltype(G)::value, ks = g >> 1, c = ks % 3;
            if (DO_A) {
                if ((g & 1) == 0) {
                    if (ks + 2 < 8) ldqr(ks + 2, (ks + 2) % 3);
                    if (ks == 0) mfma_first_vv(acc.q0, fq[c], fx[c]);
                    else mfma_acc_vv(acc.q0, fq[c], fx[c]);
                } else {
                    if (ks == 0) mfma_first_vv(acc.q1, fq[c], fy[c]);
                    else mfma_acc_vv(acc.q1, fq[c], fy[c]);
                }
                if constexpr (g == 11) Lrow = row_consts(T, 0);
                if constexpr (g >= 13) lds1(g - 13);
            }
#ifndef KV_ABL_NODMA
            if constexpr (g < NDMA) dma_piece(g, t + 1 + DEPTH);
#endif
#ifndef KV_ABL_NOSTORE
            if constexpr (g == 1 || g == 2) stv[g - 1] = store_read(g - 1, sb ^ 1);
            if constexpr (g == NDMA || g == NDMA + 1) store_piece(g - NDMA, stv[g - NDMA], i0 - QT, t >= 1);
#endif
            if constexpr (g >= 2) stage_a(std::integral_constant<int, g - 2>{});
            if constexpr (g >= 14) stage_a(std::integral_constant<int, g>{});
            if constexpr (g >= 6) stage_b(std::integral_constant<int, g - 6>{});
            SB();
        });
        // ---- phase 2: S' chain (tile t's s is dead), then dP' chain (its dp
        // dies at the stage b of gap 5)
        char* st = smem + O_T + sb * T_BYTES + 4 * lhh * T_PITCH + (32 * w + lc32) * 2;
        const char* cQ = smem + O_Q + buf * TILE;
        const char* cO = smem + O_O + buf * TILE;
        bf16x8 fo[3], fqq[3];  // two MFMA pairs ahead
        static_for<16>([&](auto G) {
            constexpr int g = decltype(G)::value, ks = g & 7;
            if (DO_A) {
                if constexpr (g + 3 < 16) lds1(g + 3);
                if constexpr (g == 2) Drow = row_consts(T, 1);
                if constexpr (g == 0) mfma_init_va(acc.s, fa[g & 3], kf[ks], Lrow);
                else if constexpr (g < 8) mfma_acc_va(acc.s, fa[g & 3], kf[ks]);
                else if constexpr (g == 8) mfma_init_va(acc.dp, fa[g & 3], vf[ks], Drow);
                else mfma_acc_va(acc.dp, fa[g & 3], vf[ks]);
            }
            if constexpr (g < 6) stage_b(std::integral_constant<int, 10 + g>{});
            if constexpr (g >= 8) {  // dS(t) staging for the next iteration's row stores
                constexpr int u = g - 8, e0 = 2 * u;
                *(uint16_t*)(st + acc_row(e0, 0) * T_PITCH) = (uint16_t)(dw[u] & 0xffffu);
                *(uint16_t*)(st + acc_row(e0 + 1, 0) * T_PITCH) = (uint16_t)(dw[u] >> 16);
            }
            if constexpr (g == 14) {
                fo[0] = tr_frag(cO, 0, 0);
                fqq[0] = tr_frag(cQ, 0, 0);
            }
            if constexpr (g == 15) {
                fo[1] = tr_frag(cO, 1, 0);
                fqq[1] = tr_frag(cQ, 1, 0);
            }
            SB();
        });
        // ---- phase 3: C(t): dV^T[d][j] += dO^T[d][i] P[i][j], dK^T[d][j] +=
        // Q^T[d][i] dS[i][j] (16 MFMAs) | skew of tile t+1
        if (DO_A) skew_setup(T);
        const bf16x8 pa[2] = {words8(pw[0], pw[1], pw[2], pw[3]), words8(pw[4], pw[5], pw[6], pw[7])};
        const bf16x8 da[2] = {words8(dw[0], dw[1], dw[2], dw[3]), words8(dw[4], dw[5], dw[6], dw[7])};
        static_for<16>([&](auto G) {
            constexpr int g = decltype(G)::value, n = g >> 1, c = n % 3, db = n >> 1, s2 = n & 1;
            if ((g & 1) == 0) {
                if (n + 2 < 8) {
                    fo[(n + 2) % 3] = tr_frag(cO, (n + 2) & 1, (n + 2) >> 1);
                    fqq[(n + 2) % 3] = tr_frag(cQ, (n + 2) & 1, (n + 2) >> 1);
                }
                mfma_acc_a(dv[db], fo[c], pa[s2]);
            } else {
                mfma_acc_a(dk[db], fqq[c], da[s2]);
            }
            if (DO_A) skew(std::integral_constant<int, g>{});
            SB();
        });
    };

    // prologue: tiles 0..DEPTH and the R chunks of their windows, A(0), skew(0)
#pragma unroll
    for (int d = 0; d <= DEPTH; ++d)
#pragma unroll
        for (int p = 0; p < NDMA; ++p) dma_piece(p, d);
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // chunks 0..3 (dma_piece covers chunk T + 4 of tile T)
        const int r0 = rw0 + 128 - 32 * c;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int rg = r0 + lrow[k];
            dma16(rr, sR + (c % NCH) * TILE + w * 2048 + k * 1024,
                  (rg >= 0 && rg < S) ? offR[k] + (uint32_t)(r0 * HS * 2) : OOB);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    {
        const char* cQ = smem + O_Q;
        const char* cO = smem + O_O;
        const char* rb0 = sR + ((4 - w) % NCH) * TILE;
        const char* rb1 = sR + ((3 - w) % NCH) * TILE;
        const f32x16 L0 = row_consts(0, 0), D0 = row_consts(0, 1);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const int off = rof[ks & 1] + 1024 * ks;
            const bf16x8 fq = *(const bf16x8*)(cQ + off), fo = *(const bf16x8*)(cO + off);
            const bf16x8 fx = *(const bf16x8*)(rb0 + off), fy = *(const bf16x8*)(rb1 + off);
            if (ks == 0) {
                mfma_first_vv(acc.q0, fq, fx);
                mfma_first_vv(acc.q1, fq, fy);
                mfma_init_va(acc.s, fq, kf[0], L0);
                mfma_init_va(acc.dp, fo, vf[0], D0);
            } else {
                mfma_acc_vv(acc.q0, fq, fx);
                mfma_acc_vv(acc.q1, fq, fy);
                mfma_acc_va(acc.s, fq, kf[ks]);
                mfma_acc_va(acc.dp, fo, vf[ks]);
            }
        }
        // (four distinct operands: an asm naming one tuple twice made the
        // compiler copy it ahead of the wait states, reading the last MFMAs'
        // results too early)
        drain4(acc.s, acc.dp, acc.q0, acc.q1);
        skew_setup(0);
        static_for<16>([&](auto E) { skew(E); });
    }
    // tiles 0..3 cross the causal diagonal (masked softmax), the rest do not
    int t = 0;
    for (; t + 1 < nqt && t < 4; ++t) iter(std::true_type{}, std::true_type{}, t);
    for (; t + 1 < nqt; ++t) iter(std::true_type{}, std::false_type{}, t);
    if (nqt - 1 < 4) iter(std::false_type{}, std::true_type{}, nqt - 1);
    else iter(std::false_type{}, std::false_type{}, nqt - 1);
    // the last tile's dS rows
    bar();
#pragma unroll
    for (int k = 0; k < 2; ++k) store_piece(k, store_read(k, (nqt - 1) & 1), it0 + QT * (nqt - 1), true);
    // the staging DMA issued for tiles past the end (zero-filled) lands before
    // the workgroup gives its LDS back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // lane holds dK^T / dV^T [d = 32 db + acc_row(e)][key c32]; dV was
    // accumulated from P ks scale: dV = acc / scale
    drain_a(dk, dv);
    if (jk < S) {
        const float vs = 1.f / a.scale;
        bf16* dkp = dqkv + ((int64_t)b * S + jk) * ldd + (H + h) * HS;
        bf16* dvp = dkp + H * HS;
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
                const int d = 32 * db + 8 * e4 + 4 * hh;
                store4(dkp + d, (f32x4){dk[db][4 * e4], dk[db][4 * e4 + 1], dk[db][4 * e4 + 2], dk[db][4 * e4 + 3]});
                store4(dvp + d, (f32x4){dv[db][4 * e4] * vs, dv[db][4 * e4 + 1] * vs, dv[db][4 * e4 + 2] * vs,
                                        dv[db][4 * e4 + 3] * vs});
            }
    }
}

}  // namespace

int flash_bwd_kv5(const AttnArgs& a, const float* nls, const float* ndk, const bf16* dout, int64_t ldo, bf16* dqkv,
                  int64_t ldd, bf16* dqr, int64_t ldr, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_bwd_kv5_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)flash_bwd_kv5_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        attr = true;
    }
    // rows up to S + 127 (the staging DMA of the tiles past the end) stay below 2^32 bytes
    if ((a.S + 128) * a.ldq * 2 >= (int64_t)OOB || (a.S + 128) * ldo * 2 >= (int64_t)OOB || a.n_meta > 8) return -1;
    if ((a.S + 128) * ldr * 2 >= (int64_t)OOB) return -1;
    if (a.colmask && mask_bh_bytes(a.mask_ld) >= (int64_t)OOB) return -1;
    if (ldr < a.S + 128) return -1;
    const dim3 grid((unsigned)((a.S + KB - 1) / KB), (unsigned)a.H, (unsigned)a.B);
    if (a.colmask)
        hipLaunchKernelGGL((flash_bwd_kv5_kernel<true>), grid, dim3(NT), LDS_BYTES, s, a, nls, ndk, dout, ldo, dqkv, ldd,
                           dqr, ldr);
    else
        hipLaunchKernelGGL((flash_bwd_kv5_kernel<false>), grid, dim3(NT), LDS_BYTES, s, a, nls, ndk, dout, ldo, dqkv,
                           ldd, dqr, ldr);
    return 0;
}
