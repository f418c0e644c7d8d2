// Relative-position flash attention backward, key/value-major pass, v4.
// (model_transformer.py:54-90 differentiated; P recomputed from the forward's
// row log-sum-exp.)  Same outputs as v3 (attn_bwd3.hip):
//   P_ij  = exp(scale (q_i.k_j + q_i.R[S-1-i+j]) - lse_i)
//   dS_ij = P_ij (dO_i.v_j - D_i) scale,           D_i = dO_i.O_i
//   dV_j  = sum_i P_ij dO_i,  dK_j = sum_i dS_ij q_i   (accumulated here)
//   dS written j-indexed (dSj) and r-indexed (dQR, r = S-1-i+j) for the dq / dR
//   products; metadata-block entries j > i go to meta_ds.
//
// One workgroup = 4 waves (one per SIMD, the whole register file each) = 128
// keys of one (b, h); a wave owns 32 keys on the lanes of v_mfma_f32_32x32x16
// (lane & 31 = key). Its K / V rows stay in registers as the B operands of
// S = Q.K^T and dP = dO.V^T; those accumulators (key on the lane, 16 query rows
// in registers) are directly the B operands of dV^T += dO^T.P and
// dK^T += Q^T.dS (cdna_hip_programming.md §3, "accumulator tile as the next
// MFMA's operand"); dK^T / dV^T accumulate in registers across query tiles.
// The relative term: a 64-row R window per wave and 32-query tile,
// QR[i][w] = q_i.R[base + w] (two 32x32 blocks, window row on the lane);
// BD[i][key] = QR[i][key - i + 31] is a rotation inside each 32-lane half
// (the query row, hence the register, is the same on source and
// destination): one ds_bpermute per register after a source-side select of
// the block. Query tiles of 32 rows (Q, dO) and 32-row R chunks (a 6-chunk
// ring) stream through LDS by LDS-DMA one tile ahead, in a chunk-major image
// (16-B chunk ch of row r at ch*512 + (16 r ^ 64 (ch & 3))): the 32 rows of
// one chunk are one 512-B run, so a row read (ds_read_b128) and a transposed
// quad read (ds_read_b64_tr_b16) are conflict-free and every fragment of a
// tile is one lane base + an immediate offset (two bases per read kind),
// which keeps the per-tile instruction count and the VGPR budget of a
// one-wave-per-SIMD kernel down.
#include <type_traits>

#include "attn_tiles.h"

namespace {
using namespace attn;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// KV4_SCHED=1 pins each k-step's fragment loads one step ahead of its MFMAs
// (sched_barrier per step); 0 leaves the order to the scheduler
#ifndef KV4_SCHED
#define KV4_SCHED 0
#endif
// KV4_LATE_STORE=1 issues the previous tile's dS stores after the QK/QR/dP
// MFMAs instead of right after the prefetch
#ifndef KV4_LATE_STORE
#define KV4_LATE_STORE 1
#endif
#if KV4_SCHED
#define KV4_SB() __builtin_amdgcn_sched_barrier(0)
#else
#define KV4_SB() ((void)0)
#endif

constexpr int NT = 256;
// KV4_REGSTAGE=1 (default): the next tile's Q / dO / R chunk / row constants
// are loaded into registers at the top of a tile and written to LDS
// (ds_write_b128) at its end; an LDS-DMA wave-instruction costs 60-185 issue
// cycles (MI355X_MICROARCH.md, LDS-DMA piece), ~7x a register-staged KB, and
// at one wave per SIMD nothing hides it. KV4_REGSTAGE=0: LDS-DMA KV4_DEPTH
// tiles ahead.
#ifndef KV4_REGSTAGE
#define KV4_REGSTAGE 0
#endif
// KV4_AHEAD: k-steps of phase-1 fragments read ahead of their MFMAs (1 or 2)
#ifndef KV4_AHEAD
#define KV4_AHEAD 1
#endif
#if KV4_REGSTAGE
#undef KV4_DEPTH
#define KV4_DEPTH 1
#endif
#ifndef KV4_DEPTH
#define KV4_DEPTH 2
#endif
// KV4_PIPE=1: the dV / dK MFMAs of tile t-1 are issued inside tile t's skew
// and softmax (same basic block, no data dependence), so the MFMA pipe runs
// under that VALU / LDS work; tile t-1's Q / dO buffer stays live one more tile
#ifndef KV4_PIPE
#define KV4_PIPE 0
#endif
constexpr int DEPTH = KV4_DEPTH, NB = DEPTH + 1 + KV4_PIPE;
constexpr int KB = 128, QT = 32, NCH = 5 + DEPTH;
constexpr int TILE = QT * 256;  // 32 rows x 128 bf16
constexpr int O_Q = 0, O_O = NB * TILE, O_R = 2 * NB * TILE;
constexpr int O_L = O_R + NCH * TILE;       // lse, D: NB tiles x 2 x 64 floats
constexpr int O_D = O_L + NB * 2 * 64 * 4;  // dropout keep words of the 128 keys, NB tiles
constexpr int O_M = O_D + NB * KB * 4;      // metadata-block BD table
// vector memory ops per thread: NDMA per staged tile (Q 2, dO 2, R 2, one
// 4-byte piece: lse / D on waves 0-1, keep words or a dummy on waves 2-3),
// NST dS stores per tile
constexpr int NDMA = 7, NST = 4;
// dS staging for the coalesced row stores: 32 query rows x 128 keys bf16
constexpr int T_PITCH = 272, T_BYTES = QT * T_PITCH;
constexpr int O_T = O_M + 64 * 4;
constexpr int LDS_BYTES = O_T + 2 * T_BYTES;
constexpr uint32_t OOB = 0xFFFF0000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* dst_wave, uint32_t vo) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_char*)dst_wave, 16, vo, 0, 0, 0);
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, char* dst_wave, uint32_t vo) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_char*)dst_wave, 4, vo, 0, 0, 0);
}
__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// Register-file split by hand: every MFMA is an asm statement so that the
// allocator sees fixed classes (left to itself it moved 64-128 registers per
// tile between the VGPR and AGPR files). AGPRs: dK^T / dV^T (128) and the
// key-side K / V operands (64); VGPRs: the per-tile S, dP, QR accumulators
// (read by VALU) and the streamed fragments. Hazards hipcc does not pad inside
// asm (cdna_hip_programming.md §5.7 item 2): an operand may be a fresh VALU or
// accvgpr_write result (s_nop 1 first); a D register is read only by the next
// MFMA of its chain as C, or after kv4_drain* (>= 12 wait states).
__device__ __forceinline__ void mfma_acc_a(f32x16& acc, bf16x8 a, bf16x8 b) {  // D = C in AGPRs
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_first_va(f32x16& acc, bf16x8 a, const bf16x8& b) {  // D = A.B (B in AGPRs)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma_acc_va(f32x16& acc, bf16x8 a, const bf16x8& b) {  // D += A.B (B in AGPRs)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma_first_vv(f32x16& acc, bf16x8 a, bf16x8 b) {
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc_vv(f32x16& acc, bf16x8 a, bf16x8 b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// the four per-tile accumulators are complete for VALU readers after this
__device__ __forceinline__ void kv4_drain4(f32x16& a, f32x16& b, f32x16& c, f32x16& d) {
    asm volatile("s_nop 15\n\ts_nop 7" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void kv4_drain_a(f32x16 (&x)[4], f32x16 (&y)[4]) {
    asm volatile("s_nop 15\n\ts_nop 7" : "+a"(x[0]), "+a"(x[1]), "+a"(x[2]), "+a"(x[3]), "+a"(y[0]), "+a"(y[1]),
                 "+a"(y[2]), "+a"(y[3]));
}
// KV4_PROF (lab builds only): s_memtime cycles per loop phase, summed over all
// waves into kv4_prof[0..5] (wait+barrier, prefetch + dS stores, QK/QR/dP,
// skew + softmax, dV/dK + staging, tiles)
#ifdef KV4_PROF
__device__ unsigned long long kv4_prof[8];
#define KV4_T(k) const uint64_t tm##k = __builtin_amdgcn_s_memtime()
#else
#define KV4_T(k) ((void)0)
#endif
// chunk-major image of a 32-row x 128-bf16 tile
__device__ __forceinline__ int off_cm(int row, int ch) { return ch * 512 + ((row * 16) ^ ((ch & 3) << 6)); }
// query row of accumulator register e in lane half hh (32x32 C/D map)
__device__ __forceinline__ int acc_row(int e, int hh) { return (e & 3) + 8 * (e >> 2) + 4 * hh; }

// LAB: ablation switches for tools/lab (0 in the library): 1 no dS stores,
// 2 no MFMA, 4 no skew / softmax, 16 no DMA in the loop
template <bool DROP, int LAB = 0>
__global__ __launch_bounds__(NT, 1) void flash_bwd_kv4_kernel(AttnArgs a, const float* __restrict__ lse,
                                                              const float* __restrict__ Dv,
                                                              const bf16* __restrict__ dout, int64_t ldo,
                                                              bf16* __restrict__ dqkv, int64_t ldd,
                                                              bf16* __restrict__ dqr, bf16* __restrict__ dsj,
                                                              int64_t ldr, float* __restrict__ meta_ds) {
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
    const float* Lp = lse + ((int64_t)b * H + h) * S;
    const float* Dp = Dv + ((int64_t)b * H + h) * S;
    const __amdgpu_buffer_rsrc_t rl = make_rsrc(Lp, (uint32_t)(S * 4));
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(Dp, (uint32_t)(S * 4));
    bf16* qr_rows = dqr + ((int64_t)h * a.B + b) * S * ldr;
    bf16* sj_rows = dsj + ((int64_t)h * a.B + b) * S * ldr;
    float* mbd = (float*)(smem + O_M);
    const int nm = (int)min<int64_t>(a.n_meta, S);
    const float c2 = a.scale * LOG2E;

    // metadata-block relative terms BD(i, j >= i+2) = q_{i+1} . R[j-i-2]
    if (kb == 0 && w == 0) {
        for (int i = 0; i + 2 < nm; ++i)
            for (int j = i + 2; j < nm; ++j) {
                const bf16* q1 = qkv_b + (int64_t)(i + 1) * ldq + h * HS;
                const bf16* rrow = (const bf16*)a.R + ((int64_t)h * a.S_max + (j - i - 2)) * HS;
                float v = (float)q1[2 * lane] * (float)rrow[2 * lane] + (float)q1[2 * lane + 1] * (float)rrow[2 * lane + 1];
                v = wave_sum(v);
                if (lane == 0) mbd[i * 8 + j] = v;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }

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
    }
    f32x16 dk[4], dv[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) dk[n][e] = dv[n][e] = 0.f;

    // query tiles i0 = j0 + 32 t (causal: i >= j0; block 0 also the metadata rows)
    const int it0 = j0;
    const int nqt = (S - it0 + QT - 1) / QT;
    // R window of tile t: rows rw0 - 32 t + [0, 160); chunk c = rows rw0 + 128 - 32 c + [0, 32)
    const int rw0 = S - QT - it0 + j0;

    // DMA: wave-instruction k (0, 1) of wave w fills chunks 4w + 2k + hh (a
    // 1-KB run of the chunk-major image); lane c32 of half hh lands in slot c32,
    // which holds row c32 ^ 4 (ch & 3) = c32 ^ 4 (2k + hh)
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
    auto stage_q = [&](int t) {  // Q, dO, lse, D of query tile t
        const int i0 = it0 + QT * t, buf = t % NB;
        char* dq_ = smem + O_Q + buf * TILE + w * 2048;
        char* do_ = smem + O_O + buf * TILE + w * 2048;
        const uint32_t bq = (uint32_t)i0 * (uint32_t)(ldq * 2), bo = (uint32_t)i0 * (uint32_t)(ldo * 2);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const bool ok = i0 + lrow[k] < S;
            dma16(rq, dq_ + k * 1024, ok ? offQ[k] + bq : OOB);
            dma16(ro, do_ + k * 1024, ok ? offO[k] + bo : OOB);
        }
        if (w < 2) {
            const bool okl = i0 + lane < S;
            dma4(w == 0 ? rl : rd, smem + O_L + (buf * 2 + w) * 256, okl ? (uint32_t)((i0 + lane) * 4) : OOB);
        }
    };
    const int64_t mld = a.mask_ld;
    const __amdgpu_buffer_rsrc_t rm =
        make_rsrc(DROP ? (const void*)(a.colmask + (int64_t)(b * H + h) * (mask_bh_bytes(mld) / 4)) : (const void*)a.R,
                  DROP ? (uint32_t)mask_bh_bytes(mld) : 0u);
    auto stage_m = [&](int t) {  // keep words colmask[b,h,j][i0/32] of the block's keys (waves 2-3)
        if (w >= 2) {
            const int i0 = it0 + QT * t, key = j0 + 64 * (w - 2) + lane;
            // without dropout a dummy (zero-filling the unused keep-word slots)
            // keeps every wave's per-tile op count at NDMA
            dma4(rm, smem + O_D + (t % NB) * KB * 4 + (w - 2) * 256,
                 DROP && key < S && i0 < S ? (uint32_t)(mask_word(mld, key, i0) * 4) : OOB);
        }
    };
    auto stage_r = [&](int c) {  // R chunk c into ring slot c % NCH
        const int r0 = rw0 + 128 - 32 * c;
        char* dst = sR + (c % NCH) * TILE + w * 2048;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int rg = r0 + lrow[k];
            dma16(rr, dst + k * 1024, (rg >= 0 && rg < S) ? offR[k] + (uint32_t)(r0 * HS * 2) : OOB);
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

    // skew: register e of lane c32 takes the window value from lane
    // (c32 - row(e) - 1) mod 32 of the same half; the source selects block 0
    // when c32 + row(e) >= 31 (z = c32 + 4 hh against 31 - (e&3) - 8 (e>>2))
    const int z = c32 + 4 * hh, bpb = (c32 - 4 * hh - 1) * 4;

    // dV^T[d][j] += dO^T[d][i] P[i][j] ;  dK^T[d][j] += Q^T[d][i] dS[i][j]  (16 MFMAs)
    auto phase_b = [&](const char* cQb, const char* cOb, const bf16x8 (&pb)[2], const bf16x8 (&db_)[2]) {
        bf16x8 fo[2], fq[2];
        fo[0] = tr_frag(cOb, 0, 0);
        fq[0] = tr_frag(cQb, 0, 0);
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int c = n & 1, nx = c ^ 1, db = n >> 1, s2 = n & 1;
            if (n + 1 < 8) {
                fo[nx] = tr_frag(cOb, (n + 1) & 1, (n + 1) >> 1);
                fq[nx] = tr_frag(cQb, (n + 1) & 1, (n + 1) >> 1);
            }
            if (LAB & 2) {
                asm volatile("" ::"v"(fo[c]), "v"(fq[c]), "v"(pb[s2]), "v"(db_[s2]));
            } else {
                mfma_acc_a(dv[db], fo[c], pb[s2]);
                mfma_acc_a(dk[db], fq[c], db_[s2]);
            }
            KV4_SB();
        }
    };
#if KV4_PIPE
    // P / dS of the previous tile (zero before tile 0; its buffer is zeroed below)
    bf16x8 pa_prev[2] = {}, da_prev[2] = {};
    {
        const u32x4 zz = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            *(u32x4*)(smem + O_Q + (NB - 1) * TILE + tid * 32 + k * 16) = zz;
            *(u32x4*)(smem + O_O + (NB - 1) * TILE + tid * 32 + k * 16) = zz;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // published by the first tile's barrier
    }
#endif

#if KV4_REGSTAGE
    // register staging of tile tn (and R chunk tn + 4) for the write at the end
    // of the previous tile; out-of-range rows load zeros (buffer OOB)
    u32x4 gq[2], go[2], gr[2];
    uint32_t gl = 0u;
    auto load_next = [&](int tn) {
        const int i0 = it0 + QT * tn;
        const uint32_t bq = (uint32_t)i0 * (uint32_t)(ldq * 2), bo = (uint32_t)i0 * (uint32_t)(ldo * 2);
        const int r0 = rw0 + 128 - 32 * (tn + NCH - 2);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const bool ok = i0 + lrow[k] < S;
            gq[k] = __builtin_amdgcn_raw_buffer_load_b128(rq, ok ? offQ[k] + bq : OOB, 0, 0);
            go[k] = __builtin_amdgcn_raw_buffer_load_b128(ro, ok ? offO[k] + bo : OOB, 0, 0);
            const int rg = r0 + lrow[k];
            gr[k] = __builtin_amdgcn_raw_buffer_load_b128(rr, (rg >= 0 && rg < S) ? offR[k] + (uint32_t)(r0 * HS * 2) : OOB,
                                                          0, 0);
        }
        if (w < 2) {
            gl = __builtin_amdgcn_raw_buffer_load_b32(w == 0 ? rl : rd, i0 + lane < S ? (uint32_t)((i0 + lane) * 4) : OOB,
                                                      0, 0);
        } else if (DROP) {
            const int key = j0 + 64 * (w - 2) + lane;
            gl = __builtin_amdgcn_raw_buffer_load_b32(
                rm, key < S && i0 < S ? (uint32_t)(mask_word(mld, key, i0) * 4) : OOB, 0, 0);
        }
    };
    auto write_next = [&](int tn) {
        const int buf = tn % NB;
        char* dq_ = smem + O_Q + buf * TILE + w * 2048 + lane * 16;
        char* do_ = smem + O_O + buf * TILE + w * 2048 + lane * 16;
        char* dr_ = sR + ((tn + NCH - 2) % NCH) * TILE + w * 2048 + lane * 16;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            *(u32x4*)(dq_ + k * 1024) = gq[k];
            *(u32x4*)(do_ + k * 1024) = go[k];
            *(u32x4*)(dr_ + k * 1024) = gr[k];
        }
        if (w < 2) *(uint32_t*)(smem + O_L + (buf * 2 + w) * 256 + lane * 4) = gl;
        else if (DROP) *(uint32_t*)(smem + O_D + buf * KB * 4 + (w - 2) * 256 + lane * 4) = gl;
    };
#endif

    // prologue: tile 0 and the 5 R chunks of its window
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        stage_q(d);
        stage_m(d);
    }
#pragma unroll
    for (int c = 0; c < NCH - 1; ++c) stage_r(c);

    // dS of a tile (j <= i, else 0) is staged in LDS and stored in the NEXT
    // iteration after that iteration's prefetch, as whole rows: thread t writes
    // 8 keys of query rows t/16 and 16 + t/16, once j-indexed (dSj, aligned
    // 16-B chunks) and once r-indexed (dQR, r = S-1-i+j: 2-byte aligned rows,
    // unaligned 16-B chunks; entries j > i land at r >= S, in the row padding,
    // ldr >= S + 128, that no reader touches). The 4 stores per thread are the
    // youngest vector memory ops at the next tile's wait (vmcnt(4)); invalid
    // rows use the out-of-range offset, so the count is exact.
    const uint32_t ds_bytes = (uint32_t)min<int64_t>((int64_t)S * ldr * 2, OOB - 1);
    auto store_ds = [&](int ip, int sbuf) {
        // descriptors rebuilt here from readfirstlane'd halves: kept live across
        // the loop they ended up in VGPRs and every store ran a waterfall loop
        const __amdgpu_buffer_rsrc_t rqr = make_rsrc(qr_rows, ds_bytes);
        const __amdgpu_buffer_rsrc_t rsj = make_rsrc(sj_rows, ds_bytes);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int row = (tid >> 4) + 16 * k, ch = tid & 15;
            const u32x4 v = *(const u32x4*)(smem + O_T + sbuf * T_BYTES + row * T_PITCH + ch * 16);
            const int i = ip + row, j = j0 + 8 * ch;
            const bool in = i < S;
            const uint32_t os = in ? (uint32_t)(((int64_t)i * ldr + j) * 2) : OOB;
            const uint32_t oq = in ? (uint32_t)(((int64_t)i * ldr + (S - 1 - i + j)) * 2) : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(v, rsj, os, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(v, rqr, oq, 0, 0);
        }
    };

#ifdef KV4_PROF
    uint64_t pr[6] = {0, 0, 0, 0, 0, 0};
#endif
    for (int t = 0; t < nqt; ++t) {
        const int i0 = it0 + QT * t, buf = t % NB, sb = t & 1;
        KV4_T(0);
        // tile t's DMA was issued in iteration t - DEPTH; younger: that
        // iteration's NST stores and DEPTH - 1 iterations of NDMA + NST (every
        // iteration issues all of them, out-of-range ones as zero-fill)
#if KV4_REGSTAGE
        // tile 0 came by LDS-DMA (prologue); later tiles by this wave's own
        // ds_writes at the end of the previous iteration
        if (t == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();  // tile t published everywhere; tile t-1's buffers (and dS staging) are free
        KV4_T(1);
        if (t + 1 < nqt && !(LAB & 16)) load_next(t + 1);
#else
        if (t > DEPTH && !(LAB & 17)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST + (NDMA + NST) * (DEPTH - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();  // tile t landed everywhere; tile t-1's buffers (and dS staging) are free / published
        KV4_T(1);
        if (!(LAB & 16)) {
            stage_q(t + DEPTH);
            stage_r(t + NCH - 1);
            stage_m(t + DEPTH);
        }
#endif
        asm volatile("" ::: "memory");
#if !KV4_LATE_STORE
        if (t >= 1 && !(LAB & 1)) store_ds(i0 - QT, sb ^ 1);
#endif
        KV4_T(2);
        const char* cQ = smem + O_Q + buf * TILE;
        const char* cO = smem + O_O + buf * TILE;
        const float* cL = (const float*)(smem + O_L + buf * 512);
        const float* cD = cL + 64;
        char* st = smem + O_T + sb * T_BYTES + 4 * hh * T_PITCH + (32 * w + c32) * 2;
        // (a wave whose keys all follow the tile's queries computes zeros through
        // the mask: skipping it as a branch costs the register allocator a copy
        // of every accumulator at the join)
        f32x16 sacc, dpacc, qr0, qr1;
        // this wave's 64-row window starts at ring chunk t + 4 - w (block 0), t + 3 - w (block 1)
        const char* rb0 = sR + ((t + 4 - w) % NCH) * TILE;
        const char* rb1 = sR + ((t + 3 - w) % NCH) * TILE;
        // S = Q.K^T, QR = Q.Rwin^T (two blocks), dP = dO.V^T: 32 MFMAs, each Q
        // fragment read once; fragments one k-step ahead
        {
            // fragments KV4_AHEAD k-steps ahead (KV4_AHEAD + 1 register sets)
            constexpr int NF = KV4_AHEAD + 1;
            bf16x8 fq[NF], fo[NF], f0[NF], f1[NF];
            auto ld = [&](int ks, int n) {
                const int o = rof[ks & 1] + 1024 * ks;
                fq[n] = *(const bf16x8*)(cQ + o);
                fo[n] = *(const bf16x8*)(cO + o);
                f0[n] = *(const bf16x8*)(rb0 + o);
                f1[n] = *(const bf16x8*)(rb1 + o);
            };
#pragma unroll
            for (int k = 0; k < KV4_AHEAD; ++k) ld(k, k);
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const int c = ks % NF;
                if (ks + KV4_AHEAD < 8) ld(ks + KV4_AHEAD, (ks + KV4_AHEAD) % NF);
                if (LAB & 2) {
                    asm volatile("" ::"v"(fq[c]), "v"(fo[c]), "v"(f0[c]), "v"(f1[c]));
                } else if (ks == 0) {
                    mfma_first_vv(qr0, fq[c], f0[c]);
                    mfma_first_vv(qr1, fq[c], f1[c]);
                    mfma_first_va(sacc, fq[c], kf[ks]);
                    mfma_first_va(dpacc, fo[c], vf[ks]);
                } else {
                    mfma_acc_vv(qr0, fq[c], f0[c]);
                    mfma_acc_vv(qr1, fq[c], f1[c]);
                    mfma_acc_va(sacc, fq[c], kf[ks]);
                    mfma_acc_va(dpacc, fo[c], vf[ks]);
                }
                KV4_SB();
            }
        }
#if KV4_LATE_STORE
        // the previous tile's dS rows leave while the last MFMAs drain
        if (t >= 1 && !(LAB & 1)) store_ds(i0 - QT, sb ^ 1);
#endif
        if (!(LAB & 2)) kv4_drain4(sacc, dpacc, qr0, qr1);
        KV4_T(3);
        // BD added to S through the skew (z, bpb made opaque per tile: hoisted out
        // of the loop, the 16 lane masks and 16 addresses would pin 32 SGPRs and
        // 16 VGPRs for the whole kernel)
        {
            int zt = z, bt = bpb;
            asm volatile("" : "+v"(zt), "+v"(bt));
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int k = (e & 3) + 8 * (e >> 2);
                const float sel = (zt >= 31 - k) ? qr0[e] : qr1[e];
                const int adr = ((bt - 4 * k) & 124) | (hh << 7);
                sacc[e] += (LAB & 4) ? sel : __int_as_float(__builtin_amdgcn_ds_bpermute(adr, __float_as_int(sel)));
            }
        }
        bf16x8 pa[2], da[2];
#if KV4_PIPE
        const char* cQp = smem + O_Q + ((t + NB - 1) % NB) * TILE;
        const char* cOp = smem + O_O + ((t + NB - 1) % NB) * TILE;
#endif
        if (LAB & 4) {
#if KV4_PIPE
            phase_b(cQp, cOp, pa_prev, da_prev);
#endif
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                pa[e >> 3][e & 7] = (bf16)sacc[e];
                da[e >> 3][e & 7] = (bf16)dpacc[e];
            }
        } else {
            // mode 0: the whole wave tile below the diagonal and inside the sequence;
            // 1: causal / sequence-end mask; 2: the metadata tile (i0 < n_meta:
            // keys j < n_meta visible to every query, BD(i, j >= i+2) from the
            // table, dS of j > i to meta_ds). All three wave-uniform.
            const int mode = (i0 < nm) ? 2 : ((i0 >= jw0 + QT - 1) && (i0 + QT <= S)) ? 0 : 1;
            const uint32_t kw = DROP ? ((const uint32_t*)(smem + O_D + buf * KB * 4))[32 * w + c32] : 0u;
            auto softmax = [&](auto MODE) {
                constexpr int md = decltype(MODE)::value;
                auto elem = [&](int e) {
                    const int e4 = e >> 2, r = e & 3, iq = 8 * e4 + 4 * hh + r, i = i0 + iq;
                    float x = sacc[e];
                    const float l2 = cL[8 * e4 + 4 * hh + r] * LOG2E, dd = cD[8 * e4 + 4 * hh + r];
                    const float kbv = DROP ? ((kw >> iq) & 1u ? a.keep_scale : 0.f) : 1.f;
                    bool ok = true;
                    if (md == 1) ok = (i < S) && (jk <= i);
                    if (md == 2) {
                        ok = (i < S) && (jk < S) && (jk <= i || jk < nm);
                        if (ok && jk >= i + 2) x += mbd[i * 8 + jk];
                    }
                    float p = __builtin_amdgcn_exp2f(fmaf(x, c2, -l2));
                    float ds = p * (DROP ? fmaf(dpacc[e], kbv, -dd) : dpacc[e] - dd) * a.scale;
                    if (md != 0) {
                        p = ok ? p : 0.f;
                        ds = ok ? ds : 0.f;
                    }
                    if (md == 2 && ok && jk > i) meta_ds[(((int64_t)b * H + h) * 8 + i) * 8 + jk] = ds;
                    if (DROP) p *= kbv;
                    pa[e >> 3][e & 7] = (bf16)p;
                    da[e >> 3][e & 7] = (bf16)ds;
                };
#if KV4_PIPE
                // the previous tile's dV / dK step n (2 MFMAs, its fragments one
                // step ahead) beside elements 2n, 2n+1 of this tile's softmax;
                // sched_barrier per step keeps the fragment reads from being
                // hoisted (register budget) while the VALU runs under the MFMAs
                bf16x8 fo[2], fq[2];
                fo[0] = tr_frag(cOp, 0, 0);
                fq[0] = tr_frag(cQp, 0, 0);
#pragma unroll
                for (int n = 0; n < 8; ++n) {
                    const int c = n & 1, nx = c ^ 1, db = n >> 1, s2 = n & 1;
                    if (n + 1 < 8) {
                        fo[nx] = tr_frag(cOp, (n + 1) & 1, (n + 1) >> 1);
                        fq[nx] = tr_frag(cQp, (n + 1) & 1, (n + 1) >> 1);
                    }
                    if (!(LAB & 2)) {
                        mfma_acc_a(dv[db], fo[c], pa_prev[s2]);
                        mfma_acc_a(dk[db], fq[c], da_prev[s2]);
                    }
                    elem(2 * n);
                    elem(2 * n + 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
#else
#pragma unroll
                for (int e = 0; e < 16; ++e) elem(e);
#endif
            };
            if (mode == 0) softmax(std::integral_constant<int, 0>{});
            else if (mode == 1) softmax(std::integral_constant<int, 1>{});
            else softmax(std::integral_constant<int, 2>{});
        }
        KV4_T(4);
#if !KV4_PIPE
        phase_b(cQ, cO, pa, da);
#endif
        // stage this tile's dS rows for the next iteration's stores (dS is 0
        // above the diagonal except the metadata keys of the first tile, which
        // went to meta_ds and are cleared here)
#if KV4_PIPE
        // (unmasked: the metadata entries j > i belong to dK)
        pa_prev[0] = pa[0];
        pa_prev[1] = pa[1];
        da_prev[0] = da[0];
        da_prev[1] = da[1];
#endif
        if (i0 < nm) {
#pragma unroll
            for (int e = 0; e < 16; ++e)
                if (jk > i0 + acc_row(e, hh)) da[e >> 3][e & 7] = (bf16)0.f;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) *(bf16*)(st + (acc_row(e, hh) - 4 * hh) * T_PITCH) = da[e >> 3][e & 7];
#if KV4_REGSTAGE
        if (t + 1 < nqt && !(LAB & 16)) write_next(t + 1);
#endif
#ifdef KV4_PROF
        {
            const uint64_t tm5 = __builtin_amdgcn_s_memtime();
            pr[0] += tm1 - tm0; pr[1] += tm2 - tm1; pr[2] += tm3 - tm2; pr[3] += tm4 - tm3; pr[4] += tm5 - tm4;
            pr[5] += 1;
        }
#endif
    }
#ifdef KV4_PROF
    if (lane == 0)
        for (int k = 0; k < 6; ++k) atomicAdd(&kv4_prof[k], (unsigned long long)pr[k]);
#endif
#if KV4_PIPE
    phase_b(smem + O_Q + ((nqt - 1) % NB) * TILE, smem + O_O + ((nqt - 1) % NB) * TILE, pa_prev, da_prev);
#endif
    if (!(LAB & 1)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        store_ds(it0 + QT * (nqt - 1), (nqt - 1) & 1);
    }
    // lane holds dK^T / dV^T [d = 32 db + acc_row(e)][key c32]
    kv4_drain_a(dk, dv);
    if (jk < S) {
        bf16* dkp = dqkv + ((int64_t)b * S + jk) * ldd + (H + h) * HS;
        bf16* dvp = dkp + H * HS;
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
                const int d = 32 * db + 8 * e4 + 4 * hh;
                store4(dkp + d, (f32x4){dk[db][4 * e4], dk[db][4 * e4 + 1], dk[db][4 * e4 + 2], dk[db][4 * e4 + 3]});
                store4(dvp + d, (f32x4){dv[db][4 * e4], dv[db][4 * e4 + 1], dv[db][4 * e4 + 2], dv[db][4 * e4 + 3]});
            }
    }
}

}  // namespace

int flash_bwd_kv4(const AttnArgs& a, const float* lse, const float* Dv, const bf16* dout, int64_t ldo, bf16* dqkv,
                  int64_t ldd, bf16* dqr, bf16* dsj, int64_t ldr, float* meta_ds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_bwd_kv4_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)flash_bwd_kv4_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        attr = true;
    }
    if (a.S * a.ldq * 2 >= (int64_t)OOB || a.S * ldo * 2 >= (int64_t)OOB || a.n_meta > 8) return -1;
    if (a.colmask && mask_bh_bytes(a.mask_ld) >= (int64_t)OOB) return -1;
    if (ldr < a.S + 128) return -1;
    const dim3 grid((unsigned)((a.S + KB - 1) / KB), (unsigned)a.H, (unsigned)a.B);
    if (a.colmask)
        hipLaunchKernelGGL(flash_bwd_kv4_kernel<true>, grid, dim3(NT), LDS_BYTES, s, a, lse, Dv, dout, ldo, dqkv, ldd,
                           dqr, dsj, ldr, meta_ds);
    else
        hipLaunchKernelGGL(flash_bwd_kv4_kernel<false>, grid, dim3(NT), LDS_BYTES, s, a, lse, Dv, dout, ldo, dqkv, ldd,
                           dqr, dsj, ldr, meta_ds);
    return 0;
}
