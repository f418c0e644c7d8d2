// Relative-position flash attention backward, key/value-major pass, v3.
// (model_transformer.py:54-90 differentiated; the recompute of P uses the
// forward's row log-sum-exp.)
//   P_ij  = exp(scale (q_i.k_j + q_i.R[S-1-i+j]) - lse_i)
//   dS_ij = P_ij (dO_i.v_j - D_i) scale,           D_i = dO_i.O_i
//   dV_j  = sum_i P_ij dO_i,  dK_j = sum_i dS_ij q_i   (accumulated here)
//   dS is written in the r-indexed layout dQR[h][b][i][r = S-1-i+j] for the
//   dq / dR products (attn_flash.hip); metadata-block entries j > i go to
//   meta_ds.
// One workgroup = 8 waves = 128 keys of one (b, h), 16 keys per wave on the
// lanes (lane & 15 = key), two waves per SIMD; the key-side operands K^T, V^T
// stay in registers, dK^T / dV^T accumulate in registers. Query tiles of 32
// stream through LDS by LDS-DMA one tile ahead (Q and dO in a dual-swizzle
// image read both as rows and, transposed, as quads); R is a 192-row ring —
// the window of query tile t+1 is the window of tile t shifted DOWN by 32 rows,
// so each tile stages one new 32-row chunk. One barrier per tile.
#include "attn_tiles.h"

namespace {
using namespace attn;

constexpr int NT = 512;
constexpr int KB = 128, QT = 32, NCH = 6, SCR = 36;
constexpr int O_Q = 0, O_O = 2 * QT * 256, O_L = 4 * QT * 256, O_R = O_L + 2 * 2 * 64 * 4;
constexpr int O_S = O_R + NCH * 32 * 256, O_M = O_S + 8 * 2 * 16 * SCR * 4;
constexpr int O_D = O_M + 64 * 4;  // dropout keep words of the block's 128 keys, 2 tiles
// dS staging for the coalesced stores: 2 tiles x 32 query rows x 128 keys, rows
// 288 B apart (the four rows one wave writes at a time fall on disjoint banks)
constexpr int T_PITCH = 288, T_BYTES = QT * T_PITCH;
constexpr int O_T = O_D + 2 * KB * 4;
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
// dual image (row reads and transposed quads reads, cdna_hip_programming.md T10 (b))
__device__ __forceinline__ int sw_dual(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// DROP: attention-probability dropout (model_transformer.py:80); the keep word
// (key, query tile) of colmask is staged with the tile: dV uses P keep/(1-p),
// dS = P (dP keep/(1-p) - D) scale
// LAB: ablation switches for tools/lab (0 in the library): 1 no dS stores,
// 2 no MFMA, 4 no skew / softmax, 16 no DMA in the loop
template <bool DROP, int LAB = 0>
__global__ __launch_bounds__(NT, 1) void flash_bwd_kv3_kernel(AttnArgs a, const float* __restrict__ lse,
                                                              const float* __restrict__ Dv,
                                                              const bf16* __restrict__ dout, int64_t ldo,
                                                              bf16* __restrict__ dqkv, int64_t ldd,
                                                              bf16* __restrict__ dqr, bf16* __restrict__ dsj,
                                                              int64_t ldr, float* __restrict__ meta_ds) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sR = smem + O_R;
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, il = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = (int)a.S, H = (int)a.H;
    const int64_t ldq = a.ldq;
    const int kb = (int)blockIdx.x;  // 0 = keys 0..127 (the heaviest block)
    const int h = blockIdx.y, b = blockIdx.z;
    const int j0 = kb * KB, jw0 = j0 + 16 * w, jk = jw0 + il;  // this lane's key
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
    float* scw = (float*)(smem + O_S) + w * 2 * 16 * SCR;
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

    // key-side operands (B of S = Q.K^T and dP = dO.V^T): this lane's key
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        if (jk < S) {
            kf[ks] = *(const bf16x8*)(qkv_b + (int64_t)jk * ldq + (H + h) * HS + ks * 32 + g * 8);
            vf[ks] = *(const bf16x8*)(qkv_b + (int64_t)jk * ldq + (2 * H + h) * HS + ks * 32 + g * 8);
        } else {
            kf[ks] = vf[ks] = (bf16x8){};
        }
    }
    f32x4 dk[8], dv[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) dk[n] = dv[n] = zero4();

    // query tiles: i0 = it0 + 32 t (causal: i >= j0; block 0 also the metadata rows)
    const int it0 = (j0 / QT) * QT;
    const int nqt = (S - it0 + QT - 1) / QT;
    // R window of tile t: rows rw0 - 32 t + [0, 160); chunk c = rows rw0 + 128 - 32 c + [0, 32)
    const int rw0 = S - QT - it0 + j0;

    // per-lane DMA constants (row tid/16 of a 32-row tile, chunk slot lane%16)
    const int lrow = 4 * w + (lane >> 4);
    const int chD = (lane & 15) ^ sw_dual(lrow), chR = (lane & 15) ^ (lrow & 15);
    const uint32_t offQ = (uint32_t)((lrow * ldq + (int64_t)h * HS + chD * 8) * 2);
    const uint32_t offO = (uint32_t)((lrow * ldo + (int64_t)h * HS + chD * 8) * 2);
    const uint32_t offR = (uint32_t)((lrow * HS + chR * 8) * 2);
    auto stage_q = [&](int t) {  // Q, dO, lse, D of query tile t
        const int i0 = it0 + QT * t, buf = t & 1;
        const bool ok = i0 + lrow < S;
        dma16(rq, smem + O_Q + buf * QT * 256 + w * 1024, ok ? offQ + (uint32_t)i0 * (uint32_t)(ldq * 2) : OOB);
        dma16(ro, smem + O_O + buf * QT * 256 + w * 1024, ok ? offO + (uint32_t)i0 * (uint32_t)(ldo * 2) : OOB);
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
        if (DROP && w >= 2 && w < 4) {
            const int i0 = it0 + QT * t, key = j0 + 64 * (w - 2) + lane;
            dma4(rm, smem + O_D + (t & 1) * KB * 4 + (w - 2) * 256,
                 key < S ? (uint32_t)(mask_word(mld, key, i0) * 4) : OOB);
        }
    };
    auto stage_r = [&](int c) {  // R chunk c into ring slot c % NCH
        const int r0 = rw0 + 128 - 32 * c, rg = r0 + lrow;
        dma16(rr, sR + (c % NCH) * 32 * 256 + w * 1024,
              (rg >= 0 && rg < S) ? offR + (uint32_t)(r0 * HS * 2) : OOB);
    };
    // per-lane LDS fragment offsets: rows of the dual image (A operand) and
    // quads (transposed A operand of dV^T / dK^T), rows of the R ring (B operand)
    int rowo[4], quado[8], ro_R[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        rowo[ks] = il * 256 + (((ks * 4 + g) ^ sw_dual(il)) << 4);
        ro_R[ks] = il * 256 + (((ks * 4 + g) ^ il) << 4);
    }
    {
        const int q = il >> 2, p = il & 3, r1 = 4 * g + q;
#pragma unroll
        for (int n = 0; n < 8; ++n) quado[n] = r1 * 256 + (((2 * n + (p >> 1)) ^ sw_dual(r1)) << 4) + (p & 1) * 8;
    }

    // prologue: tile 0 and the 5 R chunks of its window
    stage_q(0);
    stage_m(0);
#pragma unroll
    for (int c = 0; c < NCH - 1; ++c) stage_r(c);

    // dS of a tile (j <= i, else 0) is staged in LDS and stored in the NEXT
    // iteration, right AFTER that iteration's prefetch, as whole rows: thread t
    // writes 8 keys of query row t/16, once j-indexed (dSj, aligned 16-B
    // chunks of 256-B row runs) and once r-indexed (dQR, r = S-1-i+j: the
    // row's 128 values start 2-byte aligned, stored as unaligned 16-B chunks;
    // entries j > i land at r >= S, in the row padding (ldr >= S + 128) that no
    // reader touches). The 2 stores per thread are then the youngest vector
    // memory ops at the following tile's wait (vmcnt(2) leaves them in flight);
    // invalid rows use the out-of-range offset, so the count is exact.
    int i0_prev = -1;
    const __amdgpu_buffer_rsrc_t rqr = make_rsrc(qr_rows, (uint32_t)min<int64_t>((int64_t)S * ldr * 2, OOB - 1));
    const __amdgpu_buffer_rsrc_t rsj = make_rsrc(sj_rows, (uint32_t)min<int64_t>((int64_t)S * ldr * 2, OOB - 1));
    auto store_ds = [&](int ip, int sbuf) {
        const int row = tid >> 4, ch = tid & 15;
        const u32x4 v = *(const u32x4*)(smem + O_T + sbuf * T_BYTES + row * T_PITCH + ch * 16);
        const int i = ip + row, j = j0 + 8 * ch;
        const bool in = i < S;
        const uint32_t os = in ? (uint32_t)(((int64_t)i * ldr + j) * 2) : OOB;
        const uint32_t oq = in ? (uint32_t)(((int64_t)i * ldr + (S - 1 - i + j)) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(v, rsj, os, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v, rqr, oq, 0, 0);
    };

    for (int t = 0; t < nqt; ++t) {
        const int i0 = it0 + QT * t, buf = t & 1;
        // tile t's DMA (issued in iteration t-1, or the prologue) is older than
        // the 2 dS stores of iteration t-1 (present from t = 2 on)
        if (t >= 2 && !(LAB & 1)) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();  // tile t landed everywhere; tile t-1's buffers (and dS staging) are free / published
        if (t + 1 < nqt && !(LAB & 16)) {
            stage_q(t + 1);
            stage_r(t + NCH - 1);
            stage_m(t + 1);
        }
        asm volatile("" ::: "memory");
        if (i0_prev >= 0 && !(LAB & 1)) store_ds(i0_prev, buf ^ 1);
        const char* cQ = smem + O_Q + buf * QT * 256;
        const char* cO = smem + O_O + buf * QT * 256;
        const float* cL = (const float*)(smem + O_L + buf * 512);
        const float* cD = cL + 64;
        // this wave's 48-row window (32 queries x 16 keys) starts at block-window
        // row 16 w; sub-tile s (queries i0+16s ..) uses its blocks 1-s, 2-s
        const int wbase = 16 * w;
        bf16x8 pa, da;
        // whole sub-tile below the diagonal and inside the sequence: no mask
        const bool unmasked = (i0 >= jw0 + 15) && (i0 + QT <= S);
        const uint32_t kw = DROP ? ((const uint32_t*)(smem + O_D + buf * KB * 4))[16 * w + il] >> (4 * g) : 0u;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            f32x4 sacc = zero4(), dpacc = zero4(), qa = zero4(), qb2 = zero4();
            const int rb_a = wbase + 16 * (1 - s);  // window rows of the two blocks
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const bf16x8 qx = *(const bf16x8*)(cQ + s * 4096 + rowo[ks]);
                const bf16x8 ox = *(const bf16x8*)(cO + s * 4096 + rowo[ks]);
                if (LAB & 2) {
                    asm volatile("" ::"v"(qx), "v"(ox));
                } else {
                    sacc = mfma(qx, kf[ks], sacc);
                    dpacc = mfma(ox, vf[ks], dpacc);
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int wr = rb_a + 16 * u;  // window row of the block (multiple of 16)
                    const int c = t + 4 - (wr >> 5);
                    const int ringrow = (c % NCH) * 32 + (wr & 31);
                    const bf16x8 rx = *(const bf16x8*)(sR + ringrow * 256 + ro_R[ks]);
                    if (LAB & 2) asm volatile("" ::"v"(rx));
                    else if (u == 0) qa = mfma(qx, rx, qa);
                    else qb2 = mfma(qx, rx, qb2);
                }
            }
            if (LAB & 4) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    pa[4 * s + r] = (bf16)(sacc[r] + qa[r]);
                    da[4 * s + r] = (bf16)(dpacc[r] + qb2[r]);
                }
                continue;
            }
            // skew: QR[i = 4g+r][wl = il (+16)] -> BD[i][j = il], wl = j - i + 15
            float* sc = scw + s * 16 * SCR;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sc[(4 * g + r) * SCR + il] = qa[r];
                sc[(4 * g + r) * SCR + 16 + il] = qb2[r];
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ir = 4 * g + r;
                const int i = i0 + 16 * s + ir;
                float x = sacc[r] + sc[ir * SCR + il - ir + 15];
                const float l2 = cL[16 * s + ir] * LOG2E, dd = cD[16 * s + ir];
                float p, ds;
                const float kb = DROP ? ((kw >> (16 * s + r)) & 1u ? a.keep_scale : 0.f) : 1.f;
                if (unmasked) {
                    p = __builtin_amdgcn_exp2f(fmaf(x, c2, -l2));
                    ds = p * (DROP ? fmaf(dpacc[r], kb, -dd) : dpacc[r] - dd) * a.scale;
                } else {
                    const bool ok = (i < S) && (jk < S) && (jk <= i || jk < nm);
                    if (ok && jk >= i + 2) x += mbd[i * 8 + jk];
                    p = ok ? __builtin_amdgcn_exp2f(fmaf(x, c2, -l2)) : 0.f;
                    ds = ok ? p * (DROP ? fmaf(dpacc[r], kb, -dd) : dpacc[r] - dd) * a.scale : 0.f;
                    if (ok && jk > i) meta_ds[(((int64_t)b * H + h) * 8 + i) * 8 + jk] = ds;
                }
                if (DROP) p *= kb;
                pa[4 * s + r] = (bf16)p;
                da[4 * s + r] = (bf16)ds;
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
        }
        // dV^T[d][j] += dO^T[d][i] P[i][j] ;  dK^T[d][j] += Q^T[d][i] dS[i][j]
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const bf16x8 ofr = cat8(tr_read(cO, quado[n]), tr_read(cO, 4096 + quado[n]));
            const bf16x8 qfr = cat8(tr_read(cQ, quado[n]), tr_read(cQ, 4096 + quado[n]));
            if (LAB & 2) {
                asm volatile("" ::"v"(ofr), "v"(qfr), "v"(pa), "v"(da));
            } else {
                dv[n] = mfma(ofr, pa, dv[n]);
                dk[n] = mfma(qfr, da, dk[n]);
            }
        }
        {  // stage this tile's dS rows (0 above the diagonal) for the next iteration's stores
            char* st = smem + O_T + buf * T_BYTES + (16 * w + il) * 2;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int row = 16 * (e >> 2) + 4 * g + (e & 3);
                *(bf16*)(st + row * T_PITCH) = jk <= i0 + row ? da[e] : (bf16)0.f;
            }
        }
        i0_prev = i0;
    }
    if (i0_prev >= 0 && !(LAB & 1)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        store_ds(i0_prev, (nqt - 1) & 1);
    }
    // lane holds dK^T / dV^T [d = 16n + 4g + r][key il]
    if (jk < S) {
        bf16* dkp = dqkv + ((int64_t)b * S + jk) * ldd + (H + h) * HS;
        bf16* dvp = dkp + H * HS;
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            store4(dkp + n * 16 + 4 * g, dk[n]);
            store4(dvp + n * 16 + 4 * g, dv[n]);
        }
    }
}

}  // namespace

int flash_bwd_kv3(const AttnArgs& a, const float* lse, const float* Dv, const bf16* dout, int64_t ldo, bf16* dqkv,
                  int64_t ldd, bf16* dqr, bf16* dsj, int64_t ldr, float* meta_ds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_bwd_kv3_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)flash_bwd_kv3_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        attr = true;
    }
    if (a.S * a.ldq * 2 >= (int64_t)OOB || a.S * ldo * 2 >= (int64_t)OOB || a.n_meta > 8) return -1;
    if (a.colmask && mask_bh_bytes(a.mask_ld) >= (int64_t)OOB) return -1;
    const dim3 grid((unsigned)((a.S + KB - 1) / KB), (unsigned)a.H, (unsigned)a.B);
    if (a.colmask)
        hipLaunchKernelGGL(flash_bwd_kv3_kernel<true>, grid, dim3(NT), LDS_BYTES, s, a, lse, Dv, dout, ldo, dqkv, ldd,
                           dqr, dsj, ldr, meta_ds);
    else
        hipLaunchKernelGGL(flash_bwd_kv3_kernel<false>, grid, dim3(NT), LDS_BYTES, s, a, lse, Dv, dout, ldo, dqkv, ldd,
                           dqr, dsj, ldr, meta_ds);
    return 0;
}
