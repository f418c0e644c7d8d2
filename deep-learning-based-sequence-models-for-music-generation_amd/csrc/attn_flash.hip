// Relative-position flash attention, bf16 MFMA path (hs = 128).
//
// Forward (one workgroup = 4 waves = 64 query rows of one (b, h); each wave
// owns 16 queries; key tiles of 64):
//   * scores are computed "swapped" (S^T = K.Q^T) so each lane owns ONE query
//     row (lane & 15) and 16 of the tile's keys: row max / sum need only two
//     cross-lane steps, P is already the B operand of the next MFMA and the
//     output accumulator O^T keeps the query on the lane too (no shuffles);
//   * the relative term BD(i,j) = q_i . R[S-1-i+j] (model_transformer.py:70-75,
//     84-90) is a GEMM against a 80-row window of R per wave (R tile staged per
//     key tile), followed by a per-wave skew through LDS: QR[i][w] -> BD[i][j]
//     with w = j - i + 15;
//   * online softmax in the exp2 domain, mask j <= i || j < n_meta implicit;
//   * the meta-block terms BD(i, j >= i+2) = q_{i+1}.R[j-i-2] (only i < 5) are
//     added by the single wave that sees tile (0, 0).
// Backward:
//   pre : D_i = sum_d dO.O
//   A   : per 64-key block: recompute S, P; dP = dO.V^T; dS = P (dP - D) scale;
//         dK, dV accumulated in registers; dS written in the r-indexed layout
//         dQR[h][b][i][r = S-1-i+j] (bf16) for the GEMMs below;
//   B   : dq_ac = sum_j dS_ij k_j  from dQR with a K window + LDS skew;
//   GEMM: dq = dQR . R + dq_ac (batched over heads);  dR += dQR^T . Q;
//   fix : meta-block terms (j > i inside the metadata prefix).
#include "attn_tiles.h"
#include "gemm.h"
#include <stdlib.h>

namespace {

using namespace attn;
constexpr int NT = 256;

// copy `rows` rows of 128 bf16 (row r from src + r*ld, zero if !valid) into an image
template <int MODE>  // 0 row, 1 pairs, 2 quads
__device__ __forceinline__ void stage_rows(char* dst, const bf16* src, int64_t ld, int rows, int64_t first,
                                           int64_t lo, int64_t hi, int tid) {
    for (int c = tid; c < rows * 16; c += NT) {
        const int row = c >> 4, ch = c & 15;
        const int64_t gr = first + row;
        u32x4 v = (u32x4){0u, 0u, 0u, 0u};
        if (gr >= lo && gr < hi) v = *(const u32x4*)(src + gr * ld + ch * 8);
        const int off = MODE == 0 ? off_row(row, ch) : (MODE == 1 ? off_pairs(row, ch) : off_quads(row, ch));
        *(u32x4*)(dst + off) = v;
    }
}

// --------------------------------------------------------------------- forward
constexpr int F_QB = 64, F_KB = 64, F_RW = 128, F_SCR = 84;
constexpr int F_LDS_K = F_KB * 256, F_LDS_R = F_RW * 256, F_LDS_S = 4 * 16 * F_SCR * 4;

__global__ __launch_bounds__(NT, 2) void flash_fwd_kernel(AttnArgs a, bf16* __restrict__ out, int64_t ldo,
                                                          float* __restrict__ lse) {
    __shared__ __attribute__((aligned(16))) char smem[F_LDS_K + F_LDS_R + F_LDS_S];
    char* sK = smem;
    char* sR = smem + F_LDS_K;  // R window; V overlays it after the QR products
    float* scr = (float*)(smem + F_LDS_K + F_LDS_R);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, il = lane & 15;
    const int64_t S = a.S;
    const int nqb = (int)((S + F_QB - 1) / F_QB);
    const int qb = nqb - 1 - (int)blockIdx.x;  // heaviest blocks first
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int64_t i0 = (int64_t)qb * F_QB + 16 * w;
    const int64_t iq = i0 + il;  // this lane's query row
    const int64_t ldq = a.ldq;
    const bf16* qkv = (const bf16*)a.qkv;
    const bf16* Qp = qkv + b * S * ldq + h * HS;
    const bf16* Kp = Qp + a.H * HS;
    const bf16* Vp = Kp + a.H * HS;
    const bf16* Rp = (const bf16*)a.R + h * a.S_max * HS;
    float* scw = scr + w * 16 * F_SCR;

    // Q fragments (Y operand): Q[iq][32ks + 8g .. +7]
    bf16x8 qf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        if (iq < S) qf[ks] = *(const bf16x8*)(Qp + iq * ldq + ks * 32 + g * 8);
        else qf[ks] = (bf16x8){};
    }

    f32x4 oacc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) oacc[n] = zero4();
    float m_run = -INFINITY, l_part = 0.f;
    const float c2 = a.scale * LOG2E;

    const int64_t last_q = min<int64_t>((int64_t)qb * F_QB + F_QB - 1, S - 1);
    const int nkt = (int)(last_q / F_KB) + 1;
    for (int kt = 0; kt < nkt; ++kt) {
        const int64_t j0 = (int64_t)kt * F_KB;
        const int64_t rbase = S - F_QB - (int64_t)qb * F_QB + j0;  // R row of window row 0
        __syncthreads();
        stage_rows<0>(sK, Kp, ldq, F_KB, j0, 0, S, tid);
        stage_rows<0>(sR, Rp, HS, F_RW, rbase, 0, S, tid);
        __syncthreads();

        // S^T tile: sacc[nt][r] = S_ac[key 16nt+4g+r][query il]
        f32x4 sacc[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            sacc[nt] = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) sacc[nt] = mfma(frag_row(sK, nt * 16, ks, lane), qf[ks], sacc[nt]);
        }
        // QR window of this wave: rows wb .. wb+79 of the R tile
        const int wb = 48 - 16 * w;
        f32x4 qacc[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            qacc[t] = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qacc[t] = mfma(frag_row(sR, wb + t * 16, ks, lane), qf[ks], qacc[t]);
        }
        __syncthreads();  // every wave is done with the R tile
        stage_rows<2>(sR, Vp, ldq, F_KB, j0, 0, S, tid);

        // skew QR[i][w] -> BD[i][j] through this wave's scratch
#pragma unroll
        for (int t = 0; t < 5; ++t) *(f32x4*)(scw + il * F_SCR + t * 16 + 4 * g) = qacc[t];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        float sv[4][4];
        float mx = -INFINITY;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jl = nt * 16 + 4 * g + r;
                const int64_t j = j0 + jl;
                float s = sacc[nt][r] + scw[il * F_SCR + jl - il + 15];
                const bool ok = (j < S) && (j <= iq || j < a.n_meta);
                if (ok && j >= iq + 2) {  // meta block, BD = q_{i+1}.R[j-i-2]
                    const bf16* q1 = Qp + (iq + 1) * ldq;
                    const bf16* rr = Rp + (j - iq - 2) * HS;
                    float acc = 0.f;
                    for (int d = 0; d < HS; ++d) acc += (float)q1[d] * (float)rr[d];
                    s += acc;
                }
                s = ok ? s * c2 : -INFINITY;
                sv[nt][r] = s;
                mx = fmaxf(mx, s);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx);
        const float alpha = exp2f(m_run - m_new);
        m_run = m_new;
        float ps = 0.f;
        bf16x8 pf[2];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = exp2f(sv[nt][r] - m_new);
                ps += p;
                pf[nt >> 1][(nt & 1) * 4 + r] = (bf16)p;
            }
        }
        l_part = l_part * alpha + ps;
#pragma unroll
        for (int n = 0; n < 8; ++n) oacc[n] *= alpha;
        __syncthreads();  // V staged
        // O^T[d][i] += V^T[d][key] P^T[key][i]
#pragma unroll
        for (int n = 0; n < 8; ++n) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) oacc[n] = mfma(frag_quads(sR, ks * 32, n * 16, lane), pf[ks], oacc[n]);
        }
    }
    float l = l_part + __shfl_xor(l_part, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (iq < S) {
        const float inv = 1.f / l;
        bf16* op = out + (b * S + iq) * ldo + h * HS;
#pragma unroll
        for (int n = 0; n < 8; ++n) store4(op + n * 16 + 4 * g, oacc[n] * inv);
        if (g == 0) lse[(b * a.H + h) * S + iq] = (m_run + log2f(l)) / LOG2E;
    }
}

// ------------------------------------------------------------ backward: pre
// D[b,h,i] = sum_d dO[i,d] O[i,d]
__global__ void flash_bwd_pre_kernel(AttnArgs a, const bf16* __restrict__ dout, int64_t ldo,
                                     const bf16* __restrict__ out, float* __restrict__ Dv) {
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);  // over B*S*H
    const int lane = threadIdx.x & 63;
    if (row >= a.B * a.S * a.H) return;
    const int64_t h = row % a.H, bi = row / a.H;
    const int64_t b = bi / a.S, i = bi % a.S;
    const f32x2 x = (f32x2){(float)dout[bi * ldo + h * HS + 2 * lane], (float)dout[bi * ldo + h * HS + 2 * lane + 1]};
    const f32x2 y = (f32x2){(float)out[bi * ldo + h * HS + 2 * lane], (float)out[bi * ldo + h * HS + 2 * lane + 1]};
    const float s = wave_sum(x[0] * y[0] + x[1] * y[1]);
    if (lane == 0) Dv[(b * a.H + h) * a.S + i] = s;
}

// ------------------------------------------------------------ backward: A
// block = 64 keys (4 waves x 16 keys on the lane); loop over 32-query tiles.
constexpr int A_KB = 64, A_QT = 32, A_RW = 96, A_SCR = 36;
constexpr int A_LDS_Q = A_QT * 256, A_LDS_O = A_QT * 256, A_LDS_R = A_RW * 256, A_LDS_S = 4 * 2 * 16 * A_SCR * 4;

// dual-use (row + transposed-quads) image for Q and dO: guide T10 (b) swizzle
__device__ __forceinline__ int off_dual(int row, int ch) {
    return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

__global__ __launch_bounds__(NT, 2) void flash_bwd_a_kernel(AttnArgs a, const float* __restrict__ lse,
                                                            const float* __restrict__ Dv, const bf16* __restrict__ dout,
                                                            int64_t ldo, bf16* __restrict__ dqkv, int64_t ldd,
                                                            bf16* __restrict__ dqr, int64_t ldr,
                                                            float* __restrict__ meta_ds) {
    __shared__ __attribute__((aligned(16))) char smem[A_LDS_Q + A_LDS_O + A_LDS_R + A_LDS_S];
    char* sQ = smem;
    char* sO = smem + A_LDS_Q;
    char* sR = smem + A_LDS_Q + A_LDS_O;
    float* scr = (float*)(smem + A_LDS_Q + A_LDS_O + A_LDS_R);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, il = lane & 15;
    const int64_t S = a.S, H = a.H;
    const int nkb = (int)((S + A_KB - 1) / A_KB);
    const int kb = (int)blockIdx.x;
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int64_t j0 = (int64_t)kb * A_KB;
    const int64_t jw = j0 + 16 * w;
    const int64_t jk = jw + il;  // this lane's key
    const int64_t ldq = a.ldq;
    const bf16* qkv = (const bf16*)a.qkv;
    const bf16* Qp = qkv + b * S * ldq + h * HS;
    const bf16* Kp = Qp + H * HS;
    const bf16* Vp = Kp + H * HS;
    const bf16* Op = dout + b * S * ldo + h * HS;
    const bf16* Rp = (const bf16*)a.R + h * a.S_max * HS;
    const float* Lp = lse + (b * H + h) * S;
    const float* Dp = Dv + (b * H + h) * S;
    bf16* qr_rows = dqr + ((h * a.B + b) * S) * ldr;
    float* scw = scr + w * 2 * 16 * A_SCR;
    (void)nkb;

    bf16x8 kf[4], vf[4];  // Y operands: K^T / V^T of this lane's key
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        if (jk < S) {
            kf[ks] = *(const bf16x8*)(Kp + jk * ldq + ks * 32 + g * 8);
            vf[ks] = *(const bf16x8*)(Vp + jk * ldq + ks * 32 + g * 8);
        } else {
            kf[ks] = vf[ks] = (bf16x8){};
        }
    }
    f32x4 dk[8], dv[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) dk[n] = dv[n] = zero4();
    const float c2 = a.scale * LOG2E;

    // queries i >= j (causal) plus the metadata prefix rows for kb == 0
    for (int64_t i0 = (j0 / A_QT) * A_QT; i0 < S; i0 += A_QT) {
        const int64_t rb = S - A_QT - i0 + j0;  // R row of window row 0 (block)
        __syncthreads();
        for (int c = tid; c < A_QT * 16; c += NT) {
            const int row = c >> 4, ch = c & 15;
            const int64_t gi = i0 + row;
            u32x4 vq = (u32x4){0u, 0u, 0u, 0u}, vo = vq;
            if (gi < S) {
                vq = *(const u32x4*)(Qp + gi * ldq + ch * 8);
                vo = *(const u32x4*)(Op + gi * ldo + ch * 8);
            }
            *(u32x4*)(sQ + off_dual(row, ch)) = vq;
            *(u32x4*)(sO + off_dual(row, ch)) = vo;
        }
        stage_rows<0>(sR, Rp, HS, A_RW, rb, 0, S, tid);
        __syncthreads();

        // per 16-query sub-tile s: S[i][j] (i = 4g+r on regs, j = il on lane)
        float pv[2][4], dsv[2][4];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            f32x4 sacc = zero4(), dpacc = zero4(), qa = zero4(), qb2 = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const bf16x8 qx = *(const bf16x8*)(sQ + off_dual(s * 16 + il, ks * 4 + g));
                const bf16x8 ox = *(const bf16x8*)(sO + off_dual(s * 16 + il, ks * 4 + g));
                sacc = mfma(qx, kf[ks], sacc);
                dpacc = mfma(ox, vf[ks], dpacc);
                // QR: rows of the R window: wave base 16w, sub-tile offset 16 - 16s
                const int rr = 16 * w + 16 - 16 * s;
                qa = mfma(qx, frag_row(sR, rr, ks, lane), qa);
                qb2 = mfma(qx, frag_row(sR, rr + 16, ks, lane), qb2);
            }
            // skew: QR[i][wl] (i = 4g+r, wl = il (+16)) -> BD[i][j] with wl = j - i + 15
            float* sc = scw + s * 16 * A_SCR;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sc[(4 * g + r) * A_SCR + il] = qa[r];
                sc[(4 * g + r) * A_SCR + 16 + il] = qb2[r];
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ir = 4 * g + r;
                const int64_t i = i0 + s * 16 + ir;
                float sc_v = sacc[r] + sc[ir * A_SCR + il - ir + 15];
                const bool ok = (i < S) && (jk < S) && (jk <= i || jk < a.n_meta);
                if (ok && jk >= i + 2) {
                    const bf16* q1 = Qp + (i + 1) * ldq;
                    const bf16* rr2 = Rp + (jk - i - 2) * HS;
                    float acc = 0.f;
                    for (int d = 0; d < HS; ++d) acc += (float)q1[d] * (float)rr2[d];
                    sc_v += acc;
                }
                const int64_t ic = i < S ? i : S - 1;
                const float p = ok ? exp2f(sc_v * c2 - Lp[ic] * LOG2E) : 0.f;
                const float ds = ok ? p * (dpacc[r] - Dp[ic]) * a.scale : 0.f;
                pv[s][r] = p;
                dsv[s][r] = ds;
                if (ok) {
                    const int64_t rr3 = S - 1 - i + jk;
                    if (jk <= i) qr_rows[i * ldr + rr3] = (bf16)ds;
                    else meta_ds[((b * H + h) * 8 + i) * 8 + jk] = ds;
                }
            }
        }
        // dV[j][d] += sum_i P[i][j] dO[i][d] ;  dK[j][d] += sum_i dS[i][j] q_i[d]
        bf16x8 pa, da;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            pa[r] = (bf16)pv[0][r];
            pa[4 + r] = (bf16)pv[1][r];
            da[r] = (bf16)dsv[0][r];
            da[4 + r] = (bf16)dsv[1][r];
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            // transposed reads of the dual images: rows {4g+q, 16+4g+q}, cols 16n..16n+15
            const int i = lane & 15, q = i >> 2, p = i & 3;
            const int ch = 2 * n + (p >> 1), sub = (p & 1) * 8;
            const int r1 = 4 * g + q, r2 = r1 + 16;
            const bf16x8 ofr = cat8(tr_read(sO, off_dual(r1, ch) + sub), tr_read(sO, off_dual(r2, ch) + sub));
            const bf16x8 qfr = cat8(tr_read(sQ, off_dual(r1, ch) + sub), tr_read(sQ, off_dual(r2, ch) + sub));
            dv[n] = mfma(pa, ofr, dv[n]);
            dk[n] = mfma(da, qfr, dk[n]);
        }
    }
    // lane holds dK/dV[j = jw + 4g + r][d = 16n + il]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t j = jw + 4 * g + r;
        if (j >= S) continue;
        bf16* dkp = dqkv + (b * S + j) * ldd + H * HS + h * HS;
        bf16* dvp = dkp + H * HS;
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            dkp[n * 16 + il] = (bf16)dk[n][r];
            dvp[n * 16 + il] = (bf16)dv[n][r];
        }
    }
}

// ------------------------------------------------------------ backward: B
// dq_ac[i][d] = sum_j dS_ij k_j, read from dQR[i][r] (r = S-1-i+j) per r-tile:
// j = r - (S-1-i) -> window row wl = (r - r0) + (i - i0) of a 80-row K window.
constexpr int B_QB = 64, B_RT = 64, B_KW = 144, B_WLD = 104;  // window row stride (bf16)
constexpr int B_LDS_K = B_KW * 256, B_LDS_W = 4 * 16 * B_WLD * 2;

__global__ __launch_bounds__(NT, 2) void flash_bwd_b_kernel(AttnArgs a, const bf16* __restrict__ dqr, int64_t ldr,
                                                            float* __restrict__ dq_ac, int64_t ld_ac) {
    __shared__ __attribute__((aligned(16))) char smem[B_LDS_K + B_LDS_W];
    char* sK = smem;
    bf16* swin = (bf16*)(smem + B_LDS_K);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, il = lane & 15;
    const int64_t S = a.S, H = a.H;
    const int nqb = (int)((S + B_QB - 1) / B_QB);
    const int qb = nqb - 1 - (int)blockIdx.x;
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int64_t i0b = (int64_t)qb * B_QB;
    const int64_t i0 = i0b + 16 * w;
    const int64_t iq = i0 + il;
    const int64_t ldq = a.ldq;
    const bf16* Kp = (const bf16*)a.qkv + b * S * ldq + H * HS + h * HS;
    const bf16* qr_rows = dqr + ((h * a.B + b) * S) * ldr;
    bf16* wwin = swin + w * 16 * B_WLD;

    f32x4 acc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[n] = zero4();

    // r range touched by the block: r >= S-1-(i0b+63)
    const int64_t rmin = max<int64_t>(0, S - 1 - (i0b + B_QB - 1));
    for (int64_t r0 = (rmin / B_RT) * B_RT; r0 < S; r0 += B_RT) {
        // block K window: j = r - S + 1 + i  for r in [r0, r0+64), i in [i0b, i0b+64)
        const int64_t jb = r0 - S + 1 + i0b;
        __syncthreads();
        stage_rows<1>(sK, Kp, ldq, B_KW, jb, 0, S, tid);
        // this wave's dQR tile [16 rows][64 r] -> skewed window [il][rl + il]
        for (int e = lane; e < 16 * B_WLD / 8; e += 64) *(u32x4*)(wwin + e * 8) = (u32x4){0u, 0u, 0u, 0u};
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < 16 * 8; e += 64) {
            const int row = e >> 3, ch = e & 7;
            const int64_t i = i0 + row, r = r0 + ch * 8;
            if (i < S && r < S) {
                union { u32x4 v; bf16 x[8]; } u;
                u.v = *(const u32x4*)(qr_rows + i * ldr + r);
#pragma unroll
                for (int t = 0; t < 8; ++t) wwin[row * B_WLD + ch * 8 + t + row] = u.x[t];
            }
        }
        __syncthreads();
        // window of wave w starts at block-window row 16w: wl = (r-r0) + (i-i0)
        // acc^T[d][i] += K_win^T[d][wl] . X^T[wl][i],  X[i][wl] = window
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            const bf16x8 xf = *(const bf16x8*)(wwin + il * B_WLD + ks * 32 + 8 * g);
#pragma unroll
            for (int n = 0; n < 8; ++n) acc[n] = mfma(frag_pairs(sK, 16 * w + ks * 32, n * 16, lane), xf, acc[n]);
        }
    }
    if (iq < S) {
        float* p = dq_ac + (b * S + iq) * ld_ac + h * HS;
#pragma unroll
        for (int n = 0; n < 8; ++n) *(f32x4*)(p + n * 16 + 4 * g) = acc[n];
    }
}

// ------------------------------------------------------------ backward: fix-up
// metadata prefix, j > i (only i < n_meta - 1): dS_ij was written to meta_ds.
//   dq_i     += dS_ij k_j            (AC term; pass B only sees j <= i)
//   dq_{i+1} += dS_ij R[j-i-2]        (j >= i+2)
//   dR[j-i-2] += dS_ij q_{i+1}        (j >= i+2)
__global__ void flash_bwd_meta_kernel(AttnArgs a, const float* __restrict__ meta_ds, bf16* __restrict__ dqkv,
                                      int64_t ldd, float* __restrict__ dR) {
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int d = threadIdx.x;  // 128 threads
    const int64_t S = a.S, H = a.H, ldq = a.ldq;
    const bf16* qkv = (const bf16*)a.qkv;
    const float* md = meta_ds + (b * H + h) * 64;
    const bf16* Rp = (const bf16*)a.R + h * a.S_max * HS;
    const int64_t nm = min<int64_t>(a.n_meta, S);
    for (int64_t i = 0; i + 1 < nm; ++i) {
        float gq = 0.f;
        for (int64_t j = i + 1; j < nm; ++j) gq += md[i * 8 + j] * (float)qkv[(b * S + j) * ldq + H * HS + h * HS + d];
        bf16* p = dqkv + (b * S + i) * ldd + h * HS + d;
        *p = (bf16)((float)*p + gq);
    }
    for (int64_t i = 0; i + 2 < nm; ++i) {
        float gq = 0.f;
        for (int64_t j = i + 2; j < nm; ++j) {
            const float ds = md[i * 8 + j];
            gq += ds * (float)Rp[(j - i - 2) * HS + d];
            atomicAdd(dR + (h * a.S_max + (j - i - 2)) * HS + d, ds * (float)qkv[(b * S + i + 1) * ldq + h * HS + d]);
        }
        bf16* p = dqkv + (b * S + i + 1) * ldd + h * HS + d;
        *p = (bf16)((float)*p + gq);
    }
}

}  // namespace

namespace {
// zero the part of dQR[h][b][i][r] that the consumers read but pass A does not
// write: r in [S-1-i-DQR_BAND, S-1-i) (below the written band) and the row pad
// [S, ldr). pass B and the triangular GEMMs never read further below the band.
constexpr int DQR_BAND = 256;
__global__ void dqr_band_zero_kernel(bf16* __restrict__ dqr, int64_t ldr, int64_t S, int64_t rows) {
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);  // (h, b, i) flattened
    if (row >= rows) return;
    const int64_t i = row % S;
    bf16* p = dqr + row * ldr;
    const int64_t lo = max<int64_t>(0, S - 1 - i - DQR_BAND), hi = S - 1 - i;
    for (int64_t r = lo + (threadIdx.x & 63); r < hi; r += 64) p[r] = (bf16)0.f;
    for (int64_t r = S + (threadIdx.x & 63); r < ldr; r += 64) p[r] = (bf16)0.f;
}
}  // namespace

int64_t flash_dqr_ld(int64_t S) { return (S + 7) / 8 * 8; }

// workspace: dQR bf16 [H][B][S][ldr] | D f32 [B][H][S] | meta_ds f32 [B][H][8][8] | dq_ac f32 [B*S][H*HS]
//            | dR split-K partials f32 [ksplit][H][S][HS]
static size_t align256(size_t x) { return (x + 255) / 256 * 256; }
static size_t dr_ws_bytes(int64_t B, int64_t S, int64_t H) {
    return splitk_ws_bytes(S, HS, H, gemm_bf16_tri_ksplit(2, S, HS, B * S, S, H));
}

size_t flash_bwd_workspace(int64_t B, int64_t S, int64_t H) {
    const int64_t ldr = flash_dqr_ld(S);
    return align256((size_t)H * B * S * ldr * 2) + align256((size_t)B * H * S * 4) + align256((size_t)B * H * 64 * 4) +
           align256((size_t)B * S * H * HS * 4) + align256(dr_ws_bytes(B, S, H));
}

int flash_fwd(const AttnArgs& a, bf16* out, int64_t ldo, float* lse, hipStream_t s) {
    const dim3 grid((unsigned)((a.S + F_QB - 1) / F_QB), (unsigned)a.H, (unsigned)a.B);
    hipLaunchKernelGGL(flash_fwd_kernel, grid, dim3(NT), 0, s, a, out, ldo, lse);
    return 0;
}

extern "C" int msq_gemm(int dtype, int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                        int64_t strideA, const void* B, int64_t ldb, int64_t strideB, void* C, int c_dtype,
                        int64_t ldc, int64_t strideC, int64_t batch, int epilogue, const float* bias,
                        const void* aux, int aux_dtype, int64_t ld_aux, int64_t stride_aux, void* stream);

int flash_bwd(const AttnArgs& a, const float* lse, const bf16* dout, int64_t ldo, const bf16* out, bf16* dqkv,
              int64_t ldd, float* dR, void* ws, hipStream_t s) {
    const int64_t B = a.B, S = a.S, H = a.H, ldr = flash_dqr_ld(S);
    char* p = (char*)ws;
    bf16* dqr = (bf16*)p;
    p += align256((size_t)H * B * S * ldr * 2);
    float* Dv = (float*)p;
    p += align256((size_t)B * H * S * 4);
    float* meta_ds = (float*)p;
    p += align256((size_t)B * H * 64 * 4);
    float* dq_ac = (float*)p;
    p += align256((size_t)B * S * H * HS * 4);
    float* dr_ws = (float*)p;

    hipLaunchKernelGGL(dqr_band_zero_kernel, dim3((unsigned)((H * B * S + 3) / 4)), dim3(256), 0, s, dqr, ldr, S,
                       H * B * S);
    hipMemsetAsync(meta_ds, 0, (size_t)B * H * 64 * 4, s);
    hipLaunchKernelGGL(flash_bwd_pre_kernel, dim3((unsigned)((B * S * H + 3) / 4)), dim3(256), 0, s, a, dout, ldo, out, Dv);
    // MSQ_ATTN_BWD=1 selects the first-generation key/value pass (A/B runs)
    const char* bv = getenv("MSQ_ATTN_BWD");
    const bool v1 = bv && atoi(bv) == 1 && !a.rowmask;
    if (v1 || flash_bwd_kv3(a, lse, Dv, dout, ldo, dqkv, ldd, dqr, ldr, meta_ds, s)) {
        if (a.rowmask) return msq_set_error(MSQ_ERR_UNSUPPORTED, "flash_bwd: dropout needs the v3 kernel");
        const unsigned nkb = (unsigned)((S + A_KB - 1) / A_KB);
        hipLaunchKernelGGL(flash_bwd_a_kernel, dim3(nkb, (unsigned)H, (unsigned)B), dim3(NT), 0, s, a, lse, Dv, dout,
                           ldo, dqkv, ldd, dqr, ldr, meta_ds);
    }
    const unsigned nqb = (unsigned)((S + B_QB - 1) / B_QB);
    hipLaunchKernelGGL(flash_bwd_b_kernel, dim3(nqb, (unsigned)H, (unsigned)B), dim3(NT), 0, s, a, dqr, ldr, dq_ac,
                       H * HS);
    // dq (bf16, q columns of dqkv) = dQR . R + dq_ac   (batched over heads)
    // (row i of dQR is nonzero only for r >= S-1-i: triangular K ranges, tri 1)
    int rc = gemm_bf16_tri(1, S, 0, 1, B * S, HS, S, dqr, ldr, B * S * ldr, a.R, HS, a.S_max * HS, dqkv, MSQ_BF16,
                           ldd, HS, H, MSQ_EPI_BIAS_RESID, dq_ac, MSQ_F32, H * HS, HS, s);
    if (rc) return msq_set_error(MSQ_ERR_ARG, "flash_bwd: dq product");
    // dR[h][r] += sum_{b,i} dQR[h][b,i][r] q_{b,i}   (batched over heads; per batch
    // segment only i >= S-1-r contributes: tri 2, split over segments)
    rc = gemm_bf16_tri(2, S, 1, 1, S, HS, B * S, dqr, ldr, B * S * ldr, a.qkv, a.ldq, HS, dR, MSQ_F32, HS,
                       a.S_max * HS, H, MSQ_EPI_ACCUM, nullptr, MSQ_F32, 0, 0, s, dr_ws, dr_ws_bytes(B, S, H));
    if (rc) return msq_set_error(MSQ_ERR_ARG, "flash_bwd: dR product");
    hipLaunchKernelGGL(flash_bwd_meta_kernel, dim3(1, (unsigned)H, (unsigned)B), dim3(HS), 0, s, a, meta_ds, dqkv, ldd,
                       dR);
    return 0;
}
