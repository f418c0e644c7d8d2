// Relative-position flash attention forward, v2 (bf16 MFMA, hs = 128).
// HeadRelPos (model_transformer.py:54-82, _rel_shift :84-90):
//   out_i = sum_j softmax_j(mask((q_i.k_j + q_i.R[S-1-i+j]) * C^-1/2)) v_j
//
// One workgroup = 4 waves = 128 queries of one (b, h); a wave owns 32 queries
// as two groups of 16 (lane & 15 = query, the "swapped" S^T = K.Q^T layout of
// attn_flash.hip, so softmax statistics and the O^T accumulator stay on the
// lane). Per 64-key tile a wave issues 104 MFMAs: 32 for K.Q^T, 40 for the
// relative term against a 96-row window of R (the two groups' 80-row windows
// overlap by 64 rows and share fragments), 32 for V^T.P^T (shared V
// fragments).
// HBM -> LDS traffic is LDS-DMA (buffer_load ... lds, zero-filled out of
// range) one tile ahead: K and V double-buffered, and R as a 256-row ring —
// the window of tile t+1 is the window of tile t shifted by 64 rows, so each
// tile stages only 64 new R rows. The relative term is skewed from window
// coordinates to key coordinates through a per-wave LDS scratch.
#include "attn_tiles.h"

namespace {
using namespace attn;

constexpr int NT = 256;
constexpr int QB = 128, KB = 64, RING = 256, SCR = 100;
constexpr int L_K = 2 * KB * 256, L_V = 2 * KB * 256, L_R = RING * 256, L_S = 4 * 16 * SCR * 4 + 64 * 4;
constexpr int LDS_BYTES = L_K + L_V + L_R + L_S;
constexpr uint32_t OOB = 0xFFFF0000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// DMA of 64 rows x 256 B into a row image: the lane's chunk / row inside
// each 16-row group is fixed (lane_off, lane_row), the tile moves only the
// wave-uniform base; rows outside [lo, hi) of the source come back zero.
__device__ __forceinline__ void dma64(__amdgpu_buffer_rsrc_t rs, char* dst, uint32_t lane_off, int lane_row,
                                      uint32_t base, uint32_t row_step, int lo, int hi, int w) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int r = lane_row + c * 16;
        const uint32_t vo = (r >= lo && r < hi) ? lane_off + base + c * row_step : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_char*)(dst + c * 4096 + w * 1024), 16, vo, 0, 0, 0);
    }
}

__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// LAB: ablation switches for tools/lab/attn_lab.hip only (0 in the library):
// 1 no K.Q^T MFMA, 2 no QR MFMA, 4 no skew / softmax, 8 no PV MFMA, 16 no DMA in the loop
template <int LAB = 0>
__global__ __launch_bounds__(NT, 1) void flash_fwd2_kernel(AttnArgs a, bf16* __restrict__ out, int64_t ldo,
                                                           float* __restrict__ lse) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sK = smem;
    char* sV = smem + L_K;
    char* sR = smem + L_K + L_V;
    float* scr = (float*)(smem + L_K + L_V + L_R);

    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, il = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t S = a.S, H = a.H, ldq = a.ldq;
    const int nqb = (int)((S + QB - 1) / QB);
    const int qb = nqb - 1 - (int)blockIdx.x;  // heaviest blocks first
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int64_t i0 = (int64_t)qb * QB;
    const bf16* qkv_b = (const bf16*)a.qkv + b * S * ldq;
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv_b, (uint32_t)(S * ldq * 2));
    const __amdgpu_buffer_rsrc_t rr = make_rsrc((const bf16*)a.R + h * a.S_max * HS, (uint32_t)(S * HS * 2));
    const int64_t kcol = (H + h) * HS, vcol = (2 * H + h) * HS;
    float* scw = scr + w * 16 * SCR;

    // queries of this wave: group 0 = iw .. iw+15, group 1 = iw+16 .. iw+31
    const int64_t iw = i0 + 32 * w;
    const int iwi = (int)iw, Si = (int)S, nm = (int)min<int64_t>(a.n_meta, S);
    // metadata-block relative terms BD(i, j >= i+2) = q_{i+1} . R[j-i-2]
    // (model_transformer.py:84-90 upper triangle; only i + 2 < n_meta)
    float* mbd = scr + 4 * 16 * SCR;
    if (i0 == 0 && w == 0) {
        for (int i = 0; i + 2 < nm; ++i)
            for (int j = i + 2; j < nm; ++j) {
                const bf16* q1 = qkv_b + (int64_t)(i + 1) * ldq + h * HS;
                const bf16* rrow = (const bf16*)a.R + (h * a.S_max + (j - i - 2)) * HS;
                float v = (float)q1[2 * lane] * (float)rrow[2 * lane] + (float)q1[2 * lane + 1] * (float)rrow[2 * lane + 1];
                v = wave_sum(v);
                if (lane == 0) mbd[i * 8 + j] = v;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    bf16x8 qf[2][4];
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
        const int64_t iq = iw + 16 * q2 + il;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            qf[q2][ks] = iq < S ? *(const bf16x8*)(qkv_b + iq * ldq + h * HS + ks * 32 + g * 8) : (bf16x8){};
    }
    f32x4 oacc[2][8];
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2)
#pragma unroll
        for (int n = 0; n < 8; ++n) oacc[q2][n] = zero4();
    // running max in the scaled log2 domain; finite from the first tile on
    // (key 0 is visible to every query)
    float m_run[2] = {-INFINITY, -INFINITY}, l_part[2] = {0.f, 0.f};
    const float c2 = a.scale * LOG2E;

    const int64_t last_q = min<int64_t>(i0 + QB - 1, S - 1);
    const int nkt = (int)(last_q / KB) + 1;
    // R window of tile t (block): rows rb0 + 64 t + [0, 191), ring slot 64 t mod 256
    const int64_t rb0 = S - QB - i0;

    // per-lane DMA constants: row 4w + lane/16 of each 16-row group, chunk
    // slot lane%16 holding source chunk slot ^ swizzle(row)
    const int lrow = 4 * w + (lane >> 4);
    const int chK = (lane & 15) ^ (lrow & 15), chV = (lane & 15) ^ ((lrow & 7) << 1);
    const uint32_t ldq2 = (uint32_t)(ldq * 2);
    const uint32_t offK = (uint32_t)((lrow * ldq + kcol + chK * 8) * 2);
    const uint32_t offV = (uint32_t)((lrow * ldq + vcol + chV * 8) * 2);
    const uint32_t offR = (uint32_t)((lrow * HS + chK * 8) * 2);
    const int Si32 = (int)S, rb0i = (int)rb0;
    // per-lane fragment offsets in a row image (rows rb + lane%16, k-step ks)
    int fro[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fro[ks] = (lane & 15) * 256 + (((ks * 4 + g) ^ (lane & 15)) << 4);
    // transposed V^T fragments from the quads image: rows {4g+q, 16+4g+q}
    int vqo[8];
    {
        const int q = (lane & 15) >> 2, p = lane & 3, r1 = 4 * g + q;
#pragma unroll
        for (int n = 0; n < 8; ++n) vqo[n] = off_quads(r1, 2 * n + (p >> 1)) + (p & 1) * 8;
    }

    // prologue: tile 0 (K, V, 3 R chunks)
    dma64(rq, sK, offK, lrow, 0, 16 * ldq2, 0, Si32, w);
    dma64(rq, sV, offV, lrow, 0, 16 * ldq2, 0, Si32, w);
#pragma unroll
    for (int c = 0; c < 3; ++c)
        dma64(rr, sR + c * KB * 256, offR, lrow, (uint32_t)((rb0i + c * KB) * HS * 2), 16 * HS * 2,
              -(rb0i + c * KB), Si32 - (rb0i + c * KB), w);

    for (int kt = 0; kt < nkt; ++kt) {
        const int64_t j0 = (int64_t)kt * KB;
        const int cur = kt & 1;
        if (kt + 1 < nkt && !(LAB & 16)) {  // prefetch tile kt+1 (its buffers were released by the barrier ending tile kt-1)
            const int64_t j1 = j0 + KB;
            const int j1i = (int)j1, rc = rb0i + (kt + 3) * KB;
            dma64(rq, sK + (cur ^ 1) * KB * 256, offK, lrow, (uint32_t)j1i * ldq2, 16 * ldq2, 0, Si32 - j1i, w);
            dma64(rq, sV + (cur ^ 1) * KB * 256, offV, lrow, (uint32_t)j1i * ldq2, 16 * ldq2, 0, Si32 - j1i, w);
            dma64(rr, sR + (((kt + 3) * KB) & (RING - 1)) * 256, offR, lrow, (uint32_t)(rc * HS * 2), 16 * HS * 2,
                  -rc, Si32 - rc, w);
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        const char* cK = sK + cur * KB * 256;
        const char* cV = sV + cur * KB * 256;
        // (a group whose 16 queries all precede the tile still runs its
        // MFMAs: branching per MFMA costs more than the few masked tiles)
        // S^T[key][query] = K . Q^T
        f32x4 sacc[2][4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            sacc[0][nt] = sacc[1][nt] = zero4();
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const bf16x8 kfr = *(const bf16x8*)(cK + nt * 4096 + fro[ks]);
                if (LAB & 1) {
                    asm volatile("" ::"v"(kfr));
                } else {
                    sacc[0][nt] = mfma(kfr, qf[0][ks], sacc[0][nt]);
                    sacc[1][nt] = mfma(kfr, qf[1][ks], sacc[1][nt]);
                }
            }
        }
        // QR^T[window row][query]: union window of the wave starts at block
        // window row 96 - 32 w; group 1 uses union blocks 0..4, group 0 1..5
        f32x4 qacc[2][5];
#pragma unroll
        for (int t = 0; t < 5; ++t) qacc[0][t] = qacc[1][t] = zero4();
        const int ring0 = (kt * KB + 96 - 32 * w) & (RING - 1);
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            const int rowb = (ring0 + 16 * t) & (RING - 1);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const bf16x8 rfr = *(const bf16x8*)(sR + rowb * 256 + fro[ks]);
                if (LAB & 2) {
                    asm volatile("" ::"v"(rfr));
                } else {
                    if (t >= 1) qacc[0][t - 1] = mfma(rfr, qf[0][ks], qacc[0][t - 1]);
                    if (t <= 4) qacc[1][t] = mfma(rfr, qf[1][ks], qacc[1][t]);
                }
            }
        }

        // skew + online softmax per group (scores kept unscaled until the exp:
        // max commutes with the positive scale, p = exp2(raw * c2 - m))
        bf16x8 pf[2][2];
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
            if (LAB & 4) {
                float x = 0.f;
#pragma unroll
                for (int t = 0; t < 4; ++t) x += sacc[q2][t][0] + qacc[q2][t][1];
                pf[q2][0] = pf[q2][1] = (bf16x8){(bf16)x, (bf16)x, (bf16)x, (bf16)x, (bf16)x, (bf16)x, (bf16)x, (bf16)x};
                l_part[q2] += 1.f;
                m_run[q2] = 0.f;
                continue;
            }
            const int iq = iwi + 16 * q2 + il;
            const int jt = (int)j0;
#pragma unroll
            for (int t = 0; t < 5; ++t) *(f32x4*)(scw + il * SCR + t * 16 + 4 * g) = qacc[q2][t];
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            float sv[4][4];
            float mx = -INFINITY;
            // masking needed only where a key may follow a query of the group
            // or pass the sequence end (wave-uniform)
            const bool masked = (jt + KB - 1 > iwi + 16 * q2) || (jt + KB > Si);
            if (!masked) {
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int jl = nt * 16 + 4 * g + r;
                        const float x = sacc[q2][nt][r] + scw[il * SCR + jl - il + 15];
                        sv[nt][r] = x;
                        mx = fmaxf(mx, x);
                    }
            } else {
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int jl = nt * 16 + 4 * g + r;
                        const int j = jt + jl;
                        float x = sacc[q2][nt][r] + scw[il * SCR + jl - il + 15];
                        const bool ok = (j < Si) && (j <= iq || j < nm);
                        // metadata block j >= i+2: BD = q_{i+1} . R[j-i-2] (table below)
                        if (j >= iq + 2 && j < nm) x += mbd[iq * 8 + j];
                        x = ok ? x : -INFINITY;
                        sv[nt][r] = x;
                        mx = fmaxf(mx, x);
                    }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();  // scratch reads done before the next group's writes
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float m_new = fmaxf(m_run[q2], mx * c2);
            // rescale O only when some query's running max moved (T13)
            if (__any(m_new > m_run[q2])) {
                const float alpha = __builtin_amdgcn_exp2f(m_run[q2] - m_new);
                l_part[q2] *= alpha;
#pragma unroll
                for (int n = 0; n < 8; ++n) oacc[q2][n] *= alpha;
            }
            m_run[q2] = m_new;
            float ps = 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float p = __builtin_amdgcn_exp2f(fmaf(sv[nt][r], c2, -m_new));
                    ps += p;
                    pf[q2][nt >> 1][(nt & 1) * 4 + r] = (bf16)p;
                }
            }
            l_part[q2] += ps;
        }
        // O^T[d][query] += V^T[d][key] . P^T[key][query]
#pragma unroll
        for (int n = 0; n < 8; ++n) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const bf16x8 vfr = cat8(tr_read(cV, ks * 8192 + vqo[n]), tr_read(cV, ks * 8192 + 4096 + vqo[n]));
                if (LAB & 8) {
                    asm volatile("" ::"v"(vfr), "v"(pf[0][ks]), "v"(pf[1][ks]));
                } else {
                    oacc[0][n] = mfma(vfr, pf[0][ks], oacc[0][n]);
                    oacc[1][n] = mfma(vfr, pf[1][ks], oacc[1][n]);
                }
            }
        }
        bar();  // tile kt's K / V / oldest R chunk may now be overwritten
    }

#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
        const int64_t iq = iw + 16 * q2 + il;
        float l = l_part[q2] + __shfl_xor(l_part[q2], 16, 64);
        l += __shfl_xor(l, 32, 64);
        if (iq < S) {
            const float inv = 1.f / l;
            bf16* op = out + (b * S + iq) * ldo + h * HS;
#pragma unroll
            for (int n = 0; n < 8; ++n) store4(op + n * 16 + 4 * g, oacc[q2][n] * inv);
            if (g == 0) lse[(b * H + h) * S + iq] = (m_run[q2] + log2f(l)) / LOG2E;
        }
    }
}

}  // namespace

int flash_fwd2(const AttnArgs& a, bf16* out, int64_t ldo, float* lse, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_fwd2_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_BYTES);
        attr = true;
    }
    if (a.S * a.ldq * 2 >= (int64_t)OOB || a.S * HS * 2 >= (int64_t)OOB || a.n_meta > 8) return -1;
    const dim3 grid((unsigned)((a.S + QB - 1) / QB), (unsigned)a.H, (unsigned)a.B);
    hipLaunchKernelGGL(flash_fwd2_kernel<0>, grid, dim3(NT), LDS_BYTES, s, a, out, ldo, lse);
    return 0;
}
