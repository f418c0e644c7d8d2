// Relative-position flash attention forward, v3 (bf16 MFMA, hs = 128).
// HeadRelPos (model_transformer.py:54-82, _rel_shift :84-90):
//   out_i = sum_j softmax_j(mask((q_i.k_j + q_i.R[S-1-i+j]) * C^-1/2)) v_j
//
// Two waves per SIMD: one workgroup = 8 waves = 256 queries of one (b, h),
// 32 queries per wave as two groups of 16 on the lanes (the "swapped"
// S^T = K.Q^T layout: a lane owns one query row, so row statistics and the
// O^T accumulator never leave the lane). Key tiles of 32. Per tile a wave
// issues 56 MFMAs: 16 K.Q^T, 24 for the relative term against a 64-row
// window of R (the groups' 48-row windows overlap and share fragments), 16
// for V^T.P^T.
// Query blocks are aligned to the END of the sequence (block 0 = the last
// 256 queries, the heaviest), so the ragged block is the first one and holds
// the metadata rows (S = 2048 + 6: a 6-query block with one key tile).
// LDS (139 KB): K and V double-buffered (8 KB tiles), R as a 320-row ring
// (the window of tile t+1 is the window of tile t shifted by 32 rows: one
// 32-row chunk per tile), a per-wave skew scratch and the metadata table.
// All HBM -> LDS traffic is LDS-DMA one tile ahead, zero-filled out of range.
#include "attn_tiles.h"

namespace {
using namespace attn;

constexpr int NT = 512;
constexpr int QB = 256, KB = 32, NCH = 10, RING = NCH * KB, SCR = 52;
constexpr int O_K = 0, O_V = 2 * KB * 256, O_R = 4 * KB * 256, O_S = O_R + RING * 256;
constexpr int O_M = O_S + 8 * 16 * SCR * 4;
constexpr int O_D = O_M + 64 * 4;  // dropout keep words of the block's 256 queries, 2 tiles
constexpr int LDS_BYTES = O_D + 2 * QB * 4;
constexpr uint32_t OOB = 0xFFFF0000u;
// lazy-rescale threshold of the running row maximum, log2 units (P <= 2^RESCALE)
constexpr float RESCALE = 8.f;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// one DMA per thread: 32 rows x 256 B; this lane's row / chunk are fixed,
// rows outside [lo, hi) (relative to the chunk) come back zero
__device__ __forceinline__ void dma32(__amdgpu_buffer_rsrc_t rs, char* dst, uint32_t lane_off, int lane_row,
                                      uint32_t base, int lo, int hi, int w) {
    const uint32_t vo = (lane_row >= lo && lane_row < hi) ? lane_off + base : OOB;
    // the builtin, not lds_dma16: here the compiler's wait before the V reads
    // (for the next tile's DMA) measured 8-10 % faster than the asm form
    // (same box, 1 007-1 038 vs 905-933 us per launch at cfg 2)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_char*)(dst + w * 1024), 16, vo, 0, 0, 0);
}

// max over the four lanes l, l^16, l^32, l^48 (one query's 4 key groups):
// v_permlane16/32_swap instead of ds_bpermute round trips
__device__ __forceinline__ float max_rows(float x) {
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// DROP: attention-probability dropout (model_transformer.py:80): the keep word
// of (query, key tile) is staged by LDS-DMA with the tile; P.V uses p * keep,
// the softmax normaliser the undropped p, the output is scaled by 1/(1-p)
template <bool DROP>
__global__ __launch_bounds__(NT, 1) void flash_fwd3_kernel(AttnArgs a, bf16* __restrict__ out, int64_t ldo,
                                                           float* __restrict__ lse) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sR = smem + O_R;
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, il = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int S = (int)a.S, H = (int)a.H;
    const int64_t ldq = a.ldq;
    const Blk3 blk = xcd_blk3_heavy_first(a.xcd);
    const int qb = blk.x;  // 0 = last (heaviest) 256 queries
    const int h = blk.y, b = blk.z;
    const int qhi = S - QB * qb, i0 = qhi - QB;  // queries [max(i0, 0), qhi)
    const bf16* qkv_b = (const bf16*)a.qkv + (int64_t)b * S * ldq;
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(qkv_b, (uint32_t)((int64_t)S * ldq * 2));
    const __amdgpu_buffer_rsrc_t rr = make_rsrc((const bf16*)a.R + (int64_t)h * a.S_max * HS, (uint32_t)(S * HS * 2));
    float* scw = (float*)(smem + O_S) + w * 16 * SCR;
    float* mbd = (float*)(smem + O_M);
    const int nm = (int)min<int64_t>(a.n_meta, S);

    const int iw = i0 + 32 * w;  // wave queries iw .. iw+31 (group q2: iw+16 q2 ..)
    const bool live = iw + 31 >= 0;
    // metadata-block relative terms BD(i, j >= i+2) = q_{i+1} . R[j-i-2]
    // (upper triangle of the skew inside the metadata prefix, only i+2 < n_meta)
    if (iw <= 0 && iw + 32 > 0) {
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
    bf16x8 qf[2][4];
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
        const int iq = iw + 16 * q2 + il;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            qf[q2][ks] = (iq >= 0 && iq < S) ? *(const bf16x8*)(qkv_b + (int64_t)iq * ldq + h * HS + ks * 32 + g * 8)
                                            : (bf16x8){};
    }
    f32x4 oacc[2][8];
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2)
#pragma unroll
        for (int n = 0; n < 8; ++n) oacc[q2][n] = zero4();
    // running max in the scaled log2 domain; finite after the first tile (key 0
    // is visible to every query)
    float m_run[2] = {-INFINITY, -INFINITY}, l_part[2] = {0.f, 0.f};
    const float c2 = a.scale * LOG2E;

    const int nkt = (qhi - 1) / KB + 1;
    // keep words rowmask[b,h,i][kt]: waves 0-3 stage the block's 256 queries
    const int64_t mld = a.mask_ld;
    const __amdgpu_buffer_rsrc_t rm =
        make_rsrc(DROP ? (const void*)(a.rowmask + (int64_t)(b * H + h) * (mask_bh_bytes(mld) / 4)) : (const void*)a.R,
                  DROP ? (uint32_t)mask_bh_bytes(mld) : 0u);
    auto stage_m = [&](int kt, int buf) {
        if (DROP && w < 4) {
            const int iq = i0 + 64 * w + lane;
            const uint32_t vo = (iq >= 0 && iq < S) ? (uint32_t)(mask_word(mld, iq, 32 * kt) * 4) : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lds_char*)(smem + O_D + buf * QB * 4 + w * 256), 4, vo, 0,
                                                     0, 0);
        }
    };
    const int rb0 = S - qhi;  // R row of block-window row 0 at tile 0; chunk c = rows rb0 + 32 c ..

    // per-lane DMA constants: row tid/16 of a 32-row tile, chunk slot lane%16
    const int lrow = 4 * w + (lane >> 4);
    const int chK = (lane & 15) ^ (lrow & 15), chV = (lane & 15) ^ ((lrow & 7) << 1);
    const uint32_t ldq2 = (uint32_t)(ldq * 2);
    const uint32_t offK = (uint32_t)((lrow * ldq + (int64_t)(H + h) * HS + chK * 8) * 2);
    const uint32_t offV = (uint32_t)((lrow * ldq + (int64_t)(2 * H + h) * HS + chV * 8) * 2);
    const uint32_t offR = (uint32_t)((lrow * HS + chK * 8) * 2);
    int fro[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fro[ks] = (lane & 15) * 256 + (((ks * 4 + g) ^ (lane & 15)) << 4);
    int vqo[8];
    {
        const int q = (lane & 15) >> 2, p = lane & 3, r1 = 4 * g + q;
#pragma unroll
        for (int n = 0; n < 8; ++n) vqo[n] = off_quads(r1, 2 * n + (p >> 1)) + (p & 1) * 8;
    }

    // prologue: tile 0 and the 9 R chunks of its window
    stage_m(0, 0);
    dma32(rq, smem + O_K, offK, lrow, 0, 0, S, w);
    dma32(rq, smem + O_V, offV, lrow, 0, 0, S, w);
#pragma unroll
    for (int c = 0; c < NCH - 1; ++c) {
        const int r0 = rb0 + c * KB;
        dma32(rr, sR + c * KB * 256, offR, lrow, (uint32_t)(r0 * HS * 2), -r0, S - r0, w);
    }

    // one barrier per tile: it publishes tile kt (DMA'd in the prologue, or
    // one tile ahead) and releases tile kt-1's buffers
    auto sync = [&](int kt) {
        const int cur = kt & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
        if (kt + 1 < nkt) {
            const int j1 = (kt + 1) * KB, c = kt + NCH - 1, r0 = rb0 + c * KB;
            dma32(rq, smem + O_K + (cur ^ 1) * KB * 256, offK, lrow, (uint32_t)j1 * ldq2, 0, S - j1, w);
            dma32(rq, smem + O_V + (cur ^ 1) * KB * 256, offV, lrow, (uint32_t)j1 * ldq2, 0, S - j1, w);
            dma32(rr, sR + (c % NCH) * KB * 256, offR, lrow, (uint32_t)(r0 * HS * 2), -r0, S - r0, w);
            stage_m(kt + 1, cur ^ 1);
        }
    };
    // tiles past the wave's last query are masked for all its queries (the
    // metadata keys are in tile 0): the wave only meets their barriers and
    // issues their DMA (a second loop, so the accumulators' registers stay
    // put through the first)
    const int nkw = live ? min(nkt, (iw + 31) / KB + 1) : 0;
    int kt = 0;
    for (; kt < nkw; ++kt) {
        const int j0 = kt * KB, cur = kt & 1;
        sync(kt);
        {
            const char* cK = smem + O_K + cur * KB * 256;
            const char* cV = smem + O_V + cur * KB * 256;
            // S^T[key][query] = K . Q^T
            f32x4 sacc[2][2];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                sacc[0][nt] = sacc[1][nt] = zero4();
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const bf16x8 kfr = *(const bf16x8*)(cK + nt * 4096 + fro[ks]);
                    sacc[0][nt] = mfma(kfr, qf[0][ks], sacc[0][nt]);
                    sacc[1][nt] = mfma(kfr, qf[1][ks], sacc[1][nt]);
                }
            }
            // QR^T[window row][query]: the wave's 64-row union window starts at
            // block-window row 224 - 32 w; group 1 uses blocks 0..2, group 0 1..3
            f32x4 qacc[2][3];
#pragma unroll
            for (int t = 0; t < 3; ++t) qacc[0][t] = qacc[1][t] = zero4();
            // window rows (from rb0) j0 + 224 - 32 w .. +63: ring chunks ca, cb
            // (16-row blocks t = 0, 1 in ca, t = 2, 3 in cb: one lane address
            // per chunk and k-step, the block an immediate offset)
            const int ca = (kt + 7 - w) % NCH, cb = ca + 1 == NCH ? 0 : ca + 1;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const char* rch = sR + (t < 2 ? ca : cb) * KB * 256 + (t & 1) * 16 * 256;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const bf16x8 rfr = *(const bf16x8*)(rch + fro[ks]);
                    if (t >= 1) qacc[0][t - 1] = mfma(rfr, qf[0][ks], qacc[0][t - 1]);
                    if (t <= 2) qacc[1][t] = mfma(rfr, qf[1][ks], qacc[1][t]);
                }
            }

            // skew + online softmax per group (scores unscaled until the exp:
            // max commutes with the positive scale, p = exp2(raw * c2 - m))
            bf16x8 pf[2];
            // skewed QR values of both groups: group 0's window written and read
            // back, then group 1's into the same scratch rows, all issued before
            // either is used (a wave's LDS operations execute in issue order, so
            // each read sees its group's writes and group 1's writes follow group
            // 0's reads without an lgkmcnt(0) between: one LDS round trip per
            // tile instead of one per group)
            float xs[2][2][4];
#pragma unroll
            for (int q2 = 0; q2 < 2; ++q2) {
#pragma unroll
                for (int t = 0; t < 3; ++t) *(f32x4*)(scw + il * SCR + t * 16 + 4 * g) = qacc[q2][t];
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) xs[q2][nt][r] = scw[il * SCR + nt * 16 + 4 * g + r - il + 15];
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int q2 = 0; q2 < 2; ++q2) {
                const int iq = iw + 16 * q2 + il;
                float sv[2][4];
                float mx = -INFINITY;
                // masking only where a key may follow a query of the group or
                // pass the sequence end (wave-uniform)
                const bool masked = (j0 + KB - 1 > iw + 16 * q2) || (j0 + KB > S);
                if (!masked) {
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int jl = nt * 16 + 4 * g + r;
                            const float x = sacc[q2][nt][r] + xs[q2][nt][r];
                            sv[nt][r] = x;
                            mx = fmaxf(mx, x);
                        }
                } else if (j0 >= nm) {  // the diagonal or the sequence end only
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int jl = nt * 16 + 4 * g + r;
                            const int j = j0 + jl;
                            const float x = sacc[q2][nt][r] + xs[q2][nt][r];
                            // (& not &&: no branch per element)
                            sv[nt][r] = ((j < S) & (j <= iq)) ? x : -INFINITY;
                            mx = fmaxf(mx, sv[nt][r]);
                        }
                } else {  // tile 0: the metadata keys every query sees
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int jl = nt * 16 + 4 * g + r;
                            const int j = j0 + jl;
                            float x = sacc[q2][nt][r] + xs[q2][nt][r];
                            const bool ok = (j < S) & ((j <= iq) | (j < nm));
                            const bool md = (j >= iq + 2) & (j < nm) & (iq >= 0);
                            const float b = mbd[md ? iq * 8 + j : 0];  // (read unconditionally)
                            x = md ? x + b : x;
                            x = ok ? x : -INFINITY;
                            sv[nt][r] = x;
                            mx = fmaxf(mx, x);
                        }
                }
                __builtin_amdgcn_wave_barrier();  // (code motion only)
                // lazy rescale (T13): the running max moves only when some row's
                // new maximum passes it by more than RESCALE (log2 units), so
                // p = exp2(raw c2 - m) <= 2^RESCALE; l and O always see the same m.
                // A row passes iff one of its four lanes does, so the test runs on
                // the lane maxima and the row maxima are formed only when it fires
                float m_new = m_run[q2];
                if (__any(mx * c2 > m_run[q2] + RESCALE)) {
                    mx = max_rows(mx);
                    m_new = fmaxf(m_run[q2], mx * c2);
                    const float alpha = __builtin_amdgcn_exp2f(m_run[q2] - m_new);
                    l_part[q2] *= alpha;
#pragma unroll
                    for (int n = 0; n < 8; ++n) oacc[q2][n] *= alpha;
                }
                m_run[q2] = m_new;
                float ps = 0.f;
                uint32_t kw = 0;
                if (DROP) kw = ((const uint32_t*)(smem + O_D + cur * QB * 4))[32 * w + 16 * q2 + il] >> (4 * g);
                // p packed two keys per register; a dropped key's half is
                // cleared by a mask of its sign-extended keep bit (v_bfe_i32,
                // v_bfi_b32: 2.5 VALU per key instead of 4.5)
                union { bf16x8 v; bf16x2 h[4]; uint32_t u[4]; } pk;
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const float p0 = __builtin_amdgcn_exp2f(fmaf(sv[nt][r], c2, -m_new));
                        const float p1 = __builtin_amdgcn_exp2f(fmaf(sv[nt][r + 1], c2, -m_new));
                        ps += p0;
                        ps += p1;
                        pk.h[nt * 2 + r / 2] = (bf16x2){(bf16)p0, (bf16)p1};
                        if (DROP) {
                            const int k = nt * 16 + r;
                            const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)kw, k, 1);
                            const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)kw, k + 1, 1);
                            pk.u[nt * 2 + r / 2] &= (m0 & 0xFFFFu) | (m1 & 0xFFFF0000u);
                        }
                    }
                pf[q2] = pk.v;
                l_part[q2] += ps;
            }
            // O^T[d][query] += V^T[d][key] . P^T[key][query]
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const bf16x8 vfr = cat8(tr_read(cV, vqo[n]), tr_read(cV, 4096 + vqo[n]));
                oacc[0][n] = mfma(vfr, pf[0], oacc[0][n]);
                oacc[1][n] = mfma(vfr, pf[1], oacc[1][n]);
            }
        }
    }
    for (; kt < nkt; ++kt) sync(kt);

    if (!live) return;
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
        const int iq = iw + 16 * q2 + il;
        float l = l_part[q2] + __shfl_xor(l_part[q2], 16, 64);
        l += __shfl_xor(l, 32, 64);
        if (iq >= 0 && iq < S) {
            const float inv = (DROP ? a.keep_scale : 1.f) / l;
            bf16* op = out + ((int64_t)b * S + iq) * ldo + h * HS;
#pragma unroll
            for (int n = 0; n < 8; ++n) store4(op + n * 16 + 4 * g, oacc[q2][n] * inv);
            if (g == 0) lse[((int64_t)b * H + h) * S + iq] = (m_run[q2] + log2f(l)) / LOG2E;
        }
    }
}

}  // namespace

int flash_fwd3(const AttnArgs& a, bf16* out, int64_t ldo, float* lse, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)flash_fwd3_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)flash_fwd3_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        attr = true;
    }
    if (a.rowmask && mask_bh_bytes(a.mask_ld) >= (int64_t)OOB) return -1;
    if (a.S * a.ldq * 2 >= (int64_t)OOB || a.S * HS * 2 >= (int64_t)OOB || a.n_meta > 8) return -1;
    const dim3 grid((unsigned)((a.S + QB - 1) / QB), (unsigned)a.H, (unsigned)a.B);
    if (a.rowmask)
        hipLaunchKernelGGL((flash_fwd3_kernel<true>), grid, dim3(NT), LDS_BYTES, s, a, out, ldo, lse);
    else hipLaunchKernelGGL((flash_fwd3_kernel<false>), grid, dim3(NT), LDS_BYTES, s, a, out, ldo, lse);
    return 0;
}
