// Persistent 256x256 GEMM tile for the forward / dX products (see the comment
// block below and gemm256.hip for the tile itself).
#include "gemm256_tile.h"

namespace {

using namespace g256;

// ---------------------------------------------------------------------------
// Persistent form of the same tile for the forward / dX products (K ~ 1024 to
// 18 k, one workgroup per CU walking the tiles round-robin).
//
// At K = 1024 a tile is 16 K-steps, and the non-persistent kernel pays a fixed
// prologue (every CU loading its first 96 KB at once) and epilogue (every CU
// storing its 128 KB C tile at once) around each one. Here the next tile's
// prologue LDS-DMA is issued as soon as the last MFMA phase of the current tile
// has read its fragments, BEFORE the current tile's epilogue, and the epilogue
// stores are not waited for: the next tile's first K-step counts them in its
// vmcnt waits (vm_wait<8 + S>: the S stores were issued after the prologue
// halves it waits for), so the C write burst drains under the next tile's
// MFMAs. For the count to be exact every lane issues exactly S stores per tile
// (buffer stores; rows / columns past M / N get an offset beyond the
// descriptor's num_records and are dropped), and before the first tile S
// dropped stores stand in for the previous epilogue.
//
// bf16 C: a 16x16 accumulator leaves each lane 4 columns of a row; lanes l and
// l + 16 hold the two halves of 8 consecutive columns of the neighbouring
// 16-column block, so one v_permlane16_swap per dword turns 2 x 8-B pieces into
// one 16-B store (cdna_hip_programming.md T21, in its 16-lane form).
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <typename TC>
constexpr int p_stores() {
    return sizeof(TC) == 2 ? 16 : 32;
}

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    const bf16x2 v = (bf16x2){(bf16)a, (bf16)b};
    return __builtin_bit_cast(uint32_t, v);
}

template <typename TX>
__device__ __forceinline__ f32x4 p_aux_load(__amdgpu_buffer_rsrc_t rx, uint32_t off) {
    if (sizeof(TX) == 4) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    } else {
        const bf16x4 h = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, 0));
        return (f32x4){(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    }
}

// MSQ_MASK1 aux: read as the ReLU mask of the dX product (RELU_MASK), written
// beside C by the FFN1 forward (BIAS_RELU: 16 more stores per lane and tile)
template <int EPI, typename TX>
constexpr bool p_writes_bits() {
    return EPI == MSQ_EPI_BIAS_RELU && std::is_same<TX, mask1_t>::value;
}

// epilogue of one tile: exactly p_stores<TC>() buffer stores per lane
// CS: also the column sums of the written values (fp32, before the rounding
// to TC) over the tile's rows, one partial row per (M-tile, wave-row) into
// g.cs_ws[(m0 / 256) * 2 + wr][n] (the layout gemm256_kernel's CS variant
// writes; colsum_partials_kernel reduces it in a fixed order): 4 more buffer
// stores per lane, rows / lanes that do not write get the dropped offset
template <int EPI, typename TC, typename TX, int CSM = 0>
__device__ __forceinline__ void p_epilogue(const GemmArgs& g, __amdgpu_buffer_rsrc_t rc, __amdgpu_buffer_rsrc_t rx,
                                           __amdgpu_buffer_rsrc_t rbias, __amdgpu_buffer_rsrc_t rcs, int64_t m0,
                                           int64_t n0, int wr, int wc, int lane, f32x4 (&acc)[2][2][4][2]) {
    constexpr bool HAS_BIAS = EPI == MSQ_EPI_BIAS || EPI == MSQ_EPI_BIAS_RELU || EPI == MSQ_EPI_BIAS_RESID ||
                              EPI == MSQ_EPI_BIAS_DROP_RESID;
    constexpr bool CS = CSM == 1, ST = CSM == 2;
    constexpr bool M1 = std::is_same<TX, mask1_t>::value, WB = p_writes_bits<EPI, TX>();
    const int r = lane & 15, gq = lane >> 4;
    f32x4 bv[2][2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            bv[b][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (HAS_BIAS && g.bias) {
                const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * gq;
                bv[b][j] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(rbias, n < g.N ? (uint32_t)(n * 4) : OOB, 0, 0));
            }
        }
    f32x4 csum[2][2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) csum[b][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // ST: the column max over the wave's 128 rows of the values as stored
    // (bias added, rounded to TC), first over the lane's 8 rows, then over the
    // 16 row-lanes; rows past M do not count
    constexpr float L2E = 1.4426950408889634f;
    f32x4 cmax[2][2];
    if (ST) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x4 mx = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int64_t m = m0 + a * 128 + wr * 64 + i * 16 + r;
                        if (m < g.M) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) mx[e] = fmaxf(mx[e], (float)(TC)(acc[a][b][i][j][e] + bv[b][j][e]));
                        }
                    }
#pragma unroll
                for (int o = 1; o < 16; o <<= 1)
#pragma unroll
                    for (int e = 0; e < 4; ++e) mx[e] = fmaxf(mx[e], __shfl_xor(mx[e], o, 64));
                cmax[b][j] = mx;
            }
    }
    // aux rows in groups of 2 of the lane's 8 rows (4 x 16-B loads in flight
    // per row; a whole half-tile's 64 VGPRs of aux would spill beside acc)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int ih = 0; ih < 2; ++ih) {
        f32x4 xp[4][2][2];
        if constexpr (M1 && epi_reads_aux<EPI>()) {
            // one mask word per (row, 32-column span): the lane's 2 x 4 columns of it
#pragma unroll
            for (int i = 2 * ih; i < 2 * ih + 2; ++i)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int64_t m = m0 + a * 128 + wr * 64 + i * 16 + r;
                    const int64_t wd = (n0 + b * 128 + wc * 32) >> 5;
                    const uint32_t off = (m < g.M && wd * 32 < g.N) ? (uint32_t)((m * g.ldx + wd) * 4) : OOB;
                    const uint32_t wv = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rx, off, 0, 0);
#pragma unroll
                    for (int j = 0; j < 2; ++j) xp[i][b][j] = mask1_bits(wv, j * 16 + 4 * gq);
                }
        } else if (epi_reads_aux<EPI>()) {
#pragma unroll
            for (int i = 2 * ih; i < 2 * ih + 2; ++i)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int64_t m = m0 + a * 128 + wr * 64 + i * 16 + r;
                        const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * gq;
                        const uint32_t off =
                            (m < g.M && n < g.N) ? (uint32_t)((m * g.ldx + n) * (int64_t)sizeof(TX)) : OOB;
                        xp[i][b][j] = p_aux_load<TX>(rx, off);
                    }
        }
#pragma unroll
        for (int i = 2 * ih; i < 2 * ih + 2; ++i) {
            const int64_t m = m0 + a * 128 + wr * 64 + i * 16 + r;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                f32x4 v[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * gq;
                    f32x4 t = acc[a][b][i][j];
                    if (HAS_BIAS) t += bv[b][j];
                    if (EPI == MSQ_EPI_BIAS_DROP_RESID) t = epi_drop(g, m, n, t) + xp[i][b][j];
                    if (EPI == MSQ_EPI_BIAS_RELU) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) t[e] = fmaxf(t[e], 0.f);
                    }
                    if (EPI == MSQ_EPI_BIAS_RESID) t += xp[i][b][j];
                    if (EPI == MSQ_EPI_RELU_MASK) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) t[e] = xp[i][b][j][e] > 0.f ? t[e] : 0.f;
                    }
                    v[j] = t;
                    if (CS && m < g.M) csum[b][j] += t;
                    if (ST && m < g.M) {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (cmax[b][j][e] != -INFINITY)
                                csum[b][j][e] += __builtin_amdgcn_exp2f(((float)(TC)t[e] - cmax[b][j][e]) * L2E);
                    }
                }
                if constexpr (WB) {
                    // bit (j 16 + 4 gq + e) of the span's word = (C as stored > 0); the
                    // four gq lanes of a row OR their bits, lane gq = 0 stores the word
                    uint32_t bits = 0u;
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            bits |= ((float)(TC)v[j][e] > 0.f ? 1u : 0u) << (j * 16 + 4 * gq + e);
                    bits |= (uint32_t)__shfl_xor((int)bits, 16, 64);
                    bits |= (uint32_t)__shfl_xor((int)bits, 32, 64);
                    const int64_t wd = (n0 + b * 128 + wc * 32) >> 5;
                    const uint32_t off =
                        (gq == 0 && m < g.M && wd * 32 < g.N) ? (uint32_t)((m * g.ldx + wd) * 4) : OOB;
                    __builtin_amdgcn_raw_buffer_store_b32(bits, rx, off, 0, 0);
                }
                if (sizeof(TC) == 2) {
                    uint32_t p0x = pack_bf16(v[0][0], v[0][1]), p0y = pack_bf16(v[0][2], v[0][3]);
                    uint32_t p1x = pack_bf16(v[1][0], v[1][1]), p1y = pack_bf16(v[1][2], v[1][3]);
                    // rows (lane >> 4) 1, 3 of the block-0 pieces <-> rows 0, 2 of the block-1 pieces
                    const auto sx = __builtin_amdgcn_permlane16_swap(p0x, p1x, false, false);
                    const auto sy = __builtin_amdgcn_permlane16_swap(p0y, p1y, false, false);
                    const int64_t n = n0 + b * 128 + wc * 32 + (gq & 1) * 16 + (gq >> 1) * 8;
                    const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)((m * g.ldc + n) * 2) : OOB;
                    const u32x4 d = (u32x4){(uint32_t)sx[0], (uint32_t)sy[0], (uint32_t)sx[1], (uint32_t)sy[1]};
                    __builtin_amdgcn_raw_buffer_store_b128(d, rc, off, 0, 0);
                } else {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * gq;
                        const uint32_t off = (m < g.M && n < g.N) ? (uint32_t)((m * g.ldc + n) * 4) : OOB;
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[j]), rc, off, 0, 0);
                    }
                }
            }
        }
    }
    if (ST) {
        // partial (max, sum exp) rows per (M-tile, wave-row) p = (m0 / 256) * 2 + wr:
        // cs_ws[(2 p) * ldx + n] = max, cs_ws[(2 p + 1) * ldx + n] = sum (ldx: the row stride)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x4 v = csum[b][j];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1)
#pragma unroll
                    for (int t = 0; t < 4; ++t) v[t] += __shfl_xor(v[t], o, 64);
                const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * gq;
                const int64_t p = (m0 >> 8) * 2 + wr;
                const bool ok = r == 0 && n < g.N;
                const uint32_t om = ok ? (uint32_t)(((2 * p) * g.ldx + n) * 4) : OOB;
                const uint32_t os = ok ? (uint32_t)(((2 * p + 1) * g.ldx + n) * 4) : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, cmax[b][j]), rcs, om, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rcs, os, 0, 0);
            }
    }
    if (CS) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x4 v = csum[b][j];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1)
#pragma unroll
                    for (int t = 0; t < 4; ++t) v[t] += __shfl_xor(v[t], o, 64);
                const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * gq;
                const uint32_t off = (r == 0 && n < g.N) ? (uint32_t)((((m0 >> 8) * 2 + wr) * g.N + n) * 4) : OOB;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rcs, off, 0, 0);
            }
    }
}

// tile id -> (m0, n0): 8 row panels share each sweep over the columns
__device__ __forceinline__ void p_tile_mn(const GemmArgs& g, int id, int64_t& m0, int64_t& n0) {
    const int GROUP = 8;
    const int per_group = GROUP * g.tiles_n;
    const int grp = id / per_group, first_m = grp * GROUP;
    const int gsz = min(g.tiles_m - first_m, GROUP);
    m0 = (int64_t)(first_m + (id % per_group) % gsz) * 256;
    n0 = (int64_t)((id % per_group) / gsz) * 256;
}

// Wave quantisation: M = B*S rows leave ntiles % G tiles (at cfg 2 the
// 192-row last row panel: 4 tiles at N = 1 024) for a last round on a few
// CUs. With a workspace those tail tiles run as K slices, one per idle CU:
// work item id >= n_full is slice (id - n_full) % tail_s of tail tile
// n_full + (id - n_full) / tail_s, stored as an fp32 partial 256 x 256 tile
// at ws + (id - n_full) * 64 K floats; p_tail_fixup_kernel sums each tile's
// slices in order and applies the epilogue. Every workgroup has at most one
// slice and it is its last item (tail_tiles * tail_s <= G).
template <int EPI, typename TC, typename TX>
__global__ __launch_bounds__(256) void p_tail_fixup_kernel(GemmArgs g) {
    const int n_full = g.tiles_m * g.tiles_n - g.tail_tiles;
    constexpr int64_t QPT = 256 * 64;  // 4-column quads per tile
    const int64_t total = (int64_t)g.tail_tiles * QPT;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int tt = (int)(e / QPT), q = (int)(e % QPT), r = q >> 6, c = (q & 63) * 4;
        int64_t m0, n0;
        p_tile_mn(g, n_full + tt, m0, n0);
        const int64_t m = m0 + r, n = n0 + c;
        if (m >= g.M || n >= g.N) continue;
        const float* P = g.ws + (int64_t)tt * g.tail_s * 65536 + r * 256 + c;
        f32x4 v = load4(P);
        for (int sl = 1; sl < g.tail_s; ++sl) v += load4(P + (int64_t)sl * 65536);
        epi_apply<EPI, TC, TX>(g, (TC*)g.C, (const TX*)g.aux, m, n, v);
    }
}

template <int TA, int TB, int EPI, typename TC, typename TX, int CSM = 0>
__global__ __launch_bounds__(NT, 1) void gemm256p_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    lds_t* smem = (lds_t*)smem_raw;
    constexpr int S = p_stores<TC>() + (CSM == 1 ? 4 : CSM == 2 ? 8 : 0) + (p_writes_bits<EPI, TX>() ? 16 : 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    const int ntiles = g.tiles_m * g.tiles_n;
    const int G = gridDim.x;
    // item id of round q for this workgroup: q * G + widx; blocks sharing an
    // XCD take consecutive ids (T1), which the grouped order turns into
    // shared A / B panels in that XCD's L2. Items past n_full are the K
    // slices of the tail tiles (p_tail_fixup_kernel)
    const int widx = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, G));
    const int n_full = ntiles - g.tail_tiles;
    const int n_items = n_full + g.tail_tiles * g.tail_s;

    const __amdgpu_buffer_rsrc_t ra = make_rsrc((const char*)g.A, g.a_ext);
    const __amdgpu_buffer_rsrc_t rb = make_rsrc((const char*)g.B, g.b_ext);
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const char*)g.C, g.c_ext);
    const __amdgpu_buffer_rsrc_t rbias =
        make_rsrc((const char*)(g.bias ? (const void*)g.bias : g.C), g.bias ? (uint32_t)(g.N * 4) : 0u);
    // CSM 1: colsum partials [tiles_m * 2][N]; 2: (max, sum) partials [tiles_m * 2][2][ldx]
    const uint32_t cs_bytes =
        CSM == 1 ? (uint32_t)(g.tiles_m * 2 * g.N * 4) : CSM == 2 ? (uint32_t)(g.tiles_m * 4 * g.ldx * 4) : 0u;
    const __amdgpu_buffer_rsrc_t rx =
        make_rsrc((const char*)(g.aux && CSM != 2 ? g.aux : g.C), g.aux && CSM != 2 ? g.x_ext : 0u);
    const __amdgpu_buffer_rsrc_t rcs = make_rsrc((const char*)(CSM ? (const void*)g.cs_ws : g.C), cs_bytes);

    int loA[4], loB[4];
    {
        const int r = lane & 15, gq = lane >> 4;
        if (TA == 0) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) loA[ks] = r * 128 + ((ks * 4 + gq) ^ ((r >> 1) & 7)) * 16;
            loA[2] = loA[3] = 0;
        } else {
            const int q = r >> 2, p = r & 3, k = 8 * gq + q;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                loA[i] = k * 256 + ((((wr * 64 + i * 16) >> 3) ^ gmn(k)) | (p >> 1)) * 16 + (p & 1) * 8;
        }
        if (TB == 0) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) loB[ks] = r * 128 + ((ks * 4 + gq) ^ ((r >> 1) & 7)) * 16;
            loB[2] = loB[3] = 0;
        } else {
            const int q = r >> 2, p = r & 3, k = 8 * gq + q;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                loB[i] = k * 256 + ((((wc * 32 + i * 16) >> 3) ^ gmn(k)) | (p >> 1)) * 16 + (p & 1) * 8;
            loB[2] = loB[3] = 0;
        }
    }

    const int nkt = (int)((g.K + 63) / 64);
    // item -> tile origin, first k-step, k-steps
    auto item = [&](int id, int64_t& m0, int64_t& n0, int& kb, int& nkk) {
        if (id < n_full) {
            p_tile_mn(g, id, m0, n0);
            kb = 0;
            nkk = nkt;
        } else {
            const int u = id - n_full;
            p_tile_mn(g, n_full + u / g.tail_s, m0, n0);
            kb = (u % g.tail_s) * g.tail_kst;
            nkk = min(g.tail_kst, nkt - kb);
        }
    };
    Stage<TA == 0> sa;
    Stage<TB == 0> sb;
    auto slot = [&](int b, int s) { return smem + (b * 4 + s) * HALF; };
    // k-step u of an item whose k-steps start at kb (slot parity by u)
    auto issue = [&](int kb, int u, int h) {
        const int64_t k0 = (int64_t)(kb + u) * 64;
        lds_t* dst = slot(u & 1, h);
        if (h == 0) sa.issue(ra, dst, 0, k0, g.K - k0, w);
        else if (h == 1) sb.issue(rb, dst, 0, k0, g.K - k0, w);
        else if (h == 2) sa.issue(ra, dst, 1, k0, g.K - k0, w);
        else sb.issue(rb, dst, 1, k0, g.K - k0, w);
    };
    auto prologue = [&](int64_t m0, int64_t n0, int kb, int nkk) {
        sa.init(m0, g.M, g.lda, w, lane);
        sb.init(n0, g.N, g.ldb, w, lane);
        issue(kb, 0, 0);
        issue(kb, 0, 1);
        issue(kb, 0, 2);
        issue(kb, 0, 3);
        if (nkk > 1) {
            issue(kb, 1, 0);
            issue(kb, 1, 1);
        }
    };

    int id = widx;
    if (id >= n_items) return;
    int64_t m0, n0;
    int kb, nk;
    item(id, m0, n0, kb, nk);
    prologue(m0, n0, kb, nk);
    order_fence();
    // the S stores a previous tile's epilogue would have left outstanding (to
    // distinct, non-adjacent dropped offsets: identical ones would be merged
    // into one store by dead-store elimination, adjacent ones widened)
#pragma unroll
    for (int e = 0; e < S; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(0u, rc, OOB + 64u * e, 0, 0);
    order_fence();

    f32x4 acc[2][2][4][2];
    bf16x8 af[2][2][4];
    bf16x8 bfr[2][2][2];

    // one phase (gemm256_kernel's MSQ_PHASE) with the wait count of its K-step
#define MSQ_PPHASE(Q, BUF, WAITN)                                                                       \
    {                                                                                                   \
        constexpr int mi = (Q == 1 || Q == 2) ? 1 : 0;                                                  \
        constexpr int ni = (Q >= 2) ? 1 : 0;                                                            \
        if (Q == 0) {                                                                                   \
            read_set<TA == 0, 4>(af[0], slot(BUF, 0), wr * 64, loA);                                    \
            read_set<TB == 0, 2>(bfr[0], slot(BUF, 1), wc * 32, loB);                                   \
        } else if (Q == 1) {                                                                            \
            read_set<TA == 0, 4>(af[1], slot(BUF, 2), wr * 64, loA);                                    \
        } else if (Q == 2) {                                                                            \
            read_set<TB == 0, 2>(bfr[1], slot(BUF, 3), wc * 32, loB);                                   \
        }                                                                                               \
        const int su = (Q < 2) ? t + 1 : t + 2;                                                         \
        if (su < nk) {                                                                                  \
            issue(kb, su, (Q + 2) & 3);                                                                 \
            vm_wait<WAITN>();                                                                           \
        } else {                                                                                        \
            vm_wait0();                                                                                 \
        }                                                                                               \
        barrier();                                                                                      \
        __builtin_amdgcn_s_setprio(1);                                                                  \
        _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                \
            _Pragma("unroll") for (int i = 0; i < 4; ++i)                                               \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                           \
                    acc[mi][ni][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni][ks][j], af[mi][ks][i], \
                                                                                acc[mi][ni][i][j], 0, 0, 0); \
        __builtin_amdgcn_s_setprio(0);                                                                  \
        barrier();                                                                                      \
    }

    for (;;) {
        // A0 / B0 of K-step 0 landed: younger are 4 half-tiles (8 DMA) and the S stores
        if (nk > 1) vm_wait<8 + S>();
        else vm_wait0();
        barrier();
        if (wr == 1) barrier();
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        {
            int t = 0;  // K-step 0: the stores sit between its prologue halves and its own DMA
            MSQ_PPHASE(0, 0, 8 + S)
            MSQ_PPHASE(1, 0, 8 + S)
            MSQ_PPHASE(2, 0, 8 + S)
            MSQ_PPHASE(3, 0, 8 + S)
        }
        for (int t = 1; t < nk; t += 2) {
            MSQ_PPHASE(0, 1, 8)
            MSQ_PPHASE(1, 1, 8)
            MSQ_PPHASE(2, 1, 8)
            MSQ_PPHASE(3, 1, 8)
            if (t + 1 < nk) {
                ++t;
                MSQ_PPHASE(0, 0, 8)
                MSQ_PPHASE(1, 0, 8)
                MSQ_PPHASE(2, 0, 8)
                MSQ_PPHASE(3, 0, 8)
                --t;
            }
        }
        if (wr == 0) barrier();
        // every wave has read its last fragments: the next tile's prologue may
        // overwrite the LDS slots while this tile's epilogue runs
        const int nid = id + G;
        const bool more = nid < n_items;
        int64_t m1 = 0, n1 = 0;
        int kb1 = 0, nk1 = 0;
        if (more) {
            item(nid, m1, n1, kb1, nk1);
            prologue(m1, n1, kb1, nk1);
        }
        order_fence();
        if (id < n_full) {
            p_epilogue<EPI, TC, TX, CSM>(g, rc, rx, rbias, rcs, m0, n0, wr, wc, lane, acc);
        } else {
            // a tail slice (always the workgroup's last item): its fp32 partial
            // tile, buffer stores from one lane offset (constant soffsets)
            const __amdgpu_buffer_rsrc_t rw = make_rsrc((const char*)(g.ws + (int64_t)(id - n_full) * 65536), 65536u * 4);
            const uint32_t lo = (uint32_t)(((wr * 64 + (lane & 15)) * 256 + wc * 32 + 4 * (lane >> 4)) * 4);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][b][i][j]), rw, lo,
                                                                   ((a * 128 + i * 16) * 256 + b * 128 + j * 16) * 4, 0);
        }
        order_fence();
        if (!more) break;
        id = nid;
        m0 = m1;
        n0 = n1;
        kb = kb1;
        nk = nk1;
    }
#undef MSQ_PPHASE
}

}  // namespace

namespace {
int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

template <int TA, int TB, int EPI, typename TC, typename TX, int CSM = 0>
void launch_p(const GemmArgs& g, hipStream_t s) {
    static bool attr = false;
    auto k = gemm256p_kernel<TA, TB, EPI, TC, TX, CSM>;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * HALF);
        attr = true;
    }
    const int ntiles = g.tiles_m * g.tiles_n;
    hipLaunchKernelGGL(k, dim3(std::min(ntiles, num_cus())), dim3(NT), 8 * HALF, s, g);
    if constexpr (CSM == 0) {
        if (g.tail_tiles > 0) {
            const int64_t total = (int64_t)g.tail_tiles * 256 * 64;
            hipLaunchKernelGGL((p_tail_fixup_kernel<EPI, TC, TX>), dim3((unsigned)std::min<int64_t>((total + 255) / 256, 2048)),
                               dim3(256), 0, s, g);
        }
    }
}

template <int EPI, typename TC, typename TX>
void dispatch_p_t(const GemmArgs& g, int ta, int tb, hipStream_t s) {
    if (ta == 0 && tb == 0) launch_p<0, 0, EPI, TC, TX>(g, s);
    else if (ta == 0 && tb == 1) launch_p<0, 1, EPI, TC, TX>(g, s);
    else if (ta == 1 && tb == 1) launch_p<1, 1, EPI, TC, TX>(g, s);
    else launch_p<1, 0, EPI, TC, TX>(g, s);
}

template <typename TC>
void dispatch_p(const GemmArgs& g, int ta, int tb, int epi, int aux_dtype, hipStream_t s) {
    switch (epi) {
        case MSQ_EPI_NONE: dispatch_p_t<MSQ_EPI_NONE, TC, float>(g, ta, tb, s); break;
        case MSQ_EPI_BIAS: dispatch_p_t<MSQ_EPI_BIAS, TC, float>(g, ta, tb, s); break;
        case MSQ_EPI_BIAS_RELU:
            if (aux_dtype == MSQ_MASK1 && g.aux) dispatch_p_t<MSQ_EPI_BIAS_RELU, TC, mask1_t>(g, ta, tb, s);
            else dispatch_p_t<MSQ_EPI_BIAS_RELU, TC, float>(g, ta, tb, s);
            break;
        // the aux operand is read as aux_dtype (bf16 residual streams included)
        case MSQ_EPI_BIAS_RESID:
            if (aux_dtype == MSQ_BF16) dispatch_p_t<MSQ_EPI_BIAS_RESID, TC, bf16>(g, ta, tb, s);
            else dispatch_p_t<MSQ_EPI_BIAS_RESID, TC, float>(g, ta, tb, s);
            break;
        case MSQ_EPI_BIAS_DROP_RESID:
            if (aux_dtype == MSQ_BF16) dispatch_p_t<MSQ_EPI_BIAS_DROP_RESID, TC, bf16>(g, ta, tb, s);
            else dispatch_p_t<MSQ_EPI_BIAS_DROP_RESID, TC, float>(g, ta, tb, s);
            break;
        case MSQ_EPI_RELU_MASK:
            if (aux_dtype == MSQ_MASK1) dispatch_p_t<MSQ_EPI_RELU_MASK, TC, mask1_t>(g, ta, tb, s);
            else if (aux_dtype == MSQ_BF16) dispatch_p_t<MSQ_EPI_RELU_MASK, TC, bf16>(g, ta, tb, s);
            else dispatch_p_t<MSQ_EPI_RELU_MASK, TC, float>(g, ta, tb, s);
            break;
    }
}
}  // namespace

// the K-split tail of a persistent launch (p_tail_fixup_kernel): on when the
// last round holds at most a quarter of the grid's workgroups, the epilogue
// is one p_tail_fixup_kernel applies (no mask-bit writes, no column sums),
// and K spans >= 8 k-steps; tail_s slices of >= 4 k-steps, tail_tiles *
// tail_s <= G. Returns the partials' bytes (0: off)
struct PTail {
    int tiles, s, kst;
};
static size_t p_tail_plan(int64_t M, int64_t N, int64_t K, int epi, int aux_dtype, PTail& t) {
    t = PTail{0, 0, 0};
    if (aux_dtype == MSQ_MASK1 || epi == MSQ_EPI_ACCUM) return 0;
    const int64_t ntiles = ((M + 255) / 256) * ((N + 255) / 256);
    const int64_t G = std::min<int64_t>(ntiles, num_cus());
    const int64_t rem = ntiles % G, nk = (K + 63) / 64;
    if (rem == 0 || rem * 4 > G || nk < 8) return 0;
    int64_t S = std::min<int64_t>(std::min<int64_t>(G / rem, nk / 4), 32);
    if (S < 2) return 0;
    const int64_t kst = (nk + S - 1) / S;
    S = (nk + kst - 1) / kst;
    t = PTail{(int)rem, (int)S, (int)kst};
    return (size_t)rem * S * 65536 * 4;
}

size_t gemm256p_tail_ws_bytes(int64_t M, int64_t N, int64_t K, int epi, int aux_dtype) {
    PTail t;
    return p_tail_plan(M, N, K, epi, aux_dtype, t);
}

// C / aux / bias preconditions of the persistent tile and its descriptor extents
static bool p_prepare(GemmArgs& g, int ta, int tb, int epi, int c_dtype, int aux_dtype) {
    if (epi == MSQ_EPI_ACCUM || g.batch != 1) return false;
    const int esz = c_dtype == MSQ_BF16 ? 2 : 4, xsz = aux_dtype == MSQ_BF16 ? 2 : 4;
    // MASK1: words of 32 columns (its writer needs bf16 C: the bits are of the stored values)
    if (aux_dtype == MSQ_MASK1 && g.aux && (c_dtype != MSQ_BF16 || (epi != MSQ_EPI_RELU_MASK && epi != MSQ_EPI_BIAS_RELU)))
        return false;
    // 16-B C pieces (bf16: 8 columns, fp32: 4), 16-B aligned rows
    if (g.N % 8 || g.ldc % 8 || ((uintptr_t)g.C % 16)) return false;
    if (g.bias && ((uintptr_t)g.bias % 16)) return false;
    if (g.aux && aux_dtype != MSQ_MASK1 && (g.ldx % 4 || ((uintptr_t)g.aux % 16))) return false;
    if (g.aux && aux_dtype == MSQ_MASK1 && ((uintptr_t)g.aux % 4)) return false;
    const int64_t cext = ((g.M - 1) * g.ldc + g.N) * esz;
    const int64_t xext = !g.aux ? 0
                         : aux_dtype == MSQ_MASK1 ? ((g.M - 1) * g.ldx + (g.N + 31) / 32) * 4
                                                  : ((g.M - 1) * g.ldx + g.N) * xsz;
    if (cext >= (int64_t)OOB || xext >= (int64_t)OOB || g.N * 4 >= (int64_t)OOB) return false;
    if (!gemm256_plan(g, ta, tb, epi) || g.ksplit != 1) return false;
    g.c_ext = (uint32_t)cext;
    g.x_ext = (uint32_t)xext;
    PTail t;
    const size_t tb_bytes = p_tail_plan(g.M, g.N, g.K, epi, aux_dtype, t);
    if (tb_bytes && g.ws && g.ws_bytes >= (int64_t)tb_bytes && ((uintptr_t)g.ws % 16) == 0) {
        g.tail_tiles = t.tiles;
        g.tail_s = t.s;
        g.tail_kst = t.kst;
    } else {
        g.tail_tiles = g.tail_s = g.tail_kst = 0;
    }
    return true;
}

bool gemm256p_applies(GemmArgs g, int ta, int tb, int epi, int c_dtype, int aux_dtype) {
    return p_prepare(g, ta, tb, epi, c_dtype, aux_dtype);
}

bool gemm256p_launch(GemmArgs g, int ta, int tb, int epi, int c_dtype, int aux_dtype, hipStream_t s) {
    if (!p_prepare(g, ta, tb, epi, c_dtype, aux_dtype)) return false;
    if (c_dtype == MSQ_BF16) dispatch_p<bf16>(g, ta, tb, epi, aux_dtype, s);
    else dispatch_p<float>(g, ta, tb, epi, aux_dtype, s);
    return true;
}

// the persistent tile with the column-sum partials (bf16 C, epilogue NONE /
// RELU_MASK, A / B not transposed or B transposed); the caller reduces g.cs_ws
bool gemm256p_colsum_launch(GemmArgs g, int ta, int tb, int epi, int aux_dtype, hipStream_t s) {
    if (ta != 0 || (epi != MSQ_EPI_NONE && epi != MSQ_EPI_RELU_MASK)) return false;
    if (!p_prepare(g, ta, tb, epi, MSQ_BF16, aux_dtype)) return false;
    g.tail_tiles = g.tail_s = g.tail_kst = 0;  // (the column sums need every tile's epilogue)
    if ((int64_t)g.tiles_m * 2 * g.N * 4 >= (int64_t)OOB) return false;
    const bool bx = aux_dtype == MSQ_BF16, b1 = aux_dtype == MSQ_MASK1;
    if (tb == 0) {
        if (epi == MSQ_EPI_NONE) launch_p<0, 0, MSQ_EPI_NONE, bf16, float, 1>(g, s);
        else if (b1) launch_p<0, 0, MSQ_EPI_RELU_MASK, bf16, mask1_t, 1>(g, s);
        else if (bx) launch_p<0, 0, MSQ_EPI_RELU_MASK, bf16, bf16, 1>(g, s);
        else launch_p<0, 0, MSQ_EPI_RELU_MASK, bf16, float, 1>(g, s);
    } else {
        if (epi == MSQ_EPI_NONE) launch_p<0, 1, MSQ_EPI_NONE, bf16, float, 1>(g, s);
        else if (b1) launch_p<0, 1, MSQ_EPI_RELU_MASK, bf16, mask1_t, 1>(g, s);
        else if (bx) launch_p<0, 1, MSQ_EPI_RELU_MASK, bf16, bf16, 1>(g, s);
        else launch_p<0, 1, MSQ_EPI_RELU_MASK, bf16, float, 1>(g, s);
    }
    return true;
}


// bias epilogue + per-(M-tile, wave-row) column (max, sum exp) partials of the
// stored bf16 values into part (row stride pld): the lm_head forward feeding
// the time-axis logsumexp of the filtered loss (train.py:133-138)
static bool colstats_prepare(GemmArgs& g, int ta, int tb, const float* part, int64_t pld) {
    if (ta != 0 || g.aux) return false;
    if (!p_prepare(g, ta, tb, MSQ_EPI_BIAS, MSQ_BF16, MSQ_F32)) return false;
    return !(pld < g.N || pld % 4 || ((uintptr_t)part % 16) || (int64_t)g.tiles_m * 4 * pld * 4 >= (int64_t)OOB);
}

bool gemm256p_colstats_applies(GemmArgs g, int tb, const float* part, int64_t pld) {
    return colstats_prepare(g, 0, tb, part, pld);
}

bool gemm256p_colstats_launch(GemmArgs g, int ta, int tb, float* part, int64_t pld, hipStream_t s) {
    if (!colstats_prepare(g, ta, tb, part, pld)) return false;
    g.cs_ws = part;
    g.ldx = pld;
    if (tb == 0) launch_p<0, 0, MSQ_EPI_BIAS, bf16, float, 2>(g, s);
    else launch_p<0, 1, MSQ_EPI_BIAS, bf16, float, 2>(g, s);
    return true;
}
