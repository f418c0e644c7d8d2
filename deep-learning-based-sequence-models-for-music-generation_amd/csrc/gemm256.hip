// 256x256x64 bf16 GEMM tile for the large products of the train step
// (QKV / proj / FFN / lm_head forward, their dX and dW products).
//
// Structure (cdna_hip_programming.md §5 "256² 8-phase template", rebuilt for
// the three operand layouts this path needs):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); a wave owns 128x64 outputs as
//     2x2 quadrants of 64x32 (32 accumulators of v_mfma_f32_16x16x32_bf16).
//   * LDS (128 KiB, one dynamic array) = 2 K-tile buffers x 4 half-tile slots
//     {A rows 0-127, B rows 0-127, A rows 128-255, B rows 128-255}, 16 KiB each.
//     A wave's quadrant (mi, ni) reads A-half mi and B-half ni only.
//   * Half-tiles are filled by buffer_load_dwordx4 ... lds (LDS DMA, 2 per
//     thread per half) whose buffer descriptor zero-fills every out-of-range
//     chunk, so M / N / K edges and split-K slices need no masking in LDS.
//     The XOR swizzle is applied on the SOURCE address (the LDS image is
//     lane-linear) and again on the ds_read address (rule 21).
//   * A K-tile is 4 phases, one per quadrant: (0,0) (1,0) (1,1) (0,1). Each
//     phase = {ds_reads of the fragments it introduces; LDS-DMA of one
//     half-tile 5 phases ahead; s_waitcnt vmcnt(8)} barrier {16 MFMA} barrier.
//     Waves 4-7 run one barrier behind waves 0-3 (ping-pong), so on every SIMD
//     one wave issues MFMAs while the other issues LDS / global traffic.
//   * vmcnt(8) in a phase retires the half-tile read in the next phase and
//     leaves four half-tiles (8 DMA per thread) in flight; a slot is re-filled
//     >= 2 phases after its last ds_read (the staggered groups' WAR distance).
// Operands: K-contiguous ([rows][K], e.g. activations, nn.Linear weights) use
// 128-B LDS rows read with ds_read_b128; M/N-contiguous ([K][rows], the dY of
// a dW product or W in dX = dY.W) use 256-B LDS rows read with
// ds_read_b64_tr_b16 (hardware transpose), so no operand is ever transposed.
#include "gemm256_tile.h"

namespace {

using namespace g256;

// LAB: ablation switches for tools/gemm256_lab.hip only (0 in the library):
// 1 = no LDS-DMA in the K loop, 2 = no MFMA, 4 = no ping-pong stagger,
// 8 = K slice innermost in the block order, 16 = no epilogue stores
// CS: also the column sums of the written C, per (M-tile, wave-row) into g.cs_ws
template <int TA, int TB, int EPI, typename TC, typename TX, int LAB = 0, bool CS = false>
__global__ __launch_bounds__(NT, 1) void gemm256_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    lds_t* smem = (lds_t*)smem_raw;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;

    const int tiles = g.tiles_m * g.tiles_n;
    // every tile / slice index is wave-uniform: keep it scalar (T20)
    int bid = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
    // K slice outermost: the blocks that run together on an XCD share the
    // same K range, so their A / B panels meet in that XCD's L2
    int kslice;
    if (LAB & 8) {
        kslice = bid % g.ksplit;
        bid /= g.ksplit;
    } else {
        kslice = bid / (tiles * g.batch);
        bid -= kslice * tiles * g.batch;
    }
    const int bz = bid / tiles;
    bid -= bz * tiles;
    const int GROUP = 8;
    const int per_group = GROUP * g.tiles_n;
    const int grp = bid / per_group, first_m = grp * GROUP;
    const int gsz = min(g.tiles_m - first_m, GROUP);
    const int tm = first_m + (bid % per_group) % gsz;
    const int tn = (bid % per_group) / gsz;
    const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;

    const char* Ab = (const char*)g.A + (int64_t)bz * g.sA * 2;
    const char* Bb = (const char*)g.B + (int64_t)bz * g.sB * 2;
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab, g.a_ext);
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(Bb, g.b_ext);

    Stage<TA == 0> sa;
    Stage<TB == 0> sb;
    sa.init(m0, g.M, g.lda, w, lane);
    sb.init(n0, g.N, g.ldb, w, lane);

    // per-lane fragment offsets inside a half-tile slot
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

    const int64_t kbeg = (int64_t)kslice * g.kper;
    const int64_t kend = min<int64_t>(g.K, kbeg + g.kper);
    const int nk = (int)((kend - kbeg + 63) / 64);

    // slot s of buffer b: b*4 + {0: A0, 1: B0, 2: A1, 3: B1}
    auto slot = [&](int b, int s) { return smem + (b * 4 + s) * HALF; };
    // stage index s = 4u + h; h: 0 A0, 1 B0, 2 A1, 3 B1
    auto issue = [&](int u, int h) {
        const int64_t k0 = kbeg + (int64_t)u * 64;
        lds_t* dst = slot(u & 1, h);
        if (h == 0) sa.issue(ra, dst, 0, k0, kend - k0, w);
        else if (h == 1) sb.issue(rb, dst, 0, k0, kend - k0, w);
        else if (h == 2) sa.issue(ra, dst, 1, k0, kend - k0, w);
        else sb.issue(rb, dst, 1, k0, kend - k0, w);
    };

    f32x4 acc[2][2][4][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[a][b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // prologue: stages 0..5
    issue(0, 0);
    issue(0, 1);
    issue(0, 2);
    issue(0, 3);
    if (nk > 1) {
        issue(1, 0);
        issue(1, 1);
        vm_wait8();
    } else {
        vm_wait0();
    }
    barrier();
    if (!(LAB & 4) && wr == 1) barrier();

    bf16x8 af[2][2][4];  // [mi][ks][i]
    bf16x8 bfr[2][2][2];  // [ni][ks][j]

    // one phase: quadrant Q of K-tile t held in buffer BUF
#define MSQ_PHASE(Q, BUF)                                                                               \
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
        if (su < nk && !(LAB & 1)) {                                                                    \
            issue(su, (Q + 2) & 3);                                                                     \
            vm_wait8();                                                                                 \
        } else {                                                                                        \
            vm_wait0();                                                                                 \
        }                                                                                               \
        barrier();                                                                                      \
        __builtin_amdgcn_s_setprio(1);                                                                  \
        _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                \
            _Pragma("unroll") for (int i = 0; i < 4; ++i)                                               \
                _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                         \
                    if (LAB & 2) {                                                                      \
                        asm volatile("" ::"v"(bfr[ni][ks][j]), "v"(af[mi][ks][i]));                     \
                    } else {                                                                            \
                        acc[mi][ni][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                    \
                            bfr[ni][ks][j], af[mi][ks][i], acc[mi][ni][i][j], 0, 0, 0);                 \
                    }                                                                                   \
                }                                                                                       \
        __builtin_amdgcn_s_setprio(0);                                                                  \
        barrier();                                                                                      \
    }

    for (int t = 0; t < nk; t += 2) {
        MSQ_PHASE(0, 0)
        MSQ_PHASE(1, 0)
        MSQ_PHASE(2, 0)
        MSQ_PHASE(3, 0)
        if (t + 1 < nk) {
            ++t;
            MSQ_PHASE(0, 1)
            MSQ_PHASE(1, 1)
            MSQ_PHASE(2, 1)
            MSQ_PHASE(3, 1)
            --t;
        }
    }
#undef MSQ_PHASE
    if (!(LAB & 4) && wr == 0) barrier();

    // epilogue: lane holds C[m][n..n+3]
    TC* C = (TC*)g.C + bz * g.sC;
    const TX* X = (const TX*)g.aux + (g.aux ? bz * g.sX : 0);
    float* wsp = (EPI == MSQ_EPI_ACCUM && g.ksplit > 1 && g.ws) ? g.ws + ((int64_t)kslice * g.batch + bz) * g.M * g.N
                                                                 : nullptr;
    // per half-tile, the aux vectors the epilogue reads are all loaded before
    // its first store (C stores could alias them, so the compiler would
    // otherwise issue each load only after the previous store)
    f32x4 csum[2][2];  // CS: this lane's column sums over its 8 rows, [b][j]
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) csum[b][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        f32x4 xp[4][2][2];
        if (epi_reads_aux<EPI>()) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int64_t m = m0 + a * 128 + wr * 64 + i * 16 + (lane & 15);
                        const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * (lane >> 4);
                        xp[i][b][j] = (m < g.M && n < g.N) ? epi_aux_load(g, X, m, n) : (f32x4){0.f, 0.f, 0.f, 0.f};
                    }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t m = m0 + a * 128 + wr * 64 + i * 16 + (lane & 15);
            if (m >= g.M) continue;
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * (lane >> 4);
                    if (n >= g.N) continue;
                    if ((LAB & 16) && acc[a][b][i][j][0] != 12345.f) continue;
                    const f32x4 v = epi_apply<EPI, TC, TX>(g, C, X, m, n, acc[a][b][i][j], wsp,
                                                           epi_reads_aux<EPI>() ? &xp[i][b][j] : nullptr);
                    if (CS) csum[b][j] += v;
                }
        }
    }
    if (CS) {
        // sum over the 16 row-lanes (lane & 15) of each column group, then one
        // partial row per (M-tile, wave-row): cs_ws[(tm * 2 + wr)][n]
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x4 v = csum[b][j];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1)
#pragma unroll
                    for (int t = 0; t < 4; ++t) v[t] += __shfl_xor(v[t], o, 64);
                const int64_t n = n0 + b * 128 + wc * 32 + j * 16 + 4 * (lane >> 4);
                if ((lane & 15) == 0 && n < g.N) *(f32x4*)(g.cs_ws + ((int64_t)tm * 2 + wr) * g.N + n) = v;
            }
    }
}

// dbias[n] (+)= sum_p part[p][n], fixed order: 64 columns x 16 partial groups
__global__ __launch_bounds__(1024) void colsum_partials_kernel(const float* __restrict__ part, int64_t nparts,
                                                               int64_t N, float* __restrict__ dbias, int accumulate) {
    __shared__ float red[16][64];
    const int c = threadIdx.x & 63, gq = threadIdx.x >> 6;
    const int64_t n = (int64_t)blockIdx.x * 64 + c;
    float s = 0.f;
    if (n < N)
        for (int64_t p = gq; p < nparts; p += 16) s += part[p * N + n];
    red[gq][c] = s;
    __syncthreads();
    if (gq == 0 && n < N) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) t += red[k][c];
        dbias[n] = accumulate ? dbias[n] + t : t;
    }
}

template <int TA, int TB, int EPI, typename TC, typename TX>
void launch(const GemmArgs& g, hipStream_t s) {
    static bool attr = false;
    auto k = gemm256_kernel<TA, TB, EPI, TC, TX>;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * HALF);
        attr = true;
    }
    const int nblk = g.tiles_m * g.tiles_n * g.batch * g.ksplit;
    hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), 8 * HALF, s, g);
}

template <int EPI, typename TC, typename TX>
void dispatch_t(const GemmArgs& g, int ta, int tb, hipStream_t s) {
    if (ta == 0 && tb == 0) launch<0, 0, EPI, TC, TX>(g, s);
    else if (ta == 0 && tb == 1) launch<0, 1, EPI, TC, TX>(g, s);
    else if (ta == 1 && tb == 1) launch<1, 1, EPI, TC, TX>(g, s);
    else launch<1, 0, EPI, TC, TX>(g, s);
}

template <typename TC>
void dispatch_epi(const GemmArgs& g, int ta, int tb, int epi, int aux_dtype, hipStream_t s) {
    switch (epi) {
        case MSQ_EPI_NONE: dispatch_t<MSQ_EPI_NONE, TC, float>(g, ta, tb, s); break;
        case MSQ_EPI_BIAS: dispatch_t<MSQ_EPI_BIAS, TC, float>(g, ta, tb, s); break;
        case MSQ_EPI_BIAS_RELU: dispatch_t<MSQ_EPI_BIAS_RELU, TC, float>(g, ta, tb, s); break;
        // the aux operand is read as aux_dtype (bf16 residual streams included)
        case MSQ_EPI_BIAS_RESID:
            if (aux_dtype == MSQ_BF16) dispatch_t<MSQ_EPI_BIAS_RESID, TC, bf16>(g, ta, tb, s);
            else dispatch_t<MSQ_EPI_BIAS_RESID, TC, float>(g, ta, tb, s);
            break;
        case MSQ_EPI_RELU_MASK:
            if (aux_dtype == MSQ_MASK1) dispatch_t<MSQ_EPI_RELU_MASK, TC, mask1_t>(g, ta, tb, s);
            else if (aux_dtype == MSQ_BF16) dispatch_t<MSQ_EPI_RELU_MASK, TC, bf16>(g, ta, tb, s);
            else dispatch_t<MSQ_EPI_RELU_MASK, TC, float>(g, ta, tb, s);
            break;
        case MSQ_EPI_ACCUM: dispatch_t<MSQ_EPI_ACCUM, TC, float>(g, ta, tb, s); break;
        case MSQ_EPI_BIAS_DROP_RESID:
            if (aux_dtype == MSQ_BF16) dispatch_t<MSQ_EPI_BIAS_DROP_RESID, TC, bf16>(g, ta, tb, s);
            else dispatch_t<MSQ_EPI_BIAS_DROP_RESID, TC, float>(g, ta, tb, s);
            break;
    }
}

}  // namespace

// ksplit / kper / tiles of the 256 tile for this problem, or false when its
// preconditions fail (the caller then uses the 128x128 kernel)
bool gemm256_plan(GemmArgs& g, int ta, int tb, int epi) {
    // preconditions: chunks of 8 never straddle an edge; extents fit a descriptor
    if ((ta ? g.M : g.K) % 8 || (tb ? g.N : g.K) % 8) return false;
    const int64_t aext = ((ta ? g.K : g.M) - 1) * g.lda + (ta ? g.M : g.K);
    const int64_t bext = ((tb ? g.K : g.N) - 1) * g.ldb + (tb ? g.N : g.K);
    if (aext * 2 >= (int64_t)OOB || bext * 2 >= (int64_t)OOB) return false;
    g.tiles_m = (int)((g.M + 255) / 256);
    g.tiles_n = (int)((g.N + 255) / 256);
    const int64_t tiles = (int64_t)g.tiles_m * g.tiles_n * g.batch;
    g.ksplit = 1;
    g.kper = (g.K + 63) / 64 * 64;
    if (epi == MSQ_EPI_ACCUM) {
        // split-K for the weight-gradient products: pick the split that
        // minimises  waves(ks) x (k-steps per block + C), one block per CU,
        // C ~ prologue + partial-tile epilogue in k-step units. E.g. lm_head
        // dW (280 tiles, K = 65536): ks = 8 -> 9 waves of 136, vs ks = 1 -> 2
        // waves of 1032 (the second one 24/256 full).
        const int64_t ksteps = (g.K + 63) / 64;
        const int64_t C = 8;
        int64_t best = 1, best_cost = INT64_MAX;
        for (int64_t ks = 1; ks <= 32 && ksteps / ks >= 16; ++ks) {
            const int64_t waves = (tiles * ks + 255) / 256;
            const int64_t cost = waves * ((ksteps + ks - 1) / ks + C);
            if (cost < best_cost) best = ks, best_cost = cost;
        }
        if (best > 1) {
            g.kper = ((g.K + best - 1) / best + 63) / 64 * 64;
            g.ksplit = (int)((g.K + g.kper - 1) / g.kper);
        }
    }
    // below ~half a wave of blocks the 128x128 tile (4x the blocks) wins
    if (tiles * g.ksplit < 128) return false;
    g.a_ext = (uint32_t)(aext * 2);
    g.b_ext = (uint32_t)(bext * 2);
    return true;
}

bool gemm256_colsum_launch(GemmArgs g, int ta, int tb, int epi, int aux_dtype, float* dbias, int accumulate,
                           float* ws, size_t ws_bytes, hipStream_t s) {
    if (epi != MSQ_EPI_NONE && epi != MSQ_EPI_RELU_MASK) return false;
    if (g.N % 4 || g.batch != 1 || ws_bytes < gemm256_colsum_ws_bytes(g.M, g.N) || !gemm256_plan(g, ta, tb, epi))
        return false;
    g.cs_ws = ws;
    if (gemm256p_colsum_launch(g, ta, tb, epi, aux_dtype, s)) {
        hipLaunchKernelGGL(colsum_partials_kernel, dim3((unsigned)((g.N + 63) / 64)), dim3(1024), 0, s, ws,
                           (int64_t)g.tiles_m * 2, g.N, dbias, accumulate);
        return true;
    }
    auto go = [&](auto kern) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * HALF);
        hipLaunchKernelGGL(kern, dim3(g.tiles_m * g.tiles_n), dim3(NT), 8 * HALF, s, g);
    };
    const bool bx = aux_dtype == MSQ_BF16, b1 = aux_dtype == MSQ_MASK1;
    if (ta == 0 && tb == 1) {
        if (epi == MSQ_EPI_NONE) go(gemm256_kernel<0, 1, MSQ_EPI_NONE, bf16, float, 0, true>);
        else if (b1) go(gemm256_kernel<0, 1, MSQ_EPI_RELU_MASK, bf16, mask1_t, 0, true>);
        else if (bx) go(gemm256_kernel<0, 1, MSQ_EPI_RELU_MASK, bf16, bf16, 0, true>);
        else go(gemm256_kernel<0, 1, MSQ_EPI_RELU_MASK, bf16, float, 0, true>);
    } else if (ta == 0 && tb == 0) {
        if (epi == MSQ_EPI_NONE) go(gemm256_kernel<0, 0, MSQ_EPI_NONE, bf16, float, 0, true>);
        else if (b1) go(gemm256_kernel<0, 0, MSQ_EPI_RELU_MASK, bf16, mask1_t, 0, true>);
        else if (bx) go(gemm256_kernel<0, 0, MSQ_EPI_RELU_MASK, bf16, bf16, 0, true>);
        else go(gemm256_kernel<0, 0, MSQ_EPI_RELU_MASK, bf16, float, 0, true>);
    } else {
        return false;
    }
    hipLaunchKernelGGL(colsum_partials_kernel, dim3((unsigned)((g.N + 63) / 64)), dim3(1024), 0, s, ws,
                       (int64_t)g.tiles_m * 2, g.N, dbias, accumulate);
    return true;
}

bool gemm256_launch(GemmArgs g, int ta, int tb, int epi, int c_dtype, int aux_dtype, size_t ws_bytes,
                    hipStream_t s) {
    if (!gemm256_plan(g, ta, tb, epi)) return false;
    if (!g.ws || ws_bytes < splitk_ws_bytes(g.M, g.N, g.batch, g.ksplit) ||
        !splitk_ws_bytes(g.M, g.N, g.batch, g.ksplit))
        g.ws = nullptr;
    if (c_dtype == MSQ_BF16) dispatch_epi<bf16>(g, ta, tb, epi, aux_dtype, s);
    else dispatch_epi<float>(g, ta, tb, epi, aux_dtype, s);
    if (epi == MSQ_EPI_ACCUM && g.ws) splitk_reduce(g, s);
    return true;
}
