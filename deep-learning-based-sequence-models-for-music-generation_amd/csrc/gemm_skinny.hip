// Skinny-M bf16 GEMM for the decode steps (M = batch rows <= 64):
//   C[M][N] = A[M][K] . W[N][K]^T  (+ the msq_gemm epilogues)
// The weight W (nn.Linear layout, K contiguous) is the only large operand: it
// is streamed from HBM exactly once, straight into MFMA B-fragments (no LDS
// staging), while the <= 64 activation rows (<= 128 KiB) come from L2.
//   * block = 1024 threads = 16 waves on one 16-row slice of W; the waves split
//     K (16 x 1-4 k-steps at K = 1024-2048: every W load of a wave is issued
//     at once, 32-64 KiB in flight per CU) and their partial accumulators are
//     summed through LDS;
//   * per k-step of 32 a wave issues one 16-B W load and MT 16-B A loads per
//     lane, U k-steps ahead, then U*MT v_mfma_f32_16x16x32_bf16;
//   * MFMA roles: W rows are the MFMA A-operand (output rows), activation rows
//     the B-operand, so a lane ends with C[m][n..n+3] (4 consecutive n of one
//     row m), the layout epi_apply takes.
// Bound: HBM bytes of W (2 N K) per launch; grid = N / 16 blocks (x K slices
// when N / 16 alone would leave most CUs idle, skinny_ksplit).
#include "gemm.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int SK_WAVES = 16, SK_U = 4;

// Mamba2 decode: the depthwise causal conv of the new row fused into the
// in_proj epilogue (msq_mamba_in_proj_conv_step). Output columns c0 + c,
// c < cd, are the pre-conv xBC channels; the lane holding C[m][n..n+3] runs
// conv_step_kernel's arithmetic (csrc/mamba_step.hip) on those 4 channels of
// row m: xc = silu(b + w0 s0 + w1 s1 + w2 s2 + w3 in), (s0, s1, s2) <- (s1, s2, in),
// in = the stored bf16 value. Each (m, channel) has one owner: no race.
struct SkinnyConv {
    bf16* xc;
    int64_t ldxc;
    float* st;  // [M][3][cd]
    const float* w;  // [cd][4]
    const float* b;  // [cd]
    int64_t c0, cd;
};
// as mamba.hip's silu (v_exp_f32 + v_rcp_f32), so the decode step matches the forward
__device__ __forceinline__ float conv_silu(float x) {
    return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ void conv_apply(const SkinnyConv& cv, int64_t m, int64_t n, f32x4 v) {
    const int64_t c = n - cv.c0;
    if (c < 0 || c >= cv.cd) return;  // c0, cd % 4 == 0: the 4 columns are wholly in or out
    float* s = cv.st + m * 3 * cv.cd + c;
    const f32x4 s0 = *(const f32x4*)s, s1 = *(const f32x4*)(s + cv.cd), s2 = *(const f32x4*)(s + 2 * cv.cd);
    const f32x4 bv = *(const f32x4*)(cv.b + c);
    f32x4 xo, in;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const f32x4 wc = *(const f32x4*)(cv.w + (c + t) * 4);
        in[t] = (float)(bf16)v[t];
        float acc = bv[t];
        acc += wc[0] * s0[t];
        acc += wc[1] * s1[t];
        acc += wc[2] * s2[t];
        acc += wc[3] * in[t];
        xo[t] = conv_silu(acc);
    }
    store4(cv.xc + m * cv.ldxc + c, xo);
    *(f32x4*)s = s1;
    *(f32x4*)(s + cv.cd) = s2;
    *(f32x4*)(s + 2 * cv.cd) = in;
}

template <int EPI, typename TC, typename TX, int MT, bool PART>
__global__ __launch_bounds__(64 * SK_WAVES) void gemm_skinny_kernel(GemmArgs g) {
    __shared__ f32x4 red[SK_WAVES - 1][MT][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t n0 = (int64_t)blockIdx.x * 16;
    const bf16* W = (const bf16*)g.B;
    const bf16* A = (const bf16*)g.A;
    // PART: K slice blockIdx.y of g.kper (split-K over workgroups, fp32 partials to g.ws)
    const int64_t k0 = PART ? (int64_t)blockIdx.y * g.kper : 0, k1 = PART ? min<int64_t>(g.K, k0 + g.kper) : g.K;
    const int64_t kper = (k1 - k0 + SK_WAVES * 32 - 1) / (SK_WAVES * 32) * 32;
    const int64_t kb = k0 + w * kper, ke = min<int64_t>(k1, kb + kper);
    const int64_t wn = n0 + (lane & 15);
    const bool wok = wn < g.N;
    const bf16* wrow = W + (wok ? wn : 0) * g.ldb;
    const int kq = 8 * (lane >> 4);
    const bf16* arow[MT];
    bool aok[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int64_t m = mt * 16 + (lane & 15);
        aok[mt] = m < g.M;
        arow[mt] = A + (aok[mt] ? m : 0) * g.lda;
    }
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bf16x8 z = (bf16x8){};
    for (int64_t k = kb; k < ke; k += 32 * SK_U) {
        bf16x8 wf[SK_U], af[SK_U][MT];
#pragma unroll
        for (int u = 0; u < SK_U; ++u) {
            const int64_t kk = k + 32 * u + kq;  // K % 8 == 0: a chunk of 8 is wholly in or out
            const bool kin = kk < ke;
            wf[u] = (wok && kin) ? *(const bf16x8*)(wrow + kk) : z;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[u][mt] = (aok[mt] && kin) ? *(const bf16x8*)(arow[mt] + kk) : z;
        }
#pragma unroll
        for (int u = 0; u < SK_U; ++u)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[u], af[u][mt], acc[mt], 0, 0, 0);
    }
    if (w > 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) red[w - 1][mt][lane] = acc[mt];
    }
    __syncthreads();
    if (w != 0) return;
    TC* C = (TC*)g.C;
    const TX* X = (const TX*)g.aux;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        f32x4 v = acc[mt];
#pragma unroll
        for (int q = 0; q < SK_WAVES - 1; ++q) v += red[q][mt][lane];
        const int64_t m = mt * 16 + (lane & 15), n = n0 + 4 * (lane >> 4);
        if (m < g.M && n < g.N) {
            if (PART) store4(g.ws + ((int64_t)blockIdx.y * g.M + m) * g.N + n, v);  // N % 4 == 0
            else epi_apply<EPI, TC, TX>(g, C, X, m, n, v);
        }
    }
}

// C = epi(sum_s ws[s]) of a split-K skinny product (fixed summation order)
template <int EPI, typename TC, typename TX>
__global__ __launch_bounds__(256) void skinny_reduce_kernel(GemmArgs g, int ks) {
    const int64_t nq = g.N / 4, e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= g.M * nq) return;
    const int64_t m = e / nq, n = (e - m * nq) * 4, MN = g.M * g.N;
    f32x4 v = load4(g.ws + m * g.N + n);
    for (int s = 1; s < ks; ++s) v += load4(g.ws + s * MN + m * g.N + n);
    epi_apply<EPI, TC, TX>(g, (TC*)g.C, (const TX*)g.aux, m, n, v);
}

// Persistent variant for K <= SK_WAVES * 2 * 32 = 1024: a wave's K slice of
// the activation rows (KS k-steps x MT fragments) is loaded ONCE into
// registers and serves every 16-row W slice the block visits; the block walks
// W slices blockIdx.x, + gridDim.x, ... with the next slice's W fragments
// loaded before the current slice's MFMAs, reduction and epilogue, so each
// CU keeps streaming W without launch rounds.
template <int EPI, typename TC, typename TX, int MT, int KS, bool CONV = false>
__global__ __launch_bounds__(64 * SK_WAVES) void gemm_skinny_pk_kernel(GemmArgs g, int64_t ntiles,
                                                                     SkinnyConv cv = {}) {
    __shared__ f32x4 red[SK_WAVES][MT][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bf16* W = (const bf16*)g.B;
    const bf16* A = (const bf16*)g.A;
    const int kq = 8 * (lane >> 4);
    const int64_t kb = (int64_t)w * KS * 32;
    const bf16x8 z = (bf16x8){};
    bf16x8 af[KS][MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int64_t m = mt * 16 + (lane & 15);
        const bf16* arow = A + (m < g.M ? m : 0) * g.lda;
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            const int64_t kk = kb + 32 * u + kq;
            af[u][mt] = (m < g.M && kk < g.K) ? *(const bf16x8*)(arow + kk) : z;
        }
    }
    auto load_w = [&](int64_t tile, bf16x8 (&wf)[KS]) {
        const int64_t n = tile * 16 + (lane & 15);
        const bf16* wrow = W + (n < g.N ? n : 0) * g.ldb;
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            const int64_t kk = kb + 32 * u + kq;
            wf[u] = (n < g.N && kk < g.K) ? *(const bf16x8*)(wrow + kk) : z;
        }
    };
    TC* C = (TC*)g.C;
    const TX* X = (const TX*)g.aux;
    bf16x8 wc[KS], wn[KS];
    int64_t tile = blockIdx.x;
    if (tile < ntiles) load_w(tile, wc);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t nxt = tile + gridDim.x;
        if (nxt < ntiles) load_w(nxt, wn);
        f32x4 acc[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < KS; ++u)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc[u], af[u][mt], acc[mt], 0, 0, 0);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) red[w][mt][lane] = acc[mt];
        __syncthreads();
        if (w < MT) {  // wave q sums fragment q over the 16 K slices and applies the epilogue
            f32x4 v = red[0][w][lane];
#pragma unroll
            for (int q = 1; q < SK_WAVES; ++q) v += red[q][w][lane];
            const int64_t m = w * 16 + (lane & 15), n = tile * 16 + 4 * (lane >> 4);
            if (m < g.M && n < g.N) {
                epi_apply<EPI, TC, TX>(g, C, X, m, n, v);
                if constexpr (CONV) conv_apply(cv, m, n, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < KS; ++u) wc[u] = wn[u];
    }
}

template <int EPI, typename TC, typename TX, int MT, bool CONV = false>
void launch_pk(const GemmArgs& g, hipStream_t s, const SkinnyConv& cv = {}) {
    const int64_t ntiles = (g.N + 15) / 16;
    const dim3 grid((unsigned)std::min<int64_t>(ntiles, 256));
    const int64_t ks = (g.K + SK_WAVES * 32 - 1) / (SK_WAVES * 32);
    // (KS = 4 would not fit the activation fragments in 128 VGPRs at MT = 4)
    if (ks <= 1)
        hipLaunchKernelGGL((gemm_skinny_pk_kernel<EPI, TC, TX, MT, 1, CONV>), grid, dim3(64 * SK_WAVES), 0, s, g, ntiles, cv);
    else
        hipLaunchKernelGGL((gemm_skinny_pk_kernel<EPI, TC, TX, MT, 2, CONV>), grid, dim3(64 * SK_WAVES), 0, s, g, ntiles, cv);
}

template <int EPI, typename TC, typename TX, bool PART>
void launch_plain(const GemmArgs& g, int mt, int ks, hipStream_t s) {
    const dim3 grid((unsigned)((g.N + 15) / 16), (unsigned)ks);
    if (mt == 1) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TC, TX, 1, PART>), grid, dim3(64 * SK_WAVES), 0, s, g);
    else if (mt == 2) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TC, TX, 2, PART>), grid, dim3(64 * SK_WAVES), 0, s, g);
    else if (mt == 3) hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TC, TX, 3, PART>), grid, dim3(64 * SK_WAVES), 0, s, g);
    else hipLaunchKernelGGL((gemm_skinny_kernel<EPI, TC, TX, 4, PART>), grid, dim3(64 * SK_WAVES), 0, s, g);
}

template <int EPI, typename TC, typename TX>
void launch_mt(GemmArgs g, size_t ws_bytes, hipStream_t s) {
    const int mt = (int)((g.M + 15) / 16);
    if (g.K <= SK_WAVES * 2 * 32) {
        if (mt == 1) launch_pk<EPI, TC, TX, 1>(g, s);
        else if (mt == 2) launch_pk<EPI, TC, TX, 2>(g, s);
        else if (mt == 3) launch_pk<EPI, TC, TX, 3>(g, s);
        else launch_pk<EPI, TC, TX, 4>(g, s);
        return;
    }
    int64_t kper;
    const int ks = skinny_ksplit(g.M, g.N, g.K, &kper);
    if (ks > 1 && g.ws && ws_bytes >= skinny_ws_bytes(g.M, g.N, g.K)) {
        g.kper = kper;
        launch_plain<EPI, TC, TX, true>(g, mt, ks, s);
        hipLaunchKernelGGL((skinny_reduce_kernel<EPI, TC, TX>), dim3((unsigned)((g.M * (g.N / 4) + 255) / 256)),
                           dim3(256), 0, s, g, ks);
        return;
    }
    launch_plain<EPI, TC, TX, false>(g, mt, 1, s);
}

template <typename TC>
bool launch_epi(const GemmArgs& g, int epi, int aux_dtype, size_t wsb, hipStream_t s) {
    switch (epi) {
        case MSQ_EPI_NONE: launch_mt<MSQ_EPI_NONE, TC, float>(g, wsb, s); return true;
        case MSQ_EPI_BIAS: launch_mt<MSQ_EPI_BIAS, TC, float>(g, wsb, s); return true;
        case MSQ_EPI_BIAS_RELU: launch_mt<MSQ_EPI_BIAS_RELU, TC, float>(g, wsb, s); return true;
        case MSQ_EPI_BIAS_RESID:
            if (aux_dtype == MSQ_BF16) launch_mt<MSQ_EPI_BIAS_RESID, TC, bf16>(g, wsb, s);
            else launch_mt<MSQ_EPI_BIAS_RESID, TC, float>(g, wsb, s);
            return true;
        default: return false;  // ACCUM / RELU_MASK / dropout: not decode shapes
    }
}

}  // namespace

// split-K of a skinny product whose K > 1024 (the per-slice kernel, not the
// persistent one) and whose 16-row W slices alone would leave most CUs idle
// (the decode FFN2, N 1024 x K 4096: 64 slices -> 4 K slices of 1024 each)
int skinny_ksplit(int64_t M, int64_t N, int64_t K, int64_t* kper) {
    const int64_t ntiles = (N + 15) / 16;
    *kper = K;
    if (M > 64 || K <= SK_WAVES * 2 * 32 || ntiles >= 128 || N % 4) return 1;
    const int64_t want = std::min<int64_t>((256 + ntiles - 1) / ntiles, K / 1024);
    if (want <= 1) return 1;
    const int64_t q = SK_WAVES * 32;  // whole k-steps for every wave of a slice
    *kper = ((K + want - 1) / want + q - 1) / q * q;
    return (int)((K + *kper - 1) / *kper);
}
size_t skinny_ws_bytes(int64_t M, int64_t N, int64_t K) {
    int64_t kper;
    const int ks = skinny_ksplit(M, N, K, &kper);
    return ks > 1 ? (size_t)ks * M * N * 4 : 0;
}

// M <= 64, A [M][K] and W [N][K] bf16 (ta = tb = 0), one batch; false when
// the problem is outside these conditions (the caller then uses the tiles)
bool gemm_skinny_launch(const GemmArgs& g, int ta, int tb, int epi, int c_dtype, int aux_dtype, size_t ws_bytes,
                        hipStream_t s) {
    if (ta || tb || g.batch != 1 || g.M > 64 || g.K % 8 || g.lda % 8 || g.ldb % 8) return false;
    if (epi != MSQ_EPI_NONE && epi != MSQ_EPI_BIAS && epi != MSQ_EPI_BIAS_RELU && epi != MSQ_EPI_BIAS_RESID)
        return false;
    return c_dtype == MSQ_BF16 ? launch_epi<bf16>(g, epi, aux_dtype, ws_bytes, s)
                                : launch_epi<float>(g, epi, aux_dtype, ws_bytes, s);
}

// Mamba2 decode step, first half of a mixer: zx = x . in_w^T (bf16 [B][d_in_proj],
// msq_gemm's skinny product) and, in the same launch, the conv step of the new
// row (msq_mamba_conv_step: xc, conv_state). Outside the fused kernel's range
// (B > 64 rows, d_model > 1024) the two launches run instead.
extern "C" int msq_mamba_in_proj_conv_step(void* zx, int64_t ldz, void* xc, int64_t ldxc, float* conv_state,
                                           const void* x, int64_t ldx, const void* in_w, int64_t ldw,
                                           const float* conv_w, const float* conv_b, int64_t B, int64_t d_model,
                                           int64_t d_in_proj, int64_t d_inner, int64_t nheads, void* stream) {
    const int64_t cd = d_inner + 2 * 64;
    MSQ_CHECK_ARG(zx && xc && conv_state && x && in_w && conv_w && conv_b && B > 0 && d_model > 0 && nheads > 0 &&
                      d_inner == nheads * 64 && d_in_proj == d_inner + cd + nheads && ldz >= d_in_proj &&
                      ldxc >= cd && ldx >= d_model && ldw >= d_model,
                  "msq_mamba_in_proj_conv_step: bad args");
    hipStream_t s = (hipStream_t)stream;
    const bool fused = B <= 64 && d_model <= SK_WAVES * 2 * 32 && d_model % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0 &&
                       ldz % 4 == 0 && ldxc % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)in_w % 16 == 0 &&
                       (uintptr_t)zx % 16 == 0 && (uintptr_t)xc % 8 == 0 && (uintptr_t)conv_state % 16 == 0 &&
                       (uintptr_t)conv_w % 16 == 0 && (uintptr_t)conv_b % 16 == 0;
    if (!fused) {
        const int rc = msq_gemm_ex(MSQ_BF16, 0, 0, B, d_in_proj, d_model, x, ldx, 0, in_w, ldw, 0, zx, MSQ_BF16, ldz, 0,
                                   1, MSQ_EPI_NONE, nullptr, nullptr, MSQ_F32, 0, 0, 0u, 0u, 0.f, nullptr, 0, stream);
        if (rc != MSQ_OK) return rc;
        return msq_mamba_conv_step(xc, ldxc, conv_state, zx, ldz, MSQ_BF16, conv_w, conv_b, B, d_inner, nheads,
                                   stream);
    }
    GemmArgs g{};
    g.M = B; g.N = d_in_proj; g.K = d_model;
    g.A = x; g.lda = ldx;
    g.B = in_w; g.ldb = ldw;
    g.C = zx; g.ldc = ldz;
    g.batch = 1;
    g.vec = 1;
    const SkinnyConv cv{(bf16*)xc, ldxc, conv_state, conv_w, conv_b, d_inner, cd};
    const int mt = (int)((B + 15) / 16);
    if (mt == 1) launch_pk<MSQ_EPI_NONE, bf16, float, 1, true>(g, s, cv);
    else if (mt == 2) launch_pk<MSQ_EPI_NONE, bf16, float, 2, true>(g, s, cv);
    else if (mt == 3) launch_pk<MSQ_EPI_NONE, bf16, float, 3, true>(g, s, cv);
    else launch_pk<MSQ_EPI_NONE, bf16, float, 4, true>(g, s, cv);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ---------------------------------------------------------------------------
// Decode step: residual product + the next LayerNorm in the split-K reduce.
//   C = aux + A . W^T + bias   (fp32 [M][N], the residual stream)
//   Y = LayerNorm(C rows; gamma, beta, eps)   (the next product's input)
// The skinny product runs split over K into fp32 partials (gemm_skinny_kernel
// PART), and one workgroup per ROW then owns the whole row: it sums the
// partials in slice order, adds bias and residual (epi_apply's order), stores
// C, and normalises the row it already holds -- the LayerNorm that otherwise
// follows as its own launch (model_transformer.py:115,119: ln2 after the
// proj residual, the next block's ln1 / ln_f after the FFN residual).
template <typename TY, int NC>
__global__ __launch_bounds__(256) void skinny_reduce_ln_kernel(GemmArgs g, int ks, const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float eps,
                                                               TY* __restrict__ Y, int64_t ldy) {
    __shared__ float red[2][4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t m = blockIdx.x, MN = g.M * g.N;
    const float* X = (const float*)g.aux;
    float* C = (float*)g.C;
    f32x4 v[NC];
    float s1 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int64_t n = (int64_t)(c * 256 + tid) * 4;
        v[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (n < g.N) {
            f32x4 t = load4(g.ws + m * g.N + n);
            for (int s = 1; s < ks; ++s) t += load4(g.ws + s * MN + m * g.N + n);
            if (g.bias) t += load4(g.bias + n);
            t += load4(X + m * g.ldx + n);
            store4(C + m * g.ldc + n, t);
            v[c] = t;
            s1 += (t[0] + t[1]) + (t[2] + t[3]);
        }
    }
    s1 = wave_sum(s1);
    if (lane == 0) red[0][w] = s1;
    __syncthreads();
    const float mu = ((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) / (float)g.N;
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int64_t n = (int64_t)(c * 256 + tid) * 4;
        if (n < g.N) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float z = v[c][t] - mu;
                s2 += z * z;
            }
        }
    }
    s2 = wave_sum(s2);
    if (lane == 0) red[1][w] = s2;
    __syncthreads();
    const float rs = rsqrtf(((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])) / (float)g.N + eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int64_t n = (int64_t)(c * 256 + tid) * 4;
        if (n < g.N) {
            const f32x4 gm = load4(gamma + n), bt = load4(beta + n);
            f32x4 o;
#pragma unroll
            for (int t = 0; t < 4; ++t) o[t] = (v[c][t] - mu) * rs * gm[t] + bt[t];
            store4(Y + m * ldy + n, o);
        }
    }
}

// K slices of the fused path: the skinny split (FFN2, K = 4096: 4), at least 2
// (a K <= 1024 product otherwise runs the persistent kernel, whose epilogue
// cannot see whole rows)
static int resid_ln_ksplit(int64_t M, int64_t N, int64_t K, int64_t* kper) {
    int ks = skinny_ksplit(M, N, K, kper);
    if (ks <= 1) {
        const int64_t q = SK_WAVES * 32;
        *kper = ((K + 1) / 2 + q - 1) / q * q;
        ks = (int)((K + *kper - 1) / *kper);
    }
    return ks;
}
static bool resid_ln_fused(int dtype, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldw, int64_t ldc,
                           int64_t ldx, const void* A, const void* W, const float* C, const float* aux,
                           const float* bias, const void* Y, int y_dtype, int64_t ldy) {
    return dtype == MSQ_BF16 && M <= 64 && N % 4 == 0 && N <= 4096 && K % 8 == 0 && lda % 8 == 0 && ldw % 8 == 0 &&
           ldc % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (y_dtype == MSQ_BF16 || y_dtype == MSQ_F32) &&
           ((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)aux | (uintptr_t)Y) % 16 == 0 &&
           (!bias || (uintptr_t)bias % 16 == 0);
}

extern "C" int64_t msq_gemm_resid_ln_workspace(int dtype, int64_t M, int64_t N, int64_t K, int64_t lda,
                                               int64_t ldw) {
    // fused: the fp32 partials; otherwise msq_gemm_ex's workspace + LayerNorm mean / rstd
    int64_t kper;
    const int64_t fused = (int64_t)resid_ln_ksplit(M, N, K, &kper) * M * N * 4;
    const int64_t plain = msq_gemm_workspace_size(dtype, 0, 0, M, N, K, lda, ldw, 1, MSQ_EPI_BIAS_RESID);
    return std::max(fused, (plain + 255) / 256 * 256 + 2 * M * 4);
}

// C = aux + A . W^T + bias (fp32), Y = LayerNorm(C) (y_dtype): see
// skinny_reduce_ln_kernel. Outside the fused shapes (M > 64, N > 4096, fp32
// operands, ...) it runs msq_gemm_ex + msq_layernorm_fwd.
extern "C" int msq_gemm_resid_ln(int dtype, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                                 const void* W, int64_t ldw, float* C, int64_t ldc, const float* bias,
                                 const float* aux, int64_t ldx, const float* gamma, const float* beta, float eps,
                                 void* Y, int y_dtype, int64_t ldy, void* ws, int64_t ws_bytes, void* stream) {
    MSQ_CHECK_ARG(M > 0 && N > 0 && K > 0 && A && W && C && aux && gamma && beta && Y && ldc >= N && ldx >= N &&
                      ldy >= N && lda >= K && ldw >= K,
                  "msq_gemm_resid_ln: bad args");
    MSQ_CHECK_ARG(ws && ws_bytes >= msq_gemm_resid_ln_workspace(dtype, M, N, K, lda, ldw) && (uintptr_t)ws % 16 == 0,
                  "msq_gemm_resid_ln: workspace of msq_gemm_resid_ln_workspace() bytes, 16-B aligned");
    hipStream_t s = (hipStream_t)stream;
    if (!resid_ln_fused(dtype, M, N, K, lda, ldw, ldc, ldx, A, W, C, aux, bias, Y, y_dtype, ldy)) {
        // msq_layernorm_fwd reads C and writes Y densely: checked before anything is written
        MSQ_CHECK_ARG(ldc == N && ldy == N, "msq_gemm_resid_ln: the unfused path needs ldc == N and ldy == N");
        const int64_t plain = msq_gemm_workspace_size(dtype, 0, 0, M, N, K, lda, ldw, 1, MSQ_EPI_BIAS_RESID);
        const int64_t off = (plain + 255) / 256 * 256;
        int rc = msq_gemm_ex(dtype, 0, 0, M, N, K, A, lda, 0, W, ldw, 0, C, MSQ_F32, ldc, 0, 1, MSQ_EPI_BIAS_RESID,
                             bias, aux, MSQ_F32, ldx, 0, 0u, 0u, 0.f, plain > 0 ? ws : nullptr, plain, stream);
        if (rc != MSQ_OK) return rc;
        float* st = (float*)((char*)ws + off);
        return msq_layernorm_fwd(Y, y_dtype, st, st + M, C, gamma, beta, M, N, eps, 0, 0, stream);
    }
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = lda;
    g.B = W; g.ldb = ldw;
    g.C = C; g.ldc = ldc;
    g.bias = bias;
    g.aux = aux; g.ldx = ldx;
    g.batch = 1;
    g.vec = 1;
    g.ws = (float*)ws;
    int64_t kper;
    const int ks = resid_ln_ksplit(M, N, K, &kper);
    g.kper = kper;
    const int mt = (int)((M + 15) / 16);
    launch_plain<MSQ_EPI_NONE, float, float, true>(g, mt, ks, s);
    const int nc = (int)((N + 1023) / 1024);
#define RL_GO(TY, NCV) \
    hipLaunchKernelGGL((skinny_reduce_ln_kernel<TY, NCV>), dim3((unsigned)M), dim3(256), 0, s, g, ks, gamma, beta, eps, (TY*)Y, ldy)
    if (y_dtype == MSQ_BF16) {
        if (nc == 1) RL_GO(bf16, 1); else if (nc == 2) RL_GO(bf16, 2); else RL_GO(bf16, 4);
    } else {
        if (nc == 1) RL_GO(float, 1); else if (nc == 2) RL_GO(float, 2); else RL_GO(float, 4);
    }
#undef RL_GO
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
