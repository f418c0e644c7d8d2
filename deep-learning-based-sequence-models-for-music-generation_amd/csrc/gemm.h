// Shared declarations of the bf16 / fp32 GEMM kernels (gemm.hip: 128x128
// register-staged tile; gemm256.hip: 256x256 LDS-DMA ping-pong tile).
#pragma once
#include "common.h"

struct GemmArgs {
    int64_t M, N, K;
    const void* A; int64_t lda, sA;
    const void* B; int64_t ldb, sB;
    void* C; int64_t ldc, sC;
    const float* bias;
    const void* aux; int64_t ldx, sX;
    int tiles_m, tiles_n, batch;
    int vec;     // C / aux / bias rows allow 16-B vector access
    int ksplit;  // >1: K range split over blocks, ACCUM epilogue via fp32 atomics
    int64_t kper;
    uint32_t a_ext, b_ext;  // bytes of one batch's A / B extent (256-tile buffer descriptors)
    uint32_t c_ext, x_ext;  // bytes of the C / aux extents (persistent 256 tile's buffer stores / loads)
    // triangular K ranges of the relative-attention products (128 tile only):
    // 1 = rows m are (segment, i = m % seg) and need k >= seg-1-i (dq = dQR.R);
    // 2 = K is nseg segments of seg rows, tile rows m = r need k%seg >= seg-1-r (dR)
    int tri;
    int64_t seg;
    // MSQ_EPI_BIAS_DROP_RESID: drop_base = drop_base(seed, site), keep iff bits >= drop_thr
    uint32_t drop_base, drop_thr;
    float drop_scale;
    // split-K partials (ACCUM, ksplit > 1): slice s of batch z at
    // ws + ((s * batch + z) * M) * N (N % 4 == 0); null = fp32 atomics into C
    float* ws;
    // global row of local row 0 (the dropout hash is keyed by the global row)
    int64_t m_off;
    // column sums of the written C (msq_gemm_colsum): per-(M-tile, wave-row)
    // partials [tiles_m * 2][N], reduced in a fixed order afterwards
    float* cs_ws;
    // bytes at ws (msq_gemm_ex's workspace) for the persistent tile's K-split
    // tail: its last tail_tiles tiles run as tail_s K slices of tail_kst
    // k-steps into fp32 partials at ws, summed with the epilogue afterwards
    // (gemm256p.hip; 0 = off)
    int64_t ws_bytes;
    int tail_tiles, tail_s, tail_kst;
};

// bytes of the split-K partial workspace an ACCUM product with this split needs
inline size_t splitk_ws_bytes(int64_t M, int64_t N, int64_t batch, int ksplit) {
    return ksplit > 1 && N % 4 == 0 ? (size_t)ksplit * batch * M * N * 4 : 0;
}
// C[z][m][n] += sum_s ws[s][z][m][n] (gemm.hip)
void splitk_reduce(const GemmArgs& g, hipStream_t s);

// dropout(v + bias) of one lane's 4 outputs C[m][n..n+3] (nn.Dropout, common.h hash)
__device__ __forceinline__ f32x4 epi_drop(const GemmArgs& g, int64_t m, int64_t n, f32x4 v) {
    const uint32_t rk = drop_row(g.drop_base, (uint32_t)(m + g.m_off));
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = drop_bits(rk, (uint32_t)(n + t)) >= g.drop_thr ? v[t] * g.drop_scale : 0.f;
    return v;
}

template <typename TC>
__device__ __forceinline__ void epi_store(TC* p, f32x4 v, int nv) {
    if (nv == 4) {
        store4(p, v);
    } else {
        const int n = nv < 0 ? -nv : nv;
        for (int i = 0; i < n; ++i) p[i] = (TC)v[i];
    }
}
// load up to 4 elements (nv as in epi_store)
template <typename T>
__device__ __forceinline__ f32x4 epi_load(const T* p, int nv) {
    if (nv == 4) return load4(p);
    const int n = nv < 0 ? -nv : nv;
    f32x4 x = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < n; ++i) x[i] = (float)p[i];
    return x;
}

// epilogues that read the aux operand (their loads can be issued ahead of the stores)
template <int EPI>
constexpr bool epi_reads_aux() {
    return EPI == MSQ_EPI_RELU_MASK || EPI == MSQ_EPI_BIAS_RESID || EPI == MSQ_EPI_BIAS_DROP_RESID;
}
template <typename TX>
__device__ __forceinline__ f32x4 epi_aux_load(const GemmArgs& g, const TX* X, int64_t m, int64_t n) {
    const int nv = g.vec ? (int)min<int64_t>(4, g.N - n) : -(int)min<int64_t>(4, g.N - n);
    return epi_load(X + m * g.ldx + n, nv);
}
// MSQ_MASK1 aux: one uint32 word per 32 columns (g.ldx in words); the mask
// bits of C[m][n..n+3] (n % 4 == 0: one word) as 0 / 1
struct mask1_t {
    uint32_t w;
};
__device__ __forceinline__ f32x4 mask1_bits(uint32_t w, int64_t n) {
    const uint32_t b = w >> (n & 31);
    return (f32x4){(float)(b & 1u), (float)((b >> 1) & 1u), (float)((b >> 2) & 1u), (float)((b >> 3) & 1u)};
}
__device__ __forceinline__ f32x4 epi_aux_load(const GemmArgs& g, const mask1_t* X, int64_t m, int64_t n) {
    return mask1_bits(X[m * g.ldx + (n >> 5)].w, n);
}

// Applies the epilogue to one lane's 4 consecutive outputs C[m][n..n+3]
// (xpre: the aux vector, already loaded).
template <int EPI, typename TC, typename TX>
__device__ __forceinline__ f32x4 epi_apply(const GemmArgs& g, TC* C, const TX* X, int64_t m, int64_t n, f32x4 v,
                                           float* wsp = nullptr, const f32x4* xpre = nullptr) {
    if (EPI == MSQ_EPI_ACCUM && wsp) {  // split-K partial, reduced by splitk_reduce
        store4(wsp + m * g.N + n, v);
        return v;
    }
    const int nv = g.vec ? (int)min<int64_t>(4, g.N - n) : -(int)min<int64_t>(4, g.N - n);
    if ((EPI == MSQ_EPI_BIAS || EPI == MSQ_EPI_BIAS_RELU || EPI == MSQ_EPI_BIAS_RESID ||
         EPI == MSQ_EPI_BIAS_DROP_RESID) && g.bias)
        v += epi_load(g.bias + n, nv);
    if constexpr (EPI == MSQ_EPI_BIAS_DROP_RESID) v = epi_drop(g, m, n, v) + (xpre ? *xpre : epi_load(X + m * g.ldx + n, nv));
    if (EPI == MSQ_EPI_BIAS_RELU) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = fmaxf(v[t], 0.f);
    }
    if constexpr (EPI == MSQ_EPI_BIAS_RESID) v += xpre ? *xpre : epi_load(X + m * g.ldx + n, nv);
    if (EPI == MSQ_EPI_RELU_MASK) {
        const f32x4 x = xpre ? *xpre : epi_aux_load(g, X, m, n);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = x[t] > 0.f ? v[t] : 0.f;
    }
    TC* cp = C + m * g.ldc + n;
    if (EPI == MSQ_EPI_ACCUM && g.ksplit > 1) {
        const int na = nv < 0 ? -nv : nv;
        for (int t = 0; t < na; ++t) atomicAdd((float*)cp + t, v[t]);
        return v;
    }
    if (EPI == MSQ_EPI_ACCUM) v += epi_load(cp, nv);
    epi_store(cp, v, nv);
    return v;  // the value written (before its rounding to TC)
}

// 256x256 kernel family: returns false when the problem does not fit its
// preconditions (the caller then uses the 128x128 kernel).
bool gemm256_launch(GemmArgs g, int ta, int tb, int epi, int c_dtype, int aux_dtype, size_t ws_bytes,
                    hipStream_t s);
// persistent 256 tile (forward / dX products: no ACCUM, one batch, N % 8 == 0,
// 16-B aligned C / aux / bias); false when it does not apply
bool gemm256p_launch(GemmArgs g, int ta, int tb, int epi, int c_dtype, int aux_dtype, hipStream_t s);
// whether gemm256p_launch would take this product
bool gemm256p_applies(GemmArgs g, int ta, int tb, int epi, int c_dtype, int aux_dtype);
// workspace bytes of the persistent tile's K-split tail for this product (0: none)
size_t gemm256p_tail_ws_bytes(int64_t M, int64_t N, int64_t K, int epi, int aux_dtype);
// persistent tile with the column-sum partials of gemm256_colsum_launch (g.cs_ws set,
// reduced by the caller); false when it does not apply
bool gemm256p_colsum_launch(GemmArgs g, int ta, int tb, int epi, int aux_dtype, hipStream_t s);
// persistent tile, bias epilogue + column (max, sum exp) partials of the stored bf16
// C per (256-row tile, wave-row) p: part[2p][n] = max, part[2p+1][n] = sum (row stride
// pld); false when it does not apply
bool gemm256p_colstats_applies(GemmArgs g, int tb, const float* part, int64_t pld);
bool gemm256p_colstats_launch(GemmArgs g, int ta, int tb, float* part, int64_t pld, hipStream_t s);
// skinny-M weight-streaming kernel of the decode steps (gemm_skinny.hip):
// false when the problem is not M <= 64 / ta = tb = 0 / a forward epilogue
bool gemm_skinny_launch(const GemmArgs& g, int ta, int tb, int epi, int c_dtype, int aux_dtype, size_t ws_bytes,
                        hipStream_t s);
// K slices of a split-K skinny product (1: none) and the fp32 partial bytes it needs in ws
int skinny_ksplit(int64_t M, int64_t N, int64_t K, int64_t* kper);
size_t skinny_ws_bytes(int64_t M, int64_t N, int64_t K);
// 256 tile with the column sums of C (epilogue NONE / RELU_MASK, C bf16,
// N % 4 == 0): dbias[n] (+)= sum_m C[m][n] (fp32, before C's rounding);
// ws >= gemm256_colsum_ws_bytes(M, N); false when the 256 tile does not apply
bool gemm256_colsum_launch(GemmArgs g, int ta, int tb, int epi, int aux_dtype, float* dbias, int accumulate,
                           float* ws, size_t ws_bytes, hipStream_t s);
inline size_t gemm256_colsum_ws_bytes(int64_t M, int64_t N) { return (size_t)((M + 255) / 256) * 2 * N * 4; }
// fills tiles / ksplit / kper (and descriptor extents) of the 256 tile; false if it does not apply
bool gemm256_plan(GemmArgs& g, int ta, int tb, int epi);

// bf16 GEMM with a triangular K range (GemmArgs::tri); same operand conventions as msq_gemm
int gemm_bf16_tri(int tri, int64_t seg, int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                  int64_t sA, const void* B, int64_t ldb, int64_t sB, void* C, int c_dtype, int64_t ldc, int64_t sC,
                  int64_t batch, int epi, const void* aux, int aux_dtype, int64_t ldx, int64_t sX, hipStream_t s,
                  float* ws = nullptr, size_t ws_bytes = 0);
// K split gemm_bf16_tri uses (its split-K workspace: splitk_ws_bytes(M, N, batch, this))
int gemm_bf16_tri_ksplit(int tri, int64_t M, int64_t N, int64_t K, int64_t seg, int64_t batch);
extern "C" int msq_gemm_ex(int dtype, int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                           int64_t strideA, const void* B, int64_t ldb, int64_t strideB, void* C, int c_dtype,
                           int64_t ldc, int64_t strideC, int64_t batch, int epilogue, const float* bias,
                           const void* aux, int aux_dtype, int64_t ld_aux, int64_t stride_aux, uint32_t seed,
                           uint32_t site, float p, void* ws, int64_t ws_bytes, void* stream);
