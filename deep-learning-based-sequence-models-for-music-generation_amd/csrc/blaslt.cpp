// Plain bf16 products (no fused epilogue, or a bias / bias+ReLU epilogue)
// through hipBLASLt, the vendor GEMM library. Measured on the cfg-2 train-step
// shapes (tools/gemm_vs_blas.py, tools/gemm_square.py): hipBLASLt's kernels
// run the forward / dX products 10-35 % faster than the 256x256 tile of
// gemm256.hip and the weight-gradient (K = B*S) products slower, so
// msq_gemm_ex routes only the former here; the fused epilogues (dropout +
// residual, ReLU mask, column sums) and the accumulate products stay on the
// hand-written tiles. MSQ_NO_BLASLT=1 disables the route; MSQ_BLASLT_TUNE=1
// times hipBLASLt's candidate algorithms on the first call of a shape (a few %
// on some shapes; off by default because timing picks are not reproducible
// across processes).
//
// Layouts: msq_gemm's C[M][N] (row major, ldc) = op(A) op(B) with A [M][K]
// (ta = 0) or [K][M] (ta = 1) and B [N][K] (tb = 0) or [K][N] (tb = 1), all
// row major. hipBLASLt is column major, so the call computes
// C^T [N x M] = op(B)^T op(A)^T with our B as its A operand and our A as its B.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "../../include/midiseq.h"

namespace {

constexpr int NCAND = 8;

struct Plan {
    hipblasLtMatmulDesc_t op = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    size_t ws = 0;
    bool ok = false, tuned = false;
    float best_ms = 0.f;
    int ncand = 0;
    hipblasLtMatmulHeuristicResult_t cand[NCAND];
};

typedef std::tuple<int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int64_t, int64_t, int64_t,
                   int64_t>
    Key;

std::mutex g_mu;
hipblasLtHandle_t g_h = nullptr;
bool g_init_failed = false;
std::map<Key, Plan> g_plans;
void* g_ws = nullptr;
constexpr size_t WS_BYTES = 64ull << 20;

bool init_locked() {
    if (g_h) return true;
    if (g_init_failed) return false;
    if (hipblasLtCreate(&g_h) != HIPBLAS_STATUS_SUCCESS || hipMalloc(&g_ws, WS_BYTES) != hipSuccess) {
        g_init_failed = true;
        g_h = nullptr;
        return false;
    }
    return true;
}

Plan make_plan(int ta, int tb, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int c_dtype,
               int epilogue, int64_t batch, int64_t sA, int64_t sB, int64_t sC) {
    Plan p;
    if (hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
    // hipBLASLt A := our B (N x K after op), B := our A (K x M after op)
    const hipblasOperation_t opA = tb ? HIPBLAS_OP_N : HIPBLAS_OP_T;
    const hipblasOperation_t opB = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA));
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB));
    if (epilogue != MSQ_EPI_NONE) {
        const hipblasLtEpilogue_t e = epilogue == MSQ_EPI_BIAS_RELU ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
        const hipDataType bt = HIP_R_32F;  // msq bias vectors are fp32 (bias[n]: per row of C^T)
        hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
        hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    }
    // column-major storage shapes: our row-major [R][C] with ld is col-major [C][R]
    const uint64_t a_rows = tb ? N : K, a_cols = tb ? K : N;  // our B
    const uint64_t b_rows = ta ? M : K, b_cols = ta ? K : M;  // our A
    const hipDataType ct = c_dtype == MSQ_BF16 ? HIP_R_16BF : HIP_R_32F;
    if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, a_rows, a_cols, ldb) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, b_rows, b_cols, lda) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lc, ct, N, M, ldc) != HIPBLAS_STATUS_SUCCESS)
        return p;
    if (batch > 1) {
        const int32_t bc = (int32_t)batch;
        const int64_t strides[3] = {sB, sA, sC};  // hipBLASLt A = our B, B = our A
        hipblasLtMatrixLayout_t ls[3] = {p.la, p.lb, p.lc};
        for (int i = 0; i < 3; ++i) {
            hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc));
            hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &strides[i],
                                              sizeof(int64_t));
        }
    }
    hipblasLtMatmulPreference_t pref;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
    const uint64_t wsb = WS_BYTES;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[NCAND];
    int n = 0;
    const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(g_h, p.op, p.la, p.lb, p.lc, p.lc, pref, NCAND, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return p;
    p.ncand = 0;
    for (int i = 0; i < n; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= WS_BYTES) p.cand[p.ncand++] = res[i];
    if (p.ncand == 0) return p;
    p.algo = p.cand[0].algo;
    p.ws = p.cand[0].workspaceSize;
    p.ok = true;
    return p;
}

// First call of a shape: time every candidate algorithm twice on these
// buffers (beta = 0 into a scratch output, so accumulating products are not
// disturbed) and keep the fastest; the heuristic's first choice was up to 2x
// off the best on the weight-gradient shapes. Skipped while the stream is
// being captured into a graph (the plan then keeps the heuristic's choice).
void autotune(Plan& p, const void* A, const void* B, int64_t M, int64_t ldc, int64_t batch, int64_t sC, int c_dtype,
              const float* bias, hipStream_t s) {
    p.tuned = true;
    if (p.ncand < 2) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
    const size_t esz = c_dtype == MSQ_BF16 ? 2 : 4;
    const size_t cbytes = (size_t)((batch > 1 ? sC * (batch - 1) : 0) + ldc * M) * esz;
    void* scratch = nullptr;
    if (hipMalloc(&scratch, cbytes) != hipSuccess) return;
    if (bias) hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const float alpha = 1.f, beta = 0.f;
    float best = 1e30f;
    int bi = 0;
    for (int i = 0; i < p.ncand; ++i) {
        float ms = 1e30f;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0, s);
            const hipblasStatus_t st = hipblasLtMatmul(g_h, p.op, &alpha, B, p.la, A, p.lb, &beta, scratch, p.lc,
                                                       scratch, p.lc, &p.cand[i].algo, g_ws, p.cand[i].workspaceSize, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float t = 1e30f;
            if (st == HIPBLAS_STATUS_SUCCESS) hipEventElapsedTime(&t, e0, e1);
            ms = t;  // the second run (warm)
        }
        if (ms < best) {
            best = ms;
            bi = i;
        }
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipStreamSynchronize(s);
    hipFree(scratch);
    p.algo = p.cand[bi].algo;
    p.ws = p.cand[bi].workspaceSize;
    p.best_ms = best;
}

}  // namespace

// 1 = done, 0 = not handled (caller runs its own kernel), -1 = hipBLASLt error.
// epilogue NONE / BIAS / BIAS_RELU (C = result), or ACCUM (fp32 C += result);
// batch > 1: strided batches (element strides sA, sB, sC)
int blaslt_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                int64_t ldb, void* C, int c_dtype, int64_t ldc, int epilogue, const float* bias, hipStream_t s,
                int64_t batch, int64_t sA, int64_t sB, int64_t sC) {
    static const bool off = getenv("MSQ_NO_BLASLT") != nullptr;
    if (off) return 0;
    if (epilogue != MSQ_EPI_NONE && epilogue != MSQ_EPI_BIAS && epilogue != MSQ_EPI_BIAS_RELU &&
        epilogue != MSQ_EPI_ACCUM)
        return 0;
    if ((epilogue == MSQ_EPI_BIAS || epilogue == MSQ_EPI_BIAS_RELU) != (bias != nullptr)) return 0;
    if (epilogue == MSQ_EPI_ACCUM && c_dtype != MSQ_F32) return 0;
    const int epi_l = epilogue == MSQ_EPI_ACCUM ? MSQ_EPI_NONE : epilogue;  // accumulation is beta = 1
    Plan p;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!init_locked()) return 0;
        const Key k{ta, tb, M, N, K, lda, ldb, ldc, c_dtype, epi_l, batch, sA, sB, sC};
        auto it = g_plans.find(k);
        if (it == g_plans.end())
            it = g_plans.emplace(k, make_plan(ta, tb, M, N, K, lda, ldb, ldc, c_dtype, epi_l, batch, sA, sB, sC)).first;
        // opt-in: timing picks can differ between processes (DDP ranks would
        // then round differently), so the default is the heuristic's choice
        static const bool tune = getenv("MSQ_BLASLT_TUNE") != nullptr;
        if (it->second.ok && !it->second.tuned && tune)
            autotune(it->second, A, B, M, ldc, batch, sC, c_dtype, epi_l != MSQ_EPI_NONE ? bias : nullptr, s);
        p = it->second;
    }
    if (!p.ok) return 0;
    if (epi_l != MSQ_EPI_NONE)
        hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
    const float alpha = 1.f, beta = epilogue == MSQ_EPI_ACCUM ? 1.f : 0.f;
    const hipblasStatus_t st = hipblasLtMatmul(g_h, p.op, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &p.algo,
                                               g_ws, p.ws, s);
    return st == HIPBLAS_STATUS_SUCCESS ? 1 : -1;
}
