// Ablation harness for the 256x256 GEMM tile (not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lab/gemm256_lab.hip -o tools/lab/gemm256_lab
// Runs the FFN1 forward shape (65728 x 4096 x 1024, bf16 out) under each LAB
// switch combination and prints ms / TFLOP/s.
#include "../../deep-learning-based-sequence-models-for-music-generation_amd/csrc/gemm256.hip"
#include <cstdio>
#include <vector>

int msq_set_error(int code, const char*, ...) { return code; }
void splitk_reduce(const GemmArgs&, hipStream_t) {}

__global__ void fill(bf16* p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (bf16)(((int)(x & 0xFFFF) - 32768) / 32768.0f);
    }
}

static int g_ta = 0, g_tb = 0;
template <int LAB, int TA, int TB>
float run_t(GemmArgs g, int iters) {
    auto k = gemm256_kernel<TA, TB, MSQ_EPI_NONE, bf16, float, LAB>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * HALF);
    const int nblk = g.tiles_m * g.tiles_n * g.batch * g.ksplit;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), 8 * HALF, 0, g);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, dim3(nblk), dim3(NT), 8 * HALF, 0, g);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / iters;
}
template <int LAB>
float run(GemmArgs g, int iters) {
    if (g_ta && g_tb) return run_t<LAB, 1, 1>(g, iters);
    if (g_tb) return run_t<LAB, 0, 1>(g, iters);
    return run_t<LAB, 0, 0>(g, iters);
}

int main(int argc, char** argv) {
    int64_t M = 65728, N = 4096, K = 1024;
    int ksplit = 1;
    if (argc > 3) { M = atoll(argv[1]); N = atoll(argv[2]); K = atoll(argv[3]); }
    if (argc > 5) { g_ta = atoi(argv[4]); g_tb = atoi(argv[5]); }
    if (argc > 6) ksplit = atoi(argv[6]);
    bf16 *A, *B, *C;
    (void)hipMalloc(&A, M * K * 2);
    (void)hipMalloc(&B, N * K * 2);
    (void)hipMalloc(&C, M * N * 4);
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, A, M * K, 1u);
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, B, N * K, 2u);
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = g_ta ? M : K; g.B = B; g.ldb = g_tb ? N : K; g.C = C; g.ldc = N;
    g.batch = 1; g.vec = 1; g.ksplit = ksplit;
    g.kper = ((K + ksplit - 1) / ksplit + 63) / 64 * 64;
    g.tiles_m = (int)((M + 255) / 256); g.tiles_n = (int)((N + 255) / 256);
    g.a_ext = (uint32_t)(M * K * 2); g.b_ext = (uint32_t)(N * K * 2);
    const double fl = 2.0 * M * N * K;
    struct V { const char* name; float (*fn)(GemmArgs, int); };
    V vs[] = {{"full", run<0>}, {"no-dma", run<1>}, {"no-mfma", run<2>}, {"no-dma,no-mfma", run<3>},
              {"no-stagger", run<4>}, {"no-store", run<16>}, {"full(again)", run<0>}};
    printf("M=%lld N=%lld K=%lld ta=%d tb=%d ksplit=%d\n", (long long)M, (long long)N, (long long)K, g_ta, g_tb, ksplit);
    for (auto& v : vs) {
        float ms = v.fn(g, 20);
        printf("%-22s %8.3f ms  %7.1f TFLOP/s\n", v.name, ms, fl / ms / 1e9);
    }
    return 0;
}
