// Timing harness for the streaming filtered-CE passes at the train step's
// size (B 32, T 2048, V 17914, bf16 logits, ld 17920); not part of the
// library. Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lab/loss_lab.hip -o tools/lab/loss_lab
#include "../../deep-learning-based-sequence-models-for-music-generation_amd/csrc/loss.hip"
#include <cstdio>
#include <vector>

int msq_set_error(int code, const char*, ...) { return code; }

__global__ void fill_bf(bf16* p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (bf16)(((int)(x & 0xFFFF) - 32768) / 4096.0f);
    }
}

// roofline references: the same access pattern as finish2 without the math
__global__ __launch_bounds__(256) void copy_kernel(const bf16* __restrict__ o, bf16* __restrict__ d, int64_t ld,
                                                   int64_t T, int64_t V) {
    const int v = (blockIdx.x * 256 + threadIdx.x) * 8;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (T + 31) / 32, t0 = ts * per, t1 = min(T, t0 + per);
    if (v >= V) return;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t row = b * T + t;
        *(bf16x8*)(d + row * ld + v) = *(const bf16x8*)(o + row * ld + v);
    }
}
__global__ __launch_bounds__(256) void read_kernel(const bf16* __restrict__ o, float* __restrict__ out, int64_t ld,
                                                   int64_t T, int64_t V) {
    const int v = (blockIdx.x * 256 + threadIdx.x) * 8;
    const int64_t b = blockIdx.y, ts = blockIdx.z;
    const int64_t per = (T + 31) / 32, t0 = ts * per, t1 = min(T, t0 + per);
    if (v >= V) return;
    float s = 0.f;
    for (int64_t t = t0; t < t1; ++t) {
        const bf16x8 u = *(const bf16x8*)(o + (b * T + t) * ld + v);
        for (int i = 0; i < 8; ++i) s += (float)u[i];
    }
    if (s == 1234.5f) out[0] = s;
}

template <typename F>
float timeit(F f, int iters = 10) {
    for (int i = 0; i < 2; ++i) f();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) f();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / iters;
}

int main() {
    const int64_t B = 32, T = 2048, V = 17914, ld = 17920, Vp = (V + 15) / 16 * 16;
    bf16 *o, *d;
    int64_t *src, *trg;
    float *wtab, *loss, *col_lse, *dbias;
    (void)hipMalloc(&o, B * T * ld * 2);
    (void)hipMalloc(&d, B * T * ld * 2);
    (void)hipMalloc(&src, B * T * 8);
    (void)hipMalloc(&trg, B * T * 8);
    (void)hipMalloc(&wtab, 5 * V * 4);
    (void)hipMalloc(&loss, 4);
    (void)hipMalloc(&col_lse, B * V * 4);
    (void)hipMalloc(&dbias, V * 4);
    const size_t wsb = msq_filtered_workspace(B, T, V);
    void* ws;
    (void)hipMalloc(&ws, wsb);
    hipLaunchKernelGGL(fill_bf, dim3(4096), dim3(256), 0, 0, o, B * T * ld, 7u);
    std::vector<int64_t> h(B * T);
    // grammar-cycled tokens (pitch, dyn, length, time, tempo) and the real
    // vocabulary's weight table (oracle/loss.py weight_table)
    const int64_t st[6] = {0, 16512, 16640, 17152, 17664, V};
    for (int64_t i = 0; i < B * T; ++i) h[i] = st[i % 5] + (i * 7919) % (st[i % 5 + 1] - st[i % 5]);
    (void)hipMemcpy(src, h.data(), B * T * 8, hipMemcpyHostToDevice);
    for (int64_t i = 0; i < B * T; ++i) h[i] = st[(i + 1) % 5] + (i * 104729 + 3) % (st[(i + 1) % 5 + 1] - st[(i + 1) % 5]);
    (void)hipMemcpy(trg, h.data(), B * T * 8, hipMemcpyHostToDevice);
    std::vector<float> w(5 * V, 0.f);
    for (int64_t v = st[1]; v < st[2] - 1; ++v) w[0 * V + v] = 1.f;
    for (int64_t v = st[2]; v < st[3] - 1; ++v) w[1 * V + v] = 1.f + 2.f * (v - st[2]) / 510.f;
    for (int64_t v = st[3]; v < st[4] - 1; ++v) w[2 * V + v] = 1.f;
    for (int64_t v = st[4]; v < V; ++v) w[2 * V + v] = w[3 * V + v] = 1.f;
    for (int64_t v = 0; v < st[1] - 1; ++v) w[4 * V + v] = 10.f;
    (void)hipMemcpy(wtab, w.data(), 5 * V * 4, hipMemcpyHostToDevice);
    (void)hipMemset(dbias, 0, V * 4);

    const double gb = B * T * V * 2.0 / 1e9;
    const dim3 gc((unsigned)((V + 2047) / 2048), (unsigned)B, 32);
    float ms = timeit([&] { hipLaunchKernelGGL(read_kernel, gc, dim3(256), 0, 0, o, loss, ld, T, V); });
    printf("%-28s %8.3f ms %7.0f GB/s\n", "read (1 pass)", ms, gb / ms * 1e3);
    ms = timeit([&] { hipLaunchKernelGGL(copy_kernel, gc, dim3(256), 0, 0, o, d, ld, T, V); });
    printf("%-28s %8.3f ms %7.0f GB/s\n", "copy (read+write)", ms, 2 * gb / ms * 1e3);
    ms = timeit([&] {
        msq_filtered_ce_bias(loss, d, ld, dbias, o, MSQ_BF16, ld, src, trg, wtab, 16511, 16639, 17151, 17663, B, T, V,
                             1.f / (B * T), col_lse, ws, 0);
    });
    printf("%-28s %8.3f ms %7.0f GB/s (4 passes)\n", "msq_filtered_ce_bias", ms, 4 * gb / ms * 1e3);

    // the passes one by one (same workspace carving as msq_filtered_ce_bias)
    const LossArgs a = mk(o, ld, src, trg, wtab, 16511, 16639, 17151, 17663, B, T, V);
    char* wsc = (char*)ws;
    float* colsum = (float*)(wsc + (size_t)B * TSPLIT * 2 * V * 4);
    float* rows = colsum + B * V;
    float* part2 = (float*)(wsc + (size_t)B * TSPLIT * 2 * V * 4 + (size_t)B * V * 4 + (size_t)B * T * 4 * 2 + 256);
    float* clp = part2 + (size_t)B * TS2 * 2 * V;
    float* csp = clp + B * Vp;
    float* wtp = csp + B * Vp;
    float* row_lse = rows + B * T;
    ms = timeit([&] { hipLaunchKernelGGL(colstats2_kernel<bf16>, gc, dim3(NT), 0, 0, a, part2); });
    printf("%-28s %8.3f ms %7.0f GB/s\n", "colstats2", ms, gb / ms * 1e3);
    int* wrange = (int*)(wtp + 5 * Vp);
    ms = timeit([&] {
        hipLaunchKernelGGL(rowlse_kernel<bf16>, dim3((unsigned)((B * T + 3) / 4)), dim3(256), 0, 0, a, clp, wtp, (int)Vp,
                           wrange, rows, row_lse);
    });
    printf("%-28s %8.3f ms\n", "rowlse", ms);
    ms = timeit([&] {
        hipLaunchKernelGGL(cspart_kernel<bf16>, gc, dim3(NT), 0, 0, a, clp, wtp, (int)Vp, row_lse, 1.f, part2);
    });
    printf("%-28s %8.3f ms\n", "cspart", ms);
    ms = timeit([&] {
        hipLaunchKernelGGL(cs_reduce_kernel, dim3((unsigned)((B * Vp + 255) / 256)), dim3(256), 0, 0, part2, B, V, Vp, csp);
    });
    printf("%-28s %8.3f ms\n", "cs_reduce", ms);
    ms = timeit([&] {
        hipLaunchKernelGGL((finish2_kernel<bf16, bf16>), gc, dim3(NT), 0, 0, a, clp, wtp, (int)Vp, row_lse, csp, d, ld,
                           1.f, part2);
    });
    printf("%-28s %8.3f ms %7.0f GB/s\n", "finish2 (+dbias partials)", ms, 2 * gb / ms * 1e3);
    ms = timeit([&] {
        hipLaunchKernelGGL(dbias_reduce_kernel, dim3((unsigned)((V + 63) / 64)), dim3(1024), 0, 0, part2, B * TS2,
                           (int)Vp, V, dbias);
    });
    printf("%-28s %8.3f ms\n", "dbias_reduce", ms);
    return 0;
}
