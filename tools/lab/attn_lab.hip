// Ablation harness for the attention forward v2 (not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lab/attn_lab.hip -o tools/lab/attn_lab
#include "../../deep-learning-based-sequence-models-for-music-generation_amd/csrc/attn_fwd3.hip"
#include <cstdio>

int msq_set_error(int code, const char*, ...) { return code; }


__global__ void fill(bf16* p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (bf16)(((int)(x & 0xFFFF) - 32768) / 65536.0f);
    }
}

template <int LAB>
float run(const AttnArgs& a, bf16* out, float* lse, int iters) {
    auto k = flash_fwd3_kernel<LAB>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    const dim3 grid((unsigned)((a.S + QB - 1) / QB), (unsigned)a.H, (unsigned)a.B);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, grid, dim3(NT), LDS_BYTES, 0, a, out, (int64_t)(a.H * 128), lse);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, grid, dim3(NT), LDS_BYTES, 0, a, out, (int64_t)(a.H * 128), lse);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / iters;
}

int main() {
    const int64_t B = 32, S = 2054, H = 8, HSz = 128;
    bf16 *qkv, *R, *out;
    float* lse;
    (void)hipMalloc(&qkv, B * S * 3 * H * HSz * 2);
    (void)hipMalloc(&R, H * S * HSz * 2);
    (void)hipMalloc(&out, B * S * H * HSz * 2);
    (void)hipMalloc(&lse, B * H * S * 4);
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, qkv, B * S * 3 * H * HSz, 1u);
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, R, H * S * HSz, 2u);
    AttnArgs a{};
    a.B = B; a.S = S; a.H = H; a.hs = HSz; a.S_max = S; a.n_meta = 6; a.scale = 1.f / 32.f;
    a.qkv = qkv; a.ldq = 3 * H * HSz; a.R = R;
    const double fl = 3.0 * 1024 * S * (S + 1) * B;
    struct V { const char* n; float (*f)(const AttnArgs&, bf16*, float*, int); };
    V vs[] = {{"full", run<0>}, {"no S mfma", run<1>}, {"no QR mfma", run<2>}, {"no softmax", run<4>},
              {"no PV mfma", run<8>}, {"no DMA", run<16>}, {"no mfma at all", run<11>}, {"only mfma", run<20>},
              {"full again", run<0>}};
    for (auto& v : vs) {
        float ms = v.f(a, out, lse, 10);
        printf("%-18s %8.3f ms %7.1f TFLOP/s\n", v.n, ms, fl / ms / 1e9);
    }
}
