// Adam update variants at the cfg-2 parameter count (154.9 M fp32 params + bf16
// shadow): times each with HIP events. Build: hipcc --offload-arch=gfx950 -O3
// tools/lab/adam_lab.hip -o tools/lab/adam_lab
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cmath>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __hip_bfloat16 bf16;

__device__ __forceinline__ void upd(f32x4& pv, f32x4& mv, f32x4& vv, f32x4 gv, float b1, float b2, float eps,
                                    float step_size, float bc2s, float gs) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const float gi = gv[t] * gs;
        const float mi = mv[t] + (1.f - b1) * (gi - mv[t]);
        const float vi = vv[t] * b2 + (1.f - b2) * gi * gi;
        mv[t] = mi;
        vv[t] = vi;
        const float den = sqrtf(vi) / bc2s + eps;
        pv[t] = pv[t] - step_size * (mi / den);
    }
}
__device__ __forceinline__ void st_shadow(bf16* s, f32x4 v) {
    union { uint2 u; bf16 e[4]; } r;
#pragma unroll
    for (int t = 0; t < 4; ++t) r.e[t] = __float2bfloat16(v[t]);
    *(uint2*)s = r.u;
}

// V0: the library's form (grid-stride, one quad per iteration)
__global__ void adam_v0(float* p, const float* g, float* m, float* v, bf16* sh, int64_t n4, float b1, float b2,
                        float eps, float ss, float bc, float gs) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
        const f32x4 gv = ((const f32x4*)g)[q];
        f32x4 mv = ((f32x4*)m)[q], vv = ((f32x4*)v)[q], pv = ((f32x4*)p)[q];
        upd(pv, mv, vv, gv, b1, b2, eps, ss, bc, gs);
        ((f32x4*)m)[q] = mv;
        ((f32x4*)v)[q] = vv;
        ((f32x4*)p)[q] = pv;
        st_shadow(sh + 4 * q, pv);
    }
}
// V1: one quad per thread, no loop
__global__ void adam_v1(float* p, const float* g, float* m, float* v, bf16* sh, int64_t n4, float b1, float b2,
                        float eps, float ss, float bc, float gs) {
    const int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (q >= n4) return;
    const f32x4 gv = ((const f32x4*)g)[q];
    f32x4 mv = ((f32x4*)m)[q], vv = ((f32x4*)v)[q], pv = ((f32x4*)p)[q];
    upd(pv, mv, vv, gv, b1, b2, eps, ss, bc, gs);
    ((f32x4*)m)[q] = mv;
    ((f32x4*)v)[q] = vv;
    ((f32x4*)p)[q] = pv;
    st_shadow(sh + 4 * q, pv);
}
// V2: U quads per thread (strided by the grid), all loads first; nontemporal when NT
template <int U, bool NT>
__global__ void adam_v2(float* p, const float* g, float* m, float* v, bf16* sh, int64_t n4, float b1, float b2,
                        float eps, float ss, float bc, float gs) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q0 < n4; q0 += stride * U) {
        f32x4 gv[U], mv[U], vv[U], pv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = q0 + u * stride;
            if (q < n4) {
                if (NT) {
                    gv[u] = __builtin_nontemporal_load((const f32x4*)g + q);
                    mv[u] = __builtin_nontemporal_load((const f32x4*)m + q);
                    vv[u] = __builtin_nontemporal_load((const f32x4*)v + q);
                    pv[u] = __builtin_nontemporal_load((const f32x4*)p + q);
                } else {
                    gv[u] = ((const f32x4*)g)[q];
                    mv[u] = ((f32x4*)m)[q];
                    vv[u] = ((f32x4*)v)[q];
                    pv[u] = ((f32x4*)p)[q];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = q0 + u * stride;
            if (q < n4) {
                upd(pv[u], mv[u], vv[u], gv[u], b1, b2, eps, ss, bc, gs);
                if (NT) {
                    __builtin_nontemporal_store(mv[u], (f32x4*)m + q);
                    __builtin_nontemporal_store(vv[u], (f32x4*)v + q);
                    __builtin_nontemporal_store(pv[u], (f32x4*)p + q);
                } else {
                    ((f32x4*)m)[q] = mv[u];
                    ((f32x4*)v)[q] = vv[u];
                    ((f32x4*)p)[q] = pv[u];
                }
                st_shadow(sh + 4 * q, pv[u]);
            }
        }
    }
}

// V3: flat, Q consecutive quads per thread (lane-contiguous 16 Q bytes), NT stores / loads by flags
template <int Q, bool NTL, bool NTS>
__global__ void adam_v3(float* p, const float* g, float* m, float* v, bf16* sh, int64_t n4, float b1, float b2,
                        float eps, float ss, float bc, float gs) {
    const int64_t q0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * Q;
#pragma unroll
    for (int u = 0; u < Q; ++u) {
        const int64_t q = q0 + u;
        if (q >= n4) return;
        f32x4 gv, mv, vv, pv;
        if (NTL) {
            gv = __builtin_nontemporal_load((const f32x4*)g + q);
            mv = __builtin_nontemporal_load((const f32x4*)m + q);
            vv = __builtin_nontemporal_load((const f32x4*)v + q);
            pv = __builtin_nontemporal_load((const f32x4*)p + q);
        } else {
            gv = ((const f32x4*)g)[q]; mv = ((f32x4*)m)[q]; vv = ((f32x4*)v)[q]; pv = ((f32x4*)p)[q];
        }
        upd(pv, mv, vv, gv, b1, b2, eps, ss, bc, gs);
        if (NTS) {
            __builtin_nontemporal_store(mv, (f32x4*)m + q);
            __builtin_nontemporal_store(vv, (f32x4*)v + q);
            __builtin_nontemporal_store(pv, (f32x4*)p + q);
        } else {
            ((f32x4*)m)[q] = mv; ((f32x4*)v)[q] = vv; ((f32x4*)p)[q] = pv;
        }
        st_shadow(sh + 4 * q, pv);
    }
}

int main() {
    const int64_t n = 154861050, n4 = n / 4;
    float *p, *g, *m, *v;
    bf16* sh;
    hipMalloc(&p, n * 4); hipMalloc(&g, n * 4); hipMalloc(&m, n * 4); hipMalloc(&v, n * 4); hipMalloc(&sh, n * 2);
    std::vector<float> h(n);
    for (int64_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(g, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(m, 0, n * 4); hipMemset(v, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const double bytes = 30.0 * n;
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        const int it = 20;
        for (int i = 0; i < it; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        printf("%-22s %.3f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
    };
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, ss = 1e-4f, bc = 0.03f, gs = 1.f;
    for (int r = 0; r < 2; ++r) {
        const unsigned gb = (unsigned)((n4 + 255) / 256);
        run("v0 grid16384", [&] { hipLaunchKernelGGL(adam_v0, dim3(16384), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v1 flat", [&] { hipLaunchKernelGGL(adam_v1, dim3(gb), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v1 flat 512", [&] { hipLaunchKernelGGL(adam_v1, dim3((unsigned)((n4 + 511) / 512)), dim3(512), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v1 flat 128", [&] { hipLaunchKernelGGL(adam_v1, dim3((unsigned)((n4 + 127) / 128)), dim3(128), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v3 Q1 NTS", [&] { hipLaunchKernelGGL((adam_v3<1, false, true>), dim3(gb), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v3 Q1 NTL", [&] { hipLaunchKernelGGL((adam_v3<1, true, false>), dim3(gb), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v3 Q1 NTL NTS", [&] { hipLaunchKernelGGL((adam_v3<1, true, true>), dim3(gb), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v3 Q2", [&] { hipLaunchKernelGGL((adam_v3<2, false, false>), dim3((unsigned)((n4 + 511) / 512)), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
        run("v3 Q2 NTS", [&] { hipLaunchKernelGGL((adam_v3<2, false, true>), dim3((unsigned)((n4 + 511) / 512)), dim3(256), 0, 0, p, g, m, v, sh, n4, b1, b2, eps, ss, bc, gs); });
    }
    return 0;
}
