// Shared device/host helpers for libmidiseq (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <math.h>

#include "../../include/midiseq.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64
#define LDS_PTR(T) T __attribute__((address_space(3)))*

// ---- host-side error plumbing (capi.cpp owns the thread-local message) ----
int msq_set_error(int code, const char* fmt, ...);

#define MSQ_CHECK_ARG(cond, ...)                                   \
    do {                                                           \
        if (!(cond)) return msq_set_error(MSQ_ERR_ARG, __VA_ARGS__); \
    } while (0)

#define MSQ_LAUNCH_CHECK()                                                           \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess)                                                        \
            return msq_set_error(MSQ_ERR_HIP, "%s: %s", __func__, hipGetErrorString(e_)); \
    } while (0)

// ---- device helpers ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

template <typename T>
__device__ __forceinline__ float to_f(T v) { return (float)v; }

template <typename T>
__device__ __forceinline__ T from_f(float v) { return (T)v; }

// load/store 4 consecutive elements as float4 (T = float or bf16)
__device__ __forceinline__ f32x4 load4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 load4(const bf16* p) {
    bf16x4 v = *(const bf16x4*)p;
    return (f32x4){(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ void store4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void store4(bf16* p, f32x4 v) {
    *(bf16x4*)p = (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5, T1)
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = bid % 8, loc = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}
