// Tile images and MFMA fragment readers shared by the attention kernels
// (hs = 128 rows of 256 B in LDS; XOR chunk swizzles, see attn_flash.hip).
#pragma once
#include "attn.h"
#include "lds_dma.h"

namespace attn {

constexpr int HS = 128;
constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) char lds_char;

__device__ __forceinline__ i16x4 tr_read(const char* base, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((i16x4 __attribute__((address_space(3)))*)((lds_char*)base + off));
}
__device__ __forceinline__ bf16x8 cat8(i16x4 a, i16x4 b) {
    union { i16x4 h[2]; bf16x8 v; } u;
    u.h[0] = a;
    u.h[1] = b;
    return u.v;
}
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero4() { return (f32x4){0.f, 0.f, 0.f, 0.f}; }

// 256-B row images (128 bf16). Row-read image: chunk ^= row & 15 (ds_read_b128
// of 16 rows at one chunk is conflict-free). Transposed-read images:
//   "pairs"  rows read as {8g+q, 8g+4+q}: chunk ^= 2*gk(row) (GEMM layout)
//   "quads"  rows read as {4g+q, 16+4g+q}: chunk ^= 2*(row & 7)
__device__ __forceinline__ int off_row(int row, int ch) { return row * 256 + ((ch ^ (row & 15)) << 4); }
__device__ __forceinline__ int off_pairs(int row, int ch) {
    return row * 256 + ((ch ^ ((((row & 3) | ((row >> 1) & 4))) << 1)) << 4);
}
__device__ __forceinline__ int off_quads(int row, int ch) { return row * 256 + ((ch ^ ((row & 7) << 1)) << 4); }

// X/Y fragment: 16 rows (rb + lane&15) x 8 values (k-step ks) from a row image
__device__ __forceinline__ bf16x8 frag_row(const char* s, int rb, int ks, int lane) {
    const int row = rb + (lane & 15);
    return *(const bf16x8*)(s + off_row(row, ks * 4 + (lane >> 4)));
}
// transposed fragment from a "quads" image: rows {kb+4g+q, kb+16+4g+q}, cols cb..cb+15
__device__ __forceinline__ bf16x8 frag_quads(const char* s, int kb, int cb, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int ch = (cb >> 3) + (p >> 1), sub = (p & 1) * 8;
    const int r1 = kb + 4 * g + q, r2 = r1 + 16;
    return cat8(tr_read(s, off_quads(r1, ch) + sub), tr_read(s, off_quads(r2, ch) + sub));
}
// transposed fragment from a "pairs" image: rows {kb+8g+q, kb+8g+4+q}
__device__ __forceinline__ bf16x8 frag_pairs(const char* s, int kb, int cb, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int ch = (cb >> 3) + (p >> 1), sub = (p & 1) * 8;
    const int r1 = kb + 8 * g + q, r2 = r1 + 4;
    return cat8(tr_read(s, off_pairs(r1, ch) + sub), tr_read(s, off_pairs(r2, ch) + sub));
}

}  // namespace attn
