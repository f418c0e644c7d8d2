// Internal interface between the attention translation units.
#pragma once
#include "common.h"

struct AttnArgs {
    int64_t B, S, H, hs, S_max, n_meta;
    float scale;
    const void* qkv; int64_t ldq;  // [B*S, ldq]: q | k | v, head h at col h*hs
    const void* R;                 // [H, S_max, hs]
    // attention-probability dropout (model_transformer.py:80); null = none.
    // keep bit of (b,h,i,j) in the block-transposed words of dropout.hip:
    // rowmask (uint32) [((bh*nb + i/64)*nb + j/64)*64 + i%64][j%64 / 32] >> (j%32),
    // colmask the same with (i, j) swapped; nb = mask_ld / 2; kept p scaled by keep_scale
    const uint32_t* rowmask = nullptr;
    const uint32_t* colmask = nullptr;
    int64_t mask_ld = 0;
    float keep_scale = 1.f;
    // XCD-aware block order in the flash kernels (xcd_blk3)
    int xcd = 1;
};

__device__ __forceinline__ float keep_bit(const AttnArgs& a, int64_t bh, int64_t i, int64_t j) {
    const int64_t nb = a.mask_ld >> 1;
    const int64_t w = (((bh * nb + (i >> 6)) * nb + (j >> 6)) * 64 + (i & 63)) * 2 + ((j >> 5) & 1);
    return (a.rowmask[w] >> (j & 31)) & 1u ? a.keep_scale : 0.f;
}

// bytes of one (b,h)'s mask words in either layout
__host__ __device__ __forceinline__ int64_t mask_bh_bytes(int64_t mask_ld) {
    return (mask_ld >> 1) * (mask_ld >> 1) * 512;
}
// uint32 word offset, inside one (b,h), of the words of row `r` (query for rowmask,
// key for colmask) against 32 columns starting at c (c % 32 == 0)
__host__ __device__ __forceinline__ int64_t mask_word(int64_t mask_ld, int64_t r, int64_t c) {
    return (((r >> 6) * (mask_ld >> 1) + (c >> 6)) * 64 + (r & 63)) * 2 + ((c >> 5) & 1);
}

// exact fp32 path (attn_exact.hip)
size_t exact_bwd_workspace(int64_t B, int64_t S, int64_t H);
int exact_fwd(const AttnArgs& a, float* out, int64_t ldo, float* lse, hipStream_t s);
int exact_bwd(const AttnArgs& a, const float* lse, const float* dout, int64_t ldo, float* dqkv, int64_t ldd, float* dR,
              void* ws, hipStream_t s);

// bf16 flash path (attn_flash.hip), hs == 128
int64_t flash_dqr_ld(int64_t S);
size_t flash_bwd_workspace(int64_t B, int64_t S, int64_t H);
// v5 key/value pass (attn_bwd5.hip): dS once, r-indexed, into dqr
// [H][B][S][ldr] (its j-view: row pitch ldr - 1 from element S - 1); -1 if unsupported
int flash_bwd_kv5(const AttnArgs& a, const float* nls, const float* ndk, const bf16* dout, int64_t ldo, bf16* dqkv,
                  int64_t ldd, bf16* dqr, int64_t ldr, hipStream_t s);
// dq = dS.K (dQR's skewed view) + dQR.R into the q columns of dqkv, dQR read
// once through an LDS ring (attn_dq.hip); -1 if unsupported
int flash_bwd_dq(const AttnArgs& a, const bf16* dqr, int64_t ldr, bf16* dqkv, int64_t ldd, hipStream_t s);
// v3 forward (attn_fwd3.hip): 8 waves x 32 queries, 32-key tiles; -1 if unsupported
int flash_fwd3(const AttnArgs& a, bf16* out, int64_t ldo, float* lse, hipStream_t s);
int flash_bwd(const AttnArgs& a, const float* lse, const bf16* dout, int64_t ldo, const bf16* out, bf16* dqkv,
              int64_t ldd, float* dR, void* ws, bool ws_ready, hipStream_t s);
