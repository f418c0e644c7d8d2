// Keep-bit masks of the attention-probability dropout (nn.Dropout on the
// softmax output, model_transformer.py:80), drawn once per layer and step
// from the counter-based hash of common.h.
//
// Two bit layouts of the same mask, both block-transposed: with nb = ceil(S/64)
// one (b,h) owns nb*nb*64 uint64 words, 64 per 64x64 block, so the 64 words of
// a block are one contiguous 512-B store of the wave that draws it:
//   rowmask[((bh*nb + i/64)*nb + j/64)*64 + i%64] bit j%64 = keep(i, j)   (forward: lanes own queries)
//   colmask[((bh*nb + j/64)*nb + i/64)*64 + j%64] bit i%64 = keep(i, j)   (backward: lanes own keys)
// (as uint32 words: low word = keys / queries 0-31 of the block, high = 32-63).
// One wave computes one 64x64 block of the causal lower block triangle: lane l
// draws the keep word of query row 64 ib + l over keys 64 jb .. +63
// (attn_word_key, common.h: one hash plus one per dropped key), and the 64
// row words are bit-transposed across the wave into the column words.
// Blocks strictly above the diagonal are never read by the attention kernels
// (every such element is masked) and are not written.
#include "common.h"

namespace {

struct DropTable {
    uint32_t t[64];
};

__global__ __launch_bounds__(256) void attn_mask_kernel(uint32_t* __restrict__ rowmask, uint32_t* __restrict__ colmask,
                                                        int S, int ld, int nb, int ntri, int H, uint32_t seed,
                                                        uint32_t site0, DropTable tab, int on) {
    __shared__ uint32_t T[64];
    if (threadIdx.x < 64) T[threadIdx.x] = tab.t[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int task = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int bh = blockIdx.y;
    if (task >= ntri) return;
    // task -> (ib, jb <= ib) of the lower block triangle
    int ib = (int)((sqrtf(8.f * task + 1.f) - 1.f) * 0.5f);
    while (ib * (ib + 1) / 2 > task) --ib;
    while ((ib + 1) * (ib + 2) / 2 <= task) ++ib;
    const int jb = task - ib * (ib + 1) / 2;
    const uint32_t base = drop_base(seed, site0 + (uint32_t)bh);
    const uint32_t key = attn_word_key(drop_row(base, (uint32_t)(ib * 64 + lane)), (uint32_t)jb);
    int k = 0;  // p = 0: every key kept
    while (on && k < 64 && key >= T[k]) ++k;
    uint64_t word = ~0ull;
    for (int s = 0; s < k; ++s) {
        const uint32_t n = __umulhi(attn_drop_draw(key, (uint32_t)s), 64u - (uint32_t)s);
        word &= ~(1ull << nth_set_bit(word, n));
    }
    const uint32_t rlo = (uint32_t)word, rhi = (uint32_t)(word >> 32);
    const uint64_t myrow = ((uint64_t)rhi << 32) | rlo;
    // column words: 64x64 bit transpose across the wave, six butterfly stages;
    // at stage s element (r, c) with r&s == 0, c&s != 0 swaps with (r+s, c-s)
    uint64_t t = myrow;
    const uint64_t hi_s[6] = {0xFFFFFFFF00000000ull, 0xFFFF0000FFFF0000ull, 0xFF00FF00FF00FF00ull,
                              0xF0F0F0F0F0F0F0F0ull, 0xCCCCCCCCCCCCCCCCull, 0xAAAAAAAAAAAAAAAAull};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int sh = 32 >> k;
        const uint64_t hm = hi_s[k];
        const uint32_t plo = (uint32_t)__shfl_xor((int)(uint32_t)t, sh);
        const uint32_t phi = (uint32_t)__shfl_xor((int)(uint32_t)(t >> 32), sh);
        const uint64_t pt = ((uint64_t)phi << 32) | plo;
        const uint64_t up = 0ull - (uint64_t)((lane >> (5 - k)) & 1);  // all ones on lanes with bit sh
        t = (t & (hm ^ ~up)) | (((pt & hm) >> sh) & up) | (((pt & ~hm) << sh) & ~up);
    }
    const uint64_t mycol = t;
    (void)S;
    (void)ld;
    const int64_t bhb = (int64_t)bh * nb;
    ((uint64_t*)rowmask)[((bhb + ib) * nb + jb) * 64 + lane] = myrow;
    ((uint64_t*)colmask)[((bhb + jb) * nb + ib) * 64 + lane] = mycol;
}

}  // namespace

extern "C" int64_t msq_dropout_mask_ld(int64_t S) { return 2 * ((S + 63) / 64); }

extern "C" int64_t msq_dropout_mask_words(int64_t B, int64_t H, int64_t S) {
    const int64_t nb = (S + 63) / 64;
    return B * H * nb * nb * 128;
}

extern "C" int msq_dropout_attn_mask(uint32_t* rowmask, uint32_t* colmask, int64_t B, int64_t H, int64_t S,
                                     uint32_t seed, uint32_t site0, float p, void* stream) {
    MSQ_CHECK_ARG(rowmask && colmask && B > 0 && H > 0 && S > 0 && S < (1 << 24) && p >= 0.f && p < 1.f,
                  "msq_dropout_attn_mask: bad args");
    const int nb = (int)((S + 63) / 64), ntri = nb * (nb + 1) / 2;
    const dim3 grid((unsigned)((ntri + 3) / 4), (unsigned)(B * H));
    DropTable tab;
    attn_drop_table(p, tab.t);
    hipLaunchKernelGGL(attn_mask_kernel, grid, dim3(256), 0, (hipStream_t)stream, rowmask, colmask, (int)S,
                       (int)msq_dropout_mask_ld(S), nb, ntri, (int)H, seed, site0, tab, p > 0.f ? 1 : 0);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// the Binomial(64, p) thresholds of the attention keep words (host only):
// oracle/dropout.py's table is checked against this one bit for bit
extern "C" int msq_dropout_attn_table(float p, uint32_t* out64) {
    MSQ_CHECK_ARG(out64 && p >= 0.f && p < 1.f, "msq_dropout_attn_table: bad args");
    attn_drop_table(p, out64);
    return MSQ_OK;
}
