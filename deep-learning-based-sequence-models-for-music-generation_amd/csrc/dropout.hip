// Keep-bit masks of the attention-probability dropout (nn.Dropout on the
// softmax output, model_transformer.py:80), drawn once per layer and step
// from the counter-based hash of common.h.
//
// Two bit layouts of the same mask, both [B, H, S, ld] uint32 words
// (ld = 2 * ceil(S / 64)):
//   rowmask[b,h,i][w] bit t = keep(i, j = 32 w + t)   (forward: lanes own queries)
//   colmask[b,h,j][w] bit t = keep(i = 32 w + t, j)   (backward: lanes own keys)
// One wave computes one 64x64 block of the causal lower block triangle: lane l
// holds key j = 64 jb + l; per query row the 64 keep bits come out of one
// __ballot (the row word), and each lane collects bit l of those ballots into
// its column word. Blocks strictly above the diagonal are never read by the
// attention kernels (every such element is masked) and are not written.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void attn_mask_kernel(uint32_t* __restrict__ rowmask, uint32_t* __restrict__ colmask,
                                                        int S, int ld, int nb, int ntri, int H, uint32_t seed,
                                                        uint32_t site0, uint32_t thr) {
    const int lane = threadIdx.x & 63;
    const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int bh = blockIdx.y;
    if (task >= ntri) return;
    // task -> (ib, jb <= ib) of the lower block triangle
    int ib = (int)((sqrtf(8.f * task + 1.f) - 1.f) * 0.5f);
    while (ib * (ib + 1) / 2 > task) --ib;
    while ((ib + 1) * (ib + 2) / 2 <= task) ++ib;
    const int jb = task - ib * (ib + 1) / 2;
    (void)nb;
    const uint32_t base = drop_base(seed, site0 + (uint32_t)bh);
    const uint32_t rk = drop_row(base, (uint32_t)(ib * 64 + lane));  // lane l: query row 64 ib + l
    const uint32_t ck = (uint32_t)(jb * 64 + lane) * 0x85ebca6bu;   // lane l: key 64 jb + l
    uint64_t myrow = 0, mycol = 0;
    for (int ii = 0; ii < 64; ++ii) {
        const uint32_t rki = __builtin_amdgcn_readlane(rk, ii);
        const bool kp = drop_mix(rki ^ ck) >= thr;
        const uint64_t bal = __ballot(kp);
        myrow = lane == ii ? bal : myrow;
        mycol |= ((bal >> lane) & 1ull) << ii;
    }
    const int i = ib * 64 + lane, j = jb * 64 + lane;
    if (i < S) *(uint64_t*)(rowmask + ((int64_t)bh * S + i) * ld + 2 * jb) = myrow;
    if (j < S) *(uint64_t*)(colmask + ((int64_t)bh * S + j) * ld + 2 * ib) = mycol;
}

}  // namespace

extern "C" int64_t msq_dropout_mask_ld(int64_t S) { return 2 * ((S + 63) / 64); }

extern "C" int msq_dropout_attn_mask(uint32_t* rowmask, uint32_t* colmask, int64_t B, int64_t H, int64_t S,
                                     uint32_t seed, uint32_t site0, float p, void* stream) {
    MSQ_CHECK_ARG(rowmask && colmask && B > 0 && H > 0 && S > 0 && S < (1 << 24) && p >= 0.f && p < 1.f,
                  "msq_dropout_attn_mask: bad args");
    const int nb = (int)((S + 63) / 64), ntri = nb * (nb + 1) / 2;
    const dim3 grid((unsigned)((ntri + 3) / 4), (unsigned)(B * H));
    hipLaunchKernelGGL(attn_mask_kernel, grid, dim3(256), 0, (hipStream_t)stream, rowmask, colmask, (int)S,
                       (int)msq_dropout_mask_ld(S), nb, ntri, (int)H, seed, site0, drop_threshold(p));
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
