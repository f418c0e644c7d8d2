// Training-window gather for the data feed (processing/dataset.py:171-195
// SequenceDataset.__getitem__ + :134-168 data_augementation), run on the
// device so a batch never leaves HBM: the whole token store is resident
// (int32 tokens of every song back to back), and one launch cuts B windows
// of T+1 tokens, zero-pads short songs, applies the optional augmentation and
// writes src = w[:-1], trg = w[1:] (int64, the reference's dtype) and the
// song's 6 metadata tokens.
//
// Integer/byte work, HBM-bound: one thread per window token (coalesced reads
// of a contiguous song span, coalesced int64 writes).
#include "common.h"

namespace {

struct Aug {
    int64_t pitch0, P, C, dyn0, D, len0, L, time0, Tm, tempo0, Tp;
};

// dataset.py:18-22 shift_sequence: clamp(x + r, lb, ub-1) on lb <= x < ub
__device__ __forceinline__ int64_t aug_shift(int64_t x, int64_t r, int64_t lb, int64_t ub) {
    return (x >= lb && x < ub) ? min(max(x + r, lb), ub - 1) : x;
}
// dataset.py:24-33 shift_sequence_drums: pitch within the instrument, clamped
__device__ __forceinline__ int64_t aug_pitch(int64_t x, int64_t r, int64_t lb, int64_t ub, int64_t P) {
    if (!(x >= lb && x < ub)) return x;
    const int64_t cnt = x / P, rem = x % P;
    return cnt * P + min(max(rem + r, (int64_t)0), P - 1);
}
// dataset.py:35-39 multiply_sequence: float32 (x - lb) * f + lb, clamped, to int64
__device__ __forceinline__ int64_t aug_mul(int64_t x, float f, int64_t lb, int64_t ub) {
    if (!(x >= lb && x < ub)) return x;
    const float v = fminf(fmaxf((float)(x - lb) * f + (float)lb, (float)lb), (float)(ub - 1));
    return (int64_t)v;
}

// params[b] = {song, start, note_r, vel_r, 2 x time factor}: window token t is
// song[start + t], 0 past the song end (dataset.py:177-179 zero padding; the
// augmentation then also sees those zeros, as the reference's does)
__global__ __launch_bounds__(256) void window_gather_kernel(int64_t* __restrict__ src, int64_t* __restrict__ trg,
                                                            int64_t* __restrict__ meta_out,
                                                            const int32_t* __restrict__ tokens,
                                                            const int64_t* __restrict__ song_off,
                                                            const int64_t* __restrict__ song_len,
                                                            const int64_t* __restrict__ song_meta,
                                                            const int64_t* __restrict__ params, int n_meta,
                                                            int64_t T, int aug_on, Aug ag) {
    const int64_t b = blockIdx.y;
    const int64_t* pb = params + b * 5;
    const int64_t song = pb[0], start = pb[1];
    const int64_t off = song_off[song], len = song_len[song];
    if (blockIdx.x == 0 && threadIdx.x < n_meta) meta_out[b * n_meta + threadIdx.x] = song_meta[song * n_meta + threadIdx.x];
    for (int64_t t = blockIdx.x * 256LL + threadIdx.x; t <= T; t += (int64_t)gridDim.x * 256) {
        const int64_t pos = start + t;
        int64_t x = pos < len ? (int64_t)tokens[off + pos] : 0;
        if (aug_on) {
            const int64_t note_r = pb[2], vel_r = pb[3];
            const float f = (float)pb[4] * 0.5f;
            x = aug_pitch(x, note_r, ag.pitch0, ag.pitch0 + ag.P * ag.C - 1, ag.P);
            x = aug_shift(x, vel_r, ag.dyn0, ag.dyn0 + ag.D - 1);
            x = aug_mul(x, f, ag.time0, ag.time0 + ag.Tm - 1);
            x = aug_mul(x, f, ag.len0, ag.len0 + ag.L - 1);
            x = aug_mul(x, f, ag.tempo0, ag.tempo0 + ag.Tp - 1);
        }
        if (t < T) src[b * T + t] = x;
        if (t > 0) trg[b * T + t - 1] = x;
    }
}

}  // namespace

extern "C" int msq_window_gather(int64_t* src, int64_t* trg, int64_t* meta_out, const int32_t* tokens,
                                 const int64_t* song_off, const int64_t* song_len, const int64_t* song_meta,
                                 int n_meta, const int64_t* params, int64_t B, int64_t T, int augment,
                                 const int64_t* disc, void* stream) {
    MSQ_CHECK_ARG(src && trg && tokens && song_off && song_len && params && B > 0 && T > 0,
                  "msq_window_gather: bad args");
    MSQ_CHECK_ARG(n_meta >= 0 && n_meta <= 256 && (n_meta == 0 || (meta_out && song_meta)),
                  "msq_window_gather: bad metadata args");
    MSQ_CHECK_ARG(!augment || disc, "msq_window_gather: augmentation needs the discretization");
    Aug ag{};
    if (augment) {  // disc = {pitch, channel, dyn, length, time, tempo} (config.yaml discretization)
        ag.P = disc[0]; ag.C = disc[1]; ag.D = disc[2]; ag.L = disc[3]; ag.Tm = disc[4]; ag.Tp = disc[5];
        ag.pitch0 = 0;
        ag.dyn0 = ag.P * ag.C;
        ag.len0 = ag.dyn0 + ag.D;
        ag.time0 = ag.len0 + ag.L;
        ag.tempo0 = ag.time0 + ag.Tm;
        MSQ_CHECK_ARG(ag.P > 0 && ag.C > 0 && ag.D > 0 && ag.L > 0 && ag.Tm > 0 && ag.Tp > 0,
                      "msq_window_gather: bad discretization");
    }
    const unsigned nx = (unsigned)std::min<int64_t>((T + 1 + 255) / 256, 64);
    hipLaunchKernelGGL(window_gather_kernel, dim3(nx, (unsigned)B), dim3(256), 0, (hipStream_t)stream, src, trg,
                       meta_out, tokens, song_off, song_len, song_meta, params, n_meta, T, augment, ag);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
