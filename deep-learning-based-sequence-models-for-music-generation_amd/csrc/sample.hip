// One device kernel per decode step of scripts/generate.py:33-89, per row b:
//   recent window (generate.py:36-45): walk the history backwards summing
//     time-shift values (token - time_start for time tokens) and stop at the
//     first reversed position j where the sum reaches 1024; window = last j
//     tokens (j == 0 -> whole history; never reached -> all but the first);
//   penalties (:58-71): for every distinct pitch (dyn) token in the window,
//     z[tok] /= (float)min(1.01 ** count, 1.2)  (min(1.02 ** count, 1.2));
//   top-k (k in {1,2,3} chosen on the host with Python's `random`, :47-56),
//     p = v / sum(v), inverse-CDF pick with the row's uniform u (replaces
//     torch.multinomial, :76-80), append to the history.
// Ties in top-k prefer the lower vocabulary index.
#include "common.h"
#include <cmath>

namespace {

constexpr int NT = 1024;  // one workgroup per row: the V-long passes take 18 iterations
constexpr int MAXPEN = 16640;  // pitch + dyn token ids that can be penalised (default vocab)

struct Cand { float v; int i; };

// (float)min(base ** c, 1.2) for c < PEN_C, built on the host with libm's pow
// (what Python's ** calls), so the device needs no double-precision pow
constexpr int PEN_C = 32;
struct PenTab { float p[2][PEN_C]; };

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
    return a.v > b.v || (a.v == b.v && a.i < b.i);
}

__device__ __forceinline__ void insert3(Cand* t, Cand c) {
    if (better(c, t[2])) {
        if (better(c, t[1])) {
            t[2] = t[1];
            if (better(c, t[0])) { t[1] = t[0]; t[0] = c; }
            else t[1] = c;
        } else {
            t[2] = c;
        }
    }
}

__global__ __launch_bounds__(NT) void sample_kernel(int64_t* __restrict__ hist, int64_t ldh, int64_t cur_len,
                                                    float* __restrict__ z, int64_t ldz, int64_t V,
                                                    const int* __restrict__ ks, const float* __restrict__ us,
                                                    int64_t* __restrict__ out_tok, int64_t time_start,
                                                    int64_t tempo_start, int64_t dyn_start, int64_t len_start,
                                                    PenTab pt) {
    __shared__ unsigned short cnt[MAXPEN];
    __shared__ int s_j;
    __shared__ Cand red[NT / 64][3];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    int64_t* h = hist + b * ldh;
    float* zr = z + b * ldz;
    const int64_t npen = min<int64_t>(len_start, MAXPEN);
    for (int64_t v = tid; v < npen; v += NT) cnt[v] = 0;
    // recent window: sequential reverse prefix scan (one wave, 64 tokens per step)
    if (tid < 64) {
        int64_t acc = 0;
        int64_t jfound = -1;
        for (int64_t base = 0; base < cur_len && jfound < 0; base += 64) {
            const int64_t j = base + tid;
            int64_t val = 0;
            if (j < cur_len) {
                const int64_t t = h[cur_len - 1 - j];
                val = (t >= time_start && t < tempo_start) ? t - time_start : 0;
            }
            // inclusive prefix sum over the 64 lanes
            int64_t x = val;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int64_t y = __shfl_up(x, o, 64);
                if (tid >= o) x += y;
            }
            const bool hit = (j < cur_len) && (acc + x >= 1024);
            const unsigned long long m = __ballot(hit);
            if (m) jfound = base + __ffsll((long long)m) - 1;
            acc += __shfl(x, 63, 64);
        }
        if (tid == 0) s_j = (int)(jfound < 0 ? cur_len - 1 : jfound);
    }
    __syncthreads();
    const int64_t j = s_j;
    const int64_t wlen = j == 0 ? cur_len : j;  // cur_gen[-0:] is the whole list
    for (int64_t q = tid; q < wlen; q += NT) {
        const int64_t t = h[cur_len - wlen + q];
        if (t >= 0 && t < npen) atomicAdd((unsigned int*)((char*)cnt + ((t * 2) & ~3)), (t & 1) ? 65536u : 1u);
    }
    __syncthreads();
    for (int64_t v = tid; v < npen; v += NT) {
        const int c = cnt[v];
        if (c > 0) {
            const float pen = c < PEN_C ? pt.p[v >= dyn_start][c] : 1.2f;
            zr[v] = zr[v] / pen;
        }
    }
    __syncthreads();
    // top-3 with lower-index tie break
    Cand t3[3] = {{-INFINITY, 0x7fffffff}, {-INFINITY, 0x7fffffff}, {-INFINITY, 0x7fffffff}};
    for (int64_t v = tid; v < V; v += NT) insert3(t3, Cand{zr[v], (int)v});
    for (int o = 32; o > 0; o >>= 1) {
        Cand other[3];
        for (int q = 0; q < 3; ++q) {
            other[q].v = __shfl_xor(t3[q].v, o, 64);
            other[q].i = __shfl_xor(t3[q].i, o, 64);
        }
        for (int q = 0; q < 3; ++q) insert3(t3, other[q]);
    }
    if ((tid & 63) == 0)
        for (int q = 0; q < 3; ++q) red[tid >> 6][q] = t3[q];
    __syncthreads();
    if (tid == 0) {
        Cand f[3] = {red[0][0], red[0][1], red[0][2]};
        for (int w = 1; w < NT / 64; ++w)
            for (int q = 0; q < 3; ++q) insert3(f, red[w][q]);
        const int k = ks[b];
        float sum = f[0].v;
        for (int q = 1; q < k; ++q) sum += f[q].v;
        const float u = us[b];
        int pick = k - 1;
        float c = 0.f;
        for (int q = 0; q < k; ++q) {
            c += f[q].v / sum;
            if (c > u) { pick = q; break; }
        }
        // no finite candidate (NaN / -inf row): the reference's
        // torch.multinomial would raise; never emit an out-of-range id
        const int64_t tok = f[pick].i < V ? f[pick].i : 0;
        h[cur_len] = tok;
        out_tok[b] = tok;
    }
}

}  // namespace

extern "C" int msq_decode_sample(int64_t* hist, int64_t ld_hist, int64_t cur_len, float* z_last, int64_t ld_z,
                                 int64_t B, int64_t V, const int* ks, const float* uniforms, int64_t* out_tok,
                                 int64_t dyn_start, int64_t length_start, int64_t time_start, int64_t tempo_start,
                                 void* stream) {
    MSQ_CHECK_ARG(B > 0 && V > 0 && cur_len > 0 && cur_len < ld_hist, "msq_decode_sample: bad sizes");
    MSQ_CHECK_ARG(length_start <= MAXPEN, "msq_decode_sample: vocabulary layout too large (pitch+dyn > %d)", MAXPEN);
    static const PenTab pt = [] {
        PenTab t;
        for (int c = 0; c < PEN_C; ++c) {
            t.p[0][c] = (float)std::fmin(std::pow(1.01, (double)c), 1.2);
            t.p[1][c] = (float)std::fmin(std::pow(1.02, (double)c), 1.2);
        }
        return t;
    }();
    hipLaunchKernelGGL(sample_kernel, dim3((unsigned)B), dim3(NT), 0, (hipStream_t)stream, hist, ld_hist, cur_len,
                       z_last, ld_z, V, ks, uniforms, out_tok, time_start, tempo_start, dyn_start, length_start, pt);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
