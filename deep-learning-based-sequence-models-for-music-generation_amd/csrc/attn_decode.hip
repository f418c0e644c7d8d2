// Cached decode step of the relative-position attention (HeadRelPos,
// model_transformer.py:54-82, for the LAST row of a window only): the new
// token's query against the key/value cache of its window.
//
// For the last row i = S-1 of a window of S positions the reference's skew
// reads R[S-1-i+j] = R[j]: the relative term of key j is q . R[j], j = the
// key's position inside the window (metadata 0..5, then the window's tokens
// oldest first), and the last row sees every key (no mask). The cache is a
// ring: metadata keys in slots 0..n_meta-1, the token at sequence position p
// in slot n_meta + p % ctx; the window's first token p_first sits in slot
// n_meta + first_mod, so slot s (>= n_meta) is window position
// n_meta + (s - n_meta - first_mod) mod ctx.
//
// HBM-bound (per (b, h) the K and V rows of S keys, 2 x 256 B each at hs 128;
// the R rows are shared by every b and come from L2 / MALL). Split over the
// keys (flash decoding): one workgroup per (128-key chunk, h, b), i.e. ~8.7k
// workgroups at B 64, H 8, ctx 2048 instead of 512 — every K, R and V row of
// the chunk is requested up front (24 16-B loads per lane in flight), then
// scores, a chunk-local softmax (max m, sum l) and the unnormalised P.V go to
// a workspace partial; decode_combine_kernel merges a (b, h)'s chunks.
// A key row (hs <= 128 values) is spread over a 16-lane group, 8 values per
// lane, so one wave load instruction covers 4 consecutive rows (1 KB).
#include "common.h"

namespace {

constexpr int NT = 256, HS = 128, MAXS = 4096, CH = 128, NSTEP = CH / 16;

typedef float f32x8 __attribute__((ext_vector_type(8)));
template <typename T> struct RowT;
template <> struct RowT<bf16> { typedef bf16x8 type; };
template <> struct RowT<float> { typedef f32x8 type; };

template <typename T>
__device__ __forceinline__ typename RowT<T>::type ld_row(const T* p) { return *(const typename RowT<T>::type*)p; }
__device__ __forceinline__ void copy8(bf16* d, const bf16* s) { *(bf16x8*)d = *(const bf16x8*)s; }
__device__ __forceinline__ void copy8(float* d, const float* s) { *(f32x8*)d = *(const f32x8*)s; }

struct Pos {
    int n_tok, new_slot, first_mod;
};
// the step's window from device memory (graph-replayed steps) or the host arguments
__device__ __forceinline__ Pos window_pos(const int64_t* posp, int ctx, int n_meta, int n_tok, int new_slot,
                                          int first_mod) {
    if (posp) {
        const int64_t pos = *posp;
        n_tok = (int)min<int64_t>(pos + 1, ctx);
        new_slot = n_meta + (int)(pos % ctx);
        first_mod = (int)((pos + 1 - n_tok) % ctx);
    }
    return {n_tok, new_slot, first_mod};
}

struct DecArgs {
    int64_t ldq, S_max;
    int H, S_ring, n_meta, n_tok, new_slot, first_mod, hs, nsplit;
    float scale;
    const int64_t* posp;
};

template <typename T>
__global__ __launch_bounds__(NT) void relattn_decode_part_kernel(DecArgs a, const T* __restrict__ qkv,
                                                                 T* __restrict__ kc, T* __restrict__ vc,
                                                                 const T* __restrict__ R, float* __restrict__ po,
                                                                 float* __restrict__ pml) {
    __shared__ float part[4][HS];
    __shared__ float wm[4], wl[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int l16 = lane & 15, grp = w * 4 + (lane >> 4);  // 16 key groups per workgroup
    const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int H = a.H, hs = a.hs, n_meta = a.n_meta, ctx = a.S_ring - n_meta;
    const Pos p = window_pos(a.posp, ctx, n_meta, a.n_tok, a.new_slot, a.first_mod);
    const int S = n_meta + p.n_tok, s0 = c * CH;
    if (s0 >= S) return;  // chunk past the window (uniform over the workgroup)
    const T* qrow = qkv + (int64_t)b * a.ldq + (int64_t)h * hs;
    const T* knew = qrow + (int64_t)H * hs;
    const T* vnew = knew + (int64_t)H * hs;
    T* kcb = kc + ((int64_t)b * H + h) * a.S_ring * hs;
    T* vcb = vc + ((int64_t)b * H + h) * a.S_ring * hs;
    const T* Rh = R + (int64_t)h * a.S_max * hs;
    // the new token's key / value into its slot (this chunk reads them from qkv)
    if (p.new_slot >= s0 && p.new_slot < s0 + CH && tid < hs / 8) {
        copy8(kcb + (int64_t)p.new_slot * hs + tid * 8, knew + tid * 8);
        copy8(vcb + (int64_t)p.new_slot * hs + tid * 8, vnew + tid * 8);
    }
    const int d0 = 8 * l16;
    const bool dok = d0 < hs;

    // every row of the chunk requested before any is used
    typename RowT<T>::type kx[NSTEP], rx[NSTEP], vx[NSTEP], qx;
    if (dok) {
        qx = ld_row(qrow + d0);
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            const int s = min(s0 + st * 16 + grp, S - 1);  // rows past the window: masked below
            const int jw = s < n_meta ? s : n_meta + (s - n_meta - p.first_mod + ctx) % ctx;
            kx[st] = ld_row((s == p.new_slot ? knew : kcb + (int64_t)s * hs) + d0);
            rx[st] = ld_row(Rh + (int64_t)jw * hs + d0);
            vx[st] = ld_row((s == p.new_slot ? vnew : vcb + (int64_t)s * hs) + d0);
        }
    }
    float sc[NSTEP];
    float m = -INFINITY;
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
        float acc = 0.f;
        if (dok) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc = fmaf((float)kx[st][e] + (float)rx[st][e], (float)qx[e], acc);
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        sc[st] = s0 + st * 16 + grp < S ? acc * a.scale : -INFINITY;
        m = fmaxf(m, sc[st]);
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));  // the wave's max (>= one valid key unless the wave has none)
    float l = 0.f, o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
        const float pe = sc[st] == -INFINITY ? 0.f : __expf(sc[st] - m);
        l += pe;
        if (dok) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = fmaf(pe, (float)vx[st][e], o[e]);
        }
    }
    // the 4 key groups of the wave (l is uniform inside a group)
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 16, 64);
        o[e] += __shfl_xor(o[e], 32, 64);
    }
    if (lane < 16 && dok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) part[w][d0 + e] = o[e];
    }
    if (lane == 0) wm[w] = m, wl[w] = l;
    __syncthreads();
    // the 4 waves (the chunk holds >= 1 valid key, so M is finite)
    const float M = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    float f[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = wm[i] == -INFINITY ? 0.f : __expf(wm[i] - M);
    const int64_t pi = ((int64_t)b * H + h) * a.nsplit + c;
    if (tid < hs) po[pi * HS + tid] = f[0] * part[0][tid] + f[1] * part[1][tid] + f[2] * part[2][tid] + f[3] * part[3][tid];
    if (tid == 0) {
        pml[2 * pi] = M;
        pml[2 * pi + 1] = f[0] * wl[0] + f[1] * wl[1] + f[2] * wl[2] + f[3] * wl[3];
    }
}

// out[b, h] = sum_c e^(m_c - M) o_c / sum_c e^(m_c - M) l_c over the chunks of the window
template <typename T>
__global__ __launch_bounds__(HS) void decode_combine_kernel(DecArgs a, T* __restrict__ out, int64_t ldo,
                                                            const float* __restrict__ po,
                                                            const float* __restrict__ pml) {
    const int tid = threadIdx.x, h = blockIdx.x, b = blockIdx.y;
    const int ctx = a.S_ring - a.n_meta;
    const Pos p = window_pos(a.posp, ctx, a.n_meta, a.n_tok, a.new_slot, a.first_mod);
    const int nc = (a.n_meta + p.n_tok + CH - 1) / CH;
    const int64_t base = ((int64_t)b * a.H + h) * a.nsplit;
    float M = -INFINITY;
    for (int c = 0; c < nc; ++c) M = fmaxf(M, pml[2 * (base + c)]);
    float L = 0.f, acc = 0.f;
    for (int c = 0; c < nc; ++c) {
        const float f = __expf(pml[2 * (base + c)] - M);
        L = fmaf(f, pml[2 * (base + c) + 1], L);
        if (tid < a.hs) acc = fmaf(f, po[(base + c) * HS + tid], acc);
    }
    if (tid < a.hs) out[(int64_t)b * ldo + (int64_t)h * a.hs + tid] = (T)(acc / L);
}

int64_t n_split(int64_t S_ring) { return (S_ring + CH - 1) / CH; }

int launch(int dtype, void* out, int64_t ldo, const void* qkv, void* kcache, void* vcache, const void* R, int64_t B,
           const DecArgs& a, void* ws, size_t ws_bytes, hipStream_t s) {
    const size_t need = msq_relattn_decode_workspace(B, a.H, a.S_ring);
    MSQ_CHECK_ARG(ws && ws_bytes >= need && ((uintptr_t)ws & 15) == 0,
                  "msq_relattn_decode: workspace of %zu bytes (16-B aligned) needed, %zu given", need, ws_bytes);
    float* po = (float*)ws;
    float* pml = po + B * a.H * a.nsplit * HS;
    const dim3 grid((unsigned)a.nsplit, (unsigned)a.H, (unsigned)B), cgrid((unsigned)a.H, (unsigned)B);
    if (dtype == MSQ_BF16) {
        hipLaunchKernelGGL(relattn_decode_part_kernel<bf16>, grid, dim3(NT), 0, s, a, (const bf16*)qkv, (bf16*)kcache,
                           (bf16*)vcache, (const bf16*)R, po, pml);
        hipLaunchKernelGGL(decode_combine_kernel<bf16>, cgrid, dim3(HS), 0, s, a, (bf16*)out, ldo, po, pml);
    } else {
        hipLaunchKernelGGL(relattn_decode_part_kernel<float>, grid, dim3(NT), 0, s, a, (const float*)qkv,
                           (float*)kcache, (float*)vcache, (const float*)R, po, pml);
        hipLaunchKernelGGL(decode_combine_kernel<float>, cgrid, dim3(HS), 0, s, a, (float*)out, ldo, po, pml);
    }
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

}  // namespace

extern "C" size_t msq_relattn_decode_workspace(int64_t B, int64_t H, int64_t S_ring) {
    return (size_t)(B * H * n_split(S_ring)) * (HS + 2) * sizeof(float);
}

extern "C" int msq_relattn_decode(int dtype, void* out, int64_t ldo, const void* qkv, int64_t ldq, void* kcache, void* vcache,
                                  const void* R, int64_t S_max, int64_t B, int64_t H, int64_t hs, int64_t S_ring,
                                  int64_t n_meta, int64_t n_tok, int64_t new_slot, int64_t first_mod, float scale,
                                  void* ws, size_t ws_bytes, void* stream) {
    MSQ_CHECK_ARG(out && qkv && kcache && vcache && R, "msq_relattn_decode: null pointer");
    MSQ_CHECK_ARG(hs > 0 && hs <= HS && hs % 8 == 0, "msq_relattn_decode: head size %lld (8 | hs <= 128)",
                  (long long)hs);
    MSQ_CHECK_ARG(B > 0 && H > 0 && n_meta >= 0 && S_ring > n_meta && S_ring <= MAXS, "msq_relattn_decode: bad sizes");
    const int64_t ctx = S_ring - n_meta;
    MSQ_CHECK_ARG(n_tok >= 1 && n_tok <= ctx && n_meta + n_tok <= S_max, "msq_relattn_decode: n_tok %lld out of range",
                  (long long)n_tok);
    MSQ_CHECK_ARG(new_slot >= n_meta && new_slot < S_ring && first_mod >= 0 && first_mod < ctx,
                  "msq_relattn_decode: bad slot");
    MSQ_CHECK_ARG(ldq >= 3 * H * hs && ldo >= H * hs, "msq_relattn_decode: bad leading dims");
    MSQ_CHECK_ARG(dtype == MSQ_BF16 || dtype == MSQ_F32, "msq_relattn_decode: dtype %d", dtype);
    const DecArgs a{ldq, S_max, (int)H, (int)S_ring, (int)n_meta, (int)n_tok, (int)new_slot, (int)first_mod, (int)hs,
                    (int)n_split(S_ring), scale, nullptr};
    return launch(dtype, out, ldo, qkv, kcache, vcache, R, B, a, ws, ws_bytes, (hipStream_t)stream);
}

// msq_relattn_decode with the step's position read from device memory: n_tok =
// min(pos + 1, ctx), new slot n_meta + pos % ctx, first_mod = (pos + 1 - n_tok)
// % ctx (pos >= 0 is the caller's contract), so that a captured graph of the
// decode step replays unchanged from step to step.
extern "C" int msq_relattn_decode_pos(int dtype, void* out, int64_t ldo, const void* qkv, int64_t ldq, void* kcache,
                                      void* vcache, const void* R, int64_t S_max, int64_t B, int64_t H, int64_t hs,
                                      int64_t S_ring, int64_t n_meta, const int64_t* pos, float scale, void* ws,
                                      size_t ws_bytes, void* stream) {
    MSQ_CHECK_ARG(out && qkv && kcache && vcache && R && pos, "msq_relattn_decode_pos: null pointer");
    MSQ_CHECK_ARG(hs > 0 && hs <= HS && hs % 8 == 0, "msq_relattn_decode_pos: head size %lld (8 | hs <= 128)",
                  (long long)hs);
    MSQ_CHECK_ARG(B > 0 && H > 0 && n_meta >= 0 && S_ring > n_meta && S_ring <= MAXS && S_ring <= S_max,
                  "msq_relattn_decode_pos: bad sizes");
    MSQ_CHECK_ARG(ldq >= 3 * H * hs && ldo >= H * hs, "msq_relattn_decode_pos: bad leading dims");
    MSQ_CHECK_ARG(dtype == MSQ_BF16 || dtype == MSQ_F32, "msq_relattn_decode_pos: dtype %d", dtype);
    const DecArgs a{ldq, S_max, (int)H, (int)S_ring, (int)n_meta, 1, (int)n_meta, 0, (int)hs,
                    (int)n_split(S_ring), scale, pos};
    return launch(dtype, out, ldo, qkv, kcache, vcache, R, B, a, ws, ws_bytes, (hipStream_t)stream);
}
