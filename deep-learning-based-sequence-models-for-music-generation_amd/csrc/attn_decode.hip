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
// Memory-bound (per (b, h): K, V of S keys from HBM, R rows from L2/MALL,
// ~1.5 KB of loads per key against 3 x 256 FLOP): one workgroup of 4 waves per
// (b, h); scores with the key on the thread (16-B row loads, q from LDS), a
// workgroup softmax, then P.V with the dimension on the lane (coalesced 256-B
// V rows, one wave per key residue class) and a 4-wave combine. The new
// token's k / v come from the QKV row (and are written to its slot here).
#include "common.h"

namespace {

constexpr int NT = 256, HS = 128, MAXS = 4096;

// dot of 8 consecutive elements with q (fp32 in LDS)
__device__ __forceinline__ float dot8(const bf16* p, const float* q) {
    const bf16x8 a = *(const bf16x8*)p;
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf((float)a[e], q[e], s);
    return s;
}
__device__ __forceinline__ float dot8(const float* p, const float* q) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fmaf(a[e], q[e], s);
#pragma unroll
    for (int e = 0; e < 4; ++e) s = fmaf(b[e], q[4 + e], s);
    return s;
}
__device__ __forceinline__ void copy8(bf16* d, const bf16* s) { *(bf16x8*)d = *(const bf16x8*)s; }
__device__ __forceinline__ void copy8(float* d, const float* s) {
    *(f32x4*)d = *(const f32x4*)s;
    *(f32x4*)(d + 4) = *(const f32x4*)(s + 4);
}
__device__ __forceinline__ f32x2 load2(const bf16* p) {
    const bf16x2 v = *(const bf16x2*)p;
    return (f32x2){(float)v[0], (float)v[1]};
}
__device__ __forceinline__ f32x2 load2(const float* p) { return *(const f32x2*)p; }

__device__ __forceinline__ void load8(const bf16* p, float (&x)[8]) {
    const bf16x8 a = *(const bf16x8*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (float)a[e];
}
__device__ __forceinline__ void load8(const float* p, float (&x)[8]) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = a[e], x[4 + e] = b[e];
}

// T = bf16 (the MFMA engine) or float (the exact fp32 engine). A key's row
// (hs <= 128 values) is spread over a 16-lane group, 8 values per lane, so a
// wave reads 4 whole rows per load instruction (coalesced) and keeps 4 row
// loads of every kind in flight per unrolled step.
template <typename T>
__global__ __launch_bounds__(NT) void relattn_decode_kernel(T* __restrict__ out, int64_t ldo,
                                                            const T* __restrict__ qkv, int64_t ldq,
                                                            T* __restrict__ kc, T* __restrict__ vc,
                                                            const T* __restrict__ R, int64_t S_max, int H,
                                                            int S_ring, int n_meta, int n_tok, int new_slot,
                                                            int first_mod, float scale, int hs,
                                                            const int64_t* __restrict__ posp) {
    __shared__ float q_s[HS];
    __shared__ float p_s[MAXS];
    __shared__ float red[NT / 64];
    __shared__ float part[4][HS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int l16 = lane & 15, grp = w * 4 + (lane >> 4);  // 16 key groups per block
    const int h = blockIdx.x, b = blockIdx.y;
    const int ctx = S_ring - n_meta;
    if (posp) {  // the step's position from device memory (graph-replayed steps)
        const int64_t pos = *posp;
        n_tok = (int)min<int64_t>(pos + 1, ctx);
        new_slot = n_meta + (int)(pos % ctx);
        first_mod = (int)((pos + 1 - n_tok) % ctx);
    }
    const int S = n_meta + n_tok;
    const T* qrow = qkv + (int64_t)b * ldq + (int64_t)h * hs;
    const T* knew = qrow + (int64_t)H * hs;
    const T* vnew = knew + (int64_t)H * hs;
    T* kcb = kc + ((int64_t)b * H + h) * S_ring * hs;
    T* vcb = vc + ((int64_t)b * H + h) * S_ring * hs;
    const T* Rh = R + (int64_t)h * S_max * hs;
    if (tid < hs) q_s[tid] = (float)qrow[tid];
    // the new token's key / value into its slot (read back below from qkv)
    if (tid < hs / 8) {
        copy8(kcb + (int64_t)new_slot * hs + tid * 8, knew + tid * 8);
        copy8(vcb + (int64_t)new_slot * hs + tid * 8, vnew + tid * 8);
    }
    __syncthreads();
    const int d0 = 8 * l16;
    const bool dok = d0 < hs;
    float q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = dok ? q_s[d0 + e] : 0.f;

    // scores: group g takes slots g, g + 16, ...; lane l16 the dims 8 l16 ..
    float mx = -INFINITY;
#pragma unroll 4
    for (int s = grp; s < S; s += 16) {
        const int jw = s < n_meta ? s : n_meta + (s - n_meta - first_mod + ctx) % ctx;
        const T* kr = s == new_slot ? knew : kcb + (int64_t)s * hs;
        float kx[8], rx[8];
        if (dok) {
            load8(kr + d0, kx);
            load8(Rh + (int64_t)jw * hs + d0, rx);
        }
        float acc = 0.f;
        if (dok) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc = fmaf(kx[e] + rx[e], q[e], acc);
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        acc *= scale;
        if (l16 == 0) p_s[s] = acc;
        mx = fmaxf(mx, acc);
    }
    mx = wave_max(mx);
    if (lane == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float sum = 0.f;
    for (int s = tid; s < S; s += NT) {
        const float p = __expf(p_s[s] - mx);
        p_s[s] = p;
        sum += p;
    }
    sum = wave_sum(sum);
    if (lane == 0) red[w] = sum;
    __syncthreads();
    const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);

    // P.V: group g takes slots g, g + 16, ...; lane l16 accumulates dims 8 l16 ..
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
#pragma unroll 4
    for (int s = grp; s < S; s += 16) {
        const T* vr = s == new_slot ? vnew : vcb + (int64_t)s * hs;
        if (dok) {
            float vx[8];
            load8(vr + d0, vx);
            const float p = p_s[s];
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = fmaf(p, vx[e], o[e]);
        }
    }
    // the 4 groups of the wave, then the 4 waves
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 16, 64);
        o[e] += __shfl_xor(o[e], 32, 64);
    }
    if (lane < 16 && dok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) part[w][d0 + e] = o[e];
    }
    __syncthreads();
    if (tid < hs) {
        const float r = (part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid]) * inv;
        out[(int64_t)b * ldo + (int64_t)h * hs + tid] = (T)r;
    }
}

}  // namespace

extern "C" int msq_relattn_decode(int dtype, void* out, int64_t ldo, const void* qkv, int64_t ldq, void* kcache, void* vcache,
                                  const void* R, int64_t S_max, int64_t B, int64_t H, int64_t hs, int64_t S_ring,
                                  int64_t n_meta, int64_t n_tok, int64_t new_slot, int64_t first_mod, float scale,
                                  void* stream) {
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
    const dim3 grid((unsigned)H, (unsigned)B);
    if (dtype == MSQ_BF16)
        hipLaunchKernelGGL(relattn_decode_kernel<bf16>, grid, dim3(NT), 0, (hipStream_t)stream, (bf16*)out, ldo,
                           (const bf16*)qkv, ldq, (bf16*)kcache, (bf16*)vcache, (const bf16*)R, S_max, (int)H,
                           (int)S_ring, (int)n_meta, (int)n_tok, (int)new_slot, (int)first_mod, scale, (int)hs, nullptr);
    else
        hipLaunchKernelGGL(relattn_decode_kernel<float>, grid, dim3(NT), 0, (hipStream_t)stream, (float*)out, ldo,
                           (const float*)qkv, ldq, (float*)kcache, (float*)vcache, (const float*)R, S_max, (int)H,
                           (int)S_ring, (int)n_meta, (int)n_tok, (int)new_slot, (int)first_mod, scale, (int)hs, nullptr);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// msq_relattn_decode with the step's position read from device memory: n_tok =
// min(pos + 1, ctx), new slot n_meta + pos % ctx, first_mod = (pos + 1 - n_tok)
// % ctx (pos >= 0 is the caller's contract), so that a captured graph of the
// decode step replays unchanged from step to step.
extern "C" int msq_relattn_decode_pos(int dtype, void* out, int64_t ldo, const void* qkv, int64_t ldq, void* kcache,
                                      void* vcache, const void* R, int64_t S_max, int64_t B, int64_t H, int64_t hs,
                                      int64_t S_ring, int64_t n_meta, const int64_t* pos, float scale, void* stream) {
    MSQ_CHECK_ARG(out && qkv && kcache && vcache && R && pos, "msq_relattn_decode_pos: null pointer");
    MSQ_CHECK_ARG(hs > 0 && hs <= HS && hs % 8 == 0, "msq_relattn_decode_pos: head size %lld (8 | hs <= 128)",
                  (long long)hs);
    MSQ_CHECK_ARG(B > 0 && H > 0 && n_meta >= 0 && S_ring > n_meta && S_ring <= MAXS && S_ring <= S_max,
                  "msq_relattn_decode_pos: bad sizes");
    MSQ_CHECK_ARG(ldq >= 3 * H * hs && ldo >= H * hs, "msq_relattn_decode_pos: bad leading dims");
    MSQ_CHECK_ARG(dtype == MSQ_BF16 || dtype == MSQ_F32, "msq_relattn_decode_pos: dtype %d", dtype);
    const dim3 grid((unsigned)H, (unsigned)B);
    if (dtype == MSQ_BF16)
        hipLaunchKernelGGL(relattn_decode_kernel<bf16>, grid, dim3(NT), 0, (hipStream_t)stream, (bf16*)out, ldo,
                           (const bf16*)qkv, ldq, (bf16*)kcache, (bf16*)vcache, (const bf16*)R, S_max, (int)H,
                           (int)S_ring, (int)n_meta, 1, (int)n_meta, 0, scale, (int)hs, pos);
    else
        hipLaunchKernelGGL(relattn_decode_kernel<float>, grid, dim3(NT), 0, (hipStream_t)stream, (float*)out, ldo,
                           (const float*)qkv, ldq, (float*)kcache, (float*)vcache, (const float*)R, S_max, (int)H,
                           (int)S_ring, (int)n_meta, 1, (int)n_meta, 0, scale, (int)hs, pos);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
