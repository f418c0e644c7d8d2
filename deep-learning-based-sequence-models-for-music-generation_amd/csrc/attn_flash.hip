// Relative-position flash attention backward, bf16 MFMA path (hs = 128):
// the host side of the pass sequence and its small kernels
// (model_transformer.py:54-90 differentiated):
//   pre : D_i = sum_d dO.O (and the key/value pass's row constants -lse/scale,
//         -D/ks: the initial accumulators of its S and dP chains)
//   kv  : per 128-key block (attn_bwd5.hip): recompute S, P; dP = dO.V^T;
//         dS = P (dP - D) scale; dK, dV accumulated in registers; dS written
//         once, r-indexed: dQR[h][b][i][r = S-1-i+j];
//   dq  : dq = dS . K (the j-view of dQR: pitch ldr - 1) + dQR . R (attn_dq.hip);
//   GEMM: dR += dQR^T . Q (batched over heads, split-K partials);
//   meta: the metadata-prefix entries j > i (flash_bwd_meta5_kernel).
// The forward is attn_fwd3.hip.
#include "attn_tiles.h"
#include "gemm.h"
#include <cstdlib>
#include <stdlib.h>

namespace {

using namespace attn;
constexpr int NT = 256;

// ------------------------------------------------------------ backward: pre
// D[b,h,i] = sum_d dO[i,d] O[i,d]
// same, 16 lanes x 8 elements (one 16-B load of dO and of O each) per
// (row, head): 4 head-rows per wave; also the key/value pass's row
// constants nls = -lse / scale and ndk = -D / ks (ks = 1/(1-p) with dropout,
// else 1): the initial values of its S and dP accumulators, so that
// P = exp2(scale log2(e) (S + R term)) and dS = P ks scale (dP - D/ks)
__global__ __launch_bounds__(256) void flash_bwd_pre_vec_kernel(AttnArgs a, const bf16* __restrict__ dout,
                                                                int64_t ldo, const bf16* __restrict__ out,
                                                                const float* __restrict__ lse,
                                                                float* __restrict__ Dv, float* __restrict__ nls,
                                                                float* __restrict__ ndk) {
    const int64_t row = blockIdx.x * 16LL + (threadIdx.x >> 4);  // over B*S*H
    const int l = threadIdx.x & 15;
    const bool ok = row < a.B * a.S * a.H;
    const int64_t r = ok ? row : 0;
    const int64_t h = r % a.H, bi = r / a.H;
    const bf16x8 x = *(const bf16x8*)(dout + bi * ldo + h * HS + 8 * l);
    const bf16x8 y = *(const bf16x8*)(out + bi * ldo + h * HS + 8 * l);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (float)x[e] * (float)y[e];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (ok && l == 0) {
        const int64_t b = bi / a.S, i = bi % a.S, k = (b * a.H + h) * a.S + i;
        Dv[k] = s;
        ndk[k] = -s / (a.colmask ? a.keep_scale : 1.f);
        nls[k] = -lse[k] / a.scale;
    }
}

// ------------------------------------------------------------ backward: fix-up
// metadata prefix, v5 form: the key/value pass v5 masks the entries j > i
// inside the metadata prefix (i < j < n_meta, keys every query sees) like the
// rest of the upper triangle, so this kernel owns them whole: per (b, h) and
// pair (i, j)
//   s    = scale (q_i.k_j + [j >= i+2] q_{i+1}.R[j-i-2]),  p = exp(s - lse_i)
//   dS   = p (dO_i.v_j m_ij ks - D_i) scale
//   dV_j += p m_ij ks dO_i,  dK_j += dS q_i,  dq_i += dS k_j
//   j >= i+2: dq_{i+1} += dS R[j-i-2],  dR[j-i-2] += dS q_{i+1}
// (model_transformer.py:70-90 with the _rel_shift wrap of :84-90 for j > i).
// The dR rows go to mdr[b][h][r] (plain stores); flash_bwd_meta_dr_kernel adds
// them over b in a fixed order, so the backward has no atomics here.
__global__ __launch_bounds__(HS) void flash_bwd_meta5_kernel(AttnArgs a, const float* __restrict__ lse,
                                                             const float* __restrict__ Dv,
                                                             const bf16* __restrict__ dout, int64_t ldo,
                                                             bf16* __restrict__ dqkv, int64_t ldd,
                                                             float* __restrict__ mdr) {
    __shared__ float red[3][2];
    const int64_t h = blockIdx.y, b = blockIdx.z;
    const int d = threadIdx.x, lane = d & 63, wv = d >> 6;  // 128 threads, one per dim
    const int64_t S = a.S, H = a.H, ldq = a.ldq, bh = b * H + h;
    const bf16* qkv = (const bf16*)a.qkv + b * S * ldq;
    const bf16* Rp = (const bf16*)a.R + h * a.S_max * HS;
    const bf16* dob = dout + b * S * ldo;
    const int nm = (int)min<int64_t>(a.n_meta, S);
    float gq[8], gk[8], gv[8], gr[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) gq[r] = gk[r] = gv[r] = gr[r] = 0.f;
    auto q = [&](int i) { return (float)qkv[i * ldq + h * HS + d]; };
    auto k = [&](int j) { return (float)qkv[j * ldq + (H + h) * HS + d]; };
    auto v = [&](int j) { return (float)qkv[j * ldq + (2 * H + h) * HS + d]; };
    auto sum3 = [&](float x, float y, float z) {
        x = wave_sum(x);
        y = wave_sum(y);
        z = wave_sum(z);
        __syncthreads();
        if (lane == 0) {
            red[0][wv] = x;
            red[1][wv] = y;
            red[2][wv] = z;
        }
        __syncthreads();
    };
#pragma unroll 1
    for (int i = 0; i + 1 < nm; ++i) {
#pragma unroll 1
        for (int j = i + 1; j < nm; ++j) {
            const bool far = j >= i + 2;
            const float rr = far ? (float)Rp[(j - i - 2) * HS + d] : 0.f;
            const float q1 = far ? q(i + 1) : 0.f;
            sum3(q(i) * k(j), q1 * rr, (float)dob[i * ldo + h * HS + d] * v(j));
            const float sc = (red[0][0] + red[0][1] + red[1][0] + red[1][1]) * a.scale;
            const float dp = red[2][0] + red[2][1];
            const float p = expf(sc - lse[bh * S + i]);
            const float m = a.rowmask ? keep_bit(a, bh, i, j) : 1.f;  // ks or 0 with dropout
            const float ds = p * (dp * m - Dv[bh * S + i]) * a.scale;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (r == j) {
                    gv[r] += p * m * (float)dob[i * ldo + h * HS + d];
                    gk[r] += ds * q(i);
                }
                if (r == i) gq[r] += ds * k(j);
                if (far && r == i + 1) gq[r] += ds * rr;
                if (far && r == j - i - 2) gr[r] += ds * q1;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (r >= nm) break;
        bf16* row = dqkv + (b * S + r) * ldd;
        row[h * HS + d] = (bf16)((float)row[h * HS + d] + gq[r]);
        row[(H + h) * HS + d] = (bf16)((float)row[(H + h) * HS + d] + gk[r]);
        row[(2 * H + h) * HS + d] = (bf16)((float)row[(2 * H + h) * HS + d] + gv[r]);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) mdr[(bh * 8 + r) * HS + d] = gr[r];
}

// dR[h][r] += sum over b (in order) of mdr[b][h][r], r < 8
__global__ __launch_bounds__(HS) void flash_bwd_meta_dr_kernel(AttnArgs a, const float* __restrict__ mdr,
                                                              float* __restrict__ dR) {
    const int64_t h = blockIdx.x, r = blockIdx.y;
    const int d = threadIdx.x;
    if (r + 2 >= min<int64_t>(a.n_meta, a.S)) return;  // only j - i - 2 < n_meta - 2 occurs
    float s = 0.f;
    for (int64_t b = 0; b < a.B; ++b) s += mdr[((b * a.H + h) * 8 + r) * HS + d];
    dR[(h * a.S_max + r) * HS + d] += s;
}

}  // namespace

namespace {
// zero the part of dQR[h][b][i][r] that the consumers read but the key/value
// pass does not write: r in [S-1-i-DQR_BAND, S-1-i) (below the written band)
// and the row pad [S, ldr). The dq kernel and the dR product never read
// further below the band.
constexpr int DQR_BAND = 256;
// one wave per row; ldr % 8 == 0 (flash_dqr_ld), so the row starts are 16-B
// aligned: ragged ends with 2-B stores, the body with 16-B stores
__device__ __forceinline__ void zero_span(bf16* __restrict__ p, int64_t lo, int64_t hi, int lane) {
    if (lo >= hi) return;
    const int64_t a = min(hi, (lo + 7) & ~(int64_t)7), e = max(a, hi & ~(int64_t)7);
    if (lane < a - lo) p[lo + lane] = (bf16)0.f;
    if (lane < hi - e) p[e + lane] = (bf16)0.f;
    const u32x4 z = (u32x4){0u, 0u, 0u, 0u};
    for (int64_t r = a + 8 * lane; r < e; r += 512) *(u32x4*)(p + r) = z;
}

__global__ void dqr_band_zero_kernel(bf16* __restrict__ dqr, int64_t ldr, int64_t S, int64_t rows) {
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);  // (h, b, i) flattened
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t i = row % S;
    bf16* p = dqr + row * ldr;
    zero_span(p, max<int64_t>(0, S - 1 - i - DQR_BAND), S - 1 - i, lane);
    zero_span(p, S, ldr, lane);
}
}  // namespace

// dQR / dSj row pitch: >= S + 128 so that the key/value pass's whole-row dS
// stores of a 128-key block never reach the next row (dQR entries j > i fall
// at r = S-1-i+j in [S, S+127)), and >= S + 200 for the dq kernel's j-view of
// dQR (dS-once: row i's K range ends below i0 + 192, i.e. r < S + 191, plus
// the funnel shift's second chunk): padding, zeroed once per workspace
int64_t flash_dqr_ld(int64_t S) { return (S + 200 + 7) / 8 * 8; }

// workspace: dQR bf16 [H][B][S][ldr] | D f32 [B][H][S]
//            | dR split-K partials f32 [ksplit][H][S][HS]
//            | nls f32 [B][H][S] | ndk f32 [B][H][S] | mdr f32 [B][H][8][HS]
static size_t align256(size_t x) { return (x + 255) / 256 * 256; }
static size_t dr_ws_bytes(int64_t B, int64_t S, int64_t H) {
    return splitk_ws_bytes(S, HS, H, gemm_bf16_tri_ksplit(2, S, HS, B * S, S, H));
}

size_t flash_bwd_workspace(int64_t B, int64_t S, int64_t H) {
    const int64_t ldr = flash_dqr_ld(S);
    return align256((size_t)H * B * S * ldr * 2) + 3 * align256((size_t)B * H * S * 4) +
           align256((size_t)B * H * 8 * HS * 4) +
           align256(dr_ws_bytes(B, S, H));
}

int flash_bwd(const AttnArgs& a, const float* lse, const bf16* dout, int64_t ldo, const bf16* out, bf16* dqkv,
              int64_t ldd, float* dR, void* ws, bool ws_ready, hipStream_t s) {
    const int64_t B = a.B, S = a.S, H = a.H, ldr = flash_dqr_ld(S);
    char* p = (char*)ws;
    bf16* dqr = (bf16*)p;
    p += align256((size_t)H * B * S * ldr * 2);
    float* Dv = (float*)p;
    p += align256((size_t)B * H * S * 4);
    float* dr_ws = (float*)p;
    p += align256(dr_ws_bytes(B, S, H));
    float* nls = (float*)p;
    p += align256((size_t)B * H * S * 4);
    float* ndk = (float*)p;
    p += align256((size_t)B * H * S * 4);
    float* mdr = (float*)p;  // the metadata block's dR rows per (b, h)

    // the band and row pads are never written non-zero by the passes below
    // (their dS entries there are 0 by the mask), so a workspace that already
    // served this (B, S, H) keeps them (ws_ready)
    if (!ws_ready)
        hipLaunchKernelGGL(dqr_band_zero_kernel, dim3((unsigned)((H * B * S + 3) / 4)), dim3(256), 0, s, dqr, ldr, S,
                           H * B * S);
    if (ldo % 8 || ((uintptr_t)dout % 16) || ((uintptr_t)out % 16))
        return msq_set_error(MSQ_ERR_ARG, "flash_bwd: dout / out need 16-B aligned rows");
    hipLaunchKernelGGL(flash_bwd_pre_vec_kernel, dim3((unsigned)((B * S * H + 15) / 16)), dim3(256), 0, s, a, dout, ldo,
                       out, lse, Dv, nls, ndk);
    // key/value pass v5: dK, dV, and dS once (dQR, r-indexed; its second,
    // j-indexed copy cost the pass a quarter of its time: DESIGN.md §10)
    if (flash_bwd_kv5(a, nls, ndk, dout, ldo, dqkv, ldd, dqr, ldr, s))
        return msq_set_error(MSQ_ERR_UNSUPPORTED, "flash_bwd: shape outside the key/value pass (n_meta > 8 or > 4 GB)");
    // dq (bf16, q columns of dqkv) = dS . K (dQR's skewed view) + dQR . R
    if (flash_bwd_dq(a, dqr, ldr, dqkv, ldd, s))
        return msq_set_error(MSQ_ERR_UNSUPPORTED, "flash_bwd: shape outside the query pass (> 4 GB)");
    // dR[h][r] += sum_{b,i} dQR[h][b,i][r] q_{b,i}   (batched over heads; per batch
    // segment only i >= S-1-r contributes: tri 2, split over segments)
    // (a strided-batched hipBLASLt product over the whole K range, 2x the
    // triangle's work, measured 1.08 ms against this kernel's 0.50)
    int rc = gemm_bf16_tri(2, S, 1, 1, S, HS, B * S, dqr, ldr, B * S * ldr, a.qkv, a.ldq, HS, dR, MSQ_F32, HS,
                           a.S_max * HS, H, MSQ_EPI_ACCUM, nullptr, MSQ_F32, 0, 0, s, dr_ws, dr_ws_bytes(B, S, H));
    if (rc) return msq_set_error(MSQ_ERR_ARG, "flash_bwd: dR product");
    hipLaunchKernelGGL(flash_bwd_meta5_kernel, dim3(1, (unsigned)H, (unsigned)B), dim3(HS), 0, s, a, lse, Dv, dout,
                       ldo, dqkv, ldd, mdr);
    hipLaunchKernelGGL(flash_bwd_meta_dr_kernel, dim3((unsigned)H, 8), dim3(HS), 0, s, a, mdr, dR);
    return 0;
}
