// Memory-bound row/element kernels: embedding gather/scatter, LayerNorm
// fwd/bwd, column sums (bias grads), casts and Adam. All HBM-bound; loads are
// 16-B (fp32x4) or 8-B (bf16x4) per lane (guide §6 G13).
#include "common.h"
#include <cstdlib>

// ------------------------------------------------------------------ embedding
// model_transformer.py:152-155 / mamba.py:29-30: meta rows first, then tokens.
__global__ void embed_fwd_kernel(float* __restrict__ x, const float* __restrict__ tok, const float* __restrict__ met,
                                 const int64_t* __restrict__ idx, const int64_t* __restrict__ meta, int64_t B,
                                 int64_t T, int64_t nm, int64_t d) {
    const int64_t S = T + nm;
    const int64_t d4 = d / 4;
    const int64_t total = B * S * d4;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e % d4, row = e / d4;
        const int64_t b = row / S, s = row % S;
        const float* src = s < nm ? met + meta[b * nm + s] * d : tok + idx[b * T + (s - nm)] * d;
        *(f32x4*)(x + row * d + c * 4) = *(const f32x4*)(src + c * 4);
    }
}

__global__ void embed_bwd_kernel(float* __restrict__ gt, float* __restrict__ gm, const float* __restrict__ dx,
                                 const int64_t* __restrict__ idx, const int64_t* __restrict__ meta, int64_t B,
                                 int64_t T, int64_t nm, int64_t d) {
    const int64_t S = T + nm;
    const int64_t total = B * S * d;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e % d, row = e / d;
        const int64_t b = row / S, s = row % S;
        float* dst = s < nm ? gm + meta[b * nm + s] * d : gt + idx[b * T + (s - nm)] * d;
        atomicAdd(dst + c, dx[e]);
    }
}

extern "C" int msq_embed_fwd(float* x, const float* tok_table, const float* meta_table, const int64_t* idx,
                             const int64_t* meta, int64_t B, int64_t T, int64_t n_meta, int64_t d, void* stream) {
    MSQ_CHECK_ARG(d % 4 == 0 && B > 0 && T >= 0 && n_meta >= 0, "msq_embed_fwd: d %% 4 != 0 or bad sizes");
    const int64_t total = B * (T + n_meta) * (d / 4);
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, tok_table, meta_table,
                       idx, meta, B, T, n_meta, d);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

extern "C" int msq_embed_bwd(float* g_tok, float* g_meta, const float* dx, const int64_t* idx, const int64_t* meta,
                             int64_t B, int64_t T, int64_t n_meta, int64_t d, void* stream) {
    MSQ_CHECK_ARG(B > 0 && d > 0, "msq_embed_bwd: bad sizes");
    const int64_t total = B * (T + n_meta) * d;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 16384);
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, g_tok, g_meta, dx, idx,
                       meta, B, T, n_meta, d);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ------------------------------------------------ deterministic embedding backward
// The same scatter-add as embed_bwd_kernel with a fixed summation order, so the
// gradient is bitwise reproducible (a sorted segment sum). Every
// dx row r gets one key: its token id, or V_tok + its metadata id (ids out of
// range get the dropped key K = V_tok + V_meta). An LSD radix sort with 8-bit
// digits (2 passes at the 17 914 + 568 keys of cfg 2) orders the rows by key,
// stably, so each table row then sums its rows in sequence order:
//   key:     keys[r], pos[r] = r
//   per pass rank: per 256-row chunk, a row's rank among the equal digits before
//                  it (LDS compare); the chunk's last one writes cnt[digit][chunk]
//            scan: exclusive scan of cnt (digit-major, two launches) = where each
//                  (digit, chunk) group lands
//            scatter: (key, pos) to its place
//   sum:     blocks of EMB_P sorted rows, one wave per 256 columns: a key run
//            wholly inside the block is added to its table row directly (its only
//            writer); runs crossing a block edge leave per-block partials
//   fix:     the block where a crossing run ends adds that run's partials in
//            block order
// HBM traffic: one read of dx (the row sums) plus ~50 B of index arrays per row.
#define EMB_CH 256
#define EMB_P 64

__global__ void emb_key_kernel(int* __restrict__ key, int* __restrict__ pos, const int64_t* __restrict__ idx,
                               const int64_t* __restrict__ meta, int64_t N, int64_t T, int64_t nm, int64_t Vt,
                               int64_t Vm) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const int64_t S = T + nm, K = Vt + Vm;
    const int64_t b = r / S, s = r % S;
    int64_t k;
    if (s < nm) {
        const int64_t m = meta[b * nm + s];
        k = (m >= 0 && m < Vm) ? Vt + m : K;
    } else {
        const int64_t t = idx[b * T + (s - nm)];
        k = (t >= 0 && t < Vt) ? t : K;
    }
    key[r] = (int)k;
    pos[r] = (int)r;
}

__global__ __launch_bounds__(EMB_CH) void emb_rank_kernel(int* __restrict__ cnt, int* __restrict__ rank,
                                                          const int* __restrict__ key, int64_t N, int shift,
                                                          int64_t nch) {
    __shared__ int dig[EMB_CH];
    const int tid = threadIdx.x;
    const int64_t r = (int64_t)blockIdx.x * EMB_CH + tid;
    const int dg = r < N ? (key[r] >> shift) & 255 : -1;
    dig[tid] = dg;
    __syncthreads();
    int rk = 0;
    bool last = true;
#pragma unroll 8
    for (int j = 0; j < EMB_CH; ++j) {  // broadcast LDS reads
        const int dj = dig[j];
        rk += (j < tid && dj == dg);
        last = last && !(j > tid && dj == dg);
    }
    if (r < N) {
        rank[r] = rk;
        if (last) cnt[(int64_t)dg * nch + blockIdx.x] = rk + 1;
    }
}

// exclusive scan of n ints in place (n % 4 == 0), two launches: each 1024-thread
// block scans 4096 ints (int4 per thread, LDS scan of the thread sums) and
// leaves its total; then every block adds the totals of the blocks before it.
// a[n] = the grand total.
#define EMB_SCAN 4096
__device__ __forceinline__ int block_excl_scan(int v, int* lds) {  // 1024 threads
    const int tid = threadIdx.x;
    lds[tid] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int u = tid >= off ? lds[tid - off] : 0;
        __syncthreads();
        lds[tid] += u;
        __syncthreads();
    }
    return lds[tid] - v;
}

__global__ __launch_bounds__(1024) void emb_scan_local_kernel(int* __restrict__ a, int* __restrict__ tot, int64_t n) {
    __shared__ int lds[1024];
    const int64_t i = (int64_t)blockIdx.x * EMB_SCAN + threadIdx.x * 4;
    int4 v = {0, 0, 0, 0};
    if (i < n) v = *(const int4*)(a + i);
    const int ex = block_excl_scan(v.x + v.y + v.z + v.w, lds);
    if (i < n) *(int4*)(a + i) = int4{ex, ex + v.x, ex + v.x + v.y, ex + v.x + v.y + v.z};
    if (threadIdx.x == 1023) tot[blockIdx.x] = lds[1023];
}

__global__ __launch_bounds__(1024) void emb_scan_add_kernel(int* __restrict__ a, const int* __restrict__ tot,
                                                            int64_t n) {
    __shared__ int lds[1024];
    const int g = blockIdx.x;
    int s = 0;
    for (int h = threadIdx.x; h < g; h += 1024) s += tot[h];
    lds[threadIdx.x] = s;
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) lds[threadIdx.x] += lds[threadIdx.x + off];
        __syncthreads();
    }
    const int pre = lds[0];
    const int64_t i = (int64_t)g * EMB_SCAN + threadIdx.x * 4;
    if (i < n) {
        int4 v = *(const int4*)(a + i);
        *(int4*)(a + i) = int4{v.x + pre, v.y + pre, v.z + pre, v.w + pre};
    }
    if (g == (int)gridDim.x - 1 && threadIdx.x == 0) a[n] = pre + tot[g];
}

__global__ void emb_scatter_kernel(int* __restrict__ key_out, int* __restrict__ pos_out, const int* __restrict__ off,
                                   const int* __restrict__ rank, const int* __restrict__ key_in,
                                   const int* __restrict__ pos_in, int64_t N, int shift, int64_t nch) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const int k = key_in[r];
    const int64_t dst = off[(int64_t)((k >> shift) & 255) * nch + r / EMB_CH] + rank[r];
    key_out[dst] = k;
    pos_out[dst] = pos_in[r];
}

__device__ __forceinline__ float* emb_row(float* gt, float* gm, int key, int64_t Vt, int64_t d) {
    return key < Vt ? gt + (int64_t)key * d : gm + ((int64_t)key - Vt) * d;
}

// grid (blocks of EMB_P sorted rows, column slices of 256), one wave. Lane j
// holds the block's j-th (row, key); rows are broadcast with readlane so 16
// row loads are in flight before the ordered adds.
__global__ __launch_bounds__(64) void emb_sum_kernel(float* __restrict__ gt, float* __restrict__ gm,
                                                     float* __restrict__ part, const float* __restrict__ dx,
                                                     const int* __restrict__ spos, const int* __restrict__ skey,
                                                     int64_t N, int64_t d, int64_t Vt, int K) {
    static_assert(EMB_P == 64, "one sorted row per lane");
    const int64_t blk = blockIdx.x;
    const int64_t b0 = blk * EMB_P;
    const int n = (int)std::min<int64_t>(EMB_P, N - b0);
    const int lane = threadIdx.x;
    const int64_t c = ((int64_t)blockIdx.y * 64 + lane) * 4;
    const bool on = c < d;
    const int myp = lane < n ? spos[b0 + lane] : 0;
    const int myk = lane < n ? skey[b0 + lane] : -1;
    const int prevk = b0 > 0 ? skey[b0 - 1] : -1;  // the keys either side of the block
    const int nextk = b0 + n < N ? skey[b0 + n] : -1;
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    f32x4 acc = zero;
    int cur = __builtin_amdgcn_readlane(myk, 0);
    int rs = 0;
    auto flush = [&](int key, int s0, int s1) {
        if (key == K || !on) return;
        const bool start_in = s0 > 0 || prevk != key;
        const bool end_in = s1 < n || nextk != key;
        if (start_in && end_in) {
            f32x4* dst = (f32x4*)(emb_row(gt, gm, key, Vt, d) + c);
            *dst = *dst + acc;
        } else {
            *(f32x4*)(part + (blk * 2 + (s0 == 0 ? 0 : 1)) * d + c) = acc;
        }
    };
    for (int j0 = 0; j0 < n; j0 += 16) {
        f32x4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = j0 + u;
            const int row = __builtin_amdgcn_readlane(myp, j & 63);
            v[u] = (j < n && on) ? *(const f32x4*)(dx + (int64_t)row * d + c) : zero;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int j = j0 + u;
            if (j < n) {
                const int k = __builtin_amdgcn_readlane(myk, j & 63);
                if (k != cur) {
                    flush(cur, rs, j);
                    acc = zero;
                    cur = k;
                    rs = j;
                }
                acc = acc + v[u];
            }
        }
    }
    flush(cur, rs, n);
}

// grid (blocks, column slices), one wave: the block in which a run that began in
// an earlier block ends sums the run's partials (first block's, then one per
// block) and adds them to the table row
__global__ __launch_bounds__(64) void emb_fix_kernel(float* __restrict__ gt, float* __restrict__ gm,
                                                     const float* __restrict__ part, const int* __restrict__ skey,
                                                     int64_t N, int64_t d, int64_t Vt, int K) {
    const int64_t blk = blockIdx.x;
    const int64_t b0 = blk * EMB_P, b1 = std::min<int64_t>(N, b0 + EMB_P);
    if (blk == 0) return;
    const int key = skey[b0];
    if (key == K || skey[b0 - 1] != key || (b1 < N && skey[b1] == key)) return;
    const int64_t c = ((int64_t)blockIdx.y * 64 + threadIdx.x) * 4;
    if (c >= d) return;
    int64_t lo = 0, hi = b0 - 1;  // first sorted row of the key (skey[hi] == key)
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (skey[mid] < key) lo = mid + 1; else hi = mid;
    }
    const int64_t s = lo;
    f32x4 acc = *(const f32x4*)(part + ((s / EMB_P) * 2 + (s % EMB_P == 0 ? 0 : 1)) * d + c);
    for (int64_t k = s / EMB_P + 1; k <= blk; ++k) acc = acc + *(const f32x4*)(part + k * 2 * d + c);
    f32x4* dst = (f32x4*)(emb_row(gt, gm, key, Vt, d) + c);
    *dst = *dst + acc;
}

namespace {
struct EmbWs {
    int64_t N, nch, nblk, ncnt;
    int passes;
    int64_t nscan;
    size_t o_cnt, o_tot, o_rank, o_k0, o_p0, o_k1, o_p1, o_part, total;
};
size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
EmbWs emb_ws(int64_t B, int64_t T, int64_t nm, int64_t d, int64_t Vt, int64_t Vm) {
    EmbWs w;
    w.N = B * (T + nm);
    w.nch = (w.N + EMB_CH - 1) / EMB_CH;
    w.nblk = (w.N + EMB_P - 1) / EMB_P;
    w.ncnt = 256 * w.nch;
    w.passes = 1;
    while ((Vt + Vm) >> (8 * w.passes)) ++w.passes;  // digits of the largest key K
    const size_t nb = al16(w.N * 4);
    w.nscan = (w.ncnt + EMB_SCAN - 1) / EMB_SCAN;
    w.o_cnt = 0;
    w.o_tot = al16((w.ncnt + 1) * 4);
    w.o_rank = w.o_tot + al16(w.nscan * 4);
    w.o_k0 = w.o_rank + nb;
    w.o_p0 = w.o_k0 + nb;
    w.o_k1 = w.o_p0 + nb;
    w.o_p1 = w.o_k1 + nb;
    w.o_part = w.o_p1 + nb;
    w.total = w.o_part + al16(w.nblk * 2 * d * 4);
    return w;
}
}  // namespace

extern "C" size_t msq_embed_bwd_workspace(int64_t B, int64_t T, int64_t n_meta, int64_t d, int64_t V_tok,
                                          int64_t V_meta) {
    return emb_ws(B, T, n_meta, d, V_tok, V_meta).total;
}

extern "C" int msq_embed_bwd_sorted(float* g_tok, float* g_meta, const float* dx, const int64_t* idx,
                                    const int64_t* meta, int64_t B, int64_t T, int64_t n_meta, int64_t d,
                                    int64_t V_tok, int64_t V_meta, void* workspace, void* stream) {
    MSQ_CHECK_ARG(B > 0 && T >= 0 && n_meta >= 0 && d > 0 && d % 4 == 0 && V_tok > 0 && V_meta >= 0 && workspace,
                  "msq_embed_bwd_sorted: bad sizes or no workspace");
    const EmbWs w = emb_ws(B, T, n_meta, d, V_tok, V_meta);
    MSQ_CHECK_ARG(w.N < INT32_MAX && V_tok + V_meta < INT32_MAX, "msq_embed_bwd_sorted: more than 2^31 rows or keys");
    MSQ_CHECK_ARG(((uintptr_t)workspace % 16) == 0, "msq_embed_bwd_sorted: workspace must be 16-B aligned");
    if (w.N == 0) return MSQ_OK;
    hipStream_t s = (hipStream_t)stream;
    char* ws = (char*)workspace;
    int* cnt = (int*)(ws + w.o_cnt);
    int* tot = (int*)(ws + w.o_tot);
    int* rank = (int*)(ws + w.o_rank);
    int* key[2] = {(int*)(ws + w.o_k0), (int*)(ws + w.o_k1)};
    int* pos[2] = {(int*)(ws + w.o_p0), (int*)(ws + w.o_p1)};
    float* part = (float*)(ws + w.o_part);
    const int K = (int)(V_tok + V_meta);
    const int slices = (int)((d / 4 + 63) / 64);
    const unsigned rows256 = (unsigned)((w.N + 255) / 256);
    hipLaunchKernelGGL(emb_key_kernel, dim3(rows256), dim3(256), 0, s, key[0], pos[0], idx, meta, w.N, T, n_meta,
                       V_tok, V_meta);
    for (int p = 0; p < w.passes; ++p) {
        const int in = p & 1, shift = 8 * p;
        if (hipMemsetAsync(cnt, 0, w.ncnt * 4, s) != hipSuccess)
            return msq_set_error(MSQ_ERR_HIP, "msq_embed_bwd_sorted: memset");
        hipLaunchKernelGGL(emb_rank_kernel, dim3((unsigned)w.nch), dim3(EMB_CH), 0, s, cnt, rank, key[in], w.N, shift,
                           w.nch);
        hipLaunchKernelGGL(emb_scan_local_kernel, dim3((unsigned)w.nscan), dim3(1024), 0, s, cnt, tot, w.ncnt);
        hipLaunchKernelGGL(emb_scan_add_kernel, dim3((unsigned)w.nscan), dim3(1024), 0, s, cnt, tot, w.ncnt);
        hipLaunchKernelGGL(emb_scatter_kernel, dim3(rows256), dim3(256), 0, s, key[in ^ 1], pos[in ^ 1], cnt, rank,
                           key[in], pos[in], w.N, shift, w.nch);
    }
    const int out = w.passes & 1;
    hipLaunchKernelGGL(emb_sum_kernel, dim3((unsigned)w.nblk, slices), dim3(64), 0, s, g_tok, g_meta, part, dx,
                       pos[out], key[out], w.N, d, V_tok, K);
    hipLaunchKernelGGL(emb_fix_kernel, dim3((unsigned)w.nblk, slices), dim3(64), 0, s, g_tok, g_meta, part, key[out],
                       w.N, d, V_tok, K);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ------------------------------------------------------------------ LayerNorm
// one wave per row; the row (d <= 64*4*MAXC) is held in registers.
// Row r of the compact output maps to input row
//   (r / seg) * (seg + skip) + skip + r % seg      (identity when skip == 0)
// so LN_f can normalise only the T token rows of every [meta | tokens] segment.
__device__ __forceinline__ int64_t map_row(int64_t r, int64_t seg, int64_t skip) {
    return skip == 0 ? r : (r / seg) * (seg + skip) + skip + r % seg;
}
template <typename TY, int MAXC>
__global__ __launch_bounds__(256) void ln_fwd_kernel(TY* __restrict__ y, float* __restrict__ mean,
                                                     float* __restrict__ rstd, const float* __restrict__ x,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     int64_t rows, int d, float eps, int64_t seg, int64_t skip) {
    const int lane = threadIdx.x & 63;
    const int64_t row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + map_row(row, seg, skip) * d;
    f32x4 v[MAXC];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int col = (c * 64 + lane) * 4;
        v[c] = col < d ? *(const f32x4*)(xr + col) : (f32x4){0.f, 0.f, 0.f, 0.f};
        s += v[c][0] + v[c][1] + v[c][2] + v[c][3];
    }
    const float mu = wave_sum(s) / d;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int col = (c * 64 + lane) * 4;
        if (col < d) {
#pragma unroll
            for (int t = 0; t < 4; ++t) { const float z = v[c][t] - mu; q += z * z; }
        }
    }
    const float rs = rsqrtf(wave_sum(q) / d + eps);
    if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
    TY* yr = y + row * d;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int col = (c * 64 + lane) * 4;
        if (col < d) {
            const f32x4 g = *(const f32x4*)(gamma + col), b = *(const f32x4*)(beta + col);
            f32x4 o;
#pragma unroll
            for (int t = 0; t < 4; ++t) o[t] = (v[c][t] - mu) * rs * g[t] + b[t];
            store4(yr + col, o);
        }
    }
}

// persistent grid of the LayerNorm backward: one workgroup per SIMD-wave slot
// the kernel's VGPR count allows (d <= 256: 3 per CU; d <= 1024, two rows in
// flight per wave at 216 VGPRs: 2; wider: 1); the partial-sum workspace is
// sized for the largest grid
constexpr int LN_BWD_MAX_BLOCKS = 1024;
static int ln_bwd_blocks(int64_t d) { return d <= 256 ? 768 : (d <= 1024 ? 512 : 256); }
// rows per work-queue ticket of the LayerNorm backward (2 and 8 measured slower)
constexpr int LN_QROWS = 4;

// dropout keep mask applied to the copy (the gradient into the dropped branch)
struct CopyDrop {
    uint32_t base, thr;
    float scale;
    int on;
};

// dx_acc += rstd*(dyg - mean(dyg) - xhat*mean(dyg*xhat)); per-block dgamma/dbeta
// partials, and (BIAS) the column sums of the written gradient rows (the copy
// after its dropout mask, else the updated dx_acc): the bias gradient of the
// residual branch that produced this LayerNorm's input (model_transformer.py
// :51,101 proj / FFN output biases), which would otherwise be a separate
// column-sum pass over the same rows
template <typename TD, typename TO, int MAXC, bool BIAS>
__global__ __launch_bounds__(256) void ln_bwd_kernel(float* __restrict__ dxa, TO* __restrict__ dcopy,
                                                     float* __restrict__ part, const TD* __restrict__ dy,
                                                     const float* __restrict__ x, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                     int64_t rows, int d, int64_t seg, int64_t skip, CopyDrop cd,
                                                     int* __restrict__ ctr) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    f32x4 pg[MAXC], pb[MAXC], pc[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) pg[c] = pb[c] = pc[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // row schedule: with ctr, a work queue of LNQ-row chunks per WAVE: chunk
    // (wave id) first, then tickets nwaves + atomicAdd(ctr, 1) (lane 0,
    // broadcast by readfirstlane, each requested one chunk ahead), so waves
    // that start late (their CUs held by the other stream's GEMM tiles) take
    // fewer rows instead of finishing last; without, rows blockIdx*4 + wid +
    // k gridDim*4
    constexpr int LNQ = LN_QROWS;
    const int nwaves = gridDim.x * 4;
    int64_t row, rend;
    int tk = 0;
    if (ctr) {
        row = (int64_t)(blockIdx.x * 4 + wid) * LNQ;
        rend = row + LNQ;
        if (lane == 0 && row < rows) tk = atomicAdd(ctr, 1);
    } else {
        row = blockIdx.x * 4LL + wid;
        rend = rows;
    }
    // the row after `row` in this wave's schedule
    auto advance = [&]() {
        if (!ctr) {
            row += (int64_t)gridDim.x * 4;
            return;
        }
        if (++row >= rend) {
            const int t = nwaves + __builtin_amdgcn_readfirstlane(__shfl(tk, 0, 64));
            row = (int64_t)t * LNQ;
            rend = row + LNQ;
            if (lane == 0 && row < rows) tk = atomicAdd(ctr, 1);
        }
    };
    f32x4 gm[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int col = (c * 64 + lane) * 4;
        gm[c] = col < d ? *(const f32x4*)(gamma + col) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    // two rows in flight per wave: the next row's x / dy / dx_acc are loaded
    // while this row is reduced and written (one row at a time left the
    // kernel latency-bound: 80 % of wave cycles waiting at 3.6 TB/s)
    f32x4 nx[MAXC], nacc[MAXC];
    TD ndy[MAXC][4];
    float nmu = 0.f, nrs = 0.f;
    auto fetch = [&](int64_t r) {
        nmu = mean[r];
        nrs = rstd[r];
        const int64_t xr = map_row(r, seg, skip);
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int col = (c * 64 + lane) * 4;
            if (col < d) {
                nx[c] = *(const f32x4*)(x + xr * d + col);
                nacc[c] = *(const f32x4*)(dxa + xr * d + col);
#pragma unroll
                for (int t = 0; t < 4; ++t) ndy[c][t] = dy[r * d + col + t];
            }
        }
    };
    if (row < rows) fetch(row);
    for (;;) {
        if (row >= rows) break;
        const int64_t cur = row, xrow = map_row(cur, seg, skip);
        const float mu = nmu, rs = nrs;
        f32x4 xv[MAXC], acc[MAXC], dv[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            xv[c] = nx[c];
            acc[c] = nacc[c];
            dv[c] = (f32x4){to_f(ndy[c][0]), to_f(ndy[c][1]), to_f(ndy[c][2]), to_f(ndy[c][3])};
        }
        advance();
        if (row < rows) fetch(row);
        {
        f32x4 xh[MAXC], g[MAXC];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int col = (c * 64 + lane) * 4;
            if (col < d) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    xh[c][t] = (xv[c][t] - mu) * rs;
                    g[c][t] = dv[c][t] * gm[c][t];
                    s1 += g[c][t];
                    s2 += g[c][t] * xh[c][t];
                    pg[c][t] += dv[c][t] * xh[c][t];
                    pb[c][t] += dv[c][t];
                }
            } else {
                xh[c] = g[c] = acc[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
            }
        }
        const float m1 = wave_sum(s1) / d, m2 = wave_sum(s2) / d;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int col = (c * 64 + lane) * 4;
            if (col < d) {
                float* dp = dxa + xrow * d + col;
                f32x4 o = acc[c];
#pragma unroll
                for (int t = 0; t < 4; ++t) o[t] += rs * (g[c][t] - m1 - xh[c][t] * m2);
                *(f32x4*)dp = o;
                if (dcopy) {
                    if (cd.on) {  // d(dropped branch) = g * keep / (1-p) at (row xrow, col)
                        const uint32_t rk = drop_row(cd.base, (uint32_t)xrow);
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            o[t] = drop_bits(rk, (uint32_t)(col + t)) >= cd.thr ? o[t] * cd.scale : 0.f;
                    }
                    store4(dcopy + xrow * d + col, o);
                }
                if (BIAS) pc[c] += o;
            }
        }
        }
    }
    // block reduce of the partials through LDS, then one row per block
    __shared__ f32x4 red[4][64 * MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) red[wid][c * 64 + lane] = pg[c];
    __syncthreads();
    if (wid == 0) {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int col = (c * 64 + lane) * 4;
            f32x4 t = red[0][c * 64 + lane] + red[1][c * 64 + lane] + red[2][c * 64 + lane] + red[3][c * 64 + lane];
            if (col < d) *(f32x4*)(part + (int64_t)blockIdx.x * 3 * d + col) = t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < MAXC; ++c) red[wid][c * 64 + lane] = pb[c];
    __syncthreads();
    if (wid == 0) {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const int col = (c * 64 + lane) * 4;
            f32x4 t = red[0][c * 64 + lane] + red[1][c * 64 + lane] + red[2][c * 64 + lane] + red[3][c * 64 + lane];
            if (col < d) *(f32x4*)(part + (int64_t)blockIdx.x * 3 * d + d + col) = t;
        }
    }
    if (BIAS) {
        __syncthreads();
#pragma unroll
        for (int c = 0; c < MAXC; ++c) red[wid][c * 64 + lane] = pc[c];
        __syncthreads();
        if (wid == 0) {
#pragma unroll
            for (int c = 0; c < MAXC; ++c) {
                const int col = (c * 64 + lane) * 4;
                f32x4 t = red[0][c * 64 + lane] + red[1][c * 64 + lane] + red[2][c * 64 + lane] + red[3][c * 64 + lane];
                if (col < d) *(f32x4*)(part + (int64_t)blockIdx.x * 3 * d + 2 * d + col) = t;
            }
        }
    }
}

// out[c] += sum_p part[p, c] for c < nout (dgamma | dbeta | dbias), partial rows 3d apart
// block = 64 columns x 4 waves; each wave sums every 4th partial row
__global__ __launch_bounds__(256) void ln_reduce_kernel(float* __restrict__ dg, float* __restrict__ db,
                                                        float* __restrict__ dbias, const float* __restrict__ part,
                                                        int nparts, int d, int nout) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (c < nout) {
#pragma unroll 8
        for (int p = w; p < nparts; p += 4) s += part[(int64_t)p * 3 * d + c];
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && c < nout) {
        s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        if (c < d) dg[c] += s;
        else if (c < 2 * d) db[c - d] += s;
        else dbias[c - 2 * d] += s;
    }
}

extern "C" size_t msq_layernorm_bwd_workspace(int64_t rows, int64_t d) {
    (void)rows;
    return (size_t)LN_BWD_MAX_BLOCKS * 3 * d * sizeof(float) + 64;
}

template <typename TY>
static void ln_fwd_launch(TY* y, float* mean, float* rstd, const float* x, const float* g, const float* b,
                          int64_t rows, int d, float eps, int64_t seg, int64_t skip, hipStream_t s) {
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (d <= 256) hipLaunchKernelGGL((ln_fwd_kernel<TY, 1>), grid, dim3(256), 0, s, y, mean, rstd, x, g, b, rows, d, eps, seg, skip);
    else if (d <= 1024) hipLaunchKernelGGL((ln_fwd_kernel<TY, 4>), grid, dim3(256), 0, s, y, mean, rstd, x, g, b, rows, d, eps, seg, skip);
    else hipLaunchKernelGGL((ln_fwd_kernel<TY, 8>), grid, dim3(256), 0, s, y, mean, rstd, x, g, b, rows, d, eps, seg, skip);
}

extern "C" int msq_layernorm_fwd(void* y, int y_dtype, float* mean, float* rstd, const float* x, const float* gamma,
                                 const float* beta, int64_t rows, int64_t d, float eps, int64_t seg_len,
                                 int64_t seg_skip, void* stream) {
    MSQ_CHECK_ARG(d % 4 == 0 && d <= 2048 && rows > 0, "msq_layernorm_fwd: need d %% 4 == 0, d <= 2048");
    MSQ_CHECK_ARG(seg_skip == 0 || seg_len > 0, "msq_layernorm_fwd: seg_len must be > 0 with seg_skip");
    hipStream_t s = (hipStream_t)stream;
    if (y_dtype == MSQ_BF16) ln_fwd_launch((bf16*)y, mean, rstd, x, gamma, beta, rows, (int)d, eps, seg_len, seg_skip, s);
    else ln_fwd_launch((float*)y, mean, rstd, x, gamma, beta, rows, (int)d, eps, seg_len, seg_skip, s);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

template <typename TD, typename TO, bool BIAS>
static void ln_bwd_launch_b(float* dxa, TO* dcopy, float* part, const TD* dy, const float* x, const float* mean,
                            const float* rstd, const float* gamma, int64_t rows, int d, int64_t seg, int64_t skip,
                            CopyDrop cd, bool queue, hipStream_t s) {
    // the work-queue ticket counter sits after the partials (zeroed per launch)
    int* ctr = queue ? (int*)(part + (int64_t)LN_BWD_MAX_BLOCKS * 3 * d) : nullptr;
    if (ctr) (void)hipMemsetAsync(ctr, 0, sizeof(int), s);
    const dim3 grid(ln_bwd_blocks(d));
    if (d <= 256) hipLaunchKernelGGL((ln_bwd_kernel<TD, TO, 1, BIAS>), grid, dim3(256), 0, s, dxa, dcopy, part, dy, x, mean, rstd, gamma, rows, d, seg, skip, cd, ctr);
    else if (d <= 1024) hipLaunchKernelGGL((ln_bwd_kernel<TD, TO, 4, BIAS>), grid, dim3(256), 0, s, dxa, dcopy, part, dy, x, mean, rstd, gamma, rows, d, seg, skip, cd, ctr);
    else hipLaunchKernelGGL((ln_bwd_kernel<TD, TO, 8, BIAS>), grid, dim3(256), 0, s, dxa, dcopy, part, dy, x, mean, rstd, gamma, rows, d, seg, skip, cd, ctr);
}
template <typename TD, typename TO>
static void ln_bwd_launch(float* dxa, TO* dcopy, float* part, const TD* dy, const float* x, const float* mean,
                          const float* rstd, const float* gamma, int64_t rows, int d, int64_t seg, int64_t skip,
                          CopyDrop cd, bool bias, bool queue, hipStream_t s) {
    if (bias) ln_bwd_launch_b<TD, TO, true>(dxa, dcopy, part, dy, x, mean, rstd, gamma, rows, d, seg, skip, cd, queue, s);
    else ln_bwd_launch_b<TD, TO, false>(dxa, dcopy, part, dy, x, mean, rstd, gamma, rows, d, seg, skip, cd, queue, s);
}

extern "C" int msq_layernorm_bwd(float* dx_acc, void* dx_copy, int copy_dtype, float* dgamma, float* dbeta,
                                 const void* dy, int dy_dtype, const float* x, const float* mean, const float* rstd,
                                 const float* gamma, int64_t rows, int64_t d, int64_t seg_len, int64_t seg_skip,
                                 void* workspace, void* stream) {
    return msq_layernorm_bwd_dropout(dx_acc, dx_copy, copy_dtype, dgamma, dbeta, dy, dy_dtype, x, mean, rstd, gamma,
                                     rows, d, seg_len, seg_skip, 0u, 0u, 0.f, workspace, stream);
}

extern "C" int msq_layernorm_bwd_dropout(float* dx_acc, void* dx_copy, int copy_dtype, float* dgamma, float* dbeta,
                                         const void* dy, int dy_dtype, const float* x, const float* mean,
                                         const float* rstd, const float* gamma, int64_t rows, int64_t d,
                                         int64_t seg_len, int64_t seg_skip, uint32_t seed, uint32_t site, float p,
                                         void* workspace, void* stream) {
    return msq_layernorm_bwd_bias(dx_acc, dx_copy, copy_dtype, dgamma, dbeta, nullptr, dy, dy_dtype, x, mean, rstd,
                                  gamma, rows, d, seg_len, seg_skip, seed, site, p, 0, workspace, stream);
}

extern "C" int msq_layernorm_bwd_bias(float* dx_acc, void* dx_copy, int copy_dtype, float* dgamma, float* dbeta,
                                      float* dbias, const void* dy, int dy_dtype, const float* x, const float* mean,
                                      const float* rstd, const float* gamma, int64_t rows, int64_t d, int64_t seg_len,
                                      int64_t seg_skip, uint32_t seed, uint32_t site, float p, int schedule,
                                      void* workspace, void* stream) {
    MSQ_CHECK_ARG(d % 4 == 0 && d <= 2048 && rows > 0 && workspace, "msq_layernorm_bwd: bad args");
    MSQ_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || dx_copy), "msq_layernorm_bwd: dropout needs dx_copy");
    CopyDrop cd{drop_base(seed, site), drop_threshold(p), 1.f / (1.f - p), p > 0.f ? 1 : 0};
    MSQ_CHECK_ARG(seg_skip == 0 || seg_len > 0, "msq_layernorm_bwd: seg_len must be > 0 with seg_skip");
    hipStream_t s = (hipStream_t)stream;
    float* part = (float*)workspace;
    const int di = (int)d;
    const bool bias = dbias != nullptr, queue = schedule == 1;
    MSQ_CHECK_ARG(schedule == 0 || schedule == 1, "msq_layernorm_bwd_bias: schedule must be 0 or 1");
    if (dy_dtype == MSQ_BF16) {
        if (copy_dtype == MSQ_BF16) ln_bwd_launch(dx_acc, (bf16*)dx_copy, part, (const bf16*)dy, x, mean, rstd, gamma, rows, di, seg_len, seg_skip, cd, bias, queue, s);
        else ln_bwd_launch(dx_acc, (float*)dx_copy, part, (const bf16*)dy, x, mean, rstd, gamma, rows, di, seg_len, seg_skip, cd, bias, queue, s);
    } else {
        if (copy_dtype == MSQ_BF16) ln_bwd_launch(dx_acc, (bf16*)dx_copy, part, (const float*)dy, x, mean, rstd, gamma, rows, di, seg_len, seg_skip, cd, bias, queue, s);
        else ln_bwd_launch(dx_acc, (float*)dx_copy, part, (const float*)dy, x, mean, rstd, gamma, rows, di, seg_len, seg_skip, cd, bias, queue, s);
    }
    const int nout = (bias ? 3 : 2) * di;
    hipLaunchKernelGGL(ln_reduce_kernel, dim3((unsigned)((nout + 63) / 64)), dim3(256), 0, s, dgamma, dbeta, dbias,
                       part, ln_bwd_blocks(di), di, nout);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ------------------------------------------------------------------ colsum
constexpr int CS_SPLIT = 128;

template <typename T>
__global__ void colsum_part_kernel(float* __restrict__ part, const T* __restrict__ x, int64_t rows, int64_t cols,
                                   int64_t ld) {
    // block (col chunk of 1024, row split); each thread 4 columns
    const int64_t c = (blockIdx.x * 256LL + threadIdx.x) * 4;
    const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
    const int64_t r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
    if (c >= cols) return;
    f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (c + 4 <= cols) {
        for (int64_t r = r0; r < r1; ++r) s += load4(x + r * ld + c);
    } else {
        for (int64_t r = r0; r < r1; ++r)
            for (int t = 0; c + t < cols; ++t) s[t] += (float)x[r * ld + c + t];
    }
    for (int t = 0; t < 4 && c + t < cols; ++t) part[blockIdx.y * cols + c + t] = s[t];
}

__global__ void colsum_reduce_kernel(float* __restrict__ out, const float* __restrict__ part, int nparts,
                                     int64_t cols, int accumulate) {
    const int64_t c = blockIdx.x * 256LL + threadIdx.x;
    if (c >= cols) return;
    float s = 0.f;
    for (int p = 0; p < nparts; ++p) s += part[p * cols + c];
    out[c] = accumulate ? out[c] + s : s;
}

// streaming variant: 1024-thread workgroups (16 waves) = row groups x column
// vectors of N = 16/sizeof(T) columns, 8 independent 16-B loads in flight per
// thread, the row groups folded in LDS, then one fp32 atomic per column per
// workgroup (about 256 workgroups: few atomics per address).
template <typename T>
__global__ __launch_bounds__(1024) void colsum2_kernel(float* __restrict__ out, const T* __restrict__ x, int64_t rows,
                                                       int64_t cols, int64_t ld, int tpr) {
    constexpr int N = 16 / sizeof(T), U = 8;
    __shared__ float red[1024 * 4];
    const int tid = threadIdx.x, rg = tid / tpr, rgs = 1024 / tpr, ti = tid - rg * tpr;
    const int64_t c = ((int64_t)blockIdx.x * tpr + ti) * N;
    const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
    const int64_t r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
    float s[N];
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = 0.f;
    if (c < cols) {
        const T* p = x + c;
        const bool full = c + N <= cols;
        int64_t r = r0 + rg;
        if (full) {
            for (; r + (U - 1) * rgs < r1; r += U * rgs) {
                float v[U][N];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if constexpr (N == 8) {
                        const bf16x8 q = *(const bf16x8*)(p + (r + u * rgs) * ld);
#pragma unroll
                        for (int i = 0; i < N; ++i) v[u][i] = (float)q[i];
                    } else {
                        const f32x4 q = *(const f32x4*)(p + (r + u * rgs) * ld);
#pragma unroll
                        for (int i = 0; i < N; ++i) v[u][i] = q[i];
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int i = 0; i < N; ++i) s[i] += v[u][i];
            }
        }
        for (; r < r1; r += rgs)
#pragma unroll
            for (int i = 0; i < N; ++i)
                if (c + i < cols) s[i] += (float)p[r * ld + i];
    }
    // fold the row groups: red[rg][ti][i] (N <= 8, at most 4 row groups when N == 8)
    for (int h = 0; h < N; h += 4) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(rg * tpr + ti) * 4 + i] = h + i < N ? s[h + i] : 0.f;
        __syncthreads();
        if (rg == 0 && c < cols) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (h + i >= N || c + h + i >= cols) continue;
                float t = 0.f;
                for (int q = 0; q < rgs; ++q) t += red[(q * tpr + ti) * 4 + i];
                atomicAdd(out + c + h + i, t);
            }
        }
    }
}

extern "C" size_t msq_colsum_workspace(int64_t rows, int64_t cols) {
    (void)rows;
    return (size_t)CS_SPLIT * cols * sizeof(float);
}

extern "C" int msq_colsum(float* out, int accumulate, const void* x, int dtype, int64_t rows, int64_t cols,
                          int64_t ld, void* workspace, void* stream) {
    MSQ_CHECK_ARG(rows > 0 && cols > 0 && workspace && ld % 4 == 0, "msq_colsum: bad args (ld %% 4 == 0)");
    hipStream_t s = (hipStream_t)stream;
    {
        const int N = dtype == MSQ_BF16 ? 8 : 4;
        if (ld % N == 0 && ((uintptr_t)x % 16) == 0) {
            if (!accumulate) hipMemsetAsync(out, 0, (size_t)cols * 4, s);
            const int64_t cvec = (cols + N - 1) / N;
            const int tpr = (int)std::min<int64_t>(1024, std::max<int64_t>(64, (cvec + 63) / 64 * 64 > 512 ? 1024 : (cvec + 63) / 64 * 64 > 256 ? 512 : (cvec + 63) / 64 * 64 > 128 ? 256 : (cvec + 63) / 64 * 64 > 64 ? 128 : 64));
            const int64_t nch = (cvec + tpr - 1) / tpr;
            const int64_t split = std::max<int64_t>(1, std::min<int64_t>(rows / 64 + 1, 256 / nch + 1));
            dim3 g2((unsigned)nch, (unsigned)split);
            if (dtype == MSQ_BF16) hipLaunchKernelGGL(colsum2_kernel<bf16>, g2, dim3(1024), 0, s, out, (const bf16*)x, rows, cols, ld, tpr);
            else hipLaunchKernelGGL(colsum2_kernel<float>, g2, dim3(1024), 0, s, out, (const float*)x, rows, cols, ld, tpr);
            MSQ_LAUNCH_CHECK();
            return MSQ_OK;
        }
    }
    const int split = (int)std::min<int64_t>(CS_SPLIT, rows);
    dim3 grid((unsigned)((cols + 1023) / 1024), (unsigned)split);
    if (dtype == MSQ_BF16) hipLaunchKernelGGL(colsum_part_kernel<bf16>, grid, dim3(256), 0, s, (float*)workspace, (const bf16*)x, rows, cols, ld);
    else hipLaunchKernelGGL(colsum_part_kernel<float>, grid, dim3(256), 0, s, (float*)workspace, (const float*)x, rows, cols, ld);
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, s, out,
                       (const float*)workspace, split, cols, accumulate);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ------------------------------------------------------------------ cast
template <typename TD, typename TS>
__global__ void cast_kernel(TD* __restrict__ d, const TS* __restrict__ s, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = (TD)(float)s[i];
}

extern "C" int msq_cast(void* dst, int dst_dtype, const void* src, int src_dtype, int64_t n, void* stream) {
    MSQ_CHECK_ARG(n >= 0, "msq_cast: n < 0");
    if (n == 0) return MSQ_OK;
    hipStream_t s = (hipStream_t)stream;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 16384);
    if (dst_dtype == MSQ_BF16 && src_dtype == MSQ_F32) hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(grid), dim3(256), 0, s, (bf16*)dst, (const float*)src, n);
    else if (dst_dtype == MSQ_F32 && src_dtype == MSQ_BF16) hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(grid), dim3(256), 0, s, (float*)dst, (const bf16*)src, n);
    else if (dst_dtype == MSQ_F32 && src_dtype == MSQ_F32) hipLaunchKernelGGL((cast_kernel<float, float>), dim3(grid), dim3(256), 0, s, (float*)dst, (const float*)src, n);
    else hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(grid), dim3(256), 0, s, (bf16*)dst, (const bf16*)src, n);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ------------------------------------------------------------------ transpose
// dst[c][r] = src[r][c] (bf16): the transposed weight shadows of the backward's
// dX products (dY . W reads W^T K-contiguous: the 256 tile's tb = 0 path).
// 64 x 64 tiles through LDS with 16-B global loads and stores: a wave moves 8
// rows x 128 B either way. The LDS image keeps row r's 16-B chunk ch at chunk
// ch ^ (r >> 3): the transposed reads (8 rows r0 .. r0 + 7 of one column per
// lane, lanes over 8 row octets x 8 columns) then fall on 32 distinct dwords.
// Ragged edges (rows / cols not multiples of 8, or past the tile) take the
// element path.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(bf16* __restrict__ dst, int64_t ldd,
                                                             const bf16* __restrict__ src, int64_t lds,
                                                             int64_t rows, int64_t cols) {
    __shared__ __attribute__((aligned(16))) bf16 tile[64 * 64];
    const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
    const int t = threadIdx.x;
    const bool vec = (lds % 8 == 0) && (ldd % 8 == 0) && ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int r = (t >> 3) + 32 * p, ch = t & 7;
        const int64_t gr = r0 + r, gc = c0 + ch * 8;
        union { u32x4 v; bf16 e[8]; } u;
        if (vec && gr < rows && gc + 8 <= cols) {
            u.v = *(const u32x4*)(src + gr * lds + gc);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) u.e[i] = (gr < rows && gc + i < cols) ? src[gr * lds + gc + i] : (bf16)0.f;
        }
        *(u32x4*)(tile + r * 64 + ((ch ^ (r >> 3)) * 8)) = u.v;
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int rch = t & 7, c = (t >> 3) + 32 * p;  // dst row c0 + c, columns r0 + 8 rch .. + 7
        union { u32x4 v; bf16 e[8]; } u;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = rch * 8 + i;
            u.e[i] = tile[r * 64 + (((c >> 3) ^ rch) * 8) + (c & 7)];
        }
        const int64_t gc = c0 + c, gr = r0 + rch * 8;
        if (gc >= cols) continue;
        if (vec && gr + 8 <= rows) {
            *(u32x4*)(dst + gc * ldd + gr) = u.v;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (gr + i < rows) dst[gc * ldd + gr + i] = u.e[i];
        }
    }
}

extern "C" int msq_transpose_bf16(void* dst, int64_t ld_dst, const void* src, int64_t ld_src, int64_t rows,
                                  int64_t cols, void* stream) {
    MSQ_CHECK_ARG(dst && src && rows > 0 && cols > 0 && ld_src >= cols && ld_dst >= rows,
                  "msq_transpose_bf16: bad sizes");
    const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
    hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, (bf16*)dst, ld_dst,
                       (const bf16*)src, ld_src, rows, cols);
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}

// ------------------------------------------------------------------ Adam
// torch.optim.Adam (foreach, weight_decay=0, amsgrad=False):
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16* __restrict__ shadow, int64_t n, float b1, float b2, float eps,
                            float step_size, float bc2_sqrt, float gscale) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = g[i] * gscale;
        const float mi = m[i] + (1.f - b1) * (gi - m[i]);  // exp_avg.lerp_(grad, 1-b1)
        const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float den = sqrtf(vi) / bc2_sqrt + eps;
        const float pi = p[i] - step_size * (mi / den);
        p[i] = pi;
        if (shadow) shadow[i] = (bf16)pi;
    }
}

// same update, 4 parameters per thread with 16-B loads / stores (8-B shadow
// stores); elements [4 n4, n) are left to the scalar kernel. One quad per
// thread over a flat grid: 0.86 ms at cfg 2 (5.4 TB/s over the 30 B per
// parameter) against 0.94 for a grid-stride loop and 1.0+ for 2-4 quads per
// thread (tools/lab/adam_lab.hip; nontemporal accesses: no change)
__global__ __launch_bounds__(256) void adam4_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16* __restrict__ shadow, int64_t n4, float b1, float b2,
                                                    float eps, float step_size, float bc2_sqrt, float gscale) {
    {
        const int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
        if (q >= n4) return;
        const f32x4 gv = ((const f32x4*)g)[q];
        f32x4 mv = ((f32x4*)m)[q], vv = ((f32x4*)v)[q], pv = ((f32x4*)p)[q];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float gi = gv[t] * gscale;
            const float mi = mv[t] + (1.f - b1) * (gi - mv[t]);
            const float vi = vv[t] * b2 + (1.f - b2) * gi * gi;
            mv[t] = mi;
            vv[t] = vi;
            const float den = sqrtf(vi) / bc2_sqrt + eps;
            pv[t] = pv[t] - step_size * (mi / den);
        }
        ((f32x4*)m)[q] = mv;
        ((f32x4*)v)[q] = vv;
        ((f32x4*)p)[q] = pv;
        if (shadow) store4(shadow + 4 * q, pv);
    }
}

extern "C" int msq_adam_step(float* p, const float* g, float* m, float* v, void* p_shadow, int64_t n, float lr,
                             float beta1, float beta2, float eps, int64_t step, float grad_scale, void* stream) {
    MSQ_CHECK_ARG(n >= 0 && step >= 1, "msq_adam_step: bad args");
    if (n == 0) return MSQ_OK;
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    const float step_size = (float)(lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    const bool al = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16) == 0 &&
                    ((uintptr_t)p_shadow % 8) == 0;
    const int64_t n4 = al ? n / 4 : 0;
    if (n4 > 0) {
        hipLaunchKernelGGL(adam4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (bf16*)p_shadow,
                           n4, beta1, beta2, eps, step_size, bc2s, grad_scale);
    }
    const int64_t rest = n - 4 * n4;
    if (rest > 0) {
        const int grid = (int)std::min<int64_t>((rest + 255) / 256, 16384);
        hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, p + 4 * n4, g + 4 * n4,
                           m + 4 * n4, v + 4 * n4, p_shadow ? (bf16*)p_shadow + 4 * n4 : nullptr, rest, beta1, beta2,
                           eps, step_size, bc2s, grad_scale);
    }
    MSQ_LAUNCH_CHECK();
    return MSQ_OK;
}
