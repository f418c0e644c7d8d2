/* libmidiseq — C ABI of the MI355X (gfx950) symbolic-music sequence-model path.
 *
 * Drop-in boundary for the hot path of thorGabe123/Deep-Learning-Based-Sequence-
 * Models-for-Music-Generation (reference @ 2025-08-24). Every entry point names
 * the reference interface it replaces (file:line). The reference is pure
 * Python/PyTorch, so its "FFI" for these ops is PyTorch's ATen dispatch; the
 * Python host layer of this repo binds these symbols with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions:
 *   - raw device pointers, int64 sizes/strides (in ELEMENTS), a dtype enum and
 *     a hipStream_t passed as void*;
 *   - the caller owns every buffer; scratch comes from *_workspace() queries;
 *   - launches are asynchronous on the given stream; nothing here allocates,
 *     synchronises or copies to the host (graph-capture safe);
 *   - return 0 on success, a negative MSQ_ERR_* code on failure;
 *     msq_last_error() returns a thread-local message.
 */
#ifndef MIDISEQ_H
#define MIDISEQ_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSQ_OK 0
#define MSQ_ERR_ARG (-1)
#define MSQ_ERR_HIP (-2)
#define MSQ_ERR_UNSUPPORTED (-3)

/* element types */
#define MSQ_F32 0
#define MSQ_BF16 1
/* aux of the bf16 GEMM only: a ReLU mask at 1 bit per element, bit n % 32 of
 * the uint32 word [m][n / 32] (ld_aux in words, one batch). With
 * MSQ_EPI_RELU_MASK the product reads it (C = acc * bit); with
 * MSQ_EPI_BIAS_RELU it is written: bit = (C[m][n] as stored > 0). It stands in
 * for the bf16 post-ReLU activation as the FFN dX mask (model_transformer.py:97-100)
 * at 1/16 of the bytes. */
#define MSQ_MASK1 2

/* GEMM epilogues */
#define MSQ_EPI_NONE 0       /* C = acc                                   */
#define MSQ_EPI_BIAS 1       /* C = acc + bias[n]                          */
#define MSQ_EPI_BIAS_RELU 2  /* C = relu(acc + bias[n])                    */
#define MSQ_EPI_BIAS_RESID 3 /* C = acc + bias[n] + aux[m,n]  (aux fp32)   */
#define MSQ_EPI_RELU_MASK 4  /* C = acc * (aux[m,n] > 0)                   */
#define MSQ_EPI_ACCUM 5      /* C += acc                     (C fp32)      */
/* C = aux[m,n] + dropout(acc + bias[n]) (aux fp32): msq_gemm_dropout only   */
#define MSQ_EPI_BIAS_DROP_RESID 6

const char* msq_last_error(void);
int msq_version(void);

/* ---- token + metadata embedding -------------------------------------------
 * Replaces nn.Embedding x2 + torch.cat (model_transformer.py:152-155,
 * mamba.py:29-30). x[b, 0:n_meta] = meta_table[meta[b]], x[b, n_meta+t] =
 * tok_table[idx[b,t]]; x is fp32 [B, n_meta+T, d].                           */
int msq_embed_fwd(float* x, const float* tok_table, const float* meta_table, const int64_t* idx,
                  const int64_t* meta, int64_t B, int64_t T, int64_t n_meta, int64_t d, void* stream);
/* backward: g_tok[idx[b,t]] += dx[b, n_meta+t], g_meta[meta[b,i]] += dx[b,i]
 * (fp32 atomics; caller zeroes or accumulates).                               */
int msq_embed_bwd(float* g_tok, float* g_meta, const float* dx, const int64_t* idx, const int64_t* meta,
                  int64_t B, int64_t T, int64_t n_meta, int64_t d, void* stream);
/* deterministic form of msq_embed_bwd (bitwise reproducible): a stable
 * counting sort of the dx rows by table row, then in-order segment sums.
 * Table sizes V_tok / V_meta are needed for the sort; ids outside them are
 * dropped. workspace: msq_embed_bwd_workspace() bytes, 16-B aligned.          */
size_t msq_embed_bwd_workspace(int64_t B, int64_t T, int64_t n_meta, int64_t d, int64_t V_tok, int64_t V_meta);
int msq_embed_bwd_sorted(float* g_tok, float* g_meta, const float* dx, const int64_t* idx, const int64_t* meta,
                         int64_t B, int64_t T, int64_t n_meta, int64_t d, int64_t V_tok, int64_t V_meta,
                         void* workspace, void* stream);

/* ---- LayerNorm (nn.LayerNorm, model_transformer.py:115-116,146; mamba.py:25)
 * y = (x - mean) * rstd * gamma + beta; x fp32; y in y_dtype, compact [rows, d].
 * Output row r reads input row (r/seg_len)*(seg_len+seg_skip)+seg_skip+r%seg_len
 * (seg_skip = 0: identity) -- LN_f normalises only the token rows that feed
 * lm_head (model_transformer.py:160-164 slices them off afterwards).         */
int msq_layernorm_fwd(void* y, int y_dtype, float* mean, float* rstd, const float* x, const float* gamma,
                      const float* beta, int64_t rows, int64_t d, float eps, int64_t seg_len, int64_t seg_skip,
                      void* stream);
size_t msq_layernorm_bwd_workspace(int64_t rows, int64_t d);
/* dx_acc[map(r),:] += LN'(dy[r]) (fp32, in place); if dx_copy != NULL also
 * writes the updated rows in copy_dtype; dgamma/dbeta accumulate (+=).       */
int msq_layernorm_bwd(float* dx_acc, void* dx_copy, int copy_dtype, float* dgamma, float* dbeta, const void* dy,
                      int dy_dtype, const float* x, const float* mean, const float* rstd, const float* gamma,
                      int64_t rows, int64_t d, int64_t seg_len, int64_t seg_skip, void* workspace, void* stream);

/* msq_layernorm_bwd whose dx_copy is the gradient of a dropped branch: the
 * copy of row map(r) is multiplied by keep(seed, site, map(r), col)/(1-p)
 * (the mask msq_gemm_dropout drew in the forward); dx_acc stays unmasked.   */
int msq_layernorm_bwd_dropout(float* dx_acc, void* dx_copy, int copy_dtype, float* dgamma, float* dbeta,
                              const void* dy, int dy_dtype, const float* x, const float* mean, const float* rstd,
                              const float* gamma, int64_t rows, int64_t d, int64_t seg_len, int64_t seg_skip,
                              uint32_t seed, uint32_t site, float p, void* workspace, void* stream);
/* msq_layernorm_bwd_dropout that also accumulates (+=) into dbias (fp32 [d],
 * unless NULL) the column sums of the rows it writes (the copy after its
 * mask, else the updated dx_acc): the bias gradient of the residual branch
 * feeding this LayerNorm (proj / FFN output biases, model_transformer.py
 * :46,101), fused instead of a separate pass over those rows.
 * schedule 0: every row's contribution to dgamma / dbeta / dbias is summed
 * in a fixed order (bitwise reproducible; msq_layernorm_bwd and _dropout use
 * it); 1: rows are taken from a work queue, so the fp32 summation order (the
 * last bits of those sums) depends on timing.                              */
int msq_layernorm_bwd_bias(float* dx_acc, void* dx_copy, int copy_dtype, float* dgamma, float* dbeta, float* dbias,
                           const void* dy, int dy_dtype, const float* x, const float* mean, const float* rstd,
                           const float* gamma, int64_t rows, int64_t d, int64_t seg_len, int64_t seg_skip,
                           uint32_t seed, uint32_t site, float p, int schedule, void* workspace, void* stream);
/* ---- GEMM (nn.Linear fwd/bwd: model_transformer.py:46,57-59,97-100,147;
 * Mamba2 in_proj/out_proj). C[b] = op(A[b]) . op(B[b]) with
 *   ta = 0: A stored [M,K] (K contiguous)     ta = 1: A stored [K,M]
 *   tb = 0: B stored [N,K] (K contiguous)     tb = 1: B stored [K,N]
 * dtype = MSQ_BF16: bf16 operands, fp32 accumulation on MFMA (fast path);
 * dtype = MSQ_F32 : fp32 operands and accumulation (exact/parity path).
 * c_dtype: output type (ACCUM requires fp32). aux (the residual of
 * BIAS_RESID / BIAS_DROP_RESID, the mask source of RELU_MASK) is read as
 * aux_dtype: MSQ_F32 or MSQ_BF16 (MSQ_MASK1 bits for RELU_MASK / BIAS_RELU).
 * Leading dims must be multiples of 8.                                      */
int msq_gemm(int dtype, int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
             int64_t strideA, const void* B, int64_t ldb, int64_t strideB, void* C, int c_dtype, int64_t ldc,
             int64_t strideC, int64_t batch, int epilogue, const float* bias, const void* aux, int aux_dtype,
             int64_t ld_aux, int64_t stride_aux, void* stream);

/* msq_gemm with nn.Dropout(p) on acc + bias before the residual add
 * (model_transformer.py:51 proj, :101 FFN output): epilogue
 * MSQ_EPI_BIAS_DROP_RESID; element (m, n) is kept iff
 * hash(seed, site, row m, col n) >= p*2^32 (csrc/common.h) and scaled by 1/(1-p). */
int msq_gemm_dropout(int dtype, int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                     int64_t strideA, const void* B, int64_t ldb, int64_t strideB, void* C, int c_dtype, int64_t ldc,
                     int64_t strideC, int64_t batch, int epilogue, const float* bias, const void* aux, int aux_dtype,
                     int64_t ld_aux, int64_t stride_aux, uint32_t seed, uint32_t site, float p, void* stream);
/* msq_gemm_dropout with a caller-owned split-K workspace. An ACCUM product
 * whose K is split over workgroups (the weight gradients: the dW of
 * nn.Linear in the DDP backward, train_parallel.py:166) writes each slice's
 * fp32 partial tile to ws and one reduction adds them into C, instead of
 * fp32 atomics; ws_bytes below msq_gemm_workspace_size(...) (or ws = NULL)
 * falls back to the atomics. Other epilogues ignore ws.                      */
int64_t msq_gemm_workspace_size(int dtype, int ta, int tb, int64_t M, int64_t N, int64_t K, int64_t lda,
                                int64_t ldb, int64_t batch, int epilogue);
int msq_gemm_ex(int dtype, int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                int64_t strideA, const void* B, int64_t ldb, int64_t strideB, void* C, int c_dtype, int64_t ldc,
                int64_t strideC, int64_t batch, int epilogue, const float* bias, const void* aux, int aux_dtype,
                int64_t ld_aux, int64_t stride_aux, uint32_t seed, uint32_t site, float p, void* ws,
                int64_t ws_bytes, void* stream);
/* Decode step: a residual product and the LayerNorm that follows it
 * (model_transformer.py:115,119: x + proj(attn) -> ln2, x + FFN -> the next
 * block's ln1 / ln_f at :146) in two launches instead of three:
 *   C = aux + A . W^T + bias   (fp32 [M, N], ldc; aux fp32 ldx; bias may be NULL)
 *   Y = LayerNorm(rows of C; gamma, beta, eps) in y_dtype (ldy)
 * A [M, K] and W [N, K] (nn.Linear) in dtype. For M <= 64 bf16 rows the product
 * runs split over K into fp32 partials and one workgroup per row sums them,
 * adds bias and residual and normalises the row it holds; other shapes run
 * msq_gemm_ex + msq_layernorm_fwd (ldy == N). ws of
 * msq_gemm_resid_ln_workspace(...) bytes, 16-B aligned.                       */
int64_t msq_gemm_resid_ln_workspace(int dtype, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldw);
int msq_gemm_resid_ln(int dtype, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* W,
                      int64_t ldw, float* C, int64_t ldc, const float* bias, const float* aux, int64_t ldx,
                      const float* gamma, const float* beta, float eps, void* Y, int y_dtype, int64_t ldy, void* ws,
                      int64_t ws_bytes, void* stream);
/* Which kernel family runs the large (M > 64) bf16 products (tests / A-B
 * tools; process-wide, default from the environment at the first call):
 *   MSQ_ROUTE_DEFAULT  persistent 256 tile for the forward / dX products, the
 *                      per-tile 256 tile (split-K) for the weight gradients;
 *   MSQ_ROUTE_TILE256  the per-tile 256 tile for every product (MSQ_GEMM_NOP);
 *   MSQ_ROUTE_TILE128  the 128 tile only (MSQ_GEMM128).
 * Returns the previous route.                                                 */
#define MSQ_ROUTE_DEFAULT 0
#define MSQ_ROUTE_TILE256 1
#define MSQ_ROUTE_TILE128 2
int msq_gemm_set_route(int route);
/* column sums (bias gradients): out[c] (+)= sum_r x[r, c]                      */
/* C = epi(op(A) op(B)) in bf16 (epilogue NONE or RELU_MASK with aux, no
 * batch) and dbias[n] = (accumulate ? dbias[n] : 0) + sum_m C[m][n] in fp32:
 * the FFN dX product of the backward with the gradient of the first
 * Linear's bias (model_transformer.py:95) fused into its epilogue. ws of
 * msq_gemm_colsum_workspace(M, N) bytes. Replaces the per-step bias
 * gradient of FeedFoward's nn.Linear (autograd's sum over rows). */
size_t msq_gemm_colsum_workspace(int64_t M, int64_t N);
int msq_gemm_colsum(int ta, int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                    int64_t ldb, void* C, int64_t ldc, int epilogue, const void* aux, int aux_dtype, int64_t ld_aux,
                    float* dbias, int accumulate, void* ws, int64_t ws_bytes, void* stream);
/* lm_head forward (model_transformer.py:147, nn.Linear with bias) in bf16:
 * C[m][n] = sum_k A[m][k] B[n][k] + bias[n] (A [M, K] row-major; B stored
 * [N, K] as msq_gemm's tb = 0, or [K, N] with tb = 1), and per 256-row tile / 128-row half p
 * the column max and sum of exp(C - max) of the stored bf16 values:
 * part[2p][n], part[2p+1][n] (row stride pld). The statistics are the
 * time-axis logsumexp partials of filtered_logit (train.py:136) for rows
 * ordered (b, t) with T % 256 == 0: pass part, T / 128 and pld to
 * msq_filtered_ce_bias_part. M % 256 == 0; part holds
 * msq_gemm_colstats_bytes(M, N) bytes at pld = N rounded up to 4. Returns
 * MSQ_ERR_UNSUPPORTED for shapes outside the persistent 256 tile (or with a
 * GEMM route other than MSQ_ROUTE_DEFAULT); msq_gemm_bias_colstats_applies
 * answers that for the same arguments without launching (1 / 0; host only,
 * no device needed): a caller then runs the plain bias GEMM instead. */
size_t msq_gemm_colstats_bytes(int64_t M, int64_t N);
int msq_gemm_bias_colstats_applies(int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                                   int64_t ldb, const void* C, int64_t ldc, const float* bias, const float* part,
                                   int64_t pld);
int msq_gemm_bias_colstats(int tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* B,
                           int64_t ldb, void* C, int64_t ldc, const float* bias, float* part, int64_t pld,
                           void* stream);
/* dst[c][r] = src[r][c] for a bf16 [rows][cols] matrix (leading dims in
 * elements): the transposed weight copies the backward's dX products read
 * (autograd's x.grad = dy @ W of nn.Linear, model_transformer.py:47,95,97,147). */
int msq_transpose_bf16(void* dst, int64_t ld_dst, const void* src, int64_t ld_src, int64_t rows, int64_t cols,
                       void* stream);
size_t msq_colsum_workspace(int64_t rows, int64_t cols);
int msq_colsum(float* out, int accumulate, const void* x, int dtype, int64_t rows, int64_t cols, int64_t ld,
               void* workspace, void* stream);

/* elementwise cast (weights fp32 -> bf16 shadow etc.)                        */
int msq_cast(void* dst, int dst_dtype, const void* src, int src_dtype, int64_t n, void* stream);

/* ---- Adam (torch.optim.Adam, train_parallel.py:157,183; foreach formula)
 * g is multiplied by grad_scale first (1/world after a SUM all-reduce).
 * Optional p_shadow receives the updated parameters in bf16.                 */
int msq_adam_step(float* p, const float* g, float* m, float* v, void* p_shadow, int64_t n, float lr, float beta1,
                  float beta2, float eps, int64_t step, float grad_scale, void* stream);


/* ---- relative-position causal attention (HeadRelPos x n_heads +
 * torch.cat, model_transformer.py:41-90). Per head h and batch b:
 *   s(i,j) = (q_i.k_j + BD(i,j)) * scale, allowed iff j <= i or j < n_meta,
 *   BD(i,j) = q_i.R[S-1-i+j] (j <= i) | 0 (j == i+1) | q_{i+1}.R[j-i-2] (j >= i+2)
 * qkv: [B*S, ld_qkv] with q | k | v blocks of H*hs columns (head h at h*hs);
 * R: [H, S_max, hs]; out: [B*S, ld_out]; lse: fp32 [B, H, S] (natural log).
 * dtype MSQ_BF16 (flash MFMA kernels, hs == 128) or MSQ_F32 (exact path).   */
int msq_relattn_fwd(int dtype, void* out, int64_t ld_out, float* lse, const void* qkv, int64_t ld_qkv,
                    const void* R, int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale,
                    int64_t n_meta, void* stream);
/* ---- attention-probability dropout (nn.Dropout(p) on the softmax output,
 * model_transformer.py:62,80; active in train() mode, config.yaml:16 p = 0.01).
 * Keep bits of one layer in two block-transposed layouts of
 * msq_dropout_mask_words(B, H, S) uint32 each (nb = ceil(S/64), bh = b*H + h):
 *   rowmask as uint64 [((bh*nb + i/64)*nb + j/64)*64 + i%64] bit j%64 = keep(i, j)
 *   colmask as uint64 [((bh*nb + j/64)*nb + i/64)*64 + j%64] bit i%64 = keep(i, j)
 * The keep bits of row i over keys 64 jb .. +63 are one word drawn from the
 * counter-based hash of (seed, site0 + b*H + h, i, jb) (csrc/common.h
 * attn_word_key): k ~ Binomial(64, p) dropped keys at uniformly drawn distinct
 * positions, so every element is kept with probability 1 - p independently.
 * Only the causal lower block triangle is written.
 * msq_dropout_mask_ld(S) = 2*nb, the uint32 words of one block row.          */
int64_t msq_dropout_mask_ld(int64_t S);
int64_t msq_dropout_mask_words(int64_t B, int64_t H, int64_t S);
int msq_dropout_attn_mask(uint32_t* rowmask, uint32_t* colmask, int64_t B, int64_t H, int64_t S, uint32_t seed,
                          uint32_t site0, float p, void* stream);
/* the 64 Binomial(64, p) thresholds of that draw (host only, no device):
 * out64[t] = round(2^32 P(K <= t)), clamped to 2^32 - 1                       */
int msq_dropout_attn_table(float p, uint32_t* out64);
/* msq_relattn_fwd / _bwd with dropout p on the attention probabilities: the
 * masks of msq_dropout_attn_mask; kept probabilities are scaled by 1/(1-p);
 * lse stays the undropped softmax normaliser. p = 0 = the plain entry points. */
int msq_relattn_fwd_dropout(int dtype, void* out, int64_t ld_out, float* lse, const void* qkv, int64_t ld_qkv,
                            const void* R, int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale,
                            int64_t n_meta, const uint32_t* rowmask, const uint32_t* colmask, float p, void* stream);
size_t msq_relattn_bwd_workspace(int dtype, int64_t B, int64_t S, int64_t H);
/* dqkv (same layout as qkv) is overwritten; dR (fp32 [H, S_max, hs]) accumulates. */
int msq_relattn_bwd(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout, int64_t ld_dout,
                    const void* out, const float* lse, const void* qkv, int64_t ld_qkv, const void* R, int64_t B,
                    int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale, int64_t n_meta, void* workspace,
                    void* stream);
int msq_relattn_bwd_dropout(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout, int64_t ld_dout,
                            const void* out, const float* lse, const void* qkv, int64_t ld_qkv, const void* R,
                            int64_t B, int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale, int64_t n_meta,
                            const uint32_t* rowmask, const uint32_t* colmask, float p, void* workspace, void* stream);
/* msq_relattn_bwd_dropout with ws_ready = 1 when this workspace already served
 * a backward of the same (dtype, B, S, H) and was not written by anything
 * else since: its dS layouts' zero band and row padding (which no pass writes
 * non-zero) are then not cleared again. */
int msq_relattn_bwd_ws(int dtype, void* dqkv, int64_t ld_dqkv, float* dR, const void* dout, int64_t ld_dout,
                       const void* out, const float* lse, const void* qkv, int64_t ld_qkv, const void* R, int64_t B,
                       int64_t S, int64_t H, int64_t hs, int64_t S_max, float scale, int64_t n_meta,
                       const uint32_t* rowmask, const uint32_t* colmask, float p, void* workspace, int ws_ready,
                       void* stream);

/* ---- grammar-weighted filtered loss (train.py:79-138; CrossEntropyLoss,
 * train_parallel.py:156,179). logits [B,T,ld] (ld >= V, ld % 4 == 0) in dtype;
 * wtab fp32 [5,V] (make_distributions); b0..b3 = bucketize boundaries
 * (dyn-1, length-1, time-1, tempo-1); col_lse fp32 [B,V] receives the
 * log-sum-exp over the time axis.                                            */
size_t msq_filtered_workspace(int64_t B, int64_t T, int64_t V);
int msq_filtered_colstats(float* col_lse, const void* logits, int dtype, int64_t ld, int64_t B, int64_t T, int64_t V,
                          void* workspace, void* stream);

/* Cached decode (generate mode="cached", TransformerEngine.step): column
 * log-sum-exp over the time axis of a ring of logits rows ring [B][ctx][ld]
 * (-inf rows are empty), kept as per-block partials part f32 [B][nblk][V]
 * over blocks of rows_per_block rows. Recomputes blocks [blk_lo, blk_hi)
 * leaving out row skip_row (-1: none), and block blk_extra (-1: none) whole,
 * then col_lse[b][v] = logsumexp over the blocks. Replaces the per-step
 * torch.logsumexp(out, dim=1) of train.py:133-138 as applied by
 * scripts/generate.py:33 to the sliding window. */
int msq_ring_lse(float* col_lse, float* part, const void* ring, int dtype, int64_t ld, int64_t B, int64_t ctx,
                 int64_t V, int64_t rows_per_block, int64_t blk_lo, int64_t blk_hi, int64_t skip_row,
                 int64_t blk_extra, void* stream);
/* One graph-replayable cached-decode step of the ring: copies row [B][ld_row]
 * into ring slot pos % ctx and tok[b] into tokens [B][ctx], writes col_lse =
 * the LSE over the window's other rows (what msq_ring_lse gives for that
 * slot) and advances *pos by one. pos: int64 on the device (the sequence
 * position of the new row), so the launch arguments do not change from step
 * to step. Incremental: state (msq_ring_state_bytes, 16-B aligned) holds the
 * merged partials of the blocks other than the slot's, a running prefix of
 * the slot's block and its suffix table, and (the int64 in its last 16
 * bytes) the block they describe: set that int64 to -1 after msq_ring_lse
 * has filled every block partial (the first step after a prefill); the step
 * that enters a block re-derives the tables from part and the ring.
 * scripts/generate.py:29-33 per new token. */
size_t msq_ring_state_bytes(int64_t B, int64_t V, int64_t rows_per_block);
int msq_ring_step(float* col_lse, float* part, void* state, void* ring, int dtype, int64_t ld, int64_t B, int64_t ctx,
                  int64_t V, int64_t rows_per_block, const void* row, int64_t ld_row, int64_t* tokens,
                  const int64_t* tok, int64_t* pos, void* stream);
/* loss (fp32 scalar, device) = mean over B*T of the row CE of Z. If dlogits
 * != NULL also writes grad_scale * d(sum of row CE)/dlogits (so grad_scale =
 * 1/(B*T) gives the gradient of the mean).                                  */
int msq_filtered_ce(float* loss, void* dlogits, int64_t ldd, const void* logits, int dtype, int64_t ld,
                    const int64_t* src, const int64_t* trg, const float* wtab, int64_t b0, int64_t b1, int64_t b2,
                    int64_t b3, int64_t B, int64_t T, int64_t V, float grad_scale, float* col_lse, void* workspace,
                    void* stream);
/* msq_filtered_ce that also accumulates (+=) into dbias (fp32 [V]) the column
 * sums of dlogits over the B*T rows: the gradient of the output layer's bias
 * (lm_head.bias / output_layer.bias), fused into the pass that writes dlogits. */
int msq_filtered_ce_bias(float* loss, void* dlogits, int64_t ldd, float* dbias, const void* logits, int dtype,
                         int64_t ld, const int64_t* src, const int64_t* trg, const float* wtab, int64_t b0, int64_t b1,
                         int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V, float grad_scale, float* col_lse,
                         void* workspace, void* stream);
/* msq_filtered_ce_bias with the time-axis column statistics supplied by the
 * lm_head GEMM epilogue (msq_gemm_bias_colstats): colpart holds, per
 * sequence b, nts (max, sum exp) partial row pairs of stride pld
 * (colpart[((b * nts + ts) * 2) * pld + v] = max, the next row the sum), so the
 * pass that re-reads the logits for col_lse (train.py:136, log_softmax over
 * the time axis) is skipped. Needs the streaming path: bf16 / fp32 logits and
 * dlogits with ld, ldd % 8 == 0 and 16-B aligned rows. */
int msq_filtered_ce_bias_part(float* loss, void* dlogits, int64_t ldd, float* dbias, const void* logits, int dtype,
                              int64_t ld, const int64_t* src, const int64_t* trg, const float* wtab, int64_t b0,
                              int64_t b1, int64_t b2, int64_t b3, int64_t B, int64_t T, int64_t V, float grad_scale,
                              float* col_lse, const float* colpart, int64_t nts, int64_t pld, void* workspace,
                              void* stream);
/* Z rows t_begin..T-1 (fp32, [B, T-t_begin, ldz]) = filtered_logit(src, logits). */
int msq_filtered_logit(float* z, int64_t ldz, const void* logits, int dtype, int64_t ld, const int64_t* src,
                       const float* wtab, int64_t b0, int64_t b1, int64_t b2, int64_t b3, int64_t B, int64_t T,
                       int64_t V, int64_t t_begin, float* col_lse, void* workspace, void* stream);
/* dlogits = d filtered_logit^T dz (col_lse from msq_filtered_logit).        */
int msq_filtered_logit_bwd(void* dlogits, int64_t ldd, const float* dz, int64_t ldz, const void* logits, int dtype,
                           int64_t ld, const int64_t* src, const float* wtab, int64_t b0, int64_t b1, int64_t b2,
                           int64_t b3, int64_t B, int64_t T, int64_t V, const float* col_lse, void* workspace,
                           void* stream);

/* ---- autoregressive decode step (scripts/generate.py:33-89) ---------------
 * For every row b: recent window of hist[b, :cur_len] (time-shift sum >= 1024),
 * repetition penalties on z_last[b] (in place), top-k (k = ks[b] in 1..3,
 * chosen by the host with Python's random), p = v / sum v, inverse-CDF pick
 * with uniforms[b]; the token is written to hist[b, cur_len] and out_tok[b].
 * hist: int64 [B, ld_hist]; z_last: fp32 [B, ld_z] (filtered logits of the
 * last window row, msq_filtered_logit with t_begin = T-1).                 */
int msq_decode_sample(int64_t* hist, int64_t ld_hist, int64_t cur_len, float* z_last, int64_t ld_z, int64_t B,
                      int64_t V, const int* ks, const float* uniforms, int64_t* out_tok, int64_t dyn_start,
                      int64_t length_start, int64_t time_start, int64_t tempo_start, void* stream);

/* ---- Mamba2 mixer (mamba_ssm.Mamba2 via models/mamba/mamba.py:16-24;
 * d_state 64, d_conv 4, expand 2, headdim 64, ngroups 1). zxbcdt is the
 * in_proj output [B*L, ldz] = z | xBC | dt_raw; xc the conv output [B*L, ldxc]
 * = x | B | C (post-SiLU). dtype selects bf16 (fast) or fp32 (exact) storage;
 * the scan itself always runs in fp32.                                       */
size_t msq_mamba_states_size(int64_t B, int64_t L, int64_t nheads);
int msq_mamba_conv_fwd(void* xc, int64_t ldxc, const void* zxbcdt, int64_t ldz, int dtype, const float* conv_w,
                       const float* conv_b, int64_t B, int64_t L, int64_t d_inner, int64_t nheads, void* stream);
/* y [B*L, ldy] (in dtype: bf16 as mamba_ssm stores it, or fp32) = SSD(x, dt,
 * A, B, C) + D x; states receive the fp32 chunk-entry states
 * (msq_mamba_states_size bytes) used by the backward.                        */
int msq_mamba_ssd_fwd(void* y, int64_t ldy, float* states, const void* xc, int64_t ldxc, const void* zxbcdt,
                      int64_t ldz, int dtype, const float* dt_bias, const float* A_log, const float* D, int64_t B,
                      int64_t L, int64_t d_inner, int64_t nheads, void* stream);
/* out = (y * silu(z)) * rsqrt(mean((y*silu(z))^2) + eps) * w  (RMSNormGated);
 * y in dtype (msq_mamba_ssd_fwd's output)                                    */
int msq_mamba_gnorm_fwd(void* out, int64_t ldo, float* rstd, const void* y, int64_t ldy, const void* zxbcdt,
                        int64_t ldz, int dtype, const float* w, int64_t rows, int64_t d_inner, float eps,
                        void* stream);
/* dy (in dtype, ld = ldy: bf16 in the bf16 path, as mamba_ssm's gradient of its
 * bf16 y) and dz (into dzxbcdt[:, :d_inner]); dw accumulates.               */
int msq_mamba_gnorm_bwd(void* dy, void* dzxbcdt, const void* y, int64_t ldy, const void* zxbcdt, int64_t ldz,
                        int dtype, const float* w, const float* rstd, const float* dout, int64_t ldd, float* dw,
                        int64_t rows, int64_t d_inner, void* stream);
/* dxc fp32 [B*L, ldxc]: dx (written) | dB, dC (reduced over heads); dt_raw
 * grads into dzxbcdt[:, d_inner+conv_dim+h]; gA_log / gD / gdt_bias accumulate.
 * workspace: msq_mamba_ssd_bwd_workspace() bytes (the bf16 path's per-chunk
 * state gradients; the fp32 path ignores it and accepts NULL). dY in dtype
 * (msq_mamba_gnorm_bwd's dy).                                                */
size_t msq_mamba_ssd_bwd_workspace(int64_t B, int64_t L, int64_t nheads);
int msq_mamba_ssd_bwd(float* dxc, int64_t ld_dxc, void* dzxbcdt, const void* dY, int64_t ldy, const float* states,
                      const void* xc, int64_t ldxc, const void* zxbcdt, int64_t ldz, int dtype, const float* dt_bias,
                      const float* A_log, const float* D, float* gA_log, float* gD, float* gdt_bias, int64_t B,
                      int64_t L, int64_t d_inner, int64_t nheads, void* workspace, void* stream);
/* d(xBC_raw) into dzxbcdt[:, d_inner : d_inner+conv_dim]; conv grads accumulate. */
int msq_mamba_conv_bwd(void* dzxbcdt, const float* dxc, int64_t ld_dxc, const void* zxbcdt, int64_t ldz, int dtype,
                       const float* conv_w, const float* conv_b, float* g_conv_w, float* g_conv_b, int64_t B,
                       int64_t L, int64_t d_inner, int64_t nheads, void* stream);

/* ---- Mamba cached decode (scripts/generate.py:14-95
 * with a Mamba model while prompt + new tokens <= context_len, where every
 * mixer is causal and the per-step full forward equals one recurrent step).
 * msq_mamba_ssd_fwd_state = msq_mamba_ssd_fwd + the state after the last
 * position, final_state fp32 [B][H][64][64] (NULL = none): the prefill.      */
int msq_mamba_ssd_fwd_state(void* y, int64_t ldy, float* states, float* final_state, const void* xc,
                            int64_t ldxc, const void* zxbcdt, int64_t ldz, int dtype, const float* dt_bias,
                            const float* A_log, const float* D, int64_t B, int64_t L, int64_t d_inner,
                            int64_t nheads, void* stream);
/* one position: xc[b] = silu(conv(conv_state[b] (fp32 [B][3][conv_dim], the
 * last three pre-conv xBC rows, oldest first) ++ zxbcdt[b, xBC])); the state
 * shifts in the new row.                                                     */
int msq_mamba_conv_step(void* xc, int64_t ldxc, float* conv_state, const void* zxbcdt, int64_t ldz, int dtype,
                        const float* conv_w, const float* conv_b, int64_t B, int64_t d_inner, int64_t nheads,
                        void* stream);
/* bf16 decode, first half of a mixer step (mamba_ssm Mamba2.step's in_proj
 * + conv1d update): zxbcdt = x . in_w^T (bf16 [B][d_in_proj], in_w
 * [d_in_proj][d_model]) and msq_mamba_conv_step on its xBC columns, one launch
 * for B <= 64 rows and d_model <= 1024 (the conv runs in the product's
 * epilogue), the two launches otherwise. Same results as msq_gemm +
 * msq_mamba_conv_step.                                                      */
int msq_mamba_in_proj_conv_step(void* zxbcdt, int64_t ldz, void* xc, int64_t ldxc, float* conv_state, const void* x,
                                int64_t ldx, const void* in_w, int64_t ldw, const float* conv_w, const float* conv_b,
                                int64_t B, int64_t d_model, int64_t d_in_proj, int64_t d_inner, int64_t nheads,
                                void* stream);
/* one position: h = exp(dt A) h + dt x B^T (ssm_state fp32 [B][H][64][64],
 * in place); y[b] (in dtype) = h C + D x.                                    */
int msq_mamba_ssd_step(void* y, int64_t ldy, float* ssm_state, const void* xc, int64_t ldxc, const void* zxbcdt,
                       int64_t ldz, int dtype, const float* dt_bias, const float* A_log, const float* D, int64_t B,
                       int64_t d_inner, int64_t nheads, void* stream);
/* filtered logit of one new position (train.py:133-138): col_lse fp32 [B][V]
 * (the time-axis LSE over the positions so far, e.g. msq_filtered_logit's
 * col_lse of the prefill) absorbs logits[b]; z[b] = -(o - lse) * W[class(tok[b])],
 * tok[b] = the token at that position.                                       */
int msq_filtered_logit_step(float* z, int64_t ldz, float* col_lse, const void* logits, int dtype, int64_t ld,
                            const int64_t* tok, const float* wtab, int64_t b0, int64_t b1, int64_t b2, int64_t b3,
                            int64_t B, int64_t V, void* stream);

/* ---- data feed (processing/dataset.py:171-195 SequenceDataset.__getitem__)
 * B training windows of T+1 tokens cut from the device-resident token store
 * (tokens int32, song s = tokens[song_off[s] .. + song_len[s]]): params[b] =
 * {song, start, note_shift, velocity_shift, 2 x time_factor}; tokens past the
 * song end are 0 (dataset.py:177-179); augment != 0 applies
 * data_augementation (:134-168) with disc = {pitch, channel, dyn, length,
 * time, tempo}. Writes src[b] = w[:-1], trg[b] = w[1:] (int64 [B, T]) and
 * meta_out[b] = song_meta[song] (int64 [B, n_meta]).                        */
int msq_window_gather(int64_t* src, int64_t* trg, int64_t* meta_out, const int32_t* tokens,
                      const int64_t* song_off, const int64_t* song_len, const int64_t* song_meta, int n_meta,
                      const int64_t* params, int64_t B, int64_t T, int augment, const int64_t* disc, void* stream);

/* Token -> note decode of B generated rows (replaces processing/processing.py
 * :171-214 decode + :154-169 revert_note_time, called per row by
 * scripts/generate_midi_combined.py:143-156). rows int64 [B, ld], first L <=
 * 15872 tokens used; disc = {pitch, channel, dyn, length, time, tempo}
 * (config.yaml discretization); res_per_beat = resolution.bar_res. Row b's
 * notes go to [b*cap, b*cap + min(count[b], cap)) of pitch / channel / dyn /
 * tempo (int32), beat_start / beat_end (int64 beats) and t_start / t_end
 * (fp64 seconds, bit-identical to the reference's Python floats); count[b] is
 * the row's full note count. cap >= L/4 + 1 never truncates.                 */
int msq_midi_decode(const int64_t* rows, int64_t B, int64_t L, int64_t ld, const int64_t* disc, int64_t res_per_beat,
                    int64_t cap, int32_t* pitch, int32_t* channel, int32_t* dyn, int32_t* tempo, int64_t* beat_start,
                    int64_t* beat_end, double* t_start, double* t_end, int64_t* count, void* stream);

/* Cached decode step of the relative attention (the Transformer's
 * generate(mode="cached"), an approximation of scripts/generate.py:26-31's
 * full forward per token: every row is computed once, as the last row of its
 * own window, and its keys / values are reused). For each (b, h): the new
 * token's q, k, v are the head's columns of qkv[b] (bf16 [B, ldq], q | k | v);
 * k, v are written to cache slot new_slot, then
 *   out[b, h] = softmax_j((q.k_j + q.R[jw(j)]) * scale) . v_j
 * over the window's slots j < n_meta + n_tok of kcache / vcache (bf16
 * [B, H, S_ring, hs]); jw(j) = j for metadata slots, else
 * n_meta + (j - n_meta - first_mod) mod (S_ring - n_meta) (the key's window
 * position: HeadRelPos's skew R[S-1-i+j] at the last row i = S-1). R bf16
 * [H, S_max, hs] (rel_pos_emb of the layer). 8 | hs <= 128; dtype MSQ_BF16 or
 * MSQ_F32 for every tensor (out [B, ldo] too).                              */
int msq_relattn_decode(int dtype, void* out, int64_t ldo, const void* qkv, int64_t ldq, void* kcache, void* vcache, const void* R,
                       int64_t S_max, int64_t B, int64_t H, int64_t hs, int64_t S_ring, int64_t n_meta, int64_t n_tok,
                       int64_t new_slot, int64_t first_mod, float scale, void* ws, size_t ws_bytes, void* stream);
/* Bytes of the workspace msq_relattn_decode(_pos) needs (16-B aligned): the
 * per-(b, h, 128-key chunk) partials of the split (flash-decoding) pass.   */
size_t msq_relattn_decode_workspace(int64_t B, int64_t H, int64_t S_ring);
/* msq_relattn_decode with the step's sequence position read from device
 * memory (*pos, int64): n_tok = min(pos + 1, S_ring - n_meta), new_slot =
 * n_meta + pos % ctx, first_mod = (pos + 1 - n_tok) % ctx; for a captured
 * (graph-replayed) decode step whose launch arguments stay fixed.          */
int msq_relattn_decode_pos(int dtype, void* out, int64_t ldo, const void* qkv, int64_t ldq, void* kcache, void* vcache,
                           const void* R, int64_t S_max, int64_t B, int64_t H, int64_t hs, int64_t S_ring,
                           int64_t n_meta, const int64_t* pos, float scale, void* ws, size_t ws_bytes,
                           void* stream);

/* Note -> token encode of a batch of songs (replaces processing/processing.py
 * :129-152 encode + :111-126 adjust_note_time, the preprocessing step of
 * preprocess_midi_files :24-55). Song s = notes [song_off[s], song_off[s+1])
 * of the note columns (sorted by start as extract_midi leaves them; times in
 * seconds, tempo = round(bpm)); disc as above, res_per_beat = bar_res.
 * Writes song s's tokens to tokens[5*song_off[s] ..] (5 slots per note),
 * count[s] = its token count, and each note's integer beats (the notes'
 * time_start / time_end after adjust_note_time) to beat_start / beat_end.   */
int msq_midi_encode(const int32_t* pitch, const int32_t* channel, const int32_t* dyn, const int32_t* tempo,
                    const double* t_start, const double* t_end, const int64_t* song_off, int64_t n_songs,
                    const int64_t* disc, int64_t res_per_beat, int64_t* tokens, int64_t* beat_start, int64_t* beat_end,
                    int64_t* count, void* stream);

#ifdef __cplusplus
}
#endif
#endif
