// Host-side launcher API of the HIP kernels (device code lives in csrc/*.hip).
// Pointers are device pointers; every launcher enqueues on `stream` and never synchronises, so all
// of them are safe inside hipGraph capture.  dtype codes: dph::DType (0 = fp32, 1 = bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dph {

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

// ---- RMSNorm (fsdp_tp/llama2_model.py:115-142 semantics: fp32 statistics, eps inside rsqrt) ----
void rmsnorm_fwd(const void* x, const void* w, const void* residual, void* h_out, void* y, float* rstd,
                 int64_t rows, int dim, float eps, int x_dtype, int w_dtype, hipStream_t stream);
// dx (x dtype) and dw_partial (fp32 [nblk, dim]) then dw (w dtype) by a column reduction.
// dres (optional, x dtype): a residual-stream gradient added into dx in the same pass.
void rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dres, void* dx,
                 float* dw_partial, void* dw, int nblk, int64_t rows, int dim, int x_dtype, int w_dtype,
                 hipStream_t stream);
int rmsnorm_bwd_blocks(int64_t rows);

// ---- LayerNorm (nn.LayerNorm semantics, used by ViT / pipeline transformer) ----
void layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                   int dim, float eps, int x_dtype, int w_dtype, hipStream_t stream);
void layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
                   float* dwb_partial, void* dw, void* db, int nblk, int64_t rows, int dim, int x_dtype,
                   int w_dtype, hipStream_t stream);

// ---- RoPE, interleaved pairs (llama2_model.py:74-100), in place on a [B,S,H,hd] strided view ----
void rope_apply(void* x, const float* cos_t, const float* sin_t, int64_t B, int64_t S, int64_t H, int hd,
                int64_t sb, int64_t ss, int64_t sh, int64_t pos_offset, int inverse, int dtype, hipStream_t stream);

// ---- SwiGLU on the fused [N, 2F] = [w1 x | w3 x] GEMM output (llama2_model.py:266-267) ----
void swiglu_fwd(const void* x2, void* y, int64_t n, int64_t f, int64_t ld_x2, int dtype, hipStream_t stream);
void swiglu_bwd(const void* dy, const void* x2, void* dx2, int64_t n, int64_t f, int64_t ld_x2, int dtype,
                hipStream_t stream);

// ---- GELU (tanh / erf) fwd/bwd, elementwise ----
void gelu_fwd(const void* x, void* y, int64_t n, int approximate_tanh, int dtype, hipStream_t stream);
void gelu_bwd(const void* dy, const void* x, void* dx, int64_t n, int approximate_tanh, int dtype,
              hipStream_t stream);

// ---- Fused AdamW over flat buffers (torch.optim.AdamW semantics, decoupled weight decay) ----
//   master/m/v: fp32 [n]; grad: grad_dtype [n]; param_out (optional): param_dtype [n] (rounded copy of master).
//   grad_scale_ptr (optional device fp32 scalar) multiplies the gradient (global-norm clipping, 1/world).
//   hyper (optional device fp32 [lr, step]) overrides lr and the bias corrections (HIP-graph capturable steps).
void adamw_step(float* master, float* m, float* v, const void* grad, void* param_out, int64_t n, float lr,
                float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2,
                const float* grad_scale_ptr, const float* hyper, int grad_dtype, int param_dtype, hipStream_t stream);
// ---- Fused SGD with momentum (torch.optim.SGD semantics) ----
void sgd_step(float* master, float* momentum_buf, const void* grad, void* param_out, int64_t n, float lr,
              float momentum, float dampening, float weight_decay, int nesterov, int first_step,
              const float* grad_scale_ptr, const float* hyper, int grad_dtype, int param_dtype, hipStream_t stream);
// sum of squares of a flat buffer, accumulated (atomically, fp32) into *out (caller zeroes it).
void sumsq(const void* x, int64_t n, float* out, int dtype, hipStream_t stream);

// ---- Fused softmax cross-entropy over [N, V] logits (mean over non-ignored rows) ----
//   loss_rows: fp32 [N]; if grad_inplace, logits are overwritten with d(mean loss)/d(logits)
//   using the device scalar *inv_count (1 / number of non-ignored rows).
void cross_entropy_fwd(void* logits, const int64_t* target, float* loss_rows, float* lse_rows,
                       const float* inv_count, int64_t n, int64_t v, int64_t ld, int64_t ignore_index,
                       int grad_inplace, float label_smoothing, int dtype, hipStream_t stream);

// ---- Flash attention (causal / full, GQA), bf16, head_dim in {32, 64, 128} ----
//   q: [B, Sq, Hq, D], k/v: [B, Sk, Hkv, D] with arbitrary batch/seq/head strides (last dim contiguous),
//   o: [B, Sq, Hq, D] contiguous, lse: fp32 [B, Hq, Sq] (natural log, includes the softmax scale).
struct AttnParams {
  const void* q; const void* k; const void* v; void* o; float* lse;
  int64_t q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh;
  int B, Sq, Sk, Hq, Hkv, D;
  float scale;
  int causal;
  // causal offset: query i attends keys j <= i + (Sk - Sq) (bottom-right aligned, as flash-attn).
  // Attention dropout (training): probability drop_p, keep mask regenerated bit-identically in the forward and
  // both backward kernels from a counter hash of (drop_seed, b * Hq + hq, query, key) -- see attn_keep().
  float drop_p;
  unsigned drop_seed;
  // Optional ring-attention merge (context parallelism): fp32 running output acc_o [B, Sq, Hq, D] (strides ao_*) and
  // natural-log log-sum-exp acc_lse [B, Hq, Sq] (strides al_*, unit stride along the sequence).  When acc_o is set
  // the kernel folds its normalised block result into them with the online-softmax merge in its epilogue
  // (lse' = logaddexp(lse, lse_b), acc' = acc e^(lse - lse') + o_b e^(lse_b - lse')) instead of writing o / lse.
  float* acc_o; int64_t ao_sb, ao_ss, ao_sh;
  float* acc_lse; int64_t al_sb, al_sh;
};
void flash_attn_fwd(const AttnParams& p, hipStream_t stream);

struct AttnBwdParams {
  AttnParams f;
  const void* dout; int64_t do_sb, do_ss, do_sh;
  float* delta;          // fp32 [B, Hq, Sq] workspace: rowsum(dO * O)
  void* dq; void* dk; void* dv;   // bf16 [B,S,H,D] at the strides below; dk/dv per KV head (GQA summed)
  int64_t dq_sb, dq_ss, dq_sh, dk_sb, dk_ss, dk_sh, dv_sb, dv_ss, dv_sh;
  // optional fused inverse RoPE of dq / dk (interleaved pairs, fp32 tables [max_pos, D / 2], position = row +
  // rope_off): the gradient of attention(rope(q), rope(k), v) w.r.t. the UNrotated q / k, rotated in the epilogue
  // from the fp32 accumulators (one rounding, no separate rope pass over dq / dk)
  const float* rope_cos; const float* rope_sin; int rope_off;
};
void flash_attn_bwd(const AttnBwdParams& p, hipStream_t stream);
int attn_set_variant(int v);   // flash-attention kernel forms for head dim 128: 0 = 32x32x16 (default), 2 = 16x16x32
int attn_get_variant();

// ---- Embedding gather / scatter-add backward (vocab-sharded friendly: out-of-range ids -> zero row) ----
void embedding_fwd(const int64_t* ids, const void* table, void* out, int64_t n, int64_t dim, int64_t vocab_start,
                   int64_t vocab_local, int dtype, hipStream_t stream);
void embedding_bwd(const int64_t* sorted_ids, const int64_t* perm, const void* dout, float* dtable_f32, int64_t n,
                   int64_t dim, int64_t vocab_start, int64_t vocab_local, int dtype, hipStream_t stream);

// ---- cast / scale helpers ----
// C[M, N] (+)= A^T B, A [K, M] / B [K, N] bf16 row-major (weight gradient); C bf16 or fp32.
bool gemm_tn_supported(int64_t M, int64_t N, int64_t K);
// Partial-last-wave plan (csrc/gemm.hip gemm_tn_plan): compute the tile band that would run as a partial wave with K
// split `split` ways into fp32 slabs (workspace_floats floats), keeping rows (dim 0) / columns (dim 1) [0, keep) on
// the plain kernel.  split == 0: one launch.  gemm_tn_set_tail(n): plan for n CUs (tests), 0 = device, < 0 = off.
struct GemmTnPlan {
  int split, dim;
  int64_t keep, workspace_floats;
};
GemmTnPlan gemm_tn_plan(int64_t M, int64_t N, int64_t K);
void gemm_tn_set_tail(int cus);
void gemm_tn(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
             int64_t ldc, int out_dtype, bool accumulate, hipStream_t stream, const GemmTnPlan* plan = nullptr,
             float* workspace = nullptr);

// Forward / input-gradient GEMM C[M, N] = A[M, K] B[N, K]^T with fusable epilogues (csrc/gemm_nt.hip).  bf16.
enum : int { kNtStore = 0, kNtSwiglu = 1, kNtDswiglu = 2, kNtRope = 3 };
struct GemmNtParams {
  const void* A;        // bf16 [M, K], row stride lda
  const void* B;        // bf16 [N, K] (SWIGLU: [2H, K] = [W1; W3]), row stride ldb
  void* C;              // STORE / ROPE: [M, N]; SWIGLU: x13 [M, 2H]; DSWIGLU: d13 [M, 2H]   (row stride ldc)
  void* C2;             // SWIGLU: h [M, H] (row stride ldc2)
  const void* X;        // DSWIGLU: saved x13 = [gate | up] [M, 2H] (row stride ldx)
  int M, N, K;          // SWIGLU / DSWIGLU: N = H
  int H;                // SWIGLU / DSWIGLU: hidden size (column offset of the up half)
  int64_t lda, ldb, ldc, ldc2, ldx;
  // ROPE: columns < n_rot are rotated in interleaved pairs within heads of hd, position = row % S + pos_off
  const float* rope_cos;
  const float* rope_sin;
  int S, hd, n_rot, pos_off;
  int tiles_n;          // set by gemm_nt
};
// rows % 256, N (SWIGLU: H) % 8, K % 8; shapes off the 256 / 64 grid (gemm_nt_ragged) run the ragged-edge kernel
bool gemm_nt_supported(int mode, int64_t M, int64_t N, int64_t K);
bool gemm_nt_ragged(int mode, int64_t N, int64_t K);
void gemm_nt(int mode, const GemmNtParams& p, hipStream_t stream);
int gemm_nt_set_variant(int v);   // plain-store GEMM form (A/B): 0 = 8-wave gemm_nt_k, 4 / 5 = 4-wave gemm_nt4_k
// pipeline variant: bit 0 = lookahead B0 reads (8/4/8/0 fragment reads per phase instead of 12/4/8/0), bit 1 = the
// v_mfma_f32_32x32x16_bf16 kernel (gemm_nt32_k) instead of 16x16x32 (gemm_nt_k); both take ragged shapes.

// 1x1 convolution on channels-last activations as tall-skinny GEMMs (csrc/conv1x1.hip).  bf16 operands.
// ts_gemm_nt: C[M, N] = A[M, K] B[N, K]^T (N, K % 64 == 0).  ts_gemm_tn: C[N, K] (+)= A[M, N]^T B[M, K] through
// fp32 partials over nsplit pixel chunks (partial: nsplit * N * K floats; ts_gemm_tn_splits picks nsplit).
bool conv1x1_supported(int64_t M, int64_t N, int64_t K);
// H, W > 0: 3x3 / stride-1 / pad-1 implicit GEMM over a channels-last [M = n*H*W, K/9] input (K tap-major).
// pro_ss (1x1 only): fp32 [scale K | shift K]; A (nt) / B (tn) elements enter the product as relu(v * scale + shift)
// -- a training-mode BatchNorm + ReLU folded into the convolution's operand load.
void ts_gemm_nt(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, hipStream_t stream, int H = 0, int W = 0,
                const void* D = nullptr, float* stats = nullptr, const float* pro_ss = nullptr);
// 1x1 input gradient plus the stride-2 sub-image gradient D [n * ceil(H/2) * ceil(W/2), N] added at the even pixels of
// the H x W grid (a strided 1x1 downsample's input gradient merged into the block's conv1 dgrad; s must be 2).
void ts_gemm_nt_add_sub(const void* A, const void* B, void* C, const void* D, int64_t M, int64_t N, int64_t K,
                        int64_t lda, int64_t ldb, int64_t ldc, int H, int W, int s, hipStream_t stream);
// BatchNorm backward reduction folded into the input-gradient epilogue that produces the BatchNorm's dy (the consumer
// convolution's dgrad): for 128-row block g of the bf16 output C [M, N] and column c,
//   part[g * 2N + c] = sum dz,   part[g * 2N + N + c] = sum dz * (x - mean) * invstd,   dz = C * [ReLU mask],
// the layout bn_bwd takes as pre_part (its reduction pass over dy, x and the mask is then skipped).  The mask comes
// from x * scale + shift (ss = the forward's fp32 [scale N | shift N]) or from the forward's bits (one byte per
// 8-channel vector); x is the BatchNorm's bf16 input with C's layout (leading dimension N).
struct BnRed {
  const void* x = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  const float* ss = nullptr;
  const uint8_t* bits = nullptr;
  float* part = nullptr;
};
// C = A B^T [+ D] with the BnRed epilogue: 1x1 (H = W = 0; D the residual gradient [M, N], or with adds = 2 the
// stride-2 sub-image gradient of ts_gemm_nt_add_sub over an H x W grid) or the 3x3 stride-1 LDS-DMA kernel (H, W > 0,
// no D).  part must hold cdiv(M, 128) * 2N floats.  dmask (1x1, D [M, N], adds = 0): D is added under these mask bits
// (one byte per 8-channel vector); then r.part == nullptr means no reduction (the masked add alone).
void ts_gemm_nt_bnred(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                      int64_t ldb, int64_t ldc, int H, int W, const void* D, int adds, const BnRed& r,
                      hipStream_t stream, const uint8_t* dmask = nullptr);
void conv3_gemm_bnred(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                      int64_t ldb, int64_t ldc, int H, int W, const BnRed& r, hipStream_t stream);
// The one-tap identity geometry (ConvGeo below) that makes the LDS-DMA implicit GEMM a plain C = A B^T, and whether a
// 1x1 convolution's GEMM runs better there than on ts_nt_k (deep-K shapes).
struct ConvGeo;
ConvGeo gemm1_identity_geo(int64_t M);
bool gemm1_lds_preferred(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
bool gemm1_lds_set(bool on);   // returns the previous setting
// Workgroup slots per round that the LDS-DMA weight-gradient kernels' pixel-chunk split count fills (default 512 = two
// per CU); slots <= 0 only queries.  Returns the previous value.
int64_t c3w_round_set(int64_t slots);
// 3x3 implicit GEMM with an LDS-DMA pipeline (csrc/conv3x3.hip); ts_gemm_nt's H, W > 0 path when supported.
bool conv3_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
void conv3_gemm(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, int H, int W, hipStream_t stream, float* stats = nullptr, const void* bias = nullptr,
                bool bias_bf16 = false);
// Gathered implicit GEMM: strided and parity-class (strided-dgrad) convolutions on the same LDS-DMA kernels.
// GEMM rows m = (n, oy, ox) over an Ho x Wo grid.  The gathered operand's row for output row m and tap t is the pixel
//   (n Hs + sy oy + by + tdy[t]) Ws + sx ox + bx + tdx[t]     -- zero-filled when outside the Hs x Ws image --
// of a channels-last [src_rows, Cin] tensor, K = ntaps * Cin tap-major; the forward / input-gradient kernel stores row m
// to destination row (n Hd + ty oy + tby) Wd + tx ox + tbx (a scatter for the parity classes of a strided dgrad).
struct ConvGeo {
  int Hs, Ws, Ho, Wo;
  int sy, sx, by, bx;
  int Hd, Wd, ty, tx, tby, tbx;
  int ntaps;
  int tdy[9], tdx[9];
  int64_t src_rows;
};
// chunk_taps (the 7x7 RGB stem): every 16-B chunk of the operand's K is its own tap t < ntaps at source row offset
// (t / tdx[0]) Ws + t % tdx[0] of an [src_rows, 8] operand (pairs of 4-channel pixels of a zero-padded image).
bool convg_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const ConvGeo& g,
                     bool chunk_taps = false);
void convg_gemm(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, const ConvGeo& g, hipStream_t stream, float* stats = nullptr, bool chunk_taps = false,
                const void* bias = nullptr, bool bias_bf16 = false);
// weight gradient C[N, K] (+)= dY[M, N]^T X_gathered[M, K] on c3w_k (K = ntaps * Cin, a multiple of 192)
bool c3wg_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const ConvGeo& g,
                    bool chunk_taps = false);
int c3wg_splits(int64_t M, int64_t N, int64_t K, bool chunk_taps, bool one_tap = false);
void ts_gemm_tn_geo(const void* A, const void* B, float* partial, void* C, int64_t M, int64_t N, int64_t K,
                    int64_t lda, int64_t ldb, int nsplit, int out_dtype, bool accumulate, const ConvGeo& g,
                    hipStream_t stream, bool chunk_taps = false);
int ts_gemm_tn_splits(int64_t M, int64_t N, int64_t K);
// 3x3 weight gradient on the LDS-DMA kernel (conv1x1.hip c3w_k): supported shapes and its pixel-chunk count
bool c3w_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
int c3w_splits(int64_t M, int64_t N, int64_t K);
// 1x1 weight gradient on the same LDS-DMA kernel (ts_gemm_tn's H = 0 path without pro_ss when supported)
bool w1_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
int w1_splits(int64_t M, int64_t N, int64_t K);
void ts_gemm_tn(const void* A, const void* B, float* partial, void* C, int64_t M, int64_t N, int64_t K,
                int64_t lda, int64_t ldb, int nsplit, int out_dtype, bool accumulate, hipStream_t stream, int H = 0,
                int W = 0, const float* pro_ss = nullptr);

// Fused BatchNorm(train) [+ residual] [+ ReLU] on channels-last [M, C] activations (C power of two, 8..2048).
// Workspaces (fp32): forward 2*G*C + G, backward 2*G*C + 3*C floats with G = bn_partial_blocks(M, C).
bool bn_nhwc_supported(int64_t C);
int bn_partial_blocks(int64_t M, int64_t C);
// pre_stats (optional): per-row-block partials [mean G*C | M2 G*C | rows G] already computed by the producer of x
// (ts_gemm_nt with stats), G = pre_groups: the statistics pass is skipped.
void bn_fwd_train(const void* x, const void* res, void* y, const void* w, const void* b, void* rmean, void* rvar,
                  float* mean, float* invstd, float* scale, float* shift, float* workspace, int64_t M, int64_t C,
                  float momentum, float eps, bool relu, int dtype, int param_dtype, int running_dtype,
                  hipStream_t stream, const float* pre_stats = nullptr, int pre_groups = 0,
                  int64_t* num_batches_tracked = nullptr, uint8_t* relu_mask = nullptr);
// relu_mask (optional, ReLU only): also write [y > 0] as bits, one byte per 8-channel vector ([M * C / 8] bytes).
void bn_apply(const void* x, const void* res, const float* scale, const float* shift, void* y, int64_t M, int64_t C,
              bool relu, int dtype, hipStream_t stream, uint8_t* relu_mask = nullptr);
// y = relu(x * scale + shift + round(z * zscale + zshift)) and its [y > 0] bits (ss / zss: fp32 [scale C | shift C]):
// a BatchNorm + ReLU whose residual is another BatchNorm's output (ResNet's projection shortcut), both applied in one
// pass, bitwise the unfused pair.
void bn_apply_resbn(const void* x, const void* z, const float* ss, const float* zss, void* y, uint8_t* relu_mask,
                    int64_t M, int64_t C, int dtype, hipStream_t stream);
// xmask_ss (optional, fp32 [scale | shift] of the forward): ReLU mask from x instead of reading y.
// relu_mask (optional): the forward's bit mask instead of y (takes precedence over xmask_ss).
// bn_bwd_dual: relu(bn_a(x) + bn_b(z)) with the ReLU bits relu_mask -- both BatchNorms' backward, the dx passes fused
// into one (dx for x, dz for z); workspaces as bn_bwd's, one each; pre_part_a as bn_bwd's pre_part for bn_a.
void bn_bwd_dual(const void* dy, const uint8_t* relu_mask, const void* x, const void* z, const float* mean_a,
                 const float* invstd_a, const void* w_a, const float* mean_b, const float* invstd_b, const void* w_b,
                 void* dx, void* dz, void* dw_a, void* db_a, void* dw_b, void* db_b, float* ws_a, float* ws_b,
                 int64_t M, int64_t C, int dtype, int param_dtype, hipStream_t stream, const float* pre_part_a = nullptr,
                 int pre_groups_a = 0);
// pre_part (optional): the reduction partials [pre_groups][2C] from the producer's epilogue (BnRed): no reduction pass.
void bn_bwd(const void* dy, const void* y, const void* x, const float* mean, const float* invstd, const void* w,
            void* dx, void* dres, void* dw, void* db, float* workspace, int64_t M, int64_t C, bool relu, int dtype,
            int param_dtype, hipStream_t stream, const float* xmask_ss = nullptr,
            const uint8_t* relu_mask = nullptr, const float* pre_part = nullptr, int pre_groups = 0);

// Stride-2 max pooling, channels-last [N, H, W, C] (C % 8 == 0), csrc/pool.hip: k = 3 (padding 1) or 2 (padding 0),
// floor mode.  tap: one byte per output element, the window position (0..k*k-1) of the max; the backward gathers
// through it.
inline int64_t maxpool_s2_out(int64_t n, int k) { return k == 3 ? (n - 1) / 2 + 1 : n / 2; }
void maxpool_s2_fwd(const void* x, void* y, uint8_t* tap, int64_t N, int64_t H, int64_t W, int64_t C, int k,
                    int dtype, hipStream_t stream);
// add (optional): a second gradient of the input, [N, H, W] rows of row stride lda, summed in before the store.
void maxpool_s2_bwd(const void* dy, const uint8_t* tap, void* dx, int64_t N, int64_t H, int64_t W, int64_t C, int k,
                    int dtype, hipStream_t stream, const void* add = nullptr, int64_t lda = 0);
// maxpool_s2_bwd (bf16, C / 8 dividing 256) whose input is a training-mode BatchNorm + ReLU output: also that
// BatchNorm's backward reduction partials (BnRed, mask from x) into r.part [maxpool_s2_bwd_bnred_blocks(...)][2C].
int maxpool_s2_bwd_bnred_blocks(int64_t N, int64_t H, int64_t W, int64_t C);
void maxpool_s2_bwd_bnred(const void* dy, const uint8_t* tap, void* dx, int64_t N, int64_t H, int64_t W, int64_t C,
                          int k, const BnRed& r, hipStream_t stream, const void* add = nullptr, int64_t lda = 0);

// SimpleUNet up-path, csrc/upsample.hip.  y: the ConvTranspose2d(2, 2) GEMM output [N*H*W, 4*Co] (columns (i, j, co));
// skip / out / dcat / dskip channels-last.  out[n, oh, ow, :] = [bilinear(pixel_shuffle(y) + bias)(oh, ow), skip].
// Co, Cs % 8 == 0; bias fp32 or null.
void upcat_fwd(const void* y, const float* bias, const void* skip, void* out, int64_t N, int64_t H, int64_t W,
               int64_t Co, int64_t Ho, int64_t Wo, int64_t Cs, int dtype, hipStream_t stream);
// dskip null: only dy (the skip's gradient is read from dcat by its other consumer, maxpool_s2_bwd's add).
void upcat_bwd(const void* dcat, void* dy, void* dskip, int64_t N, int64_t H, int64_t W, int64_t Co, int64_t Ho,
               int64_t Wo, int64_t Cs, int dtype, hipStream_t stream);

// out[c] = sum_m x[m, c] over a row-major [M, C] (channels-last) tensor, csrc/chsum.hip: fp32 partials
// part[chsum_partial_blocks(M, C) * C], out in out_dtype (fp32 / bf16).  Deterministic.
int chsum_partial_blocks(int64_t M, int64_t C);
void chsum(const void* x, float* part, void* out, int64_t M, int64_t C, int dtype, int out_dtype, hipStream_t stream);

// dst[C, R] = src[R, C]^T (bf16, row-major, leading dims in elements; vector path needs 16-B aligned rows).
void pad_cols(const void* src, void* dst, int64_t R, int64_t C, int64_t ld_src, int64_t Cp, hipStream_t stream);
void transpose2d(const void* src, void* dst, int64_t R, int64_t C, int64_t ld_src, int64_t ld_dst,
                 hipStream_t stream);
// 3x3 convolution input-gradient weight: channels-last w [cout][3][3][cin] -> out [cin][9 taps][cout], taps reversed
// (the flipped, channel-transposed weight of dX = conv(dY, flip(W)^T)), one launch
void conv3x3_dgrad_weight(const void* w, void* out, int64_t cout, int64_t cin, hipStream_t stream);

void cast_copy(const void* src, void* dst, int64_t n, int src_dtype, int dst_dtype, float scale, hipStream_t stream);

// Latitude-weighted MSE over [B, C, H, W] (csrc/latmse.hip).  Forward workspace: latmse_partial_blocks(n) floats.
int latmse_partial_blocks(int64_t n);
void latmse_fwd(const void* pred, const void* target, float* partial, float* out, int64_t n, int64_t H, int64_t W,
                int64_t n_global, int64_t lat_offset, int dtype, hipStream_t stream);
void latmse_bwd(const void* pred, const void* target, const float* gloss, void* dpred, void* dtarget, int64_t n,
                int64_t H, int64_t W, int64_t n_global, int64_t lat_offset, int dtype, hipStream_t stream);

// Batch assembly from a device-resident uint8 image set [N, H, W, C] (csrc/imageaug.hip): gather idx[B], random crop
// (per-sample dy, dx in [0, 2 pad], zero padding) + horizontal flip (params [B, 3] int32, or null = centre, no flip),
// scale 1/255, normalise ((v - mean) * inv_std), write NCHW or NHWC in fp32 / bf16.
void image_augment(const uint8_t* images, const int64_t* idx, const int* params, const float* mean,
                   const float* inv_std, void* out, int64_t B, int64_t H, int64_t W, int64_t C, int64_t pad,
                   bool nhwc, int out_dtype, hipStream_t stream);

// Per-tensor FP8 quantisation (csrc/fp8.hip): OCP e4m3 / e5m2.  fp8_amax: max|x| over n contiguous bf16 (n % 8 == 0)
// via fp8_amax_blocks(n) per-block partials -> scal[3] = [amax, FMAX / amax, amax / FMAX].  fp8_quant: x [R, C]
// contiguous bf16, R % 64 == C % 64 == 0 -> y [R, C] and / or yt [C, R] fp8 (null = not written), scaled by scal[1].
constexpr int kFP8E4M3 = 0, kFP8E5M2 = 1;
int fp8_amax_blocks(int64_t n);
void fp8_amax(const void* x, int64_t n, int fmt, float* partial, float* scal, hipStream_t stream);
void fp8_quant(const void* x, int64_t R, int64_t C, const float* scal, int fmt, void* y, void* yt, hipStream_t stream);

// Serving path (csrc/decode.hip).  Caches are [B, Smax, Hkv, D] bf16 (K and V at the same strides, elements);
// pos[b] (int32, device) = tokens already cached for sequence b.
struct KVAppendParams {
  void* qkv; int64_t qkv_sb, qkv_ss;     // [B, S, (Hq + 2 Hkv) * D] bf16; q rotated in place
  void* kc; void* vc; int64_t c_sb, c_ss, c_sh;
  const int* pos; const float* cos; const float* sin;   // RoPE tables fp32 [max_pos, D / 2]
  int B, S, Hq, Hkv, D, Smax;
  int kv_fp8;                            // caches hold OCP e4m3 bytes (value / kv_scale), else bf16
  float kv_scale;
};
void kv_append(const KVAppendParams& p, hipStream_t stream);
struct DecodeParams {
  const void* q; int64_t q_sb, q_sh;     // q[b, hq, :] bf16
  const void* kc; const void* vc; int64_t c_sb, c_ss, c_sh;
  const int* pos; int len_add;           // keys visible to sequence b: pos[b] + len_add
  float* opart; float* mlpart;           // workspace [B, Hq, nch, D] / [B, Hq, nch, 2] fp32
  void* out; int64_t out_sb;             // bf16 out[b, hq * D + d]
  int B, Hq, Hkv, D, nch;                // nch = 64-key chunks covered (>= ceil(max length / 64))
  int Smax;                              // cache capacity: lengths are clamped to it (no read past the cache)
  float scale;
  int kv_fp8;                            // e4m3 caches: stored value x kv_scale = key / value
  float kv_scale;
};
int decode_heads_per_wave(int Hq, int Hkv);
void decode_attention(const DecodeParams& p, hipStream_t stream);
// y[M, N] = x[M, K] W[N, K]^T for decode-sized M (<= 64): bf16, rows of x / W / y at strides ldx / ldw / ldy.
bool skinny_gemm_supported(int64_t M, int64_t N, int64_t K);
// GEMV (M <= 2 rows) with the x operand optionally produced in the kernel: xmode 0 = x [M, K]; 1 = silu(gate) * up
// from x = [M, 2K] (gate | up); 2 = RMSNorm(x + res) * g (res, h_out optional; h_out = x + res written once).
struct GemvArgs {
  const void* x; int64_t ldx;
  const void* res; int64_t ldres;
  const void* g; float eps;
  void* h_out; int64_t ldh;
  const void* w; int64_t ldw;
  void* y; int64_t ldy;
  int M, N, K;
};
bool gemv_supported(int64_t M, int64_t N, int64_t K);
void gemv(const GemvArgs& a, int xmode, hipStream_t stream);
void skinny_gemm(const void* x, int64_t ldx, const void* w, int64_t ldw, void* y, int64_t ldy, int M, int N, int K,
                 hipStream_t stream);

// Single-node all-reduce over IPC-mapped peer buffers (csrc/custom_allreduce.hip).  ctx is an opaque handle.
int64_t car_create(int rank, int world, int64_t max_bytes, double timeout_s);
void car_ipc_handle(int64_t ctx, void* out64);
void car_open(int64_t ctx, const void* handles);
int64_t car_max_bytes(int64_t ctx);
void car_allreduce(int64_t ctx, const void* in, void* out, int64_t bytes, int dtype, int algo, float scale,
                   int max_blocks, hipStream_t stream);
int64_t car_status(int64_t ctx);
void car_flag(int64_t ctx, int* flag_dev, hipStream_t st);
void car_poison(int64_t ctx, const int* flag_dev, float* gscale_dev, hipStream_t st);
int64_t car_agreed(int64_t ctx);
void car_destroy(int64_t ctx);

}  // namespace dph
