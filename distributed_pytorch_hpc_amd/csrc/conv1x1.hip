// 1x1 (and 3x3 / stride 1, as implicit GEMMs) convolutions on channels-last activations = tall-skinny GEMMs,
// for CDNA4 (gfx950).
//
// In NHWC a stride-1 1x1 convolution is Y[M, Cout] = X[M, Cin] W[Cout, Cin]^T with M = N*H*W pixels (up to
// 802,816 for ResNet-50 at B=256) and Cin, Cout in 64..2048: far more rows than columns and memory-bound
// (benchmarks/conv_bench.py).  hipBLASLt tiles these shapes badly (2-7x slower than MIOpen's NHWC implicit GEMM,
// profiles/conv_bench_miopen_vs_1x1_gemm.json); these kernels are written for them:
//
//   ts_nt_k   C[M, N] = A[M, K] B[N, K]^T  (forward: A = X, B = W;  input gradient: A = dY, B = W^T)
//             128 x BN tile per workgroup (4 waves x 32 rows, BN = 64 | 128), K-steps of 64, A fragments straight
//             from HBM into registers (each row is used by exactly one wave -- no LDS round trip), prefetched one
//             K-step ahead; the small B slab is register-staged into a double-buffered LDS image (144-B rows:
//             conflict-free ds_read_b128); v_mfma_f32_32x32x16_bf16; the C tile goes back through LDS so the
//             stores are whole 16-B row segments.  N-tiles of one row block run on one XCD (L2 reuse of A).
//   ts_tn_k   P[s][N, K] = sum over the s-th pixel chunk of A[m, N]^T B[m, K]  (weight gradient, A = dY, B = X)
//             64 x 64 output tile per workgroup (4 waves x 32x32), pixels are the reduction dim: 64-pixel slabs
//             of both operands are register-staged into unpadded 128-B LDS rows whose 16-B chunks are XOR-
//             swizzled by bit 1 of the row (the 4-row x 64-B footprint of a half-wave's transposed read then
//             covers all 64 banks once) and read back with ds_read_b64_tr_b16 (32 KB of LDS per workgroup); split
//             over pixel chunks sized to fill one resident round of workgroups, fp32 partials, then
//   ts_reduce_k  dW = sum_s P[s] (+ dW) in the weight's dtype (deterministic: fixed summation order).
#include <algorithm>
#include <cstdlib>

#include "bn_epilogue.h"
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4_c;

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr int TS_BM = 128, TS_BK = 64, TS_NT = 256;
constexpr int TS_BROW = 72;   // B slab row: 64 bf16 + 8 pad (144 B: 16 consecutive rows hit 16 distinct 16-B slots)
constexpr int TS_KF = TS_BK / 16;   // MFMA k-steps (A fragments) per K-step

// C3: 3x3 / stride 1 / pad 1 convolution as an implicit GEMM over the channels-last input A [M = N*H*W, Cin]:
// K = 9 * Cin is tap-major (k = tap * Cin + c), and the A row of output pixel m for tap (dy, dx) is the input
// pixel m + (dy-1) * W + (dx-1), or zero when that falls outside the image (padding).  A K-step never straddles
// two taps (Cin % 64 == 0), so the shift is one wave-uniform offset per K-step plus a per-lane bounds check.
// ADD: C = A B^T + D (D [M, N] bf16 with C's leading dimension), the sum rounded once like an unfused add of
// the two bf16 tensors -- merges a residual branch's input gradient into the 1x1 convolution's dgrad.
// STATS: also emit per-row-block BatchNorm statistics of the bf16 output (the values BN will read): for row block
// mb and column n, stats[mb * N + n] = mean, stats[nmb * N + mb * N + n] = M2 (sum of squared deviations),
// stats[2 * nmb * N + mb] = rows -- the partial layout bn_finalize_k merges (Chan), so the BN that follows a
// 1x1 convolution skips its own statistics pass over the activation.
// PRO: the A operand is the raw input of a training-mode BatchNorm + ReLU (the bottleneck's bn2 -> conv3): every A
// element is replaced by relu(a * scale[k] + shift[k]) (pro_ss = fp32 [scale K | shift K], the BatchNorm's forward
// coefficients) after it lands in registers, so the normalised activation is never written to HBM.
// ADDS = s > 1 (with ADD): D is the gradient of the stride-s sub-image (a strided 1x1 downsample's input gradient,
// [n * ceil(H/s) * ceil(W/s), N]) and is added only at the pixels (y, x) with y % s == x % s == 0 of the H x W grid.
// Occupancy: the plain / ADD forms fit 128 VGPRs for 4 workgroups per CU (LDS 36 KiB each); at 132 they ran 3, and
// ResNet-50's 392-row-block layers (14 x 14 at B = 256) then launch 784 workgroups for 768 slots -- a second round for
// 16 of them (benchmarks/probes/grid_tail.py: +23 % time for +2 % rows there, profiles/r4/grid_tail/).
// MINB = 4 forces the 128-VGPR build (MINB = 1, the compiler's own budget, measured slower: profiles/r4/grid_tail/).
// BRED = 1 | 2 (input gradient of a BatchNorm + ReLU output, 1x1 only): the BatchNorm backward's reduction over the
// stored gradient (kernels.h BnRed, bn_epilogue.h) -- mask from x (1) or from the forward's bits (2).
// AMASK (with ADD, ADDS = 0): D enters as D * mask, mask = dmask bits (one byte per 8-channel vector of [M, N]) -- the
// residual gradient of a BatchNorm + residual + ReLU is its output gradient under the ReLU mask, so that BatchNorm's
// backward hands over dy and its forward's bits instead of writing the masked copy.
template <int BN, bool C3, bool ADD = false, bool STATS = false, bool PRO = false, int ADDS = 0, int MINB = 4,
          int BRED = 0, bool AMASK = false>
__global__ __launch_bounds__(TS_NT, PRO ? 1 : MINB) void ts_nt_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                 bf16* __restrict__ C, int M, int N, int K, int64_t lda,
                                                 int64_t ldb, int64_t ldc, int H, int W, int Cin,
                                                 const bf16* __restrict__ D = nullptr,
                                                 float* __restrict__ stats = nullptr,
                                                 const float* __restrict__ pro_ss = nullptr, BnRed bnr = {},
                                                 const uint8_t* __restrict__ dmask = nullptr) {
  static_assert(!BRED || (!C3 && !STATS && !PRO), "BRED: 1x1 input-gradient forms only");
  static_assert(!AMASK || (ADD && ADDS == 0), "AMASK: the masked residual-gradient add");
  constexpr int NT = BN / 32;                        // 32-column tiles per wave
  constexpr int BCH = BN * (TS_BK / 8) / TS_NT;      // 16-B B chunks per thread per K-step (BN=128: 4)
  constexpr int CROW = BN + 8;                       // epilogue LDS row (bf16)
  constexpr int LDS_B = 2 * BN * TS_BROW * 2, LDS_C = TS_BM * CROW * 2 + (STATS ? 4 * BN * 4 : 0);
  __shared__ __attribute__((aligned(16))) char smem[LDS_B > LDS_C ? LDS_B : LDS_C];
  __shared__ __attribute__((aligned(16))) float pss[PRO ? 2 * 2048 : 4];   // [scale K | shift K] (K <= 2048)
  bf16* Bs = reinterpret_cast<bf16*>(smem);
  if constexpr (PRO) {
    for (int i = threadIdx.x; i < 2 * K; i += TS_NT) pss[i] = pro_ss[i];   // visible after the first barrier
  }
  // relu(a * scale + shift) of the 8 consecutive channels k0.. of an A fragment, from the LDS copy
  auto pro = [&](bf16x8 v, int k0) -> bf16x8 {
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(pss + k0), s1 = *reinterpret_cast<const f32x4*>(pss + k0 + 4);
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(pss + K + k0), t1 = *reinterpret_cast<const f32x4*>(pss + K + k0 + 4);
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = (bf16)fmaxf(fmaf((float)v[i], s0[i], t0[i]), 0.f);
      o[i + 4] = (bf16)fmaxf(fmaf((float)v[i + 4], s1[i], t1[i]), 0.f);
    }
    return o;
  };

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l32 = lane & 31, h = lane >> 5;
  const int ntn = N / BN, nmb = (M + TS_BM - 1) / TS_BM;
  const int lin = xcd_remap(blockIdx.x, nmb * ntn);
  const int mb = lin / ntn, nt0 = (lin % ntn) * BN;
  const int m0 = mb * TS_BM;

  // A: this lane's row (clamped for the ragged last block; its results are not stored)
  const int arow = min(m0 + wid * 32 + l32, M - 1);
  const bf16* ap = A + (int64_t)arow * lda + 8 * h;
  int xw = 0, yh = 0;
  if constexpr (C3) {
    xw = arow % W;
    yh = (arow / W) % H;
  }
  // A fragment f of the K-step starting at column ko (zero for a padding tap)
  auto load_a = [&](int ko, int f) -> bf16x8 {
    if constexpr (!C3) {
      return *reinterpret_cast<const bf16x8*>(ap + ko + 16 * f);
    } else {
      const int tap = ko / Cin, cb = ko - tap * Cin;
      const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
      const bool ok = (unsigned)(yh + dy) < (unsigned)H && (unsigned)(xw + dx) < (unsigned)W;
      const bf16* pp = ok ? ap + (int64_t)(dy * W + dx) * lda + cb + 16 * f : ap;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(pp);
      return ok ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  // B staging: chunk c of thread t -> slab row (t*BCH + c) / 8, 16-B column chunk (t*BCH + c) % 8
  const bf16* bp[BCH];
  int bdst[BCH];
#pragma unroll
  for (int c = 0; c < BCH; ++c) {
    const int ch = threadIdx.x * BCH + c, row = ch >> 3, col = (ch & 7) * 8;
    bp[c] = B + (int64_t)(nt0 + row) * ldb + col;
    bdst[c] = row * TS_BROW + col;
  }

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int nks = K / TS_BK;
  bf16x8 a[TS_KF];
#pragma unroll
  for (int f = 0; f < TS_KF; ++f) a[f] = load_a(0, f);
  bf16x8 bst[BCH];
#pragma unroll
  for (int c = 0; c < BCH; ++c) bst[c] = *reinterpret_cast<const bf16x8*>(bp[c]);
#pragma unroll
  for (int c = 0; c < BCH; ++c) *reinterpret_cast<bf16x8*>(Bs + bdst[c]) = bst[c];
  __syncthreads();

  for (int ks = 0; ks < nks; ++ks) {
    const int cur = ks & 1;
    bf16x8 na[TS_KF];
#pragma unroll
    for (int f = 0; f < TS_KF; ++f) na[f] = a[f];
    if (ks + 1 < nks) {   // prefetch the next K-step (A into registers, B into staging registers)
      const int ko = (ks + 1) * TS_BK;
#pragma unroll
      for (int f = 0; f < TS_KF; ++f) na[f] = load_a(ko, f);
#pragma unroll
      for (int c = 0; c < BCH; ++c) bst[c] = *reinterpret_cast<const bf16x8*>(bp[c] + ko);
    }
    const bf16* bs = Bs + cur * BN * TS_BROW;
    if constexpr (PRO) {   // this K-step's fragments have landed (the MFMAs below consume them anyway)
#pragma unroll
      for (int f = 0; f < TS_KF; ++f) a[f] = pro(a[f], ks * TS_BK + 16 * f + 8 * h);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16* br = bs + (t * 32 + l32) * TS_BROW + 8 * h;
#pragma unroll
      for (int f = 0; f < TS_KF; ++f)
        acc[t] = mfma32(a[f], *reinterpret_cast<const bf16x8*>(br + 16 * f), acc[t]);
    }
    if (ks + 1 < nks) {
      bf16* nb = Bs + (cur ^ 1) * BN * TS_BROW;
#pragma unroll
      for (int c = 0; c < BCH; ++c) *reinterpret_cast<bf16x8*>(nb + bdst[c]) = bst[c];
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < TS_KF; ++f) a[f] = na[f];
  }

  // ---- epilogue through LDS: register r of tile t holds C[row (r&3) + 8(r>>2) + 4h][col t*32 + l32] ----
  bf16* Cs = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      Cs[(wid * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * CROW + t * 32 + l32] = (bf16)acc[t][r];
  constexpr int CPR = BN / 8;   // 16-B chunks per row
  constexpr int NIT = TS_BM * CPR / TS_NT;   // store iterations per thread (its chunk column is fixed)
  // HBM operands of the store loop (the residual-gradient add, the BatchNorm input and its mask bits) are fetched PF
  // iterations ahead, the first PF before the barrier: one exposed load latency per tile instead of one per iteration
  constexpr bool PDA = ADD && ADDS == 0;
  constexpr int PF = (PDA || BRED != 0) ? (NIT < 4 ? NIT : 4) : 1;
  using BRA = BnRedAcc<BRED ? BRED : 1>;
  [[maybe_unused]] bf16x8 dq[PF], xq[PF];
  [[maybe_unused]] unsigned mq[PF], aq[PF];
  auto fetch = [&](int it, int sl) {
    const int i = threadIdx.x + it * TS_NT, ch = i % CPR;
    const int64_t r = min(m0 + i / CPR, M - 1);
    if constexpr (PDA) dq[sl] = *reinterpret_cast<const bf16x8*>(D + r * ldc + nt0 + ch * 8);
    if constexpr (AMASK) aq[sl] = dmask[r * (N >> 3) + (nt0 >> 3) + ch];
    if constexpr (BRED != 0) {
      xq[sl] = BRA::load_x(bnr, r, N, nt0 + ch * 8);
      mq[sl] = BRA::load_m(bnr, r, N, nt0 + ch * 8);
    }
  };
  if constexpr (PDA || BRED != 0) {
#pragma unroll
    for (int it = 0; it < PF; ++it) fetch(it, it);
  }
  __syncthreads();
  [[maybe_unused]] BRA bra;
  if constexpr (BRED != 0) bra.init(bnr, nt0 + (threadIdx.x % CPR) * 8, N);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = threadIdx.x + it * TS_NT, row = i / CPR, ch = i % CPR, sl = it % PF;
    [[maybe_unused]] const bf16x8 dv = dq[sl], xv = xq[sl];
    [[maybe_unused]] const unsigned mv = mq[sl], av = aq[sl];
    if constexpr (PDA || BRED != 0) {
      if (it + PF < NIT) fetch(it + PF, sl);
    }
    if (m0 + row < M) {
      const int64_t o = (int64_t)(m0 + row) * ldc + nt0 + ch * 8;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + row * CROW + ch * 8);
      if constexpr (ADD && ADDS > 1) {
        const int m = m0 + row, x = m % W, t = m / W, y = t % H, n = t / H;
        if (x % ADDS == 0 && y % ADDS == 0) {
          const int Ho = (H - 1) / ADDS + 1, Wo = (W - 1) / ADDS + 1;
          const int64_t dr = ((int64_t)n * Ho + y / ADDS) * Wo + x / ADDS;
          const bf16x8 d = *reinterpret_cast<const bf16x8*>(D + dr * ldc + nt0 + ch * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)d[j]);
        }
      } else if constexpr (AMASK) {   // bitwise the unmasked add of a materialised bf16(dy * mask)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (((av >> j) & 1u) ? (float)dv[j] : 0.f));
      } else if constexpr (ADD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)dv[j]);
      }
      *reinterpret_cast<bf16x8*>(C + o) = v;
      if constexpr (BRED != 0) bra.add(xv, mv, v);
    }
  }
  if constexpr (BRED != 0) {
    __syncthreads();   // every C-tile read is done: the tile's LDS holds the cross-wave partials
    bra.finish(reinterpret_cast<float*>(smem), CPR, TS_NT / 64, mb, N, nt0, bnr.part);
  }
  if constexpr (STATS) {
    // from the accumulator registers (rounded to bf16, the values BN will read): register r of tile t is row
    // wid*32 + (r&3) + 8(r>>2) + 4h of column t*32 + l32.  Pass 1 column sums, pass 2 squared deviations from the
    // tile mean; the lane halves (h) meet by a cross-half shuffle, the 4 waves in a [4][BN] LDS block behind the
    // C tile (it fits in the K-loop's staging footprint for BN = 128).
    float* sred = reinterpret_cast<float*>(smem + TS_BM * CROW * 2);
    const int valid = min(TS_BM, M - m0);
    const float inv_n = 1.f / (float)valid;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float sm = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wid * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        sm += row < valid ? (float)(bf16)acc[t][r] : 0.f;
      }
      sm += __shfl_xor(sm, 32);
      if (h == 0) sred[wid * BN + t * 32 + l32] = sm;
    }
    __syncthreads();
    float mean_t[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = t * 32 + l32;
      mean_t[t] = (sred[col] + sred[BN + col] + sred[2 * BN + col] + sred[3 * BN + col]) * inv_n;
    }
    const float mean_w = threadIdx.x < BN ? (sred[threadIdx.x] + sred[BN + threadIdx.x] + sred[2 * BN + threadIdx.x] +
                                             sred[3 * BN + threadIdx.x]) * inv_n
                                          : 0.f;
    __syncthreads();   // every wave has read the sums before they are overwritten by the M2 partials
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float m2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wid * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float d = (float)(bf16)acc[t][r] - mean_t[t];
        m2 += row < valid ? d * d : 0.f;
      }
      m2 += __shfl_xor(m2, 32);
      if (h == 0) sred[wid * BN + t * 32 + l32] = m2;
    }
    __syncthreads();
    if (threadIdx.x < BN) {
      const int col = threadIdx.x, nmb = (M + TS_BM - 1) / TS_BM;
      stats[(int64_t)mb * N + nt0 + col] = mean_w;
      stats[(int64_t)nmb * N + (int64_t)mb * N + nt0 + col] =
          sred[col] + sred[BN + col] + sred[2 * BN + col] + sred[3 * BN + col];
      if (col == 0 && nt0 == 0) stats[2 * (int64_t)nmb * N + mb] = (float)valid;
    }
  }
}

// ---- weight gradient: P[s][n][k] = sum_{m in chunk s} A[m][n] B[m][k] ----
constexpr int TW_ROWB = 128;   // LDS row: 64 bf16, 16-B chunks XOR-swizzled by tw_swz(row)

// chunk swizzle of LDS row r: rows 2 apart (same bank half) read complementary 64-B halves
__device__ __forceinline__ int tw_swz(int r) { return ((r >> 1) & 1) << 2; }

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_c*)p);
  return __builtin_bit_cast(bf16x4, v);
}

// C3: 3x3 weight gradient, K = 9 * Cin tap-major; B rows (input pixels) are shifted by the output tile's tap and
// zero outside the image, A (output-gradient) rows are not shifted.
// PRO (1x1 only): B is the raw input of a training-mode BatchNorm + ReLU; each staged B element becomes
// relu(b * scale[k] + shift[k]) (pro_ss = [scale K | shift K]) on its way into LDS.  A thread's B columns are fixed for
// the whole loop, so its 8 scales / shifts live in registers.  Rows past the chunk keep dY = 0, so their transformed
// B values contribute nothing.
template <bool C3, bool PRO = false>
__global__ __launch_bounds__(256) void ts_tn_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                               float* __restrict__ P, int M, int N, int K, int64_t lda,
                                               int64_t ldb, int chunk, int H, int W, int Cin,
                                               const float* __restrict__ pro_ss = nullptr) {
  constexpr int TP = 64;   // pixels per step (rows of the staged slabs)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TP * TW_ROWB];   // [buf][A|B][64 rows][128 B]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wi = wid >> 1, wj = wid & 1;             // wave's 32x32 sub-tile of the 64x64 output tile
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int tn = N / 64, tk = K / 64;
  const int nsplit = gridDim.x / (tn * tk);
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  // all output tiles of one pixel chunk are adjacent (same XCD): they read the same dY / X rows, which then come
  // from that XCD's L2 instead of HBM once per tile
  const int ntile = tn * tk;
  const int s = lin / ntile, tile = lin % ntile;
  const int n0 = (tile / tk) * 64, k0 = (tile % tk) * 64;
  const int mbeg = s * chunk, mend = min(M, mbeg + chunk);
  int bcol = k0, dy = 0, dx = 0;
  if constexpr (C3) {
    const int tap = k0 / Cin;
    bcol = k0 - tap * Cin;
    dy = tap / 3 - 1;
    dx = tap - (tap / 3) * 3 - 1;
  }

  // staging: thread t copies 16 B of rows t>>3 and 32 + (t>>3) of the 64-row slab, chunk t&7, for A and B
  const int srow = threadIdx.x >> 3, sch = threadIdx.x & 7;
  const int sdst = srow * TW_ROWB + (sch ^ tw_swz(srow)) * 16;   // row srow + 32 has the same swizzle
  // transposed-read offsets: lane 4q+p of 16-lane group g reads row (r0 + q), columns c0 + 4p .. +3 where the
  // group's half h = g >> 1 selects rows 8h.. (k-steps) and g & 1 the column half of the 32-wide operand; the
  // rows read (16kk + 8h + q, +4) all swizzle like q
  const int hh = g >> 1;
  const int tch = 2 * (g & 1) + (p >> 1), tin = 8 * (p & 1);
  const int toffA = (8 * hh + q) * TW_ROWB + (((wi * 4 + tch) ^ tw_swz(q)) << 4) + tin;
  const int toffB = (8 * hh + q) * TW_ROWB + (((wj * 4 + tch) ^ tw_swz(q)) << 4) + tin;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  auto load = [&](int m, bf16x8 (&va)[2], bf16x8 (&vb)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = m + srow + 32 * u, row = min(rr, M - 1);
      va[u] = *reinterpret_cast<const bf16x8*>(A + (int64_t)row * lda + n0 + sch * 8);
      bool bok = true;
      int brow = row;
      if constexpr (C3) {
        const int xw = row % W, yh = (row / W) % H;
        bok = (unsigned)(yh + dy) < (unsigned)H && (unsigned)(xw + dx) < (unsigned)W;
        brow = bok ? row + dy * W + dx : row;
      }
      vb[u] = *reinterpret_cast<const bf16x8*>(B + (int64_t)brow * ldb + bcol + sch * 8);
      if (!bok) vb[u] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (rr >= mend) {   // rows past this chunk contribute zero
        va[u] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        vb[u] = va[u];
      }
    }
  };
  float psc[8], psh[8];
  if constexpr (PRO) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      psc[i] = pro_ss[bcol + sch * 8 + i];
      psh[i] = pro_ss[K + bcol + sch * 8 + i];
    }
  }
  auto stage = [&](char* base, const bf16x8 (&va)[2], const bf16x8 (&vb)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      *reinterpret_cast<bf16x8*>(base + sdst + 32 * u * TW_ROWB) = va[u];
      bf16x8 b = vb[u];
      if constexpr (PRO) {
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = (bf16)fmaxf(fmaf((float)b[i], psc[i], psh[i]), 0.f);
      }
      *reinterpret_cast<bf16x8*>(base + TP * TW_ROWB + sdst + 32 * u * TW_ROWB) = b;
    }
  };
  bf16x8 va[2], vb[2];
  load(mbeg, va, vb);
  stage(smem, va, vb);
  __syncthreads();
  int buf = 0;
  for (int m = mbeg; m < mend; m += TP) {
    const bool more = m + TP < mend;
    if (more) load(m + TP, va, vb);
    const char* As = smem + buf * 2 * TP * TW_ROWB;
    const char* Bs = As + TP * TW_ROWB;
#pragma unroll
    for (int kk = 0; kk < TP / 16; ++kk) {   // 16-pixel MFMA k-steps: rows 16kk + 8h + j
      const int ro = 16 * kk * TW_ROWB;
      const bf16x4 alo = tr_read(As + ro + toffA), ahi = tr_read(As + ro + toffA + 4 * TW_ROWB);
      const bf16x4 blo = tr_read(Bs + ro + toffB), bhi = tr_read(Bs + ro + toffB + 4 * TW_ROWB);
      acc = mfma32(__builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7),
                   __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7), acc);
    }
    if (more) stage(smem + (buf ^ 1) * 2 * TP * TW_ROWB, va, vb);
    __syncthreads();
    buf ^= 1;
  }
  // register r holds P[n0 + wi*32 + (r&3) + 8(r>>2) + 4h][k0 + wj*32 + (lane & 31)]
  float* out = P + (int64_t)s * N * K;
  const int h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r)
    out[(int64_t)(n0 + wi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * K + k0 + wj * 32 + (lane & 31)] = acc[r];
}

// ---- 3x3 weight gradient with an LDS-DMA pipeline: P[s][co][k'] = sum_{m in chunk s} dY[m][co] X_tap(k')[m][ci(k')]
// Output tile TCO (64 | 128) output channels x 192 k' (three 64-channel slabs of the tap-major K' = 9 Cin, each slab
// with its own tap), 4 waves as 2 (co) x 2 (k'), wave tile TCO/2 x 96 = (TCO/64) x 3 MFMA 32x32x16 tiles.
// Pixel steps of 64 rows: the dY slab(s) and the three tap-shifted X slabs go global -> LDS by range-checked buffer
// LDS-DMA (rows past the chunk and padding taps land as zeros, no masking anywhere), 2-stage ring, one barrier per
// step, MFMA operands by ds_read_b64_tr_b16 from the ts_tn_k image layout (128-B rows, XOR-swizzled by bit 1 of the
// row).  fp32 partials per pixel chunk, summed by ts_reduce_k.
constexpr int C3W_TK = 192, C3W_SLABS = 3, C3W_SLAB = 64 * TW_ROWB;   // 8 KB per [64 px][64 ch] slab

// q = r / d, m = r % d for 0 <= r < 2^24 through the fp32 reciprocal (error < 1 before the correction steps)
__device__ __forceinline__ void fdivmod(int r, int d, float inv, int& q, int& m) {
  q = (int)((float)r * inv);
  m = r - q * d;
  if (m < 0) { --q; m += d; }
  if (m >= d) { ++q; m -= d; }
}

// GEN: the X rows are gathered by kernels.h ConvGeo (strided convolutions): output row r = (n, oy, ox) over Ho x Wo,
// tap t's source pixel (n Hs + sy oy + by + tdy[t]) Ws + sx ox + bx + tdx[t] of the [src_rows, Cin] input.
// SL: X slabs (64 k' each) per output tile: 3 for the 3x3 kernels (192 k', one tap per slab), 1 or 2 for the 1x1
// weight gradient (GEN with the identity geometry).
// GEN = 2: chunk taps (the 7x7 RGB stem, conv3x3.hip conv3_k GEN = 2): every 16-B chunk of an X slab is its own tap.
// GEN = 3: identity rows (the stride-1 1x1 weight gradient): X row = dY row, no pixel -> (n, y, x) division per piece.
// NS: ring stages.  2 = the next step's DMA in flight while one step computes (two workgroups per CU); deeper rings
// (1x1 weight gradient, one workgroup per CU) keep NS - 1 steps in flight behind a counted vmcnt: at 16 MFMAs per wave
// and step the two-stage ring waits on every step's DMA round trip (1024->512 @ 14: ~22 % MFMA busy).
template <int TCO, int GEN = 0, int SL = C3W_SLABS, int NS = 2>
__global__ __launch_bounds__(256, NS > 2 ? 1 : 2) void c3w_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                float* __restrict__ P, int M, int N, int K, int64_t lda,
                                                int64_t ldb, int chunk, int H, int W, int Cin, ConvGeo geo) {
  constexpr int AS = TCO / 64;                       // dY slabs per step
  constexpr int TK = 64 * SL, WK = TK / 2;            // k' per tile, per wave
  constexpr int STG = (AS + SL) * C3W_SLAB;           // one stage
  constexpr int PCS = (AS + SL) * 8 / 4;              // 1-KB DMA pieces per wave per step
  constexpr int TI = TCO / 64;                       // co MFMA tiles per wave (wave covers TCO / 2 channels)
  __shared__ __attribute__((aligned(1024))) char smem[NS * STG];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cw = wid >> 1, kw = wid & 1;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, h = lane >> 5;
  const int tn = N / TCO, tk = K / TK, ntile = tn * tk;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int s = lin / ntile, tile = lin % ntile;    // the tiles of one pixel chunk run together (same XCD, same rows)
  const int n0 = (tile / tk) * TCO, k0 = (tile % tk) * TK;
  const int mbeg = s * chunk, mend = min(M, mbeg + chunk);

  const int Wr = GEN ? geo.Wo : W, Hr = GEN ? geo.Ho : H;   // the row space's grid
  const float invW = 1.f / (float)Wr, invH = 1.f / (float)Hr;
  const dph_rsrc ra = make_rsrc(A, (unsigned)((int64_t)M * lda * 2));
  const dph_rsrc rb = make_rsrc(B, (unsigned)((GEN ? geo.src_rows : (int64_t)M) * ldb * 2));
  const unsigned lds0 = lds_addr(smem);
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  // DMA lanes: piece i (of AS*8 + 24 per step) = slab i / 8, rows 8 (i % 8) + prow, LDS slot lane % 8
  const int prow = lane >> 3, sch = (lane & 7) ^ tw_swz(prow);
  int bdy[SL], bdx[SL], bcb[SL];
#pragma unroll
  for (int sb = 0; sb < SL; ++sb) {
    const int kk = k0 + sb * 64, tap = kk / Cin;
    bcb[sb] = kk - tap * Cin;
    if constexpr (GEN) {   // tap table lookup by selects (tap is uniform over the workgroup)
      bdy[sb] = geo.tdy[0];
      bdx[sb] = geo.tdx[0];
#pragma unroll
      for (int t = 1; t < 9; ++t)
        if (tap == t) {
          bdy[sb] = geo.tdy[t];
          bdx[sb] = geo.tdx[t];
        }
    } else {
      bdy[sb] = tap / 3 - 1;
      bdx[sb] = tap - (tap / 3) * 3 - 1;
    }
  }
  // Pixel coordinates (column, image row, image) of each piece's X row, advanced incrementally by the 64 rows of a
  // step instead of two float divisions per piece and step (that arithmetic sat in front of every step's MFMAs: the
  // identity-row 1x1 form without it measured 1.94 vs 2.45 ms per ResNet-50 step).  A piece is an X piece for the
  // whole loop or never (its slab depends on the wave only).
  constexpr bool INCR = GEN != 3;
  int pxw[PCS], pyh[PCS], pnq[PCS];
  const int adv_x = 64 % Wr, adv_q = 64 / Wr, adv_y = adv_q % Hr, adv_n = adv_q / Hr;
  if constexpr (INCR) {
#pragma unroll
    for (int j = 0; j < PCS; ++j) {
      int yq;
      fdivmod(mbeg + 8 * ((wid_u * PCS + j) & 7) + prow, Wr, invW, yq, pxw[j]);
      fdivmod(yq, Hr, invH, pnq[j], pyh[j]);
    }
  }
  // `adv`: rows moved on by one step since the previous call (every call but the first)
  auto issue = [&](int m, int stage, bool adv) {
#pragma unroll
    for (int j = 0; j < PCS; ++j) {
      const int i = wid_u * PCS + j;                 // wave-uniform piece index
      const int slab = i >> 3, prc = i & 7;
      const int r = m + 8 * prc + prow;              // pixel row of this lane
      const unsigned dst = lds0 + stage * STG + i * 1024;
      if (slab < AS) {
        const unsigned off = (unsigned)(((int64_t)r * lda + n0 + slab * 64 + sch * 8) * 2);
        lds_dma16_buf(ra, r < mend ? off : 0x80000000u, dst);
      } else {
        const int sb = SL == 1 ? 0 : slab - AS;   // (SL = 1: a constant index, no private-memory array)
        if (INCR && adv) {
          pxw[j] += adv_x;
          const int cx = pxw[j] >= Wr;
          pxw[j] -= cx ? Wr : 0;
          pyh[j] += adv_y + cx;
          const int cy = pyh[j] >= Hr;
          pyh[j] -= cy ? Hr : 0;
          pnq[j] += adv_n + cy;
        }
        const int xw = INCR ? pxw[j] : 0, yh = INCR ? pyh[j] : 0, nq = INCR ? pnq[j] : 0;
        bool ok;
        int64_t src;
        unsigned col = (unsigned)(bcb[sb] + sch * 8);
        if constexpr (GEN == 3) {
          ok = r < mend;
          src = r;
        } else if constexpr (GEN == 2) {   // this lane's chunk is tap t: the whole 8-element source row
          const int t = min((k0 + sb * 64) / 8 + sch, geo.ntaps - 1), ty = t / geo.tdx[0], tx = t - ty * geo.tdx[0];
          ok = r < mend;
          src = ((int64_t)nq * geo.Hs + geo.sy * yh + geo.by + ty) * geo.Ws + geo.sx * xw + geo.bx + tx;
          col = 0;
        } else if constexpr (GEN) {
          const int ay = geo.sy * yh + geo.by + bdy[sb], ax = geo.sx * xw + geo.bx + bdx[sb];
          ok = r < mend && (unsigned)ay < (unsigned)geo.Hs && (unsigned)ax < (unsigned)geo.Ws;
          src = ((int64_t)nq * geo.Hs + ay) * geo.Ws + ax;
        } else {
          ok = r < mend && (unsigned)(yh + bdy[sb]) < (unsigned)H && (unsigned)(xw + bdx[sb]) < (unsigned)W;
          src = r + bdy[sb] * W + bdx[sb];
        }
        const unsigned off = (unsigned)((src * ldb + col) * 2);
        lds_dma16_buf(rb, ok ? off : 0x80000000u, dst);
      }
    }
  };

  // transposed-read offsets (ts_tn_k's layout): 32-column operand at 32-column offset c32 of a slab
  const int hh = g >> 1, tch = 2 * (g & 1) + (p >> 1), tin = 8 * (p & 1);
  auto toff = [&](int c32) { return (8 * hh + q) * TW_ROWB + (((c32 * 4 + tch) ^ tw_swz(q)) << 4) + tin; };
  int aoff[TI], boff[SL];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int co = cw * (TCO / 2) + i * 32;          // within the tile
    aoff[i] = (co >> 6) * C3W_SLAB + toff((co >> 5) & 1);
  }
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    const int kc = kw * WK + j * 32;
    boff[j] = (AS + (kc >> 6)) * C3W_SLAB + toff((kc >> 5) & 1);
  }

  f32x16 acc[TI][SL];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < SL; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nsteps = (mend - mbeg + 63) / 64;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nsteps) issue(mbeg + i * 64, i, i > 0);
  for (int st = 0; st < nsteps; ++st) {
    // this wave's pieces of step st have landed: the NS - 2 later steps issued so far may stay in flight (each wave
    // issues PCS pieces per step); near the end fewer were issued, so drain
    if (NS > 2 && st + NS - 2 < nsteps) wait_vmcnt<(NS > 2 ? (NS - 2) * PCS : 0)>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();   // ... every wave's, and nobody reads step st - 1's slot any more
    const char* base = smem + (st % NS) * STG;
    // every operand of the step is read before its MFMAs (LDS returns in order, so the first k-step's products wait
    // only for their own reads): one exposed LDS round trip per step instead of one per 16-pixel k-step
    bf16x8 af[4][TI], bfr[4][SL];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {                 // 16-pixel MFMA k-steps
      // the next DMA goes out behind k-step 0's reads: its address arithmetic overlaps their LDS round trip
      if (kk == 1 && st + NS - 1 < nsteps) issue(mbeg + (st + NS - 1) * 64, (st + NS - 1) % NS, true);
      const int ro = 16 * kk * TW_ROWB;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const bf16x4 lo = tr_read(base + aoff[i] + ro), hi = tr_read(base + aoff[i] + ro + 4 * TW_ROWB);
        af[kk][i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < SL; ++j) {
        const bf16x4 lo = tr_read(base + boff[j] + ro), hi = tr_read(base + boff[j] + ro + 4 * TW_ROWB);
        bfr[kk][j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < SL; ++j) acc[i][j] = mfma32(af[kk][i], bfr[kk][j], acc[i][j]);
    // schedule: the reads run one k-step ahead of the MFMAs -- reads(0), reads(1), MFMAs(0), reads(2), MFMAs(1), ...
    // (left alone, hipcc reuses one fragment set and issues k-step kk + 1's reads only after k-step kk's MFMAs, so
    // each k-step's first MFMA waits out an LDS round trip)
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * (TI + SL), 0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < 3) __builtin_amdgcn_sched_group_barrier(0x100, 2 * (TI + SL), 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TI * SL, 0);
    }
  }
  // register r of tile (i, j): P[n0 + cw*TCO/2 + i*32 + (r&3) + 8(r>>2) + 4h][k0 + kw*96 + j*32 + (lane & 31)]
  float* out = P + (int64_t)s * N * K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < SL; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(int64_t)(n0 + cw * (TCO / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * K + k0 + kw * WK + j * 32 +
            (lane & 31)] = acc[i][j][r];
}

// dW = sum_s P[s] (+ dW).  A workgroup = 16 float4 output columns x 16 split groups; each thread sums every
// 16th split of its float4 (independent loads in flight), then the 16 partial sums meet in LDS in a fixed order.
template <typename T, bool ACC>
__global__ __launch_bounds__(256) void ts_reduce_k(const float* __restrict__ P, T* __restrict__ out, int64_t nk,
                                                   int nsplit) {
  __shared__ f32x4 red[16][16];
  const int c = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int64_t i = ((int64_t)blockIdx.x * 16 + c) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (i < nk) {
#pragma unroll 4
    for (int j = sg; j < nsplit; j += 16) s += *reinterpret_cast<const f32x4*>(P + (int64_t)j * nk + i);
  }
  red[sg][c] = s;
  __syncthreads();
  if (sg == 0 && i < nk) {
#pragma unroll
    for (int j = 1; j < 16; ++j) s += red[j][c];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = s[e];
      if (ACC) v += (float)out[i + e];
      out[i + e] = (T)v;
    }
  }
}

}  // namespace

template <int BN, bool C3, bool ADD = false, bool STATS = false, bool PRO = false, int ADDS = 0>
static void ts_nt_launch(int nblk, hipStream_t st, const void* A, const void* B, void* C, int64_t M, int64_t N,
                         int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int H, int W, int cin, const void* D,
                         float* stats, const float* pro_ss) {
  // built for 4 workgroups per CU (128 VGPRs, no scratch): +0.5 % in-step over the compiler's budget of 3
  // (profiles/r4/ts_nt_occ/)
  hipLaunchKernelGGL((ts_nt_k<BN, C3, ADD, STATS, PRO, ADDS, 4>), dim3(nblk), dim3(TS_NT), 0, st, (const bf16*)A,
                     (const bf16*)B, (bf16*)C, (int)M, (int)N, (int)K, lda, ldb, ldc, H, W, cin, (const bf16*)D,
                     stats, pro_ss);
}

bool conv1x1_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N % 64 == 0 && K % 64 == 0 && N >= 64 && K >= 64;
}

void ts_gemm_nt(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, hipStream_t st, int H, int W, const void* D, float* stats, const float* pro_ss) {
  const int nmb = (int)cdiv(M, TS_BM);
  const bool c3 = H > 0;
  const int cin = c3 ? (int)(K / 9) : 0;
  if (pro_ss != nullptr) {   // BatchNorm-apply + ReLU prologue on A (1x1 only, K <= 2048; host-checked)
    const bool w128 = N % 128 == 0;
#define DPH_TS_PRO(BN_, ST_)                                                                                     \
    ts_nt_launch<BN_, false, false, ST_, true>(nmb * (int)(N / BN_), st, A, B, C, M, N, K, lda, ldb, ldc, 0, 0, 0,   \
                                               nullptr, stats, pro_ss)
    if (stats) {
      if (w128) DPH_TS_PRO(128, true);
      else DPH_TS_PRO(64, true);
    } else {
      if (w128) DPH_TS_PRO(128, false);
      else DPH_TS_PRO(64, false);
    }
#undef DPH_TS_PRO
    return;
  }
#define DPH_TS_NT(BN_, C3_)                                                                                     \
  ts_nt_launch<BN_, C3_>(nmb * (int)(N / BN_), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, cin, nullptr, nullptr,   \
                         nullptr)
  // 128-wide column tiles whenever N allows: 64-wide tiles double the workgroup count of the short-grid 14x14 / 7x7
  // layers but measured 1.1-1.4x slower there too (profiles/conv_nt_bn_ab.log).
  const bool wide = N % 128 == 0;
  // 3x3: the LDS-DMA implicit GEMM of conv3x3.hip where it tiles; this file's register-staged C3 path otherwise
  if (c3 && D == nullptr && conv3_supported(M, N, K, lda, ldb)) {
    conv3_gemm(A, B, C, M, N, K, lda, ldb, ldc, H, W, st, stats);   // (+ BatchNorm partials of the output)
    return;
  }
  if (!c3 && D == nullptr && gemm1_lds_preferred(M, N, K, lda, ldb)) {   // deep-K 1x1: the LDS-DMA pipeline
    convg_gemm(A, B, C, M, N, K, lda, ldb, ldc, gemm1_identity_geo(M), st, stats);   // (+ BatchNorm partials)
    return;
  }
  if (stats != nullptr && !c3) {   // BatchNorm statistics of the output (1x1 forward only)
    if (wide)
      ts_nt_launch<128, false, false, true>(nmb * (int)(N / 128), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, cin,
                                            nullptr, stats, nullptr);
    else
      ts_nt_launch<64, false, false, true>(nmb * (int)(N / 64), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, cin,
                                           nullptr, stats, nullptr);
    return;
  }
  if (D != nullptr && !c3) {   // fused residual-gradient add (1x1 only)
    if (wide)
      ts_nt_launch<128, false, true>(nmb * (int)(N / 128), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, cin, D, nullptr,
                                     nullptr);
    else
      ts_nt_launch<64, false, true>(nmb * (int)(N / 64), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, cin, D, nullptr,
                                    nullptr);
    return;
  }
  if (wide) {
    if (c3) DPH_TS_NT(128, true);
    else DPH_TS_NT(128, false);
  } else {
    if (c3) DPH_TS_NT(64, true);
    else DPH_TS_NT(64, false);
  }
#undef DPH_TS_NT
}

void ts_gemm_nt_bnred(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                      int64_t ldb, int64_t ldc, int H, int W, const void* D, int adds, const BnRed& r,
                      hipStream_t st, const uint8_t* dmask) {
  if (H > 0 && adds == 0) {   // 3x3 stride-1 input gradient on the LDS-DMA kernel
    conv3_gemm_bnred(A, B, C, M, N, K, lda, ldb, ldc, H, W, r, st);
    return;
  }
  if (H == 0 && D == nullptr && dmask == nullptr && r.part != nullptr && gemm1_lds_preferred(M, N, K, lda, ldb)) {
    conv3_gemm_bnred(A, B, C, M, N, K, lda, ldb, ldc, 0, 0, r, st);   // deep-K 1x1 on the LDS-DMA pipeline
    return;
  }
  const int nmb = (int)cdiv(M, TS_BM);
  const bool wide = N % 128 == 0;
#define DPH_TS_BR(BN_, ADD_, ADDS_, MODE_, AM_)                                                                    \
  hipLaunchKernelGGL((ts_nt_k<BN_, false, ADD_, false, false, ADDS_, 4, MODE_, AM_>), dim3(nmb * (int)(N / BN_)),   \
                     dim3(TS_NT), 0, st, (const bf16*)A, (const bf16*)B, (bf16*)C, (int)M, (int)N, (int)K, lda, ldb, \
                     ldc, H, W, 0, (const bf16*)D, nullptr, nullptr, r, dmask)
#define DPH_TS_BR_W(ADD_, ADDS_, MODE_, AM_)         \
  if (wide) DPH_TS_BR(128, ADD_, ADDS_, MODE_, AM_); \
  else DPH_TS_BR(64, ADD_, ADDS_, MODE_, AM_)
  const bool bits = r.bits != nullptr;
  if (dmask != nullptr) {   // masked residual-gradient add; r.part == nullptr: no BatchNorm reduction
    if (r.part == nullptr) { DPH_TS_BR_W(true, 0, 0, true); }
    else if (bits) { DPH_TS_BR_W(true, 0, 2, true); }
    else { DPH_TS_BR_W(true, 0, 1, true); }
  } else if (adds == 2) {
    if (bits) { DPH_TS_BR_W(true, 2, 2, false); } else { DPH_TS_BR_W(true, 2, 1, false); }
  } else if (D != nullptr) {
    if (bits) { DPH_TS_BR_W(true, 0, 2, false); } else { DPH_TS_BR_W(true, 0, 1, false); }
  } else {
    if (bits) { DPH_TS_BR_W(false, 0, 2, false); } else { DPH_TS_BR_W(false, 0, 1, false); }
  }
#undef DPH_TS_BR_W
#undef DPH_TS_BR
}

void ts_gemm_nt_add_sub(const void* A, const void* B, void* C, const void* D, int64_t M, int64_t N, int64_t K,
                        int64_t lda, int64_t ldb, int64_t ldc, int H, int W, int s, hipStream_t st) {
  const int nmb = (int)cdiv(M, TS_BM);
  if (N % 128 == 0)
    ts_nt_launch<128, false, true, false, false, 2>(nmb * (int)(N / 128), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, 0,
                                                    D, nullptr, nullptr);
  else
    ts_nt_launch<64, false, true, false, false, 2>(nmb * (int)(N / 64), st, A, B, C, M, N, K, lda, ldb, ldc, H, W, 0,
                                                   D, nullptr, nullptr);
  (void)s;
}

int ts_gemm_tn_splits(int64_t M, int64_t N, int64_t K) {
  // Pick the number of pixel chunks s by a small cost model in units of one 64-pixel step:
  //   rounds(s) * (steps per chunk + 2)  +  s * N * K / 9e5
  // rounds = ceil(tiles * s / R) resident rounds of workgroups (R = 4 per CU x 256 CUs; a 1026-workgroup grid
  // runs a second, nearly empty round -- measured 1.4x slower than 1017), +2 steps of per-workgroup prologue /
  // epilogue, and the fp32 partials written here and re-read by ts_reduce_k (~1.5 us per 8 MB at the measured
  // 1.47 us per step).  Chunks of at least 1024 rows, partial buffers of at most max(256 splits, 64 MB).
  // (Modelling R = 1024 resident workgroups measured as well as any other value: profiles/r4/rejected_ts_tn_wgs/.)
  constexpr int R = 256 * 4;
  const int64_t tiles = (N / 64) * (K / 64);
  const int64_t smax = std::max<int64_t>(1, std::min<int64_t>(M / 1024,
                                                              std::max<int64_t>(256, (int64_t(64) << 20) / (N * K * 4))));
  int64_t best_s = 1;
  double best = 1e300;
  for (int64_t s = 1; s <= smax; ++s) {
    const int64_t steps = cdiv(cdiv(M, s), 64);
    const int64_t rounds = cdiv(tiles * s, (int64_t)R);
    const double cost = (double)rounds * (double)(steps + 2) + (double)s * (double)(N * K) / 9e5;
    if (cost < best) {
      best = cost;
      best_s = s;
    }
  }
  return (int)best_s;
}

bool c3w_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  // 32-bit buffer offsets below the 0x80000000 "padding" sentinel; fp32 row division exact below 2^24 pixels
  return N % 64 == 0 && K % C3W_TK == 0 && M * lda * 2 < (int64_t(1) << 31) &&
         M * ldb * 2 < (int64_t(1) << 31) && M < (int64_t(1) << 24);
}

static int64_t c3w_tiles(int64_t N, int64_t K, int64_t tk) { return (N / (N % 128 == 0 ? 128 : 64)) * (K / tk); }

// LDS ring depth of c3w_k: 2 stages, two workgroups per CU (3-5 stages = one workgroup per CU measured slower,
// profiles/r4/c3w_ring/).
static int w1_stages() { return 2; }
static int c3w_stages() { return 2; }

template <int TCO, int GEN, int SL, int NS>
static void c3w_go(unsigned nblk, hipStream_t st, const void* A, const void* B, float* P, int64_t M, int64_t N,
                   int64_t K, int64_t lda, int64_t ldb, int64_t chunk, int H, int W, int cin, const ConvGeo& g) {
  hipLaunchKernelGGL((c3w_k<TCO, GEN, SL, NS>), dim3(nblk), dim3(256), 0, st, (const bf16*)A, (const bf16*)B, P,
                     (int)M, (int)N, (int)K, lda, ldb, (int)chunk, H, W, cin, g);
}
// c3w_k with `ns` ring stages, capped at the deepest ring that fits 160 KiB
template <int TCO, int GEN, int SL>
static void c3w_launch(int ns, unsigned nblk, hipStream_t st, const void* A, const void* B, float* P, int64_t M,
                       int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t chunk, int H, int W, int cin,
                       const ConvGeo& g) {
  (void)ns;
  c3w_go<TCO, GEN, SL, 2>(nblk, st, A, B, P, M, N, K, lda, ldb, chunk, H, W, cin, g);
}
// resident workgroups per round: 2 per CU with the two-stage ring, 1 with a deeper one
static int64_t g_c3w_round = 512;   // workgroup slots of one round with the two-stage ring (c3w_round_set)
static int64_t c3w_round(int ns) { return ns > 2 ? g_c3w_round / 2 : g_c3w_round; }
int64_t c3w_round_set(int64_t slots) {
  const int64_t prev = g_c3w_round;
  if (slots > 0) g_c3w_round = slots;
  return prev;
}
// pixel-chunk splits: as many as fill ONE resident round (floor -- rounding up, e.g. 22 x 24 tiles = 528 workgroups
// for 512 slots, started a second round that cost a whole workgroup's time for 16 workgroups), chunks >= 512 rows
static int64_t c3w_split_count(int64_t M, int64_t tiles, int ns) {
  const int64_t s = std::max<int64_t>(1, c3w_round(ns) / tiles);
  return std::max<int64_t>(1, std::min<int64_t>(s, M / 512));
}

// 1x1 weight gradient on the LDS-DMA kernel (c3w_k with one tap, identity rows): k' tiles of 128 (64 when K % 128)
static int w1_tk(int64_t K) { return K % 128 == 0 ? 128 : 64; }

bool w1_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  // default since the identity-row form (GEN 3, no per-piece divisions): 1.94-2.06 ms per ResNet-50 step over its
  // twelve 1x1 shapes vs 2.50 for the register-staged ts_tn_k and 3.26 for MIOpen (profiles/r4/c3w_incr/,
  // profiles/r4/c3w_ring/identity_rows/).  The BatchNorm-prologue form stays on ts_tn_k.
  return N % 64 == 0 && K % 64 == 0 && M * lda * 2 < (int64_t(1) << 31) && M * ldb * 2 < (int64_t(1) << 31) &&
         M < (int64_t(1) << 24);
}

int w1_splits(int64_t M, int64_t N, int64_t K) {
  return (int)c3w_split_count(M, c3w_tiles(N, K, w1_tk(K)), w1_stages());
}

int c3w_splits(int64_t M, int64_t N, int64_t K) {
  return (int)c3w_split_count(M, c3w_tiles(N, K, C3W_TK), c3w_stages());
}

static void ts_reduce(const float* partial, void* C, int64_t nk, int nsplit, int out_dtype, bool accumulate,
                      hipStream_t st) {
  const dim3 grid((int)cdiv(nk / 4, 16));
  if (out_dtype == kBF16) {
    if (accumulate) hipLaunchKernelGGL((ts_reduce_k<bf16, true>), grid, dim3(256), 0, st, partial, (bf16*)C, nk, nsplit);
    else hipLaunchKernelGGL((ts_reduce_k<bf16, false>), grid, dim3(256), 0, st, partial, (bf16*)C, nk, nsplit);
  } else {
    if (accumulate) hipLaunchKernelGGL((ts_reduce_k<float, true>), grid, dim3(256), 0, st, partial, (float*)C, nk, nsplit);
    else hipLaunchKernelGGL((ts_reduce_k<float, false>), grid, dim3(256), 0, st, partial, (float*)C, nk, nsplit);
  }
}

void ts_gemm_tn(const void* A, const void* B, float* partial, void* C, int64_t M, int64_t N, int64_t K,
                int64_t lda, int64_t ldb, int nsplit, int out_dtype, bool accumulate, hipStream_t st, int H, int W,
                const float* pro_ss) {
  const int64_t tiles = (N / 64) * (K / 64);
  int64_t chunk = cdiv(M, nsplit);
  chunk = cdiv(chunk, 64) * 64;
  if (H == 0 && pro_ss == nullptr && w1_supported(M, N, K, lda, ldb)) {   // LDS-DMA 1x1 (nsplit from w1_splits)
    ConvGeo g{};
    g.Hs = g.Ho = g.Hd = 1;
    g.Ws = g.Wo = g.Wd = (int)M;
    g.sy = g.sx = g.ty = g.tx = 1;
    g.ntaps = 1;
    g.src_rows = M;
    const int tk = w1_tk(K);
    const unsigned nblk = (unsigned)((N / (N % 128 == 0 ? 128 : 64)) * (K / tk) * nsplit);
    const int ns = w1_stages();
    if (N % 128 == 0) {
      if (tk == 128) c3w_launch<128, 3, 2>(ns, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
      else c3w_launch<128, 3, 1>(ns, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
    } else {
      if (tk == 128) c3w_launch<64, 3, 2>(ns, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
      else c3w_launch<64, 3, 1>(ns, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
    }
  } else if (H > 0 && c3w_supported(M, N, K, lda, ldb)) {   // the LDS-DMA 3x3 kernel (nsplit from c3w_splits)
    const int cin = (int)(K / 9);
    const int ns = c3w_stages();
    if (N % 128 == 0)
      c3w_launch<128, 0, C3W_SLABS>(ns, (unsigned)((N / 128) * (K / C3W_TK) * nsplit), st, A, B, partial, M, N, K, lda,
                                    ldb, chunk, H, W, cin, ConvGeo{});
    else
      c3w_launch<64, 0, C3W_SLABS>(ns, (unsigned)((N / 64) * (K / C3W_TK) * nsplit), st, A, B, partial, M, N, K, lda,
                                   ldb, chunk, H, W, cin, ConvGeo{});
  } else if (pro_ss != nullptr && H == 0) {
    hipLaunchKernelGGL((ts_tn_k<false, true>), dim3((int)(tiles * nsplit)), dim3(256), 0, st, (const bf16*)A,
                       (const bf16*)B, partial, (int)M, (int)N, (int)K, lda, ldb, (int)chunk, 0, 0, 0, pro_ss);
  } else if (H > 0)
    hipLaunchKernelGGL((ts_tn_k<true>), dim3((int)(tiles * nsplit)), dim3(256), 0, st, (const bf16*)A,
                       (const bf16*)B, partial, (int)M, (int)N, (int)K, lda, ldb, (int)chunk, H, W, (int)(K / 9));
  else
    hipLaunchKernelGGL((ts_tn_k<false>), dim3((int)(tiles * nsplit)), dim3(256), 0, st, (const bf16*)A,
                       (const bf16*)B, partial, (int)M, (int)N, (int)K, lda, ldb, (int)chunk, 0, 0, 0);
  ts_reduce(partial, C, N * K, nsplit, out_dtype, accumulate, st);
}

bool c3wg_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const ConvGeo& g, bool chunk_taps) {
  if (chunk_taps)   // 128-wide k' tiles of 16 chunk taps each
    return N % 64 == 0 && K % 128 == 0 && ldb == 8 && g.ntaps >= 1 && g.ntaps <= K / 8 && g.tdx[0] > 0 &&
           M * lda * 2 < (int64_t(1) << 31) && g.src_rows * ldb * 2 < (int64_t(1) << 31) && M < (int64_t(1) << 24);
  if (g.ntaps == 1)   // a strided 1x1: the 1x1 tiles (64 / 128-wide k', no tap) over the gathered rows
    return N % 64 == 0 && K % 64 == 0 && M * lda * 2 < (int64_t(1) << 31) &&
           g.src_rows * ldb * 2 < (int64_t(1) << 31) && M < (int64_t(1) << 24);
  // c3w_k tiles: 192 k' (three 64-channel slabs of one tap each); fp32 row division exact below 2^24 rows
  return g.ntaps >= 1 && g.ntaps <= 9 && N % 64 == 0 && K % C3W_TK == 0 && K % g.ntaps == 0 &&
         (K / g.ntaps) % 64 == 0 && M * lda * 2 < (int64_t(1) << 31) && g.src_rows * ldb * 2 < (int64_t(1) << 31) &&
         M < (int64_t(1) << 24);
}

int c3wg_splits(int64_t M, int64_t N, int64_t K, bool chunk_taps, bool one_tap) {
  if (one_tap && !chunk_taps) return w1_splits(M, N, K);
  if (!chunk_taps) return c3w_splits(M, N, K);
  return (int)c3w_split_count(M, c3w_tiles(N, K, 128), c3w_stages());
}

void ts_gemm_tn_geo(const void* A, const void* B, float* partial, void* C, int64_t M, int64_t N, int64_t K,
                    int64_t lda, int64_t ldb, int nsplit, int out_dtype, bool accumulate, const ConvGeo& g,
                    hipStream_t st, bool chunk_taps) {
  int64_t chunk = cdiv(cdiv(M, nsplit), 64) * 64;
  const int ns = c3w_stages();
  if (chunk_taps) {   // the RGB stem's weight gradient: 64 output channels x 128-wide k' tiles
    if (N % 128 == 0)
      c3w_launch<128, 2, 2>(ns, (unsigned)((N / 128) * (K / 128) * nsplit), st, A, B, partial, M, N, K, lda, ldb,
                            chunk, 0, 0, 8, g);
    else
      c3w_launch<64, 2, 2>(ns, (unsigned)((N / 64) * (K / 128) * nsplit), st, A, B, partial, M, N, K, lda, ldb,
                           chunk, 0, 0, 8, g);
    ts_reduce(partial, C, N * K, nsplit, out_dtype, accumulate, st);
    return;
  }
  if (g.ntaps == 1) {   // strided 1x1: the 1x1 weight-gradient tiles over the gathered X rows (no slice copy)
    const int tk = w1_tk(K), ns1 = w1_stages();
    const unsigned nblk = (unsigned)((N / (N % 128 == 0 ? 128 : 64)) * (K / tk) * nsplit);
    if (N % 128 == 0) {
      if (tk == 128) c3w_launch<128, 1, 2>(ns1, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
      else c3w_launch<128, 1, 1>(ns1, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
    } else {
      if (tk == 128) c3w_launch<64, 1, 2>(ns1, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
      else c3w_launch<64, 1, 1>(ns1, nblk, st, A, B, partial, M, N, K, lda, ldb, chunk, 0, 0, (int)K, g);
    }
    ts_reduce(partial, C, N * K, nsplit, out_dtype, accumulate, st);
    return;
  }
  const int cin = (int)(K / g.ntaps);
  if (N % 128 == 0)
    c3w_launch<128, 1, C3W_SLABS>(ns, (unsigned)((N / 128) * (K / C3W_TK) * nsplit), st, A, B, partial, M, N, K, lda,
                                  ldb, chunk, 0, 0, cin, g);
  else
    c3w_launch<64, 1, C3W_SLABS>(ns, (unsigned)((N / 64) * (K / C3W_TK) * nsplit), st, A, B, partial, M, N, K, lda,
                                 ldb, chunk, 0, 0, cin, g);
  ts_reduce(partial, C, N * K, nsplit, out_dtype, accumulate, st);
}

}  // namespace dph
