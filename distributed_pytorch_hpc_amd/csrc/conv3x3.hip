// 3x3 / stride 1 / padding 1 convolution on channels-last activations as an implicit GEMM with an LDS-DMA pipeline,
// for CDNA4 (gfx950): the ResNet-50 bottleneck conv2 (scripts/main.py:249 builds torchvision resnet50) and, through
// ops/conv.py, any stride-1 3x3 convolution whose channel counts are multiples of 64.
//
//   C[M, N] = sum_k A_g[M, K] B[N, K]^T,   M = N_img*H*W pixels, K = 9 * Cin tap-major (k = tap * Cin + c),
//   A_g[m, tap * Cin + c] = X[m + dy * W + dx, c]  (dy, dx) = (tap / 3 - 1, tap % 3 - 1), zero outside the image.
//
// Forward: X = input, B = weight [Cout, (kh, kw, Cin)].  Input gradient: X = dY, B = the flipped, channel-transposed
// weight [Cin, (kh, kw, Cout)] (ops/conv.py) -- the same kernel.
//
// Structure (replaces the register-staged ts_nt_k<.., C3> path of conv1x1.hip, which tops out near 0.5 PFLOP/s with
// one K-step in flight and A straight from L2 into registers):
//   * 64 WM x BN output tile per workgroup (BN = 64 | 128; WM = 2: 4 waves, two workgroups per CU; WM = 4: 8 waves,
//     one workgroup per CU), waves as WM (M) x 2 (N), wave tile 64 x BN/2, v_mfma_f32_32x32x16_bf16 with the pixel
//     rows as the A operand;
//   * K-steps of 64 channels of one tap; both operands staged global -> LDS by LDS-DMA (16 B per lane, one 1-KiB
//     piece = 8 rows of 128 B per wave-instruction) into a STAGES-deep ring of XOR-swizzled images
//     (slot = chunk ^ ((row >> 1) & 7): conflict-free ds_read_b128 fragment reads); the A gather is just the per-lane
//     DMA source address (the row shifted by the tap), and rows whose tap falls outside the image (or past M) are
//     zero-filled by the DMA itself -- a range-checked buffer load with an out-of-range offset -- so neither a padded
//     copy of the input nor any register masking exists;
//   * one raw s_barrier per K-step, counted vmcnt: STAGES - 1 K-steps stay in flight behind the MFMAs;
//   * C tile through LDS, written as whole 16-B row segments; workgroups remapped XCD-aware with the N-tiles of one
//     row block adjacent (they read the same shifted input rows from one L2); epilogues: + bias, BN statistics.
#include "bn_epilogue.h"
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int C3_BK = 64;
constexpr int kConv3DefaultWm = 2;   // 4-wave tile (the 8-wave WM = 4 tile measured slower)
constexpr int C3_ROWB = 128;   // LDS image row: 64 bf16

__device__ __forceinline__ f32x16 c3_mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-B chunk c of image row r
__device__ __forceinline__ int c3_off(int r, int c) { return r * C3_ROWB + ((c ^ ((r >> 1) & 7)) << 4); }

// STATS: also the per-128-row-block BatchNorm partials of the bf16 output (the layout of conv1x1.hip's ts_nt_k
// STATS epilogue: stats[mb * N + n] = mean, stats[nmb * N + mb * N + n] = M2, stats[2 * nmb * N + mb] = rows, with
// 128-row blocks mb whatever the tile height), so the BatchNorm after the 3x3 convolution skips its statistics pass.
// WM: waves along M (2 waves along N): WM = 2 is a 128-row tile of 4 waves (two workgroups per CU), WM = 4 a 256-row
// tile of 8 waves (one workgroup per CU, 3-stage ring, the weight slab shared by twice the rows).
// Padding taps and rows past M are zero-filled by the DMA itself (buffer_load ... lds with an out-of-range offset);
// round 3 measured that 1.0-1.2x faster than fetching the row and zeroing the fragment registers.
// GEN: the gathered geometry of kernels.h ConvGeo (strided forward, the parity classes of a strided input gradient):
// per-lane source pixels from g, the K-step's tap offsets from g's tap table, rows stored to g's destination rows.
// GEN = 2 (chunk taps, the 7x7 RGB stem): every 16-B chunk of a K-step is its own tap -- K-step ks, chunk c is tap
// t = 8 ks + c of g.ntaps, source row (base + (t / g.tdx[0]) Ws + t % g.tdx[0]) of an [src_rows, 8] operand (pairs of
// 4-channel pixels of a zero-padded image, so no bounds checks); taps past ntaps read tap ntaps - 1 (zero weights).
// GEN = 0 is the stride-1 3x3 path (H, W, the fixed 3x3 taps, identity stores).
// BRED = 1 | 2 (GEN = 0, WM = 2: one partial row per 128-row tile): the input gradient of a BatchNorm + ReLU output
// also emits the BatchNorm backward's reduction partials (kernels.h BnRed, bn_epilogue.h).
template <int BN, int STAGES, int WM, bool STATS = false, int GEN = 0, int BRED = 0>
__global__ __launch_bounds__(128 * WM, WM == 2 ? 2 : 1) void conv3_k(const bf16* __restrict__ X,
                                                                   const bf16* __restrict__ B, bf16* __restrict__ C,
                                                                   int M, int N, int K, int64_t ldx, int64_t ldb,
                                                                   int64_t ldc, int H, int W, int Cin,
                                                                   float* __restrict__ stats,
                                                                   const void* __restrict__ bias, ConvGeo g,
                                                                   bool bias_bf16, BnRed bnr) {
  // (GEN = 1 only with an identity destination map -- the one-tap plain GEMM of gemm1_identity_geo -- since the
  // BatchNorm operands are fetched at the source row before the K-loop)
  static_assert(!BRED || (GEN != 2 && WM == 2 && !STATS), "BRED: 128-row tiles, no statistics");
  constexpr int NWV = 2 * WM, NTH = 64 * NWV, BM = 64 * WM;
  constexpr int AIMG = BM * C3_ROWB, BIMG = BN * C3_ROWB, STG = AIMG + BIMG;
  constexpr int AI = BM / 8 / NWV;         // A DMA pieces (8 rows) per wave per K-step (4)
  constexpr int BI = BN / 8 / NWV;         // B DMA pieces per wave per K-step (1, 2 or 4)
  static_assert(AI >= 1 && BI >= 1, "DMA pieces");
  constexpr int PER = AI + BI;             // DMA instructions per thread per K-step
  constexpr int WN = BN / 2, NTW = WN / 32;   // wave tile columns, 32-column MFMA tiles per wave
  constexpr int CROW = BN + 8;             // epilogue LDS row (bf16)
  constexpr int LDS_C = BM * CROW * 2 + (STATS ? 2 * WM * BN * 4 : 0);
  constexpr int LDS = STAGES * STG > LDS_C ? STAGES * STG : LDS_C;
  __shared__ __attribute__((aligned(1024))) char smem[LDS];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l32 = lane & 31, h = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = N / BN, nmb = (M + BM - 1) / BM;
  const int lin = xcd_remap(blockIdx.x, nmb * ntn);
  const int mb = lin / ntn, n0 = (lin % ntn) * BN;
  const int m0 = mb * BM;

  // ---- DMA lanes: piece q = wid * AI + j covers image rows 8 q + lane / 8, LDS slot lane % 8.  Image row 8 q + prow
  // has (row >> 1) & 7 = (4 q + (prow >> 1)) & 7: the lane's source chunk depends on the parity of q ----
  const int prow = lane >> 3, pslot = lane & 7;
  const int chunk0 = pslot ^ ((prow >> 1) & 7), chunk1 = pslot ^ (((prow >> 1) + 4) & 7);
  int ay[AI], ax[AI], am[AI], ach[AI];
  bool arow_in[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int q = wid * AI + j, r = q * 8 + prow;
    const int m = min(m0 + r, M - 1);
    arow_in[j] = m0 + r < M;
    if constexpr (GEN) {   // output row (n, oy, ox) -> its source base pixel (sy oy + by, sx ox + bx) of image n
      const int hw = g.Ho * g.Wo, n = m / hw, rem = m - n * hw, oy = rem / g.Wo, ox = rem - oy * g.Wo;
      ay[j] = g.sy * oy + g.by;
      ax[j] = g.sx * ox + g.bx;
      am[j] = (n * g.Hs + ay[j]) * g.Ws + ax[j];
    } else {
      am[j] = m;
      ax[j] = m % W;
      ay[j] = (m / W) % H;
    }
    ach[j] = (q & 1) ? chunk1 : chunk0;
  }
  unsigned boff[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int q = wid * BI + j, r = q * 8 + prow;
    boff[j] = (unsigned)(((int64_t)(n0 + r) * ldb + ((q & 1) ? chunk1 : chunk0) * 8) * 2);
  }
  const unsigned lds0 = lds_addr(smem);
  const dph_rsrc xres = make_rsrc(X, (unsigned)((GEN ? g.src_rows : (int64_t)M) * ldx * 2));
  const int Hs = GEN ? g.Hs : H, Ws = GEN ? g.Ws : W;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);   // the DMA destination (M0) must be provably wave-uniform

  auto issue = [&](int ks, int stage) {
    const int k0 = ks * C3_BK;
    const int tap = k0 / Cin, cb = k0 - tap * Cin;
    int dy, dx;
    if constexpr (GEN) {   // wave-uniform table lookup by selects (no dynamically indexed kernel-argument array)
      dy = g.tdy[0];
      dx = g.tdx[0];
#pragma unroll
      for (int t = 1; t < 9; ++t)
        if (tap == t) {
          dy = g.tdy[t];
          dx = g.tdx[t];
        }
    } else {
      dy = tap / 3 - 1;
      dx = tap - (tap / 3) * 3 - 1;
    }
    const unsigned sa = lds0 + stage * STG + wid_u * AI * 1024;
    if constexpr (GEN == 2) {
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int t = min(ks * 8 + ach[j], g.ntaps - 1), ty = t / g.tdx[0], tx = t - ty * g.tdx[0];
        const unsigned off = (unsigned)((int64_t)(am[j] + ty * Ws + tx) * ldx * 2);
        lds_dma16_buf(xres, arow_in[j] ? off : 0x80000000u, sa + j * 1024);
      }
    } else {
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const bool ok = arow_in[j] && (unsigned)(ay[j] + dy) < (unsigned)Hs && (unsigned)(ax[j] + dx) < (unsigned)Ws;
        const unsigned off = (unsigned)(((int64_t)(am[j] + dy * Ws + dx) * ldx + cb + ach[j] * 8) * 2);
        lds_dma16_buf(xres, ok ? off : 0x80000000u, sa + j * 1024);
      }
    }
    const unsigned sb = lds0 + stage * STG + AIMG + wid_u * BI * 1024;
#pragma unroll
    for (int j = 0; j < BI; ++j) lds_dma16(B, boff[j] + (unsigned)(k0 * 2), sb + j * 1024);
  };

  // ---- fragment readers: A rows wm*64 + i*32 + l32 (i < 2), B rows wn*WN + j*32 + l32 ----
  int aoff[2][4], bofs[NTW][4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i][f] = c3_off(wm * 64 + i * 32 + l32, 2 * f + h);
#pragma unroll
    for (int j = 0; j < NTW; ++j) bofs[j][f] = AIMG + c3_off(wn * WN + j * 32 + l32, 2 * f + h);
  }

  f32x16 acc[2][NTW];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // BRED: the BatchNorm input / mask bits at the tile's output positions are loaded into registers before the K-loop
  // (their values do not depend on it), so the epilogue never waits on HBM for them -- fetched at the epilogue instead,
  // one exposed load latency per tile cost the 56 x 56 layers ~2x the bytes' share (benchmarks/probes/bn_epi_probe.py)
  constexpr int CPR = BN / 8;
  constexpr int NIT = BM * CPR / NTH;   // store iterations per thread (its chunk column is fixed)
  constexpr int PF = BRED != 0 ? NIT : 1;
  using BRA = BnRedAcc<BRED ? BRED : 1>;
  [[maybe_unused]] bf16x8 xq[PF];
  [[maybe_unused]] unsigned mq[PF];
  if constexpr (BRED != 0) {
#pragma unroll
    for (int it = 0; it < PF; ++it) {
      const int i = threadIdx.x + it * NTH, ch = i % CPR;
      const int64_t r = min(m0 + i / CPR, M - 1);
      xq[it] = BRA::load_x(bnr, r, N, n0 + ch * 8);
      mq[it] = BRA::load_m(bnr, r, N, n0 + ch * 8);
    }
  }

  const int nks = K / C3_BK;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nks) issue(s, s);

  for (int ks = 0; ks < nks; ++ks) {
    // K-step ks landed (the later STAGES-2 steps may stay in flight), then every wave's pieces of it
    if (ks + STAGES - 2 < nks) wait_vmcnt<(STAGES - 2) * PER>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    // the stage refilled now was read in step ks - 1, which every wave finished before the barrier
    if (ks + STAGES - 1 < nks) issue(ks + STAGES - 1, (ks + STAGES - 1) % STAGES);
    const char* st = smem + (ks % STAGES) * STG;
    // all fragments of the K-step are read first (one LDS round trip per K-step, consumed in issue order by
    // counted lgkmcnt waits), then the 8 * NTW MFMAs
    bf16x8 a[4][2], b[4][NTW];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
#pragma unroll
      for (int i = 0; i < 2; ++i) a[f][i] = *reinterpret_cast<const bf16x8*>(st + aoff[i][f]);
#pragma unroll
      for (int j = 0; j < NTW; ++j) b[f][j] = *reinterpret_cast<const bf16x8*>(st + bofs[j][f]);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j] = c3_mfma(a[f][i], b[f][j], acc[i][j]);
  }
  __syncthreads();
  if (bias != nullptr) {   // per-output-channel bias (fp32 or bf16) on the accumulators: C and its statistics include it
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int bc = n0 + wn * WN + j * 32 + l32;
      const float bj = bias_bf16 ? (float)reinterpret_cast<const bf16*>(bias)[bc] : reinterpret_cast<const float*>(bias)[bc];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] += bj;
    }
  }

  // ---- epilogue through LDS: register r of tile (i, j) = C[wm*64 + i*32 + (r&3) + 8(r>>2) + 4h][wn*WN + j*32 + l32]
  bf16* Cs = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        Cs[(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * CROW + wn * WN + j * 32 + l32] = (bf16)acc[i][j][r];
  __syncthreads();
  [[maybe_unused]] BRA bra;
  if constexpr (BRED != 0) bra.init(bnr, n0 + (threadIdx.x % CPR) * 8, N);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = threadIdx.x + it * NTH, row = i / CPR, ch = i % CPR, sl = it % PF;
    [[maybe_unused]] const bf16x8 xv = xq[sl];
    [[maybe_unused]] const unsigned mv = mq[sl];
    if (m0 + row < M) {
      int64_t drow = m0 + row;
      if constexpr (GEN) {
        const int m = m0 + row, hw = g.Ho * g.Wo, n = m / hw, rem = m - n * hw, oy = rem / g.Wo, ox = rem - oy * g.Wo;
        drow = ((int64_t)n * g.Hd + g.ty * oy + g.tby) * g.Wd + g.tx * ox + g.tbx;
      }
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + row * CROW + ch * 8);
      *reinterpret_cast<bf16x8*>(C + drow * ldc + n0 + ch * 8) = v;
      if constexpr (BRED != 0) bra.add(xv, mv, v);
    }
  }
  if constexpr (BRED != 0) {
    __syncthreads();   // every C-tile read is done: the tile's LDS holds the cross-wave partials
    bra.finish(reinterpret_cast<float*>(smem), CPR, NWV, mb, N, n0, bnr.part);
  }
  if constexpr (STATS) {
    // per 128-row block g (waves 2g, 2g+1): pass 1 column sums, pass 2 squared deviations from the block mean, of the
    // bf16-rounded outputs; lane halves meet by a cross-half shuffle, the waves in [WM][BN] LDS blocks behind the tile
    constexpr int G = WM / 2;
    float* ssum = reinterpret_cast<float*>(smem + BM * CROW * 2);
    float* sm2 = ssum + WM * BN;
    const int nmb128 = (M + 127) / 128;
    const int g = wm >> 1;
    const int valid = max(0, min(128, M - m0 - 128 * g));
    const float inv_n = valid > 0 ? 1.f / (float)valid : 0.f;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm & 1) * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;   // within the 128-row block
          sm += row < valid ? (float)(bf16)acc[i][j][r] : 0.f;
        }
      sm += __shfl_xor(sm, 32);
      if (h == 0) ssum[wm * BN + wn * WN + j * 32 + l32] = sm;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int col = wn * WN + j * 32 + l32;
      const float mean = (ssum[2 * g * BN + col] + ssum[(2 * g + 1) * BN + col]) * inv_n;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm & 1) * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float d = (float)(bf16)acc[i][j][r] - mean;
          m2 += row < valid ? d * d : 0.f;
        }
      m2 += __shfl_xor(m2, 32);
      if (h == 0) sm2[wm * BN + col] = m2;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G * BN; i += NTH) {
      const int gg = i / BN, col = i % BN;
      const int blk = mb * G + gg;
      const int vg = min(128, M - m0 - 128 * gg);
      if (vg <= 0 || blk >= nmb128) continue;
      stats[(int64_t)blk * N + n0 + col] = (ssum[2 * gg * BN + col] + ssum[(2 * gg + 1) * BN + col]) / (float)vg;
      stats[(int64_t)nmb128 * N + (int64_t)blk * N + n0 + col] = sm2[2 * gg * BN + col] + sm2[(2 * gg + 1) * BN + col];
      if (col == 0 && n0 == 0) stats[2 * (int64_t)nmb128 * N + blk] = (float)vg;
    }
  }
}

}  // namespace

bool conv3_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  // 32-bit DMA source offsets: the whole input and weight must lie within 4 GiB of their bases
  // (and below the 0x80000000 offset the range-checked DMA uses for padding rows)
  return M > 0 && N % 64 == 0 && K % (9 * 64) == 0 && M * lda * 2 < (int64_t(1) << 31) &&
         N * ldb * 2 < (int64_t(1) << 31);
}

void conv3_gemm(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, int H, int W, hipStream_t st, float* stats, const void* bias, bool bias_bf16) {
  const int cin = (int)(K / 9);
  // 256-row tiles of 8 waves when that still gives >= 1 workgroup per CU
  const int64_t t256 = cdiv(M, 256) * (N / (N % 128 == 0 ? 128 : 64));
  const int wm = t256 >= 256 ? kConv3DefaultWm : 2;
  const int nmb = (int)cdiv(M, 64 * wm);
  // 128-wide tiles unless that leaves fewer than ~1.5 workgroups per CU (SimpleUNet's 22 x 45 bottleneck at B=4:
  // 124 tiles of 128 vs 248 of 64)
  const bool wide = N % 128 == 0 && (int64_t)nmb * (N / 128) * (wm == 4 ? 2 : 1) >= 384;
#define DPH_C3(BN_, ST_, WM_, STATS_)                                                                            \
  hipLaunchKernelGGL((conv3_k<BN_, ST_, WM_, STATS_>), dim3(nmb * (int)(N / BN_)), dim3(128 * WM_), 0, st,    \
                     (const bf16*)A, (const bf16*)B, (bf16*)C, (int)M, (int)N, (int)K, lda, ldb, ldc, H, W, cin,  \
                     stats, bias, ConvGeo{}, bias_bf16, BnRed{})
  if (wm == 4) {
    if (stats) {
      if (wide) DPH_C3(128, 3, 4, true);
      else DPH_C3(64, 3, 4, true);
    } else {
      if (wide) DPH_C3(128, 3, 4, false);
      else DPH_C3(64, 3, 4, false);
    }
  } else if (stats) {
    if (wide) DPH_C3(128, 2, 2, true);
    else DPH_C3(64, 3, 2, true);
  } else {
    if (wide) DPH_C3(128, 2, 2, false);
    else DPH_C3(64, 3, 2, false);
  }
#undef DPH_C3
}

void conv3_gemm_bnred(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                      int64_t ldb, int64_t ldc, int H, int W, const BnRed& r, hipStream_t st) {
  // conv3_gemm's tile choice at WM = 2 (its only one for these shapes): 128-row tiles = the partial rows.
  // H = 0: the plain GEMM C = A B^T on the same kernel (one tap, identity geometry: gemm1_identity_geo).
  const bool plain = H == 0;
  const ConvGeo g = plain ? gemm1_identity_geo(M) : ConvGeo{};
  const int cin = plain ? (int)K : (int)(K / 9);
  const int nmb = (int)cdiv(M, 128);
  const bool wide = N % 128 == 0 && (int64_t)nmb * (N / 128) >= 384;
#define DPH_C3B(BN_, ST_, GEN_, MODE_)                                                                           \
  hipLaunchKernelGGL((conv3_k<BN_, ST_, 2, false, GEN_, MODE_>), dim3(nmb * (int)(N / BN_)), dim3(256), 0, st,  \
                     (const bf16*)A, (const bf16*)B, (bf16*)C, (int)M, (int)N, (int)K, lda, ldb, ldc, H, W, cin,  \
                     nullptr, nullptr, g, false, r)
#define DPH_C3B_W(GEN_, MODE_)             \
  if (wide) DPH_C3B(128, 2, GEN_, MODE_); \
  else DPH_C3B(64, 3, GEN_, MODE_)
  if (plain) {
    if (r.bits != nullptr) { DPH_C3B_W(1, 2); } else { DPH_C3B_W(1, 1); }
  } else {
    if (r.bits != nullptr) { DPH_C3B_W(0, 2); } else { DPH_C3B_W(0, 1); }
  }
#undef DPH_C3B_W
#undef DPH_C3B
}

// off (ops/_lib.py applies DPH_GEMM1_LDS=0 through the gemm1_lds op): every 1x1 GEMM stays on ts_nt_k (A/B)
bool g_gemm1_lds = true;

bool gemm1_lds_set(bool on) {
  const bool old = g_gemm1_lds;
  g_gemm1_lds = on;
  return old;
}

ConvGeo gemm1_identity_geo(int64_t M) {
  // M images of 1 x 1 pixel, one tap at (0, 0), stored to the same row: the implicit GEMM degenerates to C = A B^T
  ConvGeo g{};
  g.Hs = g.Ws = g.Ho = g.Wo = g.Hd = g.Wd = 1;
  g.sy = g.sx = g.ty = g.tx = 1;
  g.ntaps = 1;
  g.src_rows = M;
  return g;
}

bool gemm1_lds_preferred(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  // ResNet-50's deep 1x1 convolutions (K >= 1024: layers 3-4) on small grids: the LDS-DMA pipeline hides the operand
  // latency that bounds ts_nt_k there (fwd + stats 10-26 % faster, input gradient 20-27 %; K <= 512 ties or loses,
  // profiles/r6/conv1x1_probe/probe.log)
  return g_gemm1_lds && K >= 1024 && M > 0 && M < (int64_t(1) << 31) &&
         convg_supported(M, N, K, lda, ldb, gemm1_identity_geo(M));
}

bool convg_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const ConvGeo& g, bool chunk_taps) {
  if (chunk_taps)   // 8-element rows, one tap per 16-B chunk, K = whole 64-element steps covering ntaps chunks
    return M > 0 && N % 64 == 0 && lda == 8 && K % 64 == 0 && g.ntaps >= 1 && g.ntaps <= K / 8 && g.tdx[0] > 0 &&
           g.src_rows * lda * 2 < (int64_t(1) << 31) && N * ldb * 2 < (int64_t(1) << 31) && M < (int64_t(1) << 31);
  // whole 64-channel K-steps of one tap; 32-bit DMA offsets below the padding sentinel; int row arithmetic
  return M > 0 && g.ntaps >= 1 && g.ntaps <= 9 && N % 64 == 0 && K % g.ntaps == 0 && (K / g.ntaps) % 64 == 0 &&
         g.src_rows * lda * 2 < (int64_t(1) << 31) && N * ldb * 2 < (int64_t(1) << 31) && M < (int64_t(1) << 31) &&
         (int64_t)g.Hd * g.Wd * (M / ((int64_t)g.Ho * g.Wo) + 1) < (int64_t(1) << 31);
}

void convg_gemm(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                int64_t ldc, const ConvGeo& g, hipStream_t st, float* stats, bool chunk_taps, const void* bias,
                bool bias_bf16) {
  const int cin = chunk_taps ? 8 : (int)(K / g.ntaps);
  // the stride-1 kernel's tile choice: 128-row tiles of 4 waves, 128 columns unless that leaves < 1.5 WG per CU
  const int nmb = (int)cdiv(M, 128);
  const bool wide = N % 128 == 0 && (int64_t)nmb * (N / 128) >= 384;
#define DPH_CG(BN_, ST_, STATS_, G_)                                                                              \
  hipLaunchKernelGGL((conv3_k<BN_, ST_, 2, STATS_, G_>), dim3(nmb * (int)(N / BN_)), dim3(256), 0, st,          \
                     (const bf16*)A, (const bf16*)B, (bf16*)C, (int)M, (int)N, (int)K, lda, ldb, ldc, 0, 0, cin,   \
                     stats, bias, g, bias_bf16, BnRed{})
  if (chunk_taps) {   // the RGB stem: 64 output channels
    if (stats) DPH_CG(64, 3, true, 2);
    else DPH_CG(64, 3, false, 2);
  } else if (stats) {
    if (wide) DPH_CG(128, 2, true, 1);
    else DPH_CG(64, 3, true, 1);
  } else {
    if (wide) DPH_CG(128, 2, false, 1);
    else DPH_CG(64, 3, false, 1);
  }
#undef DPH_CG
}

}  // namespace dph
