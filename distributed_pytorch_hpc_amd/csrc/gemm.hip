// Weight-gradient GEMM for CDNA4 (gfx950):  C[M, N] (+)= A^T B  with A [K, M] and B [K, N] both row-major
// (token-major activations / output gradients, K = tokens).  This is dW = dY^T X of every linear layer.
//
// hipBLASLt runs this "both operands K-strided" pattern at 0.95-1.2 PFLOP/s on the Llama-2-7B shapes while the
// K-contiguous pattern reaches 1.5-1.6 PFLOP/s (profiles/gemm_layout_*.json); transposing the operands first
// costs more than it saves.  Here the transposition happens on the LDS -> register path instead:
//   * 256 x 256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), each wave 128 x 64 = 4 x 2 MFMA
//     32x32x16 bf16 tiles (128 fp32 accumulator VGPRs);
//   * K-steps of 64 tokens: the [64][256] A and B tiles are copied global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, 16 B per lane, lane-linear destination, swizzle applied to the SOURCE address),
//     double-buffered so the copy of step t+1 overlaps the MFMAs of step t;
//   * MFMA operands (8 consecutive k of one m or n column per lane) come from ds_read_b64_tr_b16 transposed
//     reads; the LDS image XORs each 16-B slot with (row & 3) << 2, which makes the 4-row x 4-chunk footprint of
//     a half-wave's transposed read cover all 64 banks exactly once;
//   * workgroups are remapped so each XCD (blockIdx % 8 under round-robin dispatch) owns a contiguous range of
//     output tiles, grouped GROUP_M tiles tall, for L2 reuse of the shared A / B column panels.
// Requirements (checked by the host op): M % 8 == 0, N % 8 == 0, K % 64 == 0, lda / ldb % 8 == 0, 16-B aligned
// bases.  Ragged M / N (the tensor-parallel shards of Llama-2-7B: w13 2752 rows at tp=8, w2 1376 columns, the
// vocab-sharded head 4000 rows) run as partial edge tiles: the LDS-DMA source column of a lane whose 16-B chunk lies
// past the edge is clamped to the last valid chunk (finite data, never stored) and the epilogue masks rows / columns
// beyond M / N.  Other shapes use hipBLASLt.
#include <type_traits>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4_g;

constexpr int GBM = 256, GBN = 256, GBK = 64, GNT = 512;
constexpr int ROWB = GBM * 2;              // bytes per LDS image row (256 bf16)
constexpr int TILEB = GBK * ROWB;          // 32 KB per operand tile
constexpr int GROUP_M = 8;

// Tile (tm, tn) of logical workgroup lin: columns of GROUP_M-tall tile groups, m fastest, so the workgroups an XCD
// runs together share GROUP_M A panels and a few B panels in its L2.
__device__ __forceinline__ void grouped_tile(int lin, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int first_m = lin / (GROUP_M * tiles_n) * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int in_group = lin % (GROUP_M * tiles_n);
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

__device__ __forceinline__ bf16x8 tr2(const char* base, int off_lo, int off_hi) {
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_g*)(base + off_lo));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_g*)(base + off_hi));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// LDS-DMA / counted-wait helpers (dph_common.h): the DMA is issued from inline asm so hipcc does not drain it before
// the transposed ds_reads of other regions; completion is counted explicitly (wait_vm<N> + s_barrier).
__device__ __forceinline__ void glds16(const char* sbase, unsigned voff, unsigned lds) { lds_dma16(sbase, voff, lds); }
template <int N>
__device__ __forceinline__ void wait_vm() { wait_vmcnt<N>(); }

// Pipeline: one K-step (64 tokens) = 4 phases of 16 k-rows.  Phase P's operands live in LDS region R = P & 7 (tile
// parity x 16-row region; A rows at +0, B rows at +8 KB of a 16-KB region) and are filled by DMA "pair P" (one 16-B
// global_load_lds per thread per operand, inline asm: see glds16).  In slot S every wave retires its share of pair
// S+2 (counted vmcnt), meets the others at a raw s_barrier, issues pair S+5, and runs the 8 MFMAs of region S while the
// transposed reads of region S+1 go to the other fragment register set.
//
// Waves 4..7 run one barrier behind waves 0..3, so on every SIMD one wave issues its slot's MFMAs while its partner
// waits at the barrier, issues its DMA pair and transposed reads (the ping-pong of gemm_nt.hip); in lockstep (the
// round-2..4 gemm_tn_k, deleted in round 5) both waves of a SIMD reached the barrier together and the matrix pipe idled
// while they waited (PMC on the w13 shape: SQ_WAIT_ANY 40 % of wave cycles, MFMA busy 0.74 vs 0.79 staggered,
// profiles/r5/wgrad_power/).  The stagger makes an early wave's read of region S+1 at its slot S race the LATE waves'
// share of that region's DMA, hence the pipeline depth: slot S retires pair S+2 (not S+1) and issues pair S+5 (not
// S+4); regions in use at once: S..S+5 = 6 of the 8.  WAR: pair S+5 overwrites pair S-3's region, whose last reader
// (a late wave, in its slot S-4 = the early waves' slot S-3) is two barriers back.
// No tail code: a pair index past the last one re-loads the last pair (finite data) into a region whose contents are
// never multiplied, so every slot has the same DMA / counted wait / read and the loop body is one 8-slot block (plus
// one 4-slot block for an odd K-tile count) -- tail sequences cost the lockstep kernel ~400 VGPR spills and a
// vmcnt(0) drain per iteration where the waitcnt pass merged the spill reloads into the loop.
// LDS_EPI: the 16-B LDS-staged epilogue (C 16-B aligned with a 16-B row pitch); otherwise one store per element.
template <typename OutT, bool ACCUM, bool LDS_EPI = true>
__global__ __launch_bounds__(GNT, 1) void gemm_tn_stag_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         OutT* __restrict__ C, int M, int N, int K, int64_t lda,
                                                         int64_t ldb, int64_t ldc, int64_t cstride) {
  A += (int64_t)blockIdx.y * K * lda;
  B += (int64_t)blockIdx.y * K * ldb;
  C += (int64_t)blockIdx.y * cstride;
  __shared__ __attribute__((aligned(1024))) char lds[8 * 16384];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;

  const int tiles_m = (M + GBM - 1) / GBM, tiles_n = (N + GBN - 1) / GBN, nwg = tiles_m * tiles_n;
  int tm, tn;
  grouped_tile(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;

  const int x = 2 * (g & 1) + (tp >> 1);
  const int krow = 4 * (g >> 1) + tq;
  const int base = krow * ROWB + 8 * (tp & 1);
  int aoff[4], boff[2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) aoff[mt] = base + (wm << 8) + ((4 * (mt ^ tq) + x) << 4);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
    boff[nt] = 8192 + base + ((wn >> 1) << 8) + ((4 * ((((wn & 1) << 1) | nt) ^ tq) + x) << 4);

  const int srow = threadIdx.x >> 5, lr = (threadIdx.x >> 4) & 1, sslot = threadIdx.x & 15;
  const int sch = (lr << 4) | (sslot ^ ((srow & 3) << 2));
  const int colA = min(sch * 8, M - 8 - m0), colB = min(sch * 8, N - 8 - n0);
  const unsigned voffA = (unsigned)((srow * lda + colA) * 2), voffB = (unsigned)((srow * ldb + colB) * 2);
  const char* Ag = reinterpret_cast<const char*>(A + m0);
  const char* Bg = reinterpret_cast<const char*>(B + n0);
  const int64_t stepA = 16 * lda * 2, stepB = 16 * ldb * 2;
  const unsigned lds_wave = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds + (threadIdx.x >> 6) * 1024);

  auto region = [&](auto RI) -> char* { return lds + decltype(RI)::value * 16384; };
  const int NP = (K / GBK) * 4;
  auto dma_pair = [&](int P, auto RI) {
    const unsigned d = lds_wave + decltype(RI)::value * 16384;
    const int Pc = min(P, NP - 1);   // past the end: the last pair again, into a region nobody multiplies
    glds16(Ag + Pc * stepA, voffA, d);
    glds16(Bg + Pc * stepB, voffB, d + 8192);
  };
  auto read_phase = [&](auto RI, bf16x8 (&af)[4], bf16x8 (&bfr)[2]) {
    const char* rg = region(RI);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) af[mt] = tr2(rg, aoff[mt], aoff[mt] + 8 * ROWB);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) bfr[nt] = tr2(rg, boff[nt], boff[nt] + 8 * ROWB);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.f;

  auto mma = [&](const bf16x8 (&af)[4], const bf16x8 (&bfr)[2]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  // prologue: pairs 0..4 (regions 0..4), then pairs 0 and 1 retired by every wave before the common barrier
  dma_pair(0, I0{});
  dma_pair(1, I1{});
  dma_pair(2, I2{});
  dma_pair(3, I3{});
  dma_pair(4, I4{});
  wait_vm<6>();
  __builtin_amdgcn_s_barrier();
  bf16x8 af0[4], bf0[2], af1[4], bf1[2];
  read_phase(I0{}, af0, bf0);
  const bool late = __builtin_amdgcn_readfirstlane(wid) >= 4;
  if (late) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  // slot S (region S & 7): retire pair S+2 (vmcnt 4: pairs S+3, S+4 stay in flight) -> barrier -> DMA pair S+5 ->
  // reads of region S+1 into the other register set interleaved with the 8 MFMAs of region S
  auto slot = [&](int P0, auto SI, bf16x8 (&afc)[4], bf16x8 (&bfc)[2], bf16x8 (&afn)[4], bf16x8 (&bfn)[2]) {
    constexpr int S = decltype(SI)::value;
    wait_vm<4>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    dma_pair(P0 + S + 5, std::integral_constant<int, (S + 5) & 7>{});
    __builtin_amdgcn_s_setprio(1);
    read_phase(std::integral_constant<int, (S + 1) & 7>{}, afn, bfn);
    mma(afc, bfc);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
#define DPH_S(i) std::integral_constant<int, i>{}
  int P0 = 0;
  for (; P0 + 8 <= NP; P0 += 8) {
    slot(P0, DPH_S(0), af0, bf0, af1, bf1);
    slot(P0, DPH_S(1), af1, bf1, af0, bf0);
    slot(P0, DPH_S(2), af0, bf0, af1, bf1);
    slot(P0, DPH_S(3), af1, bf1, af0, bf0);
    slot(P0, DPH_S(4), af0, bf0, af1, bf1);
    slot(P0, DPH_S(5), af1, bf1, af0, bf0);
    slot(P0, DPH_S(6), af0, bf0, af1, bf1);
    slot(P0, DPH_S(7), af1, bf1, af0, bf0);
  }
  if (P0 < NP) {   // odd number of K-tiles: the last one (regions 0..3)
    slot(P0, DPH_S(0), af0, bf0, af1, bf1);
    slot(P0, DPH_S(1), af1, bf1, af0, bf0);
    slot(P0, DPH_S(2), af0, bf0, af1, bf1);
    slot(P0, DPH_S(3), af1, bf1, af0, bf0);
  }
#undef DPH_S
  if (!late) __builtin_amdgcn_s_barrier();   // balance the stagger
  wait_vm<0>();

  // ---- epilogue: register i of tile (mt, nt) holds C[row (i&3) + 8(i>>2) + 4h][col l32].  Through LDS (free after
  // the main loop) the tile leaves as 16-B row segments -- 16 (bf16) / 32 (fp32, two 128-row passes) vector stores per
  // thread instead of 128 scalar stores per lane; ACCUM keeps the per-element path (one rounding of old + acc) ----
  if constexpr (!ACCUM && LDS_EPI) {
    constexpr int VE = 16 / (int)sizeof(OutT);
    constexpr int PR = (int)(sizeof(OutT) == 2 ? 256 : 128);
    constexpr int NPASS = 256 / PR, SPR = 256 / VE;
    OutT* ct = reinterpret_cast<OutT*>(lds);
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
      __syncthreads();
      if (NPASS == 1 || wm == pass) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int r = (NPASS == 1 ? wm * 128 : 0) + mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
              ct[r * 256 + wn * 64 + nt * 32 + l32] = (OutT)acc[mt][nt][i];
            }
      }
      __syncthreads();
#pragma unroll
      for (int c = threadIdx.x; c < PR * SPR; c += GNT) {
        const int r = c / SPR, seg = c % SPR;
        const int row = m0 + pass * PR + r, col = n0 + seg * VE;
        if (row < M && col < N)
          *reinterpret_cast<u32x4*>(C + (int64_t)row * ldc + col) =
              *reinterpret_cast<const u32x4*>(ct + r * 256 + seg * VE);
      }
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int col = n0 + wn * 64 + nt * 32 + l32;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = m0 + wm * 128 + mt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (row >= M || col >= N) continue;
          OutT* pp = C + (int64_t)row * ldc + col;
          *pp = (OutT)(ACCUM ? acc[mt][nt][i] + (float)*pp : acc[mt][nt][i]);
        }
      }
  }
}

// Rejected (round 2-4, code removed in round 5): the same pipeline on v_mfma_f32_16x16x32_bf16 (same 128 x 64 tile
// per wave as 8 x 4 tiles of 16 x 16, pairs of 16-row regions per MFMA): 1045-1260 TF vs 1287-1432 TF for the
// 32x32x16 kernel on the 7B shapes -- twice the MFMA issues and 12 region-address VALU ops per slot outweighed the
// higher clock the chip holds on the 16x16x32 shape (profiles/gemm_wgrad_mfma16_vs_32.json, profiles/r4/wgrad_stagger/).

// fp32 split-K slabs W[S][Mb][Nb] -> C band (+ C when accumulating), in C's dtype.  Fixed summation order.
template <typename OutT, bool ACCUM>
__global__ __launch_bounds__(256) void gemm_split_reduce_k(const float* __restrict__ W, OutT* __restrict__ C, int Mb,
                                                           int Nb, int64_t ldc, int S) {
  const int64_t n4 = (int64_t)Mb * Nb / 4, slab = (int64_t)Mb * Nb;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n4; v += (int64_t)gridDim.x * 256) {
    const int64_t e = v * 4;
    f32x4 acc = *reinterpret_cast<const f32x4*>(W + e);
    for (int s = 1; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(W + s * slab + e);
    const int64_t r = e / Nb, c = e % Nb;
    OutT* o = C + r * ldc + c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x = acc[j];
      if (ACCUM) x += (float)o[j];
      o[j] = (OutT)x;
    }
  }
}

int g_gemm_tn_tail = 0;   // tail split: 0 = device CU count, > 0 = that many CUs (tests), < 0 = off

int gemm_tn_cus() {
  if (g_gemm_tn_tail > 0) return g_gemm_tn_tail;
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

}  // namespace



void gemm_tn_set_tail(int cus) { g_gemm_tn_tail = cus; }

bool gemm_tn_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 8 && N >= 8 && K > 0 && M % 8 == 0 && N % 8 == 0 && K % GBK == 0;
}

// Tail plan.  One 256 x 256 tile per workgroup and one workgroup per CU: T tiles run in ceil(T / CU) waves, and a
// partial last wave (w13's 1376 tiles = 5.375 waves, w2's 688 = 2.69 on the Llama-2-7B wgrad shapes) idles part of
// the chip for a whole wave.  The plan keeps a band of whole waves on the plain kernel and computes the remaining
// row or column band with K split S ways into fp32 slabs (one launch, gridDim.y = S), reduced into C afterwards:
// the band then costs ceil(band * S / CU) / S waves instead of ceil(band / CU).
GemmTnPlan gemm_tn_plan(int64_t M, int64_t N, int64_t K) {
  GemmTnPlan pl{};
  if (g_gemm_tn_tail < 0) return pl;
  if (M % GBM || N % GBN) return pl;   // ragged edge tiles: one launch
  const int cus = gemm_tn_cus();
  const int64_t tm = M / GBM, tn = N / GBN, T = tm * tn;
  if (T % cus == 0) return pl;
  const bool forced = g_gemm_tn_tail > 0;
  const int64_t min_k = forced ? GBK : 16 * GBK;   // >= 16 K-steps per slice on real shapes
  // cost in seconds: a wave of 256 x 256 x K tiles at ~1.3 PFLOP/s over 256 CUs (measured kernel rate), plus the
  // fp32 slabs written and read back at ~5 TB/s; the tail wave as it is costs one wave
  const double t_wave = (double)K * GBM * GBN * 2.0 / (1.3e15 / 256.0);
  double best = t_wave;
  for (int dim = 0; dim < 2; ++dim) {
    const int64_t along = dim == 0 ? tm : tn, other = dim == 0 ? tn : tm;
    // largest prefix of whole bands whose tiles fill whole waves
    int64_t keep = along;
    while (keep > 0 && (keep * other) % cus) --keep;
    const int64_t band = (along - keep) * other;
    if (band == 0) continue;
    for (int S : {2, 3, 4, 6, 8}) {
      if (K % (S * GBK) || K / S < min_k) continue;
      const double slab_bytes = 2.0 * S * (double)band * GBM * GBN * 4.0;
      const double cost = (double)((band * S + cus - 1) / cus) / S * t_wave + (forced ? 0.0 : slab_bytes / 5e12);
      if (cost < best * (forced ? 0.999 : 0.95)) {
        best = cost;
        pl.split = S;
        pl.dim = dim;
        pl.keep = keep * (dim == 0 ? GBM : GBN);
      }
    }
  }
  if (pl.split) {
    const int64_t bm = pl.dim == 0 ? M - pl.keep : M, bn = pl.dim == 0 ? N : N - pl.keep;
    pl.workspace_floats = (int64_t)pl.split * bm * bn;
  }
  return pl;
}

void gemm_tn(const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
             int64_t ldc, int out_dtype, bool accumulate, hipStream_t st, const GemmTnPlan* plan,
             float* workspace) {
  const size_t lds = 0;   // static: 8 x 16 KB regions
  const dim3 block(GNT);
  auto launch = [&](const bf16* a, const bf16* b, void* c, int64_t m, int64_t n, int64_t k, int64_t ldc_, int S,
                    bool f32_out, bool acc, int64_t cstride) {
    const dim3 grid((unsigned)(((m + GBM - 1) / GBM) * ((n + GBN - 1) / GBN)), (unsigned)S);
    // the LDS epilogue stores 16-B row segments: C's base and row pitch must be 16-B aligned (an offset view of C
    // falls back to the per-element epilogue)
    const int64_t esz_c = (!f32_out && out_dtype == kBF16) ? 2 : 4;
    const bool vec_c = ((uintptr_t)c & 15) == 0 && ((ldc_ * esz_c) & 15) == 0;
#define DPH_GEMM_LAUNCH(T, ACC)                                                                                \
  do {                                                                                                         \
    if (ACC || vec_c)                                                                                          \
      hipLaunchKernelGGL((gemm_tn_stag_k<T, ACC>), grid, block, lds, st, a, b, (T*)c, (int)m, (int)n, (int)k,  \
                         lda, ldb, ldc_, cstride);                                                             \
    else                                                                                                       \
      hipLaunchKernelGGL((gemm_tn_stag_k<T, false, false>), grid, block, lds, st, a, b, (T*)c, (int)m, (int)n, \
                         (int)k, lda, ldb, ldc_, cstride);                                                     \
  } while (0)
    if (!f32_out && out_dtype == kBF16) {
      if (acc) DPH_GEMM_LAUNCH(bf16, true);
      else DPH_GEMM_LAUNCH(bf16, false);
    } else {
      if (acc) DPH_GEMM_LAUNCH(float, true);
      else DPH_GEMM_LAUNCH(float, false);
    }
#undef DPH_GEMM_LAUNCH
  };
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  if (!plan || !plan->split || !workspace) {
    launch(a, b, C, M, N, K, ldc, 1, false, accumulate, 0);
    return;
  }
  const int64_t esz = out_dtype == kBF16 ? 2 : 4;
  char* c = (char*)C;
  int64_t bm = M, bn = N;
  const bf16 *ba = a, *bb = b;
  char* bc = c;
  if (plan->dim == 0) {   // band = rows [keep, M) of C = columns [keep, M) of A
    if (plan->keep) launch(a, b, C, plan->keep, N, K, ldc, 1, false, accumulate, 0);
    bm = M - plan->keep;
    ba = a + plan->keep;
    bc = c + plan->keep * ldc * esz;
  } else {                // band = columns [keep, N) of C = columns [keep, N) of B
    if (plan->keep) launch(a, b, C, M, plan->keep, K, ldc, 1, false, accumulate, 0);
    bn = N - plan->keep;
    bb = b + plan->keep;
    bc = c + plan->keep * esz;
  }
  const int S = plan->split;
  launch(ba, bb, workspace, bm, bn, K / S, bn, S, true, false, bm * bn);
  const dim3 rgrid(stream_grid(bm * bn / 4, 256));
  if (out_dtype == kBF16) {
    if (accumulate) hipLaunchKernelGGL((gemm_split_reduce_k<bf16, true>), rgrid, dim3(256), 0, st, workspace,
                                       (bf16*)bc, (int)bm, (int)bn, ldc, S);
    else hipLaunchKernelGGL((gemm_split_reduce_k<bf16, false>), rgrid, dim3(256), 0, st, workspace, (bf16*)bc,
                            (int)bm, (int)bn, ldc, S);
  } else {
    if (accumulate) hipLaunchKernelGGL((gemm_split_reduce_k<float, true>), rgrid, dim3(256), 0, st, workspace,
                                       (float*)bc, (int)bm, (int)bn, ldc, S);
    else hipLaunchKernelGGL((gemm_split_reduce_k<float, false>), rgrid, dim3(256), 0, st, workspace, (float*)bc,
                            (int)bm, (int)bn, ldc, S);
  }
}

}  // namespace dph
