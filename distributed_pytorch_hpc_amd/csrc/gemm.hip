// Weight-gradient GEMM for CDNA4 (gfx950):  C[M, N] (+)= A^T B  with A [K, M] and B [K, N] both row-major
// (token-major activations / output gradients, K = tokens).  This is dW = dY^T X of every linear layer.
//
// hipBLASLt runs this "both operands K-strided" pattern at 0.95-1.2 PFLOP/s on the Llama-2-7B shapes while the
// K-contiguous pattern reaches 1.5-1.6 PFLOP/s (profiles/gemm_layout_*.json); transposing the operands first
// costs more than it saves.  Here the transposition happens on the LDS -> register path instead:
//   * 256 x 256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), each wave 128 x 64 = 8 x 4 MFMA
//     16x16x32 bf16 tiles (128 fp32 accumulator VGPRs);
//   * slots of 32 tokens: the [32][256] A and B tiles are copied global -> LDS by LDS-DMA (global_load_lds_dwordx4,
//     16 B per lane, lane-linear destination, swizzle applied to the SOURCE address) into a 5-region ring, the
//     copies of slots t+2 and t+3 in flight under the MFMAs of slot t;
//   * MFMA operands (8 k of one m or n column per lane) come from ds_read_b64_tr_b16 transposed reads; the LDS image
//     XORs each 16-B slot so a half-wave's transposed reads cover all 64 banks exactly once;
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
// 4 tiles tall: w13 / wqkv +1.5-2 %, w2 / wo equal against 8 (16: -4 %; 2, 3, 6 no better than 4), interleaved on one
// box (profiles/r5/wgrad_tune/)
constexpr int GROUP_M = 4;

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

template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

// ---- The kernel: v_mfma_f32_16x16x32_bf16 (profiles/r5/mfma_power/: 12 % more TFLOP/J and 15 % more TFLOP/s than
// 32x32x16 on register operands, the clock held 14 % higher) ----
// Wave tile 128 x 64 = 8 x 4 tiles of 16 x 16 (32 f32x4 accumulators, 128 VGPRs).  A slot is 32 k-rows (one MFMA's
// K): region R of LDS holds A rows [32][256] at +0 and B rows [32][256] at +16 KB, 5 regions = 160 KB.
// Fragment of m-tile mt: lane L (m = L & 15, k-group g = L >> 4) reads rows 4g + tq (k 0..15 half) and 16 + 4g + tq
// (k 16..31 half) with two ds_read_b64_tr_b16 at one lane offset 16 rows apart; the k permutation is the same for the
// A and B fragments, so the products are exact.  The image swizzle XORs the 16-B slot with ((row & 3) << 2) |
// (((row >> 2) & 1) << 1): the two 16-lane groups of a half-wave read rows 4 apart, and the extra bit sends them to
// disjoint slots, so a half-wave's 32 transposed 8-B reads cover all 64 banks once.
// Pipeline: slot S retires DMA pair S+1 (pairs S+2, S+3 stay in flight: three slots of MFMA work hide each copy),
// meets the other waves at the barrier and runs the 32 MFMAs of region S while the fragments of region S+1 are read: B
// into the other B set first, then each A row refilled right after its own 4 MFMAs.  Pair S+4 goes into region
// (S+4) % 5 -- the region pair S-1 left, which every wave finished multiplying before this barrier -- one DMA
// instruction after every other MFMA row (+2-4 % over issuing all four right after the barrier, where each one's M0
// save / set / restore held the matrix pipe: profiles/r5/wgrad_spread/).  Pairs past the end re-load the last pair into
// a region nobody multiplies.
// Measured against the round-2..5 kernel (32x32x16, 128 x 64 wave tile, waves 4..7 one barrier behind; deleted), one
// box, interleaved (profiles/r5/wgrad16/): w13 / wqkv / w2 1255-1264 / 1296-1301 / 1312-1313 TFLOP/s vs 1202-1206 /
// 1245-1248 / 1252-1254 at 1.71-1.85 vs 1.60-1.64 GHz, 7B step 28 425-28 436 vs 28 225-28 316 tokens/s.  The same
// 16x16x32 body with the stagger lost (1224-1260 TFLOP/s): it fits only one slot of DMA latency in 160 KB of LDS.
constexpr int R16 = 5, REG16 = 32768;

template <typename OutT, bool ACCUM, bool LDS_EPI = true>
__global__ __launch_bounds__(GNT, 1) void gemm_tn16_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                      OutT* __restrict__ C, int M, int N, int K, int64_t lda,
                                                      int64_t ldb, int64_t ldc, int64_t cstride) {
  A += (int64_t)blockIdx.y * K * lda;
  B += (int64_t)blockIdx.y * K * ldb;
  C += (int64_t)blockIdx.y * cstride;
  __shared__ __attribute__((aligned(1024))) char lds[R16 * REG16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;

  const int tiles_m = (M + GBM - 1) / GBM, tiles_n = (N + GBN - 1) / GBN, nwg = tiles_m * tiles_n;
  int tm, tn;
  grouped_tile(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;

  // transposed-read offsets (k 0..15 half; the 16..31 half is +16 rows)
  const int swz = (tq << 2) | ((g & 1) << 1);
  const int base = (4 * g + tq) * ROWB + 8 * (tp & 1);
  int aoff[8], boff[4];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) aoff[mt] = base + (wm << 8) + (((2 * mt + (tp >> 1)) ^ swz) << 4);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
    boff[nt] = 16384 + base + ((wn >> 1) << 8) + (((8 * (wn & 1) + 2 * nt + (tp >> 1)) ^ swz) << 4);

  // LDS-DMA: thread t copies chunks t and t + 512 of a [32][32 x 16 B] operand image (rows t >> 5 and 16 + (t >> 5));
  // the destination is lane-linear, the swizzle goes into the source column
  const int srow = threadIdx.x >> 5, pslot = threadIdx.x & 31;
  const int sswz = ((srow & 3) << 2) | (((srow >> 2) & 1) << 1);
  const int lslot = (pslot & 16) | ((pslot & 15) ^ sswz);
  const int colA = min(lslot * 8, M - 8 - m0), colB = min(lslot * 8, N - 8 - n0);
  const unsigned voffA = (unsigned)((srow * lda + colA) * 2), voffB = (unsigned)((srow * ldb + colB) * 2);
  const unsigned hopA = (unsigned)(16 * lda * 2), hopB = (unsigned)(16 * ldb * 2);
  const char* Ag = reinterpret_cast<const char*>(A + m0);
  const char* Bg = reinterpret_cast<const char*>(B + n0);
  const int64_t stepA = 32 * lda * 2, stepB = 32 * ldb * 2;
  const unsigned lds_wave = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds + (threadIdx.x >> 6) * 1024);

  const int NP = K / 32;
  // DMA instruction i (< 4) of pair P: A rows 0..15 / 16..31, B rows 0..15 / 16..31
  auto dma_piece = [&](int P, auto RI, auto II) {
    constexpr int i = decltype(II)::value;
    const unsigned d = lds_wave + decltype(RI)::value * REG16 + (i >> 1) * 16384 + (i & 1) * 8192;
    const int Pc = min(P, NP - 1);   // past the end: the last pair again, into a region nobody multiplies
    if constexpr (i < 2) glds16(Ag + Pc * stepA, voffA + (i & 1) * hopA, d);
    else glds16(Bg + Pc * stepB, voffB + (i & 1) * hopB, d);
  };
  auto dma_pair = [&](int P, auto RI) {
    dma_piece(P, RI, std::integral_constant<int, 0>{});
    dma_piece(P, RI, std::integral_constant<int, 1>{});
    dma_piece(P, RI, std::integral_constant<int, 2>{});
    dma_piece(P, RI, std::integral_constant<int, 3>{});
  };
  // region base as an opaque wave-uniform value: the 12 per-lane addresses are formed per slot (12 VALU) instead of
  // being hoisted out of the loop for all 5 regions (60 live VGPRs)
  auto region = [&](auto RI) -> const char* {
    int rb = decltype(RI)::value * REG16;
    asm volatile("" : "+s"(rb));
    return lds + rb;
  };
  auto read_b = [&](const char* rg, bf16x8 (&bfr)[4]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bfr[nt] = tr2(rg, boff[nt], boff[nt] + 16 * ROWB);
  };
  auto read_a = [&](const char* rg, bf16x8 (&af)[8]) {
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) af[mt] = tr2(rg, aoff[mt], aoff[mt] + 16 * ROWB);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the 32 MFMAs of the current region, row by row; row mt's A fragment is refilled from the next region right after
  // its 4 MFMAs (one A set, rotated in place; B, used by every row, has two sets)
  // ... and the next pair's DMA issued behind the first two rows (two instructions after row 0, two after row 1): early
  // enough for the longest latency slack, yet not ahead of the slot's first MFMAs. A/B on one box (profiles/r5/dma_place,
  // 3 wgrad shapes x 2 rounds): one instruction after every odd row 1 393 / 1 420 / 1 373 TFLOP/s; after rows 0-3
  // +0.6 %; before rows 0-3 +0.8 %; after rows 1-4 +-0; two after rows 0 and 2 +1.1 %; two after rows 0 and 1 +1.4 %;
  // all four after row 0 +1.4 %
  auto mma_refill = [&](bf16x8 (&af)[8], const bf16x8 (&bfr)[4], const char* rn, int P, auto RI) {
    static_for<8>([&](auto MI) {
      constexpr int mt = decltype(MI)::value;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
      af[mt] = tr2(rn, aoff[mt], aoff[mt] + 16 * ROWB);
      if constexpr (mt < 2) {
        dma_piece(P, RI, std::integral_constant<int, 2 * mt>{});
        dma_piece(P, RI, std::integral_constant<int, 2 * mt + 1>{});
      }
    });
  };

  // prologue: pairs 0..3 (regions 0..3), pair 0 retired by every wave before the common barrier
  dma_pair(0, std::integral_constant<int, 0>{});
  dma_pair(1, std::integral_constant<int, 1>{});
  dma_pair(2, std::integral_constant<int, 2>{});
  dma_pair(3, std::integral_constant<int, 3>{});
  wait_vm<12>();
  __builtin_amdgcn_s_barrier();
  bf16x8 af[8], bf0[4], bf1[4];
  {
    const char* r0 = region(std::integral_constant<int, 0>{});
    read_b(r0, bf0);
    read_a(r0, af);
  }
  __builtin_amdgcn_sched_barrier(0);

  auto slot = [&](int P0, auto SI, bf16x8 (&bfc)[4], bf16x8 (&bfn)[4]) {
    constexpr int S = decltype(SI)::value;
    wait_vm<8>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    const char* rn = region(std::integral_constant<int, (S + 1) % R16>{});
    read_b(rn, bfn);
    mma_refill(af, bfc, rn, P0 + S + 4, std::integral_constant<int, (S + 4) % R16>{});
    // B reads (8) then per row 4 MFMAs + its 2 A reads
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
#define DPH_S(i) std::integral_constant<int, i>{}
  int P0 = 0;
  for (; P0 + 10 <= NP; P0 += 10) {
    slot(P0, DPH_S(0), bf0, bf1);
    slot(P0, DPH_S(1), bf1, bf0);
    slot(P0, DPH_S(2), bf0, bf1);
    slot(P0, DPH_S(3), bf1, bf0);
    slot(P0, DPH_S(4), bf0, bf1);
    slot(P0, DPH_S(5), bf1, bf0);
    slot(P0, DPH_S(6), bf0, bf1);
    slot(P0, DPH_S(7), bf1, bf0);
    slot(P0, DPH_S(8), bf0, bf1);
    slot(P0, DPH_S(9), bf1, bf0);
  }
  {   // the remaining NP - P0 (< 10) slots, each position compiled once
    const int rem = NP - P0;
    if (rem > 0) slot(P0, DPH_S(0), bf0, bf1);
    if (rem > 1) slot(P0, DPH_S(1), bf1, bf0);
    if (rem > 2) slot(P0, DPH_S(2), bf0, bf1);
    if (rem > 3) slot(P0, DPH_S(3), bf1, bf0);
    if (rem > 4) slot(P0, DPH_S(4), bf0, bf1);
    if (rem > 5) slot(P0, DPH_S(5), bf1, bf0);
    if (rem > 6) slot(P0, DPH_S(6), bf0, bf1);
    if (rem > 7) slot(P0, DPH_S(7), bf1, bf0);
    if (rem > 8) slot(P0, DPH_S(8), bf0, bf1);
  }
#undef DPH_S
  wait_vm<0>();

  // ---- epilogue: register r of tile (mt, nt) holds C[row 16 mt + 4 (lane >> 4) + r][col 16 nt + (lane & 15)] ----
  const int crow = 4 * g, ccol = lane & 15;
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
        for (int mt = 0; mt < 8; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = (NPASS == 1 ? wm * 128 : 0) + mt * 16 + crow + r;
              ct[row * 256 + wn * 64 + nt * 16 + ccol] = (OutT)acc[mt][nt][r];
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
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int col = n0 + wn * 64 + nt * 16 + ccol;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 128 + mt * 16 + crow + r;
          if (row >= M || col >= N) continue;
          OutT* pp = C + (int64_t)row * ldc + col;
          *pp = (OutT)(ACCUM ? acc[mt][nt][r] + (float)*pp : acc[mt][nt][r]);
        }
      }
  }
}


// Rejected (round 5, profiles/r5/wgrad_w4/): a 4-wave form, one wave per SIMD with a 128 x 128 wave tile (256
// accumulators in AGPRs, a third less LDS traffic per FLOP): 1272-1275 vs 1296-1302 TFLOP/s on w13 at 1.97 vs 1.78 GHz,
// MFMA busy 0.65 -- below the power cap, one wave cannot hide its own barrier and read latency.  With the DMA spread
// over its rows (offsets recomputed per instruction, no spills in the main loop) it fell to 1011-1074 vs 1363-1429 at
// 2.2 GHz (profiles/r5/wgrad_w4/spread_*).
// History: a round-2..4 16x16x32 form of the 32x32x16 pipeline (pairs of 16-row regions per MFMA, 12 region-address
// VALU ops per slot) lost to it, 1045-1260 vs 1287-1432 TF (profiles/gemm_wgrad_mfma16_vs_32.json); the kernel above
// differs in its 32-row regions, per-slot address formation, in-place A refill and a three-slot DMA lead.

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
  const size_t lds = 0;   // static: 5 x 32 KB regions
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
      hipLaunchKernelGGL((gemm_tn16_k<T, ACC>), grid, block, lds, st, a, b, (T*)c, (int)m, (int)n, (int)k,     \
                         lda, ldb, ldc_, cstride);                                                             \
    else                                                                                                       \
      hipLaunchKernelGGL((gemm_tn16_k<T, false, false>), grid, block, lds, st, a, b, (T*)c, (int)m, (int)n,    \
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
