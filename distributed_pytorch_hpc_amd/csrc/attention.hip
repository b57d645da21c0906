// Flash attention forward + backward for CDNA4 (gfx950), bf16 in / fp32 accumulate, MFMA 32x32x16.
// Replaces the reference's F.scaled_dot_product_attention(q, k, v, is_causal=True)
// (fsdp_tp/llama2_model.py:223) and the explicit softmax(QK^T)V of the ViT
// (scripts/03_tensor_parallel_tp/tensor_parallel_vit.py:120-122).
//
// Forward ("swapped" product, cdna_hip_programming.md App. B): one workgroup = 4 waves = 128 query rows,
// one wave = 32 query rows.  S^T = K Q^T puts ONE query per lane (lane & 31) with 16 of the tile's keys
// per half-wave, so the online-softmax state (m, l) and the O^T accumulator rescale are lane-local and
// a row reduction is 31 VALU ops + one permlane32_swap.  O^T = V^T P^T consumes the S^T accumulator
// directly as the B operand (no LDS round trip for P); V^T fragments come from ds_read_b64_tr_b16
// transposed LDS reads.  K/V tiles (64 keys) are register-staged into a double-buffered, XOR-swizzled
// LDS image (conflict-free for both ds_read_b128 row reads and tr reads), one barrier per tile.
//
// Backward (no atomics, no dS round trip through LDS): two kernels after a delta = rowsum(dO*O) pass.
//   dK/dV kernel, KV-stationary: a wave keeps its 32 keys' K^T / V^T fragments and dK^T / dV^T in registers
//   while the workgroup sweeps query tiles; S and dP are computed with the key on the lane so P and dS are
//   directly the B operands of dV^T += dO^T P and dK^T += Q^T dS.
//   dQ kernel, Q-stationary (the forward's structure): S^T, dP^T with the query on the lane, dS^T lane-local,
//   dQ^T += K^T dS^T with dS^T consumed from the accumulator.
// The split costs 2 extra MFMA products (S, dP recomputed) but removes the fp32 dQ atomics that bound a
// fused kernel at ~1.3 TB/s of atomic traffic (MI355X_MICROARCH.md 'Global float atomics').
//
// Dropout (DROP instantiations, 4-wave workgroups): the keep decision of element (query, key) is a counter hash,
// so the forward and both backward kernels regenerate the same mask without storing it: the forward drops
// P after the row sum (the softmax normaliser is the undropped one) and scales O by 1/(1-p); dK/dV uses the
// dropped, rescaled P for dV and dS = P (Z dP / (1-p) - delta) for dK; dQ the same dS.  This is the
// nn.MultiheadAttention(dropout=...) path of the pipeline transformer (03_pipeline_training.py:57-58,70).
#include <cstdlib>
#include <string>
#include <type_traits>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__device__ __forceinline__ float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }

// 32-bit integer mix (lowbias32 finalizer)
__device__ __forceinline__ unsigned attn_mix(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// per-(seed, batch*head, query) row key, then keep(query, key) = mix(row_key ^ key * C) >= threshold
__device__ __forceinline__ unsigned attn_row_key(unsigned seed, unsigned bh, unsigned q) {
  return attn_mix(seed ^ attn_mix(bh * 0x9e3779b1u + q * 0x85ebca77u));
}
__device__ __forceinline__ bool attn_keep(unsigned row_key, unsigned key, unsigned thr) {
  return attn_mix(row_key ^ (key * 0xc2b2ae3du)) >= thr;
}
__device__ __forceinline__ unsigned attn_drop_thr(float p) {
  return (unsigned)fminf(p * 4294967296.f, 4294967040.f);
}

// Byte offset of 16-B chunk `ch` of row `row` in an LDS image whose rows hold NC 16-B chunks.
// Rows are packed into 256-B lines; chunk slots are XOR-permuted per line so that (a) 32 lanes reading
// the same chunk of 32 consecutive rows with ds_read_b128 and (b) ds_read_b64_tr_b16 reads of 4
// consecutive rows x 4 consecutive chunks hit distinct bank slots.
template <int NC>
__device__ __forceinline__ int img_off(int row, int ch) {
  const int F = row * NC + ch;
  const int line = F >> 4, c = F & 15;
  const int f = ((line & 3) << 2) | ((line >> 2) & 3);
  return (line << 8) + ((c ^ f) << 4);
}

__device__ __forceinline__ bf16x8 lds_b128(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}
// Two transposed 4x16 reads -> one 8-element MFMA operand.
__device__ __forceinline__ bf16x8 lds_tr2(const char* base, int off_lo, int off_hi) {
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off_lo));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off_hi));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Stage ROWS rows x NC 16-B chunks of a strided bf16 global tile into an img_off-swizzled LDS image by
// LDS-DMA (global_load_lds_dwordx4: per-lane source address, lane-linear destination).  The swizzle is
// applied to the SOURCE address (cdna_hip_programming.md rule 21); rows >= nvalid read the last valid row
// (finite data that the caller masks), so no lane ever reads out of bounds.
template <int NC, int ROWS, int NT>
__device__ __forceinline__ void glds_stage(char* img, const bf16* base, int64_t rstride, int row0, int nvalid) {
  constexpr int CHUNKS = ROWS * NC;
  const int tid = threadIdx.x, wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < (CHUNKS + NT - 1) / NT; ++i) {
    const int L = tid + NT * i;
    if (CHUNKS % NT == 0 || L < CHUNKS) {
      const int line = L >> 4, slot = L & 15;
      const int F = (line << 4) + (slot ^ (((line & 3) << 2) | ((line >> 2) & 3)));
      const int row = min(row0 + F / NC, nvalid - 1);
      const bf16* src = base + (int64_t)row * rstride + (F % NC) * 8;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(img + (wave * 64 + NT * i) * 16),
                                       16, 0, 0);
    }
  }
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Both half-waves end up with the max / sum over the 32 keys of their shared query.
__device__ __forceinline__ float half_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Accumulator register r of a 32x32 MFMA tile holds row (r&3) + 8*(r>>2) + 4*h of column lane&31.
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}

// Epilogue of a 32 x HD accumulator set whose lane holds row l32 (columns dt * 32 + 8 gg + 4 h + j, j < 4): scale,
// optionally rotate every interleaved pair (2i, 2i + 1) back by -theta(row + rope_off, i) (the gradient of RoPE), cast
// to bf16 and store rows [0, nvalid) at base + r * rstride.  The wave goes through its own LDS slab (32 rows x 4*DT
// 16-B chunks, chunk index XOR-swizzled by the row): the lane's 4-column pieces are written to LDS, then every global
// store is a 16-B row segment and NCH lanes cover a full row -- 8 dwordx4 stores per lane instead of 16 dwordx2
// spread over 32 rows (HD = 128).  Measured against the per-lane form on the 7B shape: forward 1.405 -> 1.397 ms,
// backward 4.07 -> 3.96 ms, +0.4 % tokens/s (profiles/r3/ab_attn_lds_epilogue/).  Rows >= nvalid are not stored.  Needs the LDS slab free:
// called after the kernel's last barrier on the tile images; back-to-back calls on one slab are safe (a wave's LDS
// operations complete in order).
template <int DT>
__device__ __forceinline__ void store_rows_lds(char* slab, bf16* base, int64_t rstride, int nvalid,
                                               const f32x16 (&acc)[DT], float mul, int h, int l32, int row,
                                               const float* rc, const float* rs, int rope_off) {
  constexpr int NCH = 4 * DT, HALF = DT * 16;
  const bool ok = l32 < nvalid;   // rows past the end: no RoPE-table read (their values are never stored)
  const float* cr = rc && ok ? rc + (int64_t)(row + rope_off) * HALF : nullptr;
  const float* sr = rs && ok ? rs + (int64_t)(row + rope_off) * HALF : nullptr;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = acc[dt][4 * gg + j] * mul;
      if (cr) {
        const int i0 = dt * 16 + 4 * gg + 2 * h;
        const float2 c = *reinterpret_cast<const float2*>(cr + i0);
        const float2 sn = *reinterpret_cast<const float2*>(sr + i0);
        const float a0 = v[0], b0 = v[1], a1 = v[2], b1 = v[3];
        v[0] = fmaf(a0, c.x, b0 * sn.x);
        v[1] = fmaf(b0, c.x, -a0 * sn.x);
        v[2] = fmaf(a1, c.y, b1 * sn.y);
        v[3] = fmaf(b1, c.y, -a1 * sn.y);
      }
      bf16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (bf16)v[j];
      const int ch = 4 * dt + gg;   // columns 8 ch + 4 h .. +3
      *reinterpret_cast<bf16x4*>(slab + l32 * (NCH * 16) + ((ch ^ (l32 & (NCH - 1))) << 4) + 8 * h) = w;
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes are done
  __builtin_amdgcn_wave_barrier();
  const int lane = threadIdx.x & 63;
  constexpr int RPI = 64 / NCH;          // rows per store instruction
#pragma unroll
  for (int it = 0; it < 32 / RPI; ++it) {
    const int r = it * RPI + lane / NCH, c = lane % NCH;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(slab + r * (NCH * 16) + ((c ^ (r & (NCH - 1))) << 4));
    if (r < nvalid) *reinterpret_cast<bf16x8*>(base + (int64_t)r * rstride + c * 8) = v;
  }
}

// Per-lane plan for one 64-key K/V tile: swizzled LDS offsets of the ds_read_b128 row reads and the
// ds_read_b64_tr_b16 transposed reads, and the LDS-DMA source offsets of the staging loads.  Computed once
// per kernel so the tile loop issues loads with immediate offsets instead of recomputing the XOR swizzle.
// Row offsets repeat with period KP sub-tiles (32 rows) and tr offsets with period TRP k-steps (16 rows):
// Lane id as a value the compiler must treat as redefined here: what is derived from it is recomputed at the use
// instead of being hoisted out of the tile loop and kept live (at 256 VGPRs such hoisted lane constants were spilled,
// and the reload's compiler-inserted vmcnt(0) drained the in-flight LDS-DMA prefetch right after it was issued).
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// img_off's line permutation depends on (line & 15) only, so advancing 16 lines is a pure byte offset.
template <int HD, int NT_ = 256>
struct KVTilePlan {
  static constexpr int BN = 64, NT = NT_, NC = HD / 8, KS = HD / 16, DT = HD / 32, TILE = BN * HD * 2;
  static constexpr int KP = NC >= 8 ? 1 : 2;
  static constexpr int TRP = NC >= 16 ? 1 : (NC == 8 ? 2 : 4);
  static constexpr int NS = BN * NC / NT;
  static_assert(BN * NC % NT == 0, "tile must split evenly over the workgroup");
  int kro[KP][KS];
  int tro[TRP][DT][2];
  int kgo[NS];  // staging source offsets (elements), valid when K and V share the sequence stride

  __device__ __forceinline__ void init(int lane, int64_t k_ss) {
    const int h = lane >> 5, l32 = lane & 31, g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
#pragma unroll
    for (int sp = 0; sp < KP; ++sp)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) kro[sp][kk] = img_off<NC>(sp * 32 + l32, kk * 2 + h);
#pragma unroll
    for (int kp = 0; kp < TRP; ++kp)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int hi = 0; hi < 2; ++hi)
          tro[kp][dt][hi] = img_off<NC>(kp * 16 + 4 * (g >> 1) + tq + 8 * hi, dt * 4 + 2 * (g & 1) + (tp >> 1)) +
                            8 * (tp & 1);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int L = threadIdx.x + NT * i, line = L >> 4, slot = L & 15;
      const int F = (line << 4) + (slot ^ (((line & 3) << 2) | ((line >> 2) & 3)));
      kgo[i] = (F / NC) * (int)k_ss + (F % NC) * 8;
    }
  }
  __device__ __forceinline__ int row(int sub, int kk) const {
    return KP == 1 ? kro[0][kk] + sub * 32 * NC * 16 : kro[sub][kk];
  }
  __device__ __forceinline__ int tr(int ks, int dt, int hi) const {
    return tro[ks % TRP][dt][hi] + (ks / TRP) * TRP * 16 * NC * 16;
  }
  // K and V tile [k0, k0 + 64) -> image pair at img (K) / img + TILE (V).  Full tiles use the hoisted
  // offsets; the ragged last tile clamps rows to Sk - 1 (finite data the caller masks).
  __device__ __forceinline__ void stage(char* img, const bf16* kp, const bf16* vp, int64_t k_ss, int64_t v_ss,
                                        int k0, int Sk) const {
    if (k0 + BN <= Sk && k_ss == v_ss) {
      const bf16* kt = kp + (int64_t)k0 * k_ss;
      const bf16* vt = vp + (int64_t)k0 * v_ss;
      const int wave = threadIdx.x >> 6;
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        auto* dst = (__attribute__((address_space(3))) void*)(img + (wave * 64 + NT * i) * 16);
        __builtin_amdgcn_global_load_lds((const void*)(kt + kgo[i]), dst, 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        auto* dst = (__attribute__((address_space(3))) void*)(img + TILE + (wave * 64 + NT * i) * 16);
        __builtin_amdgcn_global_load_lds((const void*)(vt + kgo[i]), dst, 16, 0, 0);
      }
    } else {
      glds_stage<NC, BN, NT>(img, kp, k_ss, k0, Sk);
      glds_stage<NC, BN, NT>(img + TILE, vp, v_ss, k0, Sk);
    }
  }

  // The same copy issued as inline-asm LDS-DMA (lds_dma16): invisible to hipcc's wait bookkeeping, which otherwise
  // drains the in-flight prefetch (vmcnt(0)) before the first ds_read of the CURRENT tile's V image (it cannot prove
  // the two images disjoint).  The caller retires it with wait_vmcnt<0>() + s_barrier before reading `img`.
  // `lds_w` is this wave's byte address of the image pair (lds_addr(img + wave * 1 KiB)).
  // Instruction i of a lane copies chunk L = tid + NT i; with NT a multiple of 256 the swizzle of its 256-B line is that
  // of i = 0, so its source row is prow + i NT / NC and its chunk column pch: ONE row / column pair per lane (a per-i
  // table is spilled around the tile loop at high register pressure, and hipcc's vmcnt(0) for the reload would drain
  // the in-flight DMA).
  // RECOMPUTE: the row / column pair is recomputed from an opaque lane id per call (a few VALU) rather than kept
  // live across the tile loop -- the dQ kernel spilled the hoisted per-instruction offsets and each reload's vmcnt(0)
  // drained the DMA issued just before it; the forward (no spills) keeps the pair from init_async().
  static_assert(NT % 256 == 0, "stage_async assumes whole 16-line swizzle periods per instruction");
  static constexpr int RSTEP = NT / NC;   // rows between a lane's consecutive instructions
  int prow0 = 0, pch0 = 0;
  __device__ __forceinline__ static void lane_chunk(int L, int& prow, int& pch) {
    const int line = L >> 4, slot = L & 15;
    const int F = (line << 4) + (slot ^ (((line & 3) << 2) | ((line >> 2) & 3)));
    prow = F / NC;
    pch = (F % NC) * 8;
  }
  __device__ __forceinline__ void init_async() { lane_chunk(threadIdx.x, prow0, pch0); }
  template <bool RECOMPUTE = false>
  __device__ __forceinline__ void stage_async(unsigned lds_w, const bf16* kp, const bf16* vp, int64_t k_ss,
                                              int64_t v_ss, int k0, int Sk) const {
    int prow = prow0, pch = pch0;
    if constexpr (RECOMPUTE) lane_chunk(opaque_tid(), prow, pch);
    // wave-uniform by construction; readfirstlane keeps the bases in SGPRs inside divergent callers
    const bf16* kt = uniform_ptr(kp + (int64_t)k0 * k_ss);
    const bf16* vt = uniform_ptr(vp + (int64_t)k0 * v_ss);
    if (k0 + BN <= Sk) {   // full tile: byte offsets step by a wave-uniform constant
      const unsigned ok = (unsigned)((prow * k_ss + pch) * 2), ov = (unsigned)((prow * v_ss + pch) * 2);
      const unsigned sk = (unsigned)(RSTEP * k_ss * 2), sv = (unsigned)(RSTEP * v_ss * 2);
#pragma unroll
      for (int i = 0; i < NS; ++i) lds_dma16(kt, ok + i * sk, lds_w + NT * i * 16);
#pragma unroll
      for (int i = 0; i < NS; ++i) lds_dma16(vt, ov + i * sv, lds_w + TILE + NT * i * 16);
    } else {                // ragged last tile: rows past the end re-read the last valid row
      const int rmax = Sk - 1 - k0;
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int r = min(prow + i * RSTEP, rmax);
        lds_dma16(kt, (unsigned)((r * k_ss + pch) * 2), lds_w + NT * i * 16);
        lds_dma16(vt, (unsigned)((r * v_ss + pch) * 2), lds_w + TILE + NT * i * 16);
      }
    }
  }
};

// glds_stage issued through lds_dma16 (see KVTilePlan::stage_async): ROWS x NC chunks of rows [row0, row0 + ROWS) of a
// strided tile, rows past `nvalid` re-reading the last valid one.  `lds_w` = lds_addr(img + wave * 1 KiB).  A lane's
// source row / chunk are recomputed from an opaque lane id per call (a few VALU) instead of a hoisted per-lane table;
// with NT a multiple of 256 instruction i's chunk lies 16 image lines (RSTEP rows) below instruction 0's.
template <int NC, int ROWS, int NT>
struct RowStagePlan {
  static constexpr int CHUNKS = ROWS * NC, NI = (CHUNKS + NT - 1) / NT, RSTEP = NT / NC;
  static_assert(NT % 256 == 0, "RowStagePlan assumes whole 16-line swizzle periods per instruction");
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void stage(unsigned lds_w, const bf16* base, int64_t rstride, int row0,
                                        int nvalid) const {
    const int tid = opaque_tid(), line = tid >> 4, slot = tid & 15;
    const int F = (line << 4) + (slot ^ (((line & 3) << 2) | ((line >> 2) & 3)));
    const int prow = F / NC, pch = (F % NC) * 8;
    const int rmax = nvalid - 1 - row0;
    const bf16* t = uniform_ptr(base + (int64_t)row0 * rstride);   // wave-uniform: keep it in SGPRs
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if (CHUNKS % NT == 0 || tid + NT * i < CHUNKS)
        lds_dma16(t, (unsigned)(((int64_t)min(prow + i * RSTEP, rmax) * rstride + pch) * 2), lds_w + NT * i * 16);
  }
};

// Logical (x, y, z) of a workgroup launched on a 1-D grid of nx*ny*nz blocks, XCD-aware (xcd_remap) with x fastest:
// the workgroups of one (batch, head) -- which all stream the same K/V (or Q/dO) -- run on one XCD and share its L2
// instead of every XCD fetching every head.
__device__ __forceinline__ void xcd_block(int nx, int ny, int& x, int& y, int& z, int n) {
  const int logical = xcd_remap(blockIdx.x, n);
  x = logical % nx;
  y = (logical / nx) % ny;
  z = logical / (nx * ny);
}

// Number of 64-key tiles a 32-query wave (first query q0w) must visit: causal waves stop at their last
// visible key; the workgroup still loops to its own end for the shared staging / barriers.
template <bool CAUSAL>
__device__ __forceinline__ int wave_tile_count(int ntiles, int q0w, int off) {
  if (!CAUSAL) return ntiles;
  const int last = q0w + 31 + off;
  return last < 0 ? 0 : min(ntiles, last / 64 + 1);
}

// ==================================================================================================
// Forward
// ==================================================================================================
// Online softmax in log2 units with the 1/sqrt(d) scale folded into one FMA per score:
//   p = exp2(s * scale*log2e - m).  The running max m is only raised (and O, l rescaled) when some lane's
// tile max exceeds it by more than RESCALE_THR (FA4-style lazy rescaling): p is then bounded by 2^THR,
// harmless for the bf16 P operand and the fp32 accumulators, and the exact result is recovered by the
// final 1/l.  The rescale branch is wave-uniform (ballot), so steady-state tiles skip 16*DT multiplies.
// Rejected round-4/5 variants of this kernel (evidence kept under profiles/): 8-wave workgroups (819-822 vs 834-838
// TFLOP/s), waves 4..7 staggered one barrier behind (809-814), issue priority over the MFMA chains (within noise),
// and a software-pipelined body that overlaps each wave's softmax with its own next QK^T (754-788 vs 831-833,
// profiles/r5/attn_fwd_pipe/).
template <int HD, bool CAUSAL, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(AttnParams p) {
  constexpr int NW = 4;
  using Plan = KVTilePlan<HD, 64 * NW>;
  constexpr int BM = 32 * NW, BN = Plan::BN, KS = Plan::KS, DT = Plan::DT, TILE = Plan::TILE;
  constexpr float RESCALE_THR = 8.f;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (p.Sq + BM - 1) / BM;
  int bx, hq, b;
  xcd_block(nqb, p.Hq, bx, hq, b, nqb * p.Hq * p.B);
  const int qb = CAUSAL ? nqb - 1 - bx : bx;  // heaviest causal blocks first
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int myq = q0w + l32;
  const int off = p.Sk - p.Sq;

  const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[myq][16*kk + 8h .. +7].
  bf16x8 qf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
    qf[kk] = (myq < p.Sq) ? *reinterpret_cast<const bf16x8*>(qp + (int64_t)myq * p.q_ss + kk * 16 + 8 * h) : zero8();

  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + off);
  const int ntiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;
  const int wtiles = wave_tile_count<CAUSAL>(ntiles, q0w, off);

  Plan plan;
  plan.init(lane, p.k_ss);
  plan.init_async();
  const unsigned lds_w = lds_addr(smem + (threadIdx.x >> 6) * 64 * 16);

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  const f32x16 zacc = {};
  float m = -INFINITY, lsum = 0.f;  // m: running max of s*sl2; lsum: this half-wave's partial row sum
  const float sl2 = p.scale * 1.4426950408889634f;
  const unsigned drk = DROP ? attn_row_key(p.drop_seed, (unsigned)(b * p.Hq + hq), (unsigned)myq) : 0u;
  const unsigned dthr = DROP ? attn_drop_thr(p.drop_p) : 0u;

  if (ntiles > 0) plan.stage_async(lds_w, kp, vp, p.k_ss, p.v_ss, 0, p.Sk);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  auto tile = [&](const char* Kl, const char* Vl, int k0, bool need_mask) {
    // ---- S^T = K Q^T for two 32-key sub-tiles ----
    // all 2 x KS K fragments are read before the MFMA chains (counted lgkmcnt waits): read one, wait, multiply
    // exposed a full LDS round trip per MFMA
    bf16x8 kf[2][KS];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) kf[sub][kk] = lds_b128(Kl, plan.row(sub, kk));
    f32x16 s[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      s[sub] = mfma32(kf[sub][0], qf[0], zacc);
#pragma unroll
      for (int kk = 1; kk < KS; ++kk) s[sub] = mfma32(kf[sub][kk], qf[kk], s[sub]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * KS, 0);   // the DS reads first ...
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * KS, 0);   // ... then the MFMAs
    // phase fences keep the scheduler from hoisting the next phase's LDS reads into this one's live range
    __builtin_amdgcn_sched_barrier(0);
    if (need_mask) {  // wave-uniform: only diagonal / ragged tiles pay for the selects
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + sub * 32 + acc_row(r, h);
          s[sub][r] = (key >= p.Sk || (CAUSAL && key > myq + off)) ? -INFINITY : s[sub][r];
        }
    }
    float mx = fmaxf(s[0][0], s[1][0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
    mx = half_max(mx) * sl2;
    if (__ballot(mx > m + RESCALE_THR)) {
      const float mn = fmaxf(m, mx);
      const float alpha = mn == -INFINITY ? 1.f : exp2_(m - mn);
      lsum *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      m = mn;
    }
    const float mneg = m == -INFINITY ? 0.f : -m;
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[0][r] = exp2_(fmaf(s[0][r], sl2, mneg));
      s[1][r] = exp2_(fmaf(s[1][r], sl2, mneg));
      ls0 += s[0][r];
      ls1 += s[1][r];
    }
    lsum += ls0 + ls1;
    if constexpr (DROP) {   // after the row sum: the normaliser is the undropped softmax's
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (!attn_keep(drk, (unsigned)(k0 + sub * 32 + acc_row(r, h)), dthr)) s[sub][r] = 0.f;
    }

    // ---- P^T as B operand: k-step ks covers keys 16*ks .. 16*ks+15 of the tile ----
    bf16x8 pf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[ks][j] = (bf16)s[ks >> 1][8 * (ks & 1) + j];
    // no fence before the PV MFMAs: the compiler overlaps the first PV k-steps with the tail of the exp / convert work
    // (+2 % forward TFLOP/s at B 8, H 32, S 4096, D 128; the backward kernels keep their fences: -2 % without them)

    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        o[dt] = mfma32(lds_tr2(Vl, plan.tr(ks, dt, 0), plan.tr(ks, dt, 1)), pf[ks], o[dt]);
  };

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) plan.stage_async(lds_w + (buf ^ 1) * 2 * TILE, kp, vp, p.k_ss, p.v_ss, (t + 1) * BN, p.Sk);
    const char* Kl = smem + buf * 2 * TILE;
    if (t < wtiles) {
      const int k0 = t * BN;
      tile(Kl, Kl + TILE, k0, (k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0w + off)));
    }
    wait_vmcnt<0>();   // this wave's share of tile t+1 has landed ...
    __builtin_amdgcn_s_barrier();   // ... and every wave's, and nobody reads tile t's images any more
  }

  // ---- epilogue: O = O^T / l, lse ----
  lsum = half_sum(lsum);
  if (myq < p.Sq && p.acc_o) {
    // ring merge into the fp32 accumulators (both half-waves read the old lse before half 0 writes the new one:
    // one instruction stream, loads issued first)
    const float inv = lsum > 0.f ? (DROP ? 1.f / (1.f - p.drop_p) : 1.f) / lsum : 0.f;
    const float lse_b = lsum > 0.f ? (m + __log2f(lsum)) * 0.6931471805599453f : -INFINITY;
    float* al = p.acc_lse + (int64_t)b * p.al_sb + (int64_t)hq * p.al_sh + myq;
    const float old = *al;
    const float mx = fmaxf(old, lse_b);
    float w1 = 0.f, w2 = 0.f, nl = -INFINITY;
    if (mx != -INFINITY) {
      const float e1 = __expf(old - mx), e2 = __expf(lse_b - mx), sum = e1 + e2;
      nl = mx + __logf(sum);
      w1 = e1 / sum;
      w2 = e2 / sum * inv;
    }
    float* ao = p.acc_o + (int64_t)b * p.ao_sb + (int64_t)myq * p.ao_ss + (int64_t)hq * p.ao_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        f32x4* ptr = reinterpret_cast<f32x4*>(ao + dt * 32 + 8 * gg + 4 * h);
        f32x4 cur = *ptr;
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = cur[j] * w1 + o[dt][4 * gg + j] * w2;
        *ptr = cur;
      }
    if (h == 0) *al = nl;
  } else if (!p.acc_o) {
    // O = O^T / l through this wave's LDS slab (the K/V images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= 4 * TILE, "epilogue slabs exceed the forward kernel's LDS");
    const float inv = lsum > 0.f ? (DROP ? 1.f / (1.f - p.drop_p) : 1.f) / lsum : 0.f;
    bf16* o0 = (bf16*)p.o + (int64_t)b * p.o_sb + (int64_t)q0w * p.o_ss + (int64_t)hq * p.o_sh;
    store_rows_lds<DT>(smem + wid * (32 * HD * 2), o0, p.o_ss, min(32, p.Sq - q0w), o, inv, h, l32, 0, nullptr,
                       nullptr, 0);
    if (myq < p.Sq && h == 0 && p.lse)
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + myq] =
          lsum > 0.f ? (m + __log2f(lsum)) * 0.6931471805599453f : -INFINITY;
  }
}

// ==================================================================================================
// Backward
// ==================================================================================================
// delta[b, h, q] = sum_d dO[b,q,h,d] * O[b,q,h,d] (fp32).  TPR = D/8 lanes per row, 8 elements per lane;
// rows are enumerated (b, q, h) so a wave reads 64 * 16 contiguous bytes of each [B, S, H, D] operand.
template <int TPR>
__global__ __launch_bounds__(256) void attn_delta_k(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                    float* __restrict__ delta, int B, int S, int H,
                                                    int64_t o_sb, int64_t o_ss, int64_t o_sh, int64_t d_sb,
                                                    int64_t d_ss, int64_t d_sh) {
  constexpr int RPB = 256 / TPR;  // rows per block-iteration
  const int sub = threadIdx.x % TPR;
  const int64_t rows = (int64_t)B * H * S;
  for (int64_t r = (int64_t)blockIdx.x * RPB + threadIdx.x / TPR; r < rows; r += (int64_t)gridDim.x * RPB) {
    const int hh = (int)(r % H);
    const int64_t bq = r / H;
    const int q = (int)(bq % S), bb = (int)(bq / S);
    float x[8], y[8];
    Vec8<bf16>::load(o + bb * o_sb + (int64_t)q * o_ss + hh * o_sh + sub * 8, x);
    Vec8<bf16>::load(dout + bb * d_sb + (int64_t)q * d_ss + hh * d_sh + sub * 8, y);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += x[k] * y[k];
#pragma unroll
    for (int m = TPR / 2; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
    if (sub == 0) delta[((int64_t)bb * H + hh) * S + q] = acc;
  }
}

// ---- dK / dV: KV-stationary.  One workgroup = 4 waves = 128 keys of one (batch, kv head); one wave =
// 32 keys whose K^T / V^T B-operand fragments stay in registers.  The workgroup sweeps every query head
// of the GQA group x 32-row query tiles (double-buffered Q / dO LDS images, one barrier per tile).
// S and dP are computed with the key on the lane, so P and dS are directly the B operands of
// dV^T += dO^T P and dK^T += Q^T dS: no LDS round trip, no atomics.
// The dV / dK transposed reads are software-pipelined one step ahead (the first step issued before the softmax), and a
// wave runs at issue priority 1 while in its MFMA chains (S / dP, then dV / dK) and 0 in its softmax, so the partner
// wave on the SIMD (the other workgroup's) fills the chains' gaps with its softmax instead of competing for issue
// (round 3/4 A/B: +2 % and +1 %; row constants as the initial S / dP accumulators measured -2 % and were removed).
template <int HD, bool CAUSAL, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_k(AttnBwdParams P) {
  constexpr int NW = 4;
  constexpr int NT = 64 * NW, BNK = 32 * NW, BMQ = 32, NC = HD / 8, KS = HD / 16, DT = HD / 32;
  constexpr bool RINIT = false;
  constexpr bool TRPIPE = true;
  constexpr int QIMG = BMQ * HD * 2;        // Q / dO tile image [32 q][HD]
  constexpr int KIMG = BNK * HD * 2;        // K image [128 keys][HD] (B operand of S = Q K^T)
  // img_off's line permutation repeats every 16 lines.  For NC >= 8, rows r and r + 32 are a multiple of 16
  // lines apart, so the wave's K rows reuse the Q-image offsets plus a constant.
  constexpr bool KSHARE = NC >= 8;
  constexpr bool TRADD = NC >= 16;          // +16 rows is a pure byte offset for the transposed reads
  // smem: K | Q0 | dO0 | Q1 | dO1 | -lse2[2][32] | delta[2][32] | dropout row keys[2][32]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kimg = smem;
  char* Qbuf = smem + KIMG;
  float* lse_s = reinterpret_cast<float*>(Qbuf + 4 * QIMG);
  float* del_s = lse_s + 2 * BMQ;
  unsigned* rk_s = reinterpret_cast<unsigned*>(del_s + 2 * BMQ);

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int nkb = (p.Sk + BNK - 1) / BNK;
  int kbx, hk, b;
  xcd_block(nkb, p.Hkv, kbx, hk, b, nkb * p.Hkv * p.B);
  const int kb0 = kbx * BNK;   // ascending = heaviest causal key blocks first
  const int grp = p.Hq / p.Hkv;
  const int off = p.Sk - p.Sq;
  const int key0 = kb0 + wid * 32;
  const int mykey = key0 + l32;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;
  glds_stage<NC, BNK, NT>(Kimg, kp, p.k_ss, kb0, p.Sk);
  bf16x8 vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
    vf[kk] = mykey < p.Sk ? *reinterpret_cast<const bf16x8*>(vp + (int64_t)mykey * p.v_ss + kk * 16 + 8 * h)
                          : zero8();
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }
  const f32x16 zacc = {};

  // per-lane LDS offsets.  For HD = 128 (NC = 16, one 256-B image line per row) every offset is one per-lane base
  // XOR / plus compile-time constants: the row read of chunk 2kk + h is qb ^ (kk << 5), and the transposed read of
  // (dt, hi) is tb ^ (dt << 6) ^ (hi << 5) + hi * 2048 (img_off's swizzle f(row) XORs bits 4-7 only, and row + 8
  // flips bit 1 of f).  Two registers instead of 16 (at 256 VGPRs the tables were spilled around the tile loop).
  // The two bases are recomputed from an opaque lane id at the top of every tile (a few VALU), so they are not
  // carried across the loop at all.
  constexpr bool XOFS = NC == 16;
  int qro[XOFS ? 1 : KS];
#pragma unroll
  for (int kk = 0; kk < (XOFS ? 1 : KS); ++kk) qro[kk] = img_off<NC>(l32, kk * 2 + h);
  auto qofs = [&](int kk) { return XOFS ? qro[0] ^ (kk << 5) : qro[kk]; };

  auto kofs = [&](int kk) {
    return KSHARE ? qofs(kk) + wid * 32 * NC * 16 : img_off<NC>(wid * 32 + l32, kk * 2 + h);
  };
  int tro[XOFS ? 1 : (TRADD ? 1 : 2)][XOFS ? 1 : DT][XOFS ? 1 : 2];
#pragma unroll
  for (int ks = 0; ks < (XOFS ? 1 : (TRADD ? 1 : 2)); ++ks)
#pragma unroll
    for (int dt = 0; dt < (XOFS ? 1 : DT); ++dt)
#pragma unroll
      for (int hi = 0; hi < (XOFS ? 1 : 2); ++hi)
        tro[ks][dt][hi] = img_off<NC>(ks * 16 + 4 * (g >> 1) + tq + 8 * hi, dt * 4 + 2 * (g & 1) + (tp >> 1)) +
                          8 * (tp & 1);
  auto trofs = [&](int ks, int dt, int hi) {
    if constexpr (XOFS) return (tro[0][0][0] ^ (dt << 6) ^ (hi << 5)) + hi * 2048 + ks * 16 * NC * 16;
    return TRADD ? tro[0][dt][hi] + ks * 16 * NC * 16 : tro[ks][dt][hi];
  };
  auto rebase = [&]() {
    if constexpr (XOFS) {
      const int ln = opaque_tid() & 63, lh = ln >> 5, lg = ln >> 4, ltq = (ln & 15) >> 2, ltp = ln & 3;
      qro[0] = img_off<NC>(ln & 31, lh);
      tro[0][0][0] = img_off<NC>(4 * (lg >> 1) + ltq, 2 * (lg & 1) + (ltp >> 1)) + 8 * (ltp & 1);
    }
  };

  int qstart = 0;
  if (CAUSAL) qstart = max(0, kb0 - off) / BMQ * BMQ;
  const int nqt_head = qstart < p.Sq ? (p.Sq - qstart + BMQ - 1) / BMQ : 0;
  const int total = nqt_head * grp;

  // Q / dO tiles are prefetched by inline-asm LDS-DMA (RowStagePlan), retired by the explicit wait_vmcnt<0>() ahead
  // of the end-of-tile barrier: with the compiler-visible builtin, hipcc drained the whole prefetch (vmcnt(0))
  // before the transposed reads of the CURRENT tile.  The lse / delta row scalars are loaded raw and only scaled
  // when written to LDS at the end of the tile, so their loads are not waited for (and, vmcnt retiring in order,
  // the DMA behind them with it) at the top of the tile either.
  RowStagePlan<NC, BMQ, NT> qplan;
  qplan.init();
  const unsigned lds_q = lds_addr(Qbuf + wid * 64 * 16);
  float st_lse = 0.f, st_del = 0.f;
  unsigned st_rk = 0u;
  // lse / delta rows of this (batch, kv head)'s GQA group: grp * Sq floats from the group's first query head
  const int64_t grow = ((int64_t)b * p.Hq + (int64_t)hk * grp) * p.Sq;
  const auto lse_rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(p.lse + grow), 0, grp * p.Sq * 4, 0x00020000);
  const auto del_rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(P.delta + grow), 0, grp * p.Sq * 4, 0x00020000);
  const unsigned dthr = DROP ? attn_drop_thr(p.drop_p) : 0u;
  const float drs = DROP ? 1.f / (1.f - p.drop_p) : 1.f;
  auto stage = [&](int it, int buf) {
    const int hq = hk * grp + it / nqt_head;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
    const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
    const unsigned ql = lds_q + buf * 2 * QIMG;
    qplan.stage(ql, qp, p.q_ss, qt0, p.Sq);
    qplan.stage(ql + QIMG, dop, P.do_ss, qt0, p.Sq);
    const int tid = opaque_tid();
    if (tid < BMQ) {
      // buffer loads off the GQA group's lse / delta rows (scalar resources built once, below): only the 32-bit lane
      // offset is a VGPR (a per-lane 64-bit address was spilled and its reload drained the Q / dO prefetch above)
      const int q = min(qt0 + tid, p.Sq - 1);   // rows past Sq: finite, masked by the caller
      const int o = ((it / nqt_head) * p.Sq + q) * 4;
      st_lse = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lse_rs, o, 0, 0));
      st_del = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(del_rs, o, 0, 0));
      if constexpr (DROP) st_rk = attn_row_key(p.drop_seed, (unsigned)(b * p.Hq + hq), (unsigned)(qt0 + tid));
    }
  };
  // Row constants: without dropout they become the INITIAL accumulators of the S and dP chains (S' = Q K^T - lse/scale,
  // dP' = dO V^T - delta), so p = exp2(S' scale log2e) and dS = p dP' need no per-element row reads after the chains
  // (cdna_hip_programming.md 'Row constants as the initial accumulator'); dropout keeps the explicit form.
  const float inv_scale = 1.f / p.scale;
  auto stage_scalars = [&](int buf) {
    if (threadIdx.x < BMQ) {
      if constexpr (!RINIT) {
        lse_s[buf * BMQ + threadIdx.x] = -st_lse * 1.4426950408889634f;  // -lse in log2 units
        del_s[buf * BMQ + threadIdx.x] = st_del;
        if constexpr (DROP) rk_s[buf * BMQ + threadIdx.x] = st_rk;
      } else {
        lse_s[buf * BMQ + threadIdx.x] = -st_lse * inv_scale;
        del_s[buf * BMQ + threadIdx.x] = -st_del;
      }
    }
  };
  // accumulator register r holds query row acc_row(r, h) = (r & 3) + 8 (r >> 2) + 4 h: four 16-B row reads
  auto row_init = [&](const float* rows) {
    f32x16 a;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(rows + 8 * j + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[4 * j + i] = v[i];
    }
    return a;
  };

  if (total > 0) {
    stage(0, 0);
    stage_scalars(0);
  }
  wait_vmcnt<0>();
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    if (it + 1 < total) stage(it + 1, buf ^ 1);
    const char* Ql = Qbuf + buf * 2 * QIMG;
    const char* Ol = Ql + QIMG;
    // a wave whose 32 keys are all hidden from this query tile by the causal mask skips the tile
    if (!(CAUSAL && key0 > qt0 + BMQ - 1 + off)) {
      const float* ls = lse_s + buf * BMQ;
      const float* ds = del_s + buf * BMQ;
      rebase();
      __builtin_amdgcn_s_setprio(1);
      f32x16 s = mfma32(lds_b128(Ql, qofs(0)), lds_b128(Kimg, kofs(0)), RINIT ? row_init(ls) : zacc);
      f32x16 dp = mfma32(lds_b128(Ol, qofs(0)), vf[0], RINIT ? row_init(ds) : zacc);
#pragma unroll
      for (int kk = 1; kk < KS; ++kk) {
        s = mfma32(lds_b128(Ql, qofs(kk)), lds_b128(Kimg, kofs(kk)), s);
        dp = mfma32(lds_b128(Ol, qofs(kk)), vf[kk], dp);
      }
      __builtin_amdgcn_s_setprio(0);
      // wave-uniform: only diagonal / ragged tiles pay for the selects (masked scores -> -inf -> P = 0)
      if ((qt0 + BMQ > p.Sq) || (key0 + 32 > p.Sk) || (CAUSAL && key0 + 31 > qt0 + off)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = qt0 + acc_row(r, h);
          s[r] = (q >= p.Sq || mykey >= p.Sk || (CAUSAL && mykey > q + off)) ? -INFINITY : s[r];
        }
      }
      // TRPIPE: the first dV / dK step's transposed operands are read now, their latency covered by the softmax
      bf16x8 tro_o[2], tro_q[2];
      if constexpr (TRPIPE) {
        tro_o[0] = lds_tr2(Ol, trofs(0, 0, 0), trofs(0, 0, 1));
        tro_q[0] = lds_tr2(Ql, trofs(0, 0, 0), trofs(0, 0, 1));
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if constexpr (RINIT) {
          const float pv = exp2_(s[r] * sl2);
          s[r] = pv;
          dp[r] = pv * dp[r];
        } else if constexpr (DROP) {   // dV from the dropped, rescaled P; dS = P (Z dP / (1-p) - delta)
          const int qr = acc_row(r, h);
          const float pv = exp2_(fmaf(s[r], sl2, ls[qr]));
          const bool keep = attn_keep(rk_s[buf * BMQ + qr], (unsigned)mykey, dthr);
          s[r] = keep ? pv * drs : 0.f;
          dp[r] = pv * ((keep ? dp[r] * drs : 0.f) - ds[qr]);
        } else {
          const int qr = acc_row(r, h);
          const float pv = exp2_(fmaf(s[r], sl2, ls[qr]));
          s[r] = pv;
          dp[r] = pv * (dp[r] - ds[qr]);
        }
      }
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[ks][j] = (bf16)s[8 * ks + j];
          sb[ks][j] = (bf16)dp[8 * ks + j];
        }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (TRPIPE) {
        // step i = (ks, dt): its operands were read one step earlier; each step issues the next step's 4 reads
        // ahead of its own 2 MFMAs
#pragma unroll
        for (int i = 0; i < 2 * DT; ++i) {
          const int ks = i / DT, dt = i % DT;
          if (i + 1 < 2 * DT) {
            const int k2 = (i + 1) / DT, d2 = (i + 1) % DT;
            tro_o[(i + 1) & 1] = lds_tr2(Ol, trofs(k2, d2, 0), trofs(k2, d2, 1));
            tro_q[(i + 1) & 1] = lds_tr2(Ql, trofs(k2, d2, 0), trofs(k2, d2, 1));
          }
          dv[dt] = mfma32(tro_o[i & 1], pb[ks], dv[dt]);
          dk[dt] = mfma32(tro_q[i & 1], sb[ks], dk[dt]);
          if (i + 1 < 2 * DT) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int o0 = trofs(ks, dt, 0), o1 = trofs(ks, dt, 1);
            dv[dt] = mfma32(lds_tr2(Ol, o0, o1), pb[ks], dv[dt]);
            dk[dt] = mfma32(lds_tr2(Ql, o0, o1), sb[ks], dk[dt]);
          }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (it + 1 < total) stage_scalars(buf ^ 1);
    wait_vmcnt<0>();
    __syncthreads();
  }

  {   // dK then dV through this wave's LDS slab (the K and Q / dO images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= KIMG + 4 * QIMG, "epilogue slabs exceed the dK/dV kernel's LDS");
    const int nvalid = min(32, p.Sk - key0);
    bf16* dk0 = (bf16*)P.dk + (int64_t)b * P.dk_sb + (int64_t)key0 * P.dk_ss + (int64_t)hk * P.dk_sh;
    bf16* dv0 = (bf16*)P.dv + (int64_t)b * P.dv_sb + (int64_t)key0 * P.dv_ss + (int64_t)hk * P.dv_sh;
    char* slab = smem + wid * (32 * HD * 2);
    store_rows_lds<DT>(slab, dk0, P.dk_ss, nvalid, dk, p.scale, h, l32, mykey, P.rope_cos, P.rope_sin, P.rope_off);
    store_rows_lds<DT>(slab, dv0, P.dv_ss, nvalid, dv, 1.f, h, l32, mykey, nullptr, nullptr, 0);
  }
}

// ---- dQ: Q-stationary, the forward's structure.  One workgroup = 4 waves = 128 queries; a lane owns one
// query (lane & 31).  Per 64-key tile: S^T = K Q^T and dP^T = V dO^T (A = K / V rows from LDS, B = Q^T / dO^T
// fragments in registers), P^T = exp2(S^T c - lse) and dS^T = P^T (dP^T - delta) lane-locally (lse and delta
// are one scalar per lane), then dQ^T += K^T dS^T with dS^T consumed straight from the accumulator.
// K / V fragments are read a quarter sub-tile ahead of their MFMAs (KQ = 4: no register spills; the half-sub-tile form
// spilled 3 registers).  Rejected A/B variants (profiles/r4/attn_dq/, attn_prio/): the dQ product's transposed K reads
// software-pipelined one MFMA ahead, and issue priority over the MFMA chains.
template <int HD, bool CAUSAL, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_k(AttnBwdParams P) {
  constexpr int NW = 4, KQ = 4;
  constexpr bool PF = false, PRIO = false;
  using Plan = KVTilePlan<HD, 64 * NW>;
  constexpr int BM = 32 * NW, BN = Plan::BN, KS = Plan::KS, DT = Plan::DT, TILE = Plan::TILE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (p.Sq + BM - 1) / BM;
  int bx, hq, b;
  xcd_block(nqb, p.Hq, bx, hq, b, nqb * p.Hq * p.B);
  const int qb = CAUSAL ? nqb - 1 - bx : bx;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int myq = q0w + l32;
  const int off = p.Sk - p.Sq;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  bf16x8 qf[KS], df[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const bool ok = myq < p.Sq;
    qf[kk] = ok ? *reinterpret_cast<const bf16x8*>(qp + (int64_t)myq * p.q_ss + kk * 16 + 8 * h) : zero8();
    df[kk] = ok ? *reinterpret_cast<const bf16x8*>(dop + (int64_t)myq * P.do_ss + kk * 16 + 8 * h) : zero8();
  }
  float nlse2 = 0.f, delta = 0.f;  // -lse in log2 units
  if (myq < p.Sq) {
    const int64_t idx = ((int64_t)b * p.Hq + hq) * p.Sq + myq;
    nlse2 = -p.lse[idx] * 1.4426950408889634f;
    delta = P.delta[idx];
  }

  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + off);
  const int ntiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;
  const int wtiles = wave_tile_count<CAUSAL>(ntiles, q0w, off);
  const unsigned drk = DROP ? attn_row_key(p.drop_seed, (unsigned)(b * p.Hq + hq), (unsigned)myq) : 0u;
  const unsigned dthr = DROP ? attn_drop_thr(p.drop_p) : 0u;
  const float drs = DROP ? 1.f / (1.f - p.drop_p) : 1.f;

  Plan plan;
  plan.init(lane, p.k_ss);
  plan.init_async();
  const unsigned lds_w = lds_addr(smem + (threadIdx.x >> 6) * 64 * 16);

  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;
  const f32x16 zacc = {};

  if (ntiles > 0) plan.template stage_async<true>(lds_w, kp, vp, p.k_ss, p.v_ss, 0, p.Sk);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  auto tile = [&](const char* Kl, const char* Vl, int k0, bool need_mask) {
    bf16x8 sf[4];
    bf16x8 tk[2];   // PF: ring of transposed K operands, step i = (ks, dt) = (i / DT, i % DT)
    auto tk_read = [&](int i) { return lds_tr2(Kl, plan.tr(i / DT, i % DT, 0), plan.tr(i / DT, i % DT, 1)); };
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      // K and V fragments are read a half sub-tile (KH k-steps) ahead of their MFMAs with counted lgkmcnt waits
      // (one read + wait + multiply at a time exposed an LDS round trip per MFMA; all KS at once spills)
      constexpr int NQ = KS >= KQ ? KQ : KS, KH = KS / NQ;
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      f32x16 s = zacc, dp = zacc;
#pragma unroll
      for (int half = 0; half < NQ; ++half) {
        bf16x8 kf[KH], vf[KH];
#pragma unroll
        for (int j = 0; j < KH; ++j) {
          kf[j] = lds_b128(Kl, plan.row(sub, half * KH + j));
          vf[j] = lds_b128(Vl, plan.row(sub, half * KH + j));
        }
#pragma unroll
        for (int j = 0; j < KH; ++j) {
          s = mfma32(kf[j], qf[half * KH + j], s);
          dp = mfma32(vf[j], df[half * KH + j], dp);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * KH, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * KH, 0);
      }
      if constexpr (PF) {
        if (sub == 1) {
          tk[0] = tk_read(0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      if (need_mask) {  // wave-uniform; masked scores -> -inf -> p = 0
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + sub * 32 + acc_row(r, h);
          s[r] = (key >= p.Sk || (CAUSAL && key > myq + off)) ? -INFINITY : s[r];
        }
      }
      if constexpr (DROP) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool keep = attn_keep(drk, (unsigned)(k0 + sub * 32 + acc_row(r, h)), dthr);
          s[r] = exp2_(fmaf(s[r], sl2, nlse2)) * ((keep ? dp[r] * drs : 0.f) - delta);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = exp2_(fmaf(s[r], sl2, nlse2)) * (dp[r] - delta);
      }
#pragma unroll
      for (int half = 0; half < 2; ++half)
#pragma unroll
        for (int j = 0; j < 8; ++j) sf[sub * 2 + half][j] = (bf16)s[8 * half + j];
      __builtin_amdgcn_sched_barrier(0);
    }
    // dQ^T += K^T dS^T
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < 4 * DT; ++i) {
        if (i + 1 < 4 * DT) tk[(i + 1) & 1] = tk_read(i + 1);
        dq[i % DT] = mfma32(tk[i & 1], sf[i / DT], dq[i % DT]);
        if (i + 1 < 4 * DT) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          dq[dt] = mfma32(lds_tr2(Kl, plan.tr(ks, dt, 0), plan.tr(ks, dt, 1)), sf[ks], dq[dt]);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles)
      plan.template stage_async<true>(lds_w + (buf ^ 1) * 2 * TILE, kp, vp, p.k_ss, p.v_ss, (t + 1) * BN, p.Sk);
    const char* Kl = smem + buf * 2 * TILE;
    if (t < wtiles) {
      const int k0 = t * BN;
      tile(Kl, Kl + TILE, k0, (k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0w + off)));
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  }

  {   // dQ through this wave's LDS slab (the K / V images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= 4 * TILE, "epilogue slabs exceed the dQ kernel's LDS");
    bf16* dq0 = (bf16*)P.dq + (int64_t)b * P.dq_sb + (int64_t)q0w * P.dq_ss + (int64_t)hq * P.dq_sh;
    store_rows_lds<DT>(smem + wid * (32 * HD * 2), dq0, P.dq_ss, min(32, p.Sq - q0w), dq, p.scale, h, l32, myq,
                       P.rope_cos, P.rope_sin, P.rope_off);
  }
}

// ==================================================================================================
// One geometry for every kernel: 4 waves = 128 query rows (or keys) per workgroup, two workgroups per CU.
template <int HD>
static void fwd_launch(const AttnParams& p, hipStream_t st) {
  const dim3 grid((unsigned)((p.Sq + 127) / 128 * p.Hq * p.B));   // 1-D: xcd_block() maps it
  const size_t lds = 2 * 2 * 64 * HD * 2;
  if (p.drop_p > 0.f) {
    if (p.causal) hipLaunchKernelGGL((attn_fwd_k<HD, true, true>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((attn_fwd_k<HD, false, true>), grid, dim3(256), lds, st, p);
  } else {
    if (p.causal) hipLaunchKernelGGL((attn_fwd_k<HD, true>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((attn_fwd_k<HD, false>), grid, dim3(256), lds, st, p);
  }
}

void flash_attn_fwd(const AttnParams& p, hipStream_t st) {
  if (p.B == 0 || p.Sq == 0) return;
  switch (p.D) {
    case 32: fwd_launch<32>(p, st); break;
    case 64: fwd_launch<64>(p, st); break;
    case 128: fwd_launch<128>(p, st); break;
    default: break;  // rejected by the host op before launch
  }
}

template <int HD, bool DROP>
static void bwd_launch_t(const AttnBwdParams& P, hipStream_t st) {
  const AttnParams& p = P.f;
  const size_t lds_kv = 128 * HD * 2 + 4 * 32 * HD * 2 + 6 * 32 * 4;
  const dim3 grid_kv((unsigned)((p.Sk + 127) / 128 * p.Hkv * p.B));
  if (p.causal) hipLaunchKernelGGL((attn_bwd_dkdv_k<HD, true, DROP>), grid_kv, dim3(256), lds_kv, st, P);
  else hipLaunchKernelGGL((attn_bwd_dkdv_k<HD, false, DROP>), grid_kv, dim3(256), lds_kv, st, P);
  const size_t lds_q = 2 * 2 * 64 * HD * 2;
  const dim3 grid_q((unsigned)((p.Sq + 127) / 128 * p.Hq * p.B));
  if (p.causal) hipLaunchKernelGGL((attn_bwd_dq_k<HD, true, DROP>), grid_q, dim3(256), lds_q, st, P);
  else hipLaunchKernelGGL((attn_bwd_dq_k<HD, false, DROP>), grid_q, dim3(256), lds_q, st, P);
}

template <int HD>
static void bwd_launch(const AttnBwdParams& P, hipStream_t st) {
  if (P.f.drop_p > 0.f) bwd_launch_t<HD, true>(P, st);
  else bwd_launch_t<HD, false>(P, st);
}

void flash_attn_bwd(const AttnBwdParams& P, hipStream_t st) {
  const AttnParams& p = P.f;
  if (p.B == 0 || p.Sq == 0) return;
  const int64_t rows = (int64_t)p.B * p.Hq * p.Sq;
  auto delta = [&](auto kern, int tpr) {
    hipLaunchKernelGGL(kern, dim3(stream_grid(rows, 256 / tpr)), dim3(256), 0, st, (const bf16*)p.o,
                       (const bf16*)P.dout, P.delta, p.B, p.Sq, p.Hq, p.o_sb, p.o_ss, p.o_sh, P.do_sb, P.do_ss,
                       P.do_sh);
  };
  switch (p.D) {
    case 32: delta(attn_delta_k<4>, 4); break;
    case 64: delta(attn_delta_k<8>, 8); break;
    case 128: delta(attn_delta_k<16>, 16); break;
    default: return;
  }
  switch (p.D) {
    case 32: bwd_launch<32>(P, st); break;
    case 64: bwd_launch<64>(P, st); break;
    case 128: bwd_launch<128>(P, st); break;
    default: break;
  }
}

}  // namespace dph
