// Device-side building blocks shared by the flash-attention kernels (attention.hip: forward; attention_bwd.hip:
// dQ + delta, then dK/dV).  The two kernel families are separate translation units so each is compiled with the flags
// that suit it (csrc/build.py PER_FILE_HIP_FLAGS).
//
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
// Backward (no atomics, no dS round trip through LDS): two kernels; the first (dQ) also forms delta = rowsum(dO*O).
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
#pragma once

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

// glds_stage issued through lds_dma16 (see KVTilePlan::stage_async) with the per-lane swizzled source row/chunk
// hoisted out of the tile loop: ROWS x NC chunks of rows [row0, row0 + ROWS) of a strided tile, rows past `nvalid`
// re-reading the last valid one.  `lds_w` = lds_addr(img + wave * 1 KiB).
template <int NC, int ROWS, int NT>
struct RowStagePlan {
  static constexpr int CHUNKS = ROWS * NC, NI = (CHUNKS + NT - 1) / NT;
  int prow[NI], pch[NI];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int L = threadIdx.x + NT * i, line = L >> 4, slot = L & 15;
      const int F = (line << 4) + (slot ^ (((line & 3) << 2) | ((line >> 2) & 3)));
      prow[i] = F / NC;
      pch[i] = (F % NC) * 8;
    }
  }
  __device__ __forceinline__ void stage(unsigned lds_w, const bf16* base, int64_t rstride, int row0,
                                        int nvalid) const {
    const int rmax = nvalid - 1 - row0;
    const bf16* t = base + (int64_t)row0 * rstride;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if (CHUNKS % NT == 0 || (int)threadIdx.x + NT * i < CHUNKS)
        lds_dma16(t, (unsigned)(((int64_t)min(prow[i], rmax) * rstride + pch[i]) * 2), lds_w + NT * i * 16);
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
// 16x16x32 building blocks (head dim 128).  v_mfma_f32_16x16x32_bf16: lane l holds A[row l&15][k 8(l>>4) + j] and
// B[k 8(l>>4) + j][col l&15] (j < 8), and C/D[row 4(l>>4) + r][col l&15] (r < 4).  In bare loops it sustains 1.12-1.15x
// the FLOP/s of the 32x32x16 form at equal cycles per FLOP (a higher clock under load, profiles/r5/mfma_power/).
// ==================================================================================================
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS image of a [rows][128 bf16] tile, one 256-B bank row per tile row, 16-B chunk ch of row r at slot
// ch ^ 2 (r & 7).  Conflict-free for both reads the 16x16x32 kernels issue (bank rule of MI355X_MICROARCH.md §LDS):
//  * ds_read_b128 operand rows: lane (i, g) reads row r0 + i, chunk 4 kk + g.  A b128 lane group holds rows
//    {0-3, 12-15} at chunk a and rows {4-11} at chunk a ^ 1 (or the reverse); their slots a ^ {0,2,..,14} and
//    a ^ {1,3,..,15} are all 16 distinct;
//  * ds_read_b64_tr_b16 (T10): a 32-lane half reads 8 consecutive rows x chunks {2 db, 2 db + 1}: the 8 rows' XORs
//    2 (r & 7) differ above bit 0, so the 16 (row, chunk) pairs take 16 distinct slots.
// (img_off's swizzle, built for the 32x32x16 pattern, leaves the 16x16x32 row read 2-way conflicted.)
__device__ __forceinline__ int x16_off(int row, int ch) { return (row << 8) + ((ch ^ ((row & 7) << 1)) << 4); }

// Per-lane ABSOLUTE LDS byte addresses of the two operand reads of a 16x16x32 product on an x16 image whose row block
// starts at a multiple of 16 rows: a read is then `ds_read v_addr offset:<image + block>` with a compile-time
// immediate.  (Addressed as `smem + offset`, hipcc materialises the dynamic-LDS symbol with one v_add per read: 50
// vector adds per two tiles of the dK/dV body, which is bound by vector issue.)
struct X16Reads {
  unsigned row[4];   // ds_read_b128 of k-step kk: row i, chunk 4 kk + g
  unsigned tr[8];    // ds_read_b64_tr_b16 of 16-column block db, rows 4 g + q (and + 16 rows at tr + 4096)
  __device__ __forceinline__ void init(int lane, unsigned base) {
    const int i = lane & 15, g = lane >> 4, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) row[kk] = base + x16_off(i, 4 * kk + g);
#pragma unroll
    for (int db = 0; db < 8; ++db) tr[db] = base + x16_off(4 * g + q, 2 * db + (pp >> 1)) + 8 * (pp & 1);
  }
};

// Reads at an absolute LDS byte address (the X16Reads forms).
typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8_c;
__device__ __forceinline__ bf16x8 ldsa_b128(unsigned a) { return *reinterpret_cast<lds_bf16x8_c*>(a); }
__device__ __forceinline__ bf16x8 ldsa_tr(unsigned a) {
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<lds_i16x4*>(a));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<lds_i16x4*>(a + 16 * 256));
  bf16x4 x = __builtin_bit_cast(bf16x4, lo), y = __builtin_bit_cast(bf16x4, hi);
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

// A = X^T operand (16 columns of X as rows x 32 rows of X as k) for a 32-row tile: rows {4g..4g+3} and {16+4g..}, the
// k order in which a 16x16 accumulator pair (row blocks 0 and 1 of the other product) hands over as the B operand.
__device__ __forceinline__ bf16x8 x16_tr(const char* img, int off) { return lds_tr2(img, off, off + 16 * 256); }

// B operand from two 16x16 accumulators holding rows 4g + r of row blocks 0 and 1 (the x16_tr k order).
__device__ __forceinline__ bf16x8 acc_pair_b(const f32x4& lo, const f32x4& hi) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    b[j] = (bf16)lo[j];
    b[4 + j] = (bf16)hi[j];
  }
  return b;
}

// LDS-DMA of ROWS x 128 bf16 rows [row0, row0 + ROWS) of a strided tile into an x16 image (rows past nvalid re-read
// the last valid row: finite data the caller masks).  A lane's instructions are NT / 16 rows apart, a multiple of 8,
// so one (row, chunk) pair per lane serves them all.  `lds_w` = lds_addr(img + wave * 1 KiB).
// Full tiles step the wave-uniform source base by RSTEP rows per instruction (scalar adds) with one per-lane byte
// offset computed at init; only a ragged last tile clamps rows per instruction.
template <int ROWS, int NT>
struct X16Stage {
  static constexpr int NI = ROWS * 16 / NT, RSTEP = NT / 16;
  static_assert(ROWS * 16 % NT == 0 && RSTEP % 8 == 0, "x16 staging: whole 8-row swizzle periods per instruction");
  int prow = 0, pch = 0;
  unsigned voff = 0;   // (prow * rs0 + pch) * 2
  int64_t rs0 = 0;     // the row stride voff was computed for (a tile of another stride takes the general path)
  __device__ __forceinline__ void init(int64_t rstride) {
    const int L = threadIdx.x;
    prow = L >> 4;
    pch = ((L & 15) ^ ((prow & 7) << 1)) * 8;
    rs0 = rstride;
    voff = (unsigned)((prow * rstride + pch) * 2);
  }
  __device__ __forceinline__ void stage(unsigned lds_w, const bf16* base, int64_t rstride, int row0,
                                        int nvalid) const {
    const bf16* t = uniform_ptr(base + (int64_t)row0 * rstride);
    if (row0 + ROWS <= nvalid && rstride == rs0) {
#pragma unroll
      for (int i = 0; i < NI; ++i) lds_dma16(t + (int64_t)i * RSTEP * rstride, voff, lds_w + NT * i * 16);
    } else {
      const int rmax = nvalid - 1 - row0;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        lds_dma16(t, (unsigned)(((int64_t)min(prow + i * RSTEP, rmax) * rstride + pch) * 2), lds_w + NT * i * 16);
    }
  }
};

// Epilogue of a 32-row x 128-column result held as 16x16 accumulators acc[db][rb] (lane: row rb * 16 + (lane & 15),
// columns 16 db + 4 g .. + 3): scale, optional inverse RoPE of the interleaved pairs (position row + rope_off), bf16,
// rows [0, nvalid) stored at base + r * rstride as 16-B row segments through this wave's 8-KiB LDS slab.
__device__ __forceinline__ void store_rows16(char* slab, bf16* base, int64_t rstride, int nvalid,
                                             const f32x4 (&acc)[8][2], float mul, int lane, int row0,
                                             const float* rc, const float* rs, int rope_off) {
  const int i = lane & 15, g = lane >> 4;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = rb * 16 + i;
    const bool ok = r < nvalid;
    const float* cr = rc && ok ? rc + (int64_t)(row0 + r + rope_off) * 64 : nullptr;
    const float* sr = rs && ok ? rs + (int64_t)(row0 + r + rope_off) * 64 : nullptr;
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = acc[db][rb][j] * mul;
      if (cr) {
        const int i0 = db * 8 + 2 * g;   // pairs (16 db + 4 g, +1) and (+2, +3)
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
      const int ch = 2 * db + (g >> 1);
      *reinterpret_cast<bf16x4*>(slab + (r << 8) + ((ch ^ (r & 15)) << 4) + 8 * (g & 1)) = w;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes are done
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int r = it * 4 + (lane >> 4), c = lane & 15;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(slab + (r << 8) + ((c ^ (r & 15)) << 4));
    if (r < nvalid) *reinterpret_cast<bf16x8*>(base + (int64_t)r * rstride + c * 8) = v;
  }
}

}  // namespace dph
