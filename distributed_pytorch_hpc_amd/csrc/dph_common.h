// Shared device helpers for the CDNA4 (gfx950 / MI355X) kernels of distributed_pytorch_hpc_amd.
//
// Conventions used by every kernel in csrc/:
//   * wave = 64 lanes; all wave-level reductions below are written for 64 lanes.
//   * bf16 is handled as raw 16-bit storage (`__bf16` arithmetic type of amdclang); loads and stores
//     are vectorised to 16 B per lane (8 bf16 / 4 fp32), the coalescing sweet spot on CDNA4.
//   * fp32 accumulation everywhere; fp32 -> bf16 conversion is a plain cast (RNE, NaN preserving,
//     lowered to v_cvt_pk_bf16_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace dph {

typedef __bf16 bf16;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 8-element vector load/store with fp32 conversion, for T in {float, bf16}.
template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&o)[8]) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
  static __device__ __forceinline__ void store(bf16* p, const float (&o)[8]) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16)o[i];
    *reinterpret_cast<bf16x8*>(p) = v;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&o)[8]) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = a[i]; o[i + 4] = b[i]; }
  }
  static __device__ __forceinline__ void store(float* p, const float (&o)[8]) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = o[i]; b[i] = o[i + 4]; }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};

// LDS-DMA of 16 B per lane: global (wave-uniform SGPR base `sbase` + per-lane 32-bit byte offset `voff`) -> LDS
// (lane-linear destination at the wave-uniform LDS byte address `lds`).  Issued from inline asm on purpose: hipcc
// cannot tell that ds_reads of OTHER LDS regions do not alias an in-flight DMA and would drain every DMA (vmcnt(0))
// before each read; the asm form is invisible to its wait bookkeeping, so completion must be counted by hand
// (wait_vmcnt<N> + s_barrier) before any wave reads the destination.  hipcc's own counted waits for ordinary loads
// only ever over-wait around these (vmcnt retires in issue order).
__device__ __forceinline__ void lds_dma16(const void* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

// Buffer resource (V#) of a raw byte buffer [base, base + bytes): stride 0, the range-checked form -- a load whose
// offset lies past `bytes` returns zeros (gfx9 word 3 = 0x00020000).  Built from wave-uniform values.
typedef int dph_rsrc __attribute__((ext_vector_type(4)));
__device__ __forceinline__ dph_rsrc make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long b = (unsigned long long)base;
  dph_rsrc r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)((b >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA of 16 B per lane through a buffer resource: lds_dma16 with the per-lane byte offset `voff` range-checked
// against the resource (an out-of-range lane writes 16 zero bytes to its LDS slot -- zero padding without a copy).
__device__ __forceinline__ void lds_dma16_buf(dph_rsrc rsrc, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(lds)
               : "memory");
}

// s_waitcnt with only the vector-memory counter constrained (LDS-DMA completion), gfx9 encoding.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Bijective XCD-aware remap of a 1-D grid of n workgroups.  The hardware deals block ids round-robin over the 8 XCDs
// (ids congruent mod 8 share one L2), so XCD k is given the contiguous logical range [k*n/8, (k+1)*n/8): neighbouring
// logical tiles -- which share operand panels / heads -- run on one XCD and share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int xcd = bid & 7;
  return xcd * (n >> 3) + min(xcd, n & 7) + (bid >> 3);
}

// A pointer the caller knows to be wave-uniform, forced into SGPRs (lds_dma16's `sbase` operand must be scalar).
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}

// Wave-uniform LDS byte address of a __shared__ pointer (for lds_dma16's M0 operand).
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(p));
}

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

__host__ __device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid size for memory-bound grid-stride kernels: enough workgroups to fill 256 CUs x 8 resident.
__host__ __forceinline__ int stream_grid(int64_t work_items, int per_block) {
  int64_t g = cdiv(work_items, per_block);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dph

#define DPH_DISPATCH_FLOAT(dt, T, ...)                       \
  do {                                                       \
    if ((dt) == dph::kBF16) { typedef dph::bf16 T; __VA_ARGS__; } \
    else { typedef float T; __VA_ARGS__; }                   \
  } while (0)
