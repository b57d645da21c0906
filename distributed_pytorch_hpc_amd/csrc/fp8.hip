// Per-tensor FP8 quantisation for the opt-in FP8-GEMM training mode (ops/fp8.py): OCP e4m3 (activations, weights)
// and e5m2 (gradients), the formats gfx950's v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 produce.
//
//   fp8_amax_k   : amax = max |x| over a contiguous bf16 tensor (16-B loads, wave max, one atomicMax per wave on
//                  the float's bit pattern -- exact and order-independent for non-negative floats).
//   fp8_quant_k  : y = sat(x * FMAX / amax) in fp8, written row-major [R, C] and / or transposed [C, R] (the K-major
//                  operand copies hipBLASLt's FP8 GEMMs need for dY^T and X^T), plus the dequantisation scale
//                  amax / FMAX that torch._scaled_mm takes as scale_a / scale_b.  64 x 64 tiles, 256 threads; the
//                  transposed tile goes through LDS so both global writes are 16-B row segments.
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int Q_T = 64;           // tile rows / cols
constexpr int Q_PAD = 16;         // LDS row padding (bytes) for the transposed tile

template <int FMT>
__device__ __forceinline__ float fp8_max() { return FMT == kFP8E4M3 ? 448.f : 57344.f; }

// 4 floats -> 4 fp8 bytes (RNE, saturated by the caller's clamp)
template <int FMT>
__device__ __forceinline__ unsigned pack4(float a, float b, float c, float d) {
  if constexpr (FMT == kFP8E4M3) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  } else {
    int w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    return (unsigned)__builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
  }
}

__global__ __launch_bounds__(256) void fp8_amax_k(const bf16* __restrict__ x, int64_t n8, unsigned* __restrict__ amax) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<bf16>::load(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[k]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(amax, __float_as_uint(m));
}

template <int FMT, bool ROW, bool TRANS>
__global__ __launch_bounds__(256) void fp8_quant_k(const bf16* __restrict__ x, int R, int C,
                                                   const unsigned* __restrict__ amax_bits, uint8_t* __restrict__ y,
                                                   uint8_t* __restrict__ yt, float* __restrict__ dequant) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[Q_T][Q_T + Q_PAD];
  const float amax = __uint_as_float(*amax_bits);
  const float fmax = fp8_max<FMT>();
  const float s = amax > 0.f ? fmax / amax : 1.f;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *dequant = amax > 0.f ? amax / fmax : 1.f;
  const int r0 = blockIdx.y * Q_T, c0 = blockIdx.x * Q_T;
  const int t = threadIdx.x, r = t >> 2, c = (t & 3) * 16;   // this thread: row r, columns c .. c + 15
  float v[16];
  const bf16* src = x + (int64_t)(r0 + r) * C + c0 + c;
  {
    float a[8], b[8];
    Vec8<bf16>::load(src, a);
    Vec8<bf16>::load(src + 8, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) { v[k] = a[k]; v[8 + k] = b[k]; }
  }
  unsigned w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = __builtin_amdgcn_fmed3f(v[4 * k + j] * s, fmax, -fmax);
    w[k] = pack4<FMT>(q[0], q[1], q[2], q[3]);
  }
  if constexpr (ROW) {
    uint4 o = {w[0], w[1], w[2], w[3]};
    *reinterpret_cast<uint4*>(y + (int64_t)(r0 + r) * C + c0 + c) = o;
  }
  if constexpr (TRANS) {
#pragma unroll
    for (int k = 0; k < 16; ++k) tile[c + k][r] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    __syncthreads();
    // transposed row tr (= source column c0 + tr), source rows tc .. tc + 15
    const int tr = t >> 2, tc = (t & 3) * 16;
    const uint4 o = *reinterpret_cast<const uint4*>(&tile[tr][tc]);
    *reinterpret_cast<uint4*>(yt + (int64_t)(c0 + tr) * R + r0 + tc) = o;
  }
}

}  // namespace

void fp8_amax(const void* x, int64_t n, unsigned* amax_bits, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(fp8_amax_k, dim3(stream_grid(n8, 256)), dim3(256), 0, st, (const bf16*)x, n8, amax_bits);
}

void fp8_quant(const void* x, int64_t R, int64_t C, const unsigned* amax_bits, int fmt, void* y, void* yt,
               float* dequant, hipStream_t st) {
  if (R == 0 || C == 0) return;
  const dim3 grid((unsigned)(C / Q_T), (unsigned)(R / Q_T));
#define DPH_Q(F, RW, TR)                                                                                     \
  hipLaunchKernelGGL((fp8_quant_k<F, RW, TR>), grid, dim3(256), 0, st, (const bf16*)x, (int)R, (int)C,     \
                     amax_bits, (uint8_t*)y, (uint8_t*)yt, dequant)
#define DPH_QF(F)                                     \
  do {                                                \
    if (y && yt) DPH_Q(F, true, true);                \
    else if (y) DPH_Q(F, true, false);               \
    else DPH_Q(F, false, true);                       \
  } while (0)
  if (fmt == kFP8E4M3) DPH_QF(kFP8E4M3);
  else DPH_QF(kFP8E5M2);
#undef DPH_QF
#undef DPH_Q
}

}  // namespace dph
