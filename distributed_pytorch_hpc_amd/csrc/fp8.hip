// Per-tensor FP8 quantisation for the opt-in FP8-GEMM training mode (ops/fp8.py): OCP e4m3 (activations, weights)
// and e5m2 (gradients), the formats gfx950's v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 produce.
//
//   fp8_amax_k   : per-block max |x| over a contiguous bf16 tensor (16-B loads, wave then LDS max) into a partials
//                  array -- no atomics: with one atomicMax per wave on a single address the pass ran at ~2 TB/s
//                  (74 ms per Llama-2-7B step, rocprof), the atomics serialising; fp8_amax_finalize_k (one block)
//                  folds the partials into [amax, scale = FMAX / amax, dequant = amax / FMAX].
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

__device__ __forceinline__ float block_max(float m) {
  __shared__ float red[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__global__ __launch_bounds__(256) void fp8_amax_k(const bf16* __restrict__ x, int64_t n8, float* __restrict__ partial) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<bf16>::load(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[k]));
  }
  m = block_max(m);
  if (threadIdx.x == 0) partial[blockIdx.x] = m;
}

// partials [n] -> scal = [amax, FMAX / amax, amax / FMAX] (amax 0: scale 1, dequant 1)
__global__ __launch_bounds__(256) void fp8_amax_finalize_k(const float* __restrict__ partial, int n, float fmax,
                                                           float* __restrict__ scal) {
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, partial[i]);
  m = block_max(m);
  if (threadIdx.x == 0) {
    scal[0] = m;
    scal[1] = m > 0.f ? fmax / m : 1.f;
    scal[2] = m > 0.f ? m / fmax : 1.f;
  }
}

template <int FMT, bool ROW, bool TRANS>
__global__ __launch_bounds__(256) void fp8_quant_k(const bf16* __restrict__ x, int R, int C,
                                                   const float* __restrict__ scal, uint8_t* __restrict__ y,
                                                   uint8_t* __restrict__ yt) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[Q_T][Q_T + Q_PAD];
  const float fmax = fp8_max<FMT>();
  const float s = scal[1];
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

int fp8_amax_blocks(int64_t n) { return stream_grid(n / 8, 256); }

void fp8_amax(const void* x, int64_t n, int fmt, float* partial, float* scal, hipStream_t st) {
  const int64_t n8 = n / 8;
  const int g = fp8_amax_blocks(n);
  if (n8 > 0) hipLaunchKernelGGL(fp8_amax_k, dim3(g), dim3(256), 0, st, (const bf16*)x, n8, partial);
  hipLaunchKernelGGL(fp8_amax_finalize_k, dim3(1), dim3(256), 0, st, (const float*)partial, n8 > 0 ? g : 0,
                     fmt == kFP8E4M3 ? 448.f : 57344.f, scal);
}

void fp8_quant(const void* x, int64_t R, int64_t C, const float* scal, int fmt, void* y, void* yt, hipStream_t st) {
  if (R == 0 || C == 0) return;
  const dim3 grid((unsigned)(C / Q_T), (unsigned)(R / Q_T));
#define DPH_Q(F, RW, TR)                                                                                     \
  hipLaunchKernelGGL((fp8_quant_k<F, RW, TR>), grid, dim3(256), 0, st, (const bf16*)x, (int)R, (int)C,     \
                     scal, (uint8_t*)y, (uint8_t*)yt)
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
