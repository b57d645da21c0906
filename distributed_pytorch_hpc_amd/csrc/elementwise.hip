// Memory-bound elementwise kernels: RoPE, SwiGLU, GELU, cast/scale.
// All of them move 16 B per lane per access (8 bf16 or 2 x 4 fp32) and grid-stride over a capped grid
// (cdna_hip_programming.md Guideline 11/13).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

// ------------------------------------------------------------------------------------------------
// RoPE with interleaved pairs (x[2i], x[2i+1]) rotated by angle pos * theta^(-2i/hd), exactly the
// view_as_complex formulation of fsdp_tp/llama2_model.py:74-100 (fp32 math, one rounding).
// Tables cos_t/sin_t are fp32 [S_table, hd/2] precomputed on the host side (no device trig).
// One workgroup per (b, s) token row: every head of the row shares one position, so a thread loads its
// chunk's cos / sin (4 pairs) once and rotates that chunk in H * hd / 8 / 256 heads -- no per-element 64-bit
// index division (the grid-stride form spent more on index math than on the 16-B loads) and 16-B accesses.
template <typename T>
__global__ __launch_bounds__(256) void rope_k(T* __restrict__ x, const float* __restrict__ cos_t,
                                              const float* __restrict__ sin_t, int S, int H, int hd, int64_t sb,
                                              int64_t ss, int64_t sh, int64_t pos_offset, float sign) {
  const int cpr = hd >> 3;          // 8-element chunks per head row
  const int half = hd >> 1;
  const int row = blockIdx.x;
  const int b = row / S, s = row - b * S;
  const int64_t pos = pos_offset + s;
  T* base = x + (int64_t)b * sb + (int64_t)s * ss;
  const int n = H * cpr;
  int c = threadIdx.x % cpr, h = threadIdx.x / cpr;
  const int hstep = 256 / cpr, cstep = 256 % cpr;
  f32x4 cs = *reinterpret_cast<const f32x4*>(cos_t + pos * half + c * 4);
  f32x4 sn = *reinterpret_cast<const f32x4*>(sin_t + pos * half + c * 4);
  for (int i = threadIdx.x; i < n; i += 256) {
    T* p = base + (int64_t)h * sh + c * 8;
    float v[8], o[8];
    Vec8<T>::load(p, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = v[2 * k], bb = v[2 * k + 1];
      const float cc = cs[k], sv = sign * sn[k];
      o[2 * k] = a * cc - bb * sv;
      o[2 * k + 1] = a * sv + bb * cc;
    }
    Vec8<T>::store(p, o);
    h += hstep;
    if (cstep) {   // cpr does not divide 256: advance the chunk and reload the table entries
      c += cstep;
      if (c >= cpr) { c -= cpr; ++h; }
      cs = *reinterpret_cast<const f32x4*>(cos_t + pos * half + c * 4);
      sn = *reinterpret_cast<const f32x4*>(sin_t + pos * half + c * 4);
    }
  }
}

void rope_apply(void* x, const float* cos_t, const float* sin_t, int64_t B, int64_t S, int64_t H, int hd,
                int64_t sb, int64_t ss, int64_t sh, int64_t pos_offset, int inverse, int dtype,
                hipStream_t stream) {
  if (B * S * H == 0) return;
  const float sign = inverse ? -1.f : 1.f;
  const dim3 grid((unsigned)(B * S));
  if (dtype == kBF16)
    hipLaunchKernelGGL(rope_k<bf16>, grid, dim3(256), 0, stream, (bf16*)x, cos_t, sin_t, (int)S, (int)H, hd, sb,
                       ss, sh, pos_offset, sign);
  else
    hipLaunchKernelGGL(rope_k<float>, grid, dim3(256), 0, stream, (float*)x, cos_t, sin_t, (int)S, (int)H, hd, sb,
                       ss, sh, pos_offset, sign);
}

// ------------------------------------------------------------------------------------------------
// SwiGLU: y = silu(g) * u with x2 = [g | u] (row stride ld_x2, g at column 0, u at column f).
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_k(const T* __restrict__ x2, T* __restrict__ y, int64_t n,
                                                    int64_t f, int64_t ld, int64_t total) {
  const int64_t cpr = f >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cpr, c = (i % cpr) * 8;
    float g[8], u[8], o[8];
    Vec8<T>::load(x2 + r * ld + c, g);
    Vec8<T>::load(x2 + r * ld + f + c, u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * sigmoidf_(g[k]) * u[k];
    Vec8<T>::store(y + r * f + c, o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x2,
                                                    T* __restrict__ dx2, int64_t n, int64_t f, int64_t ld,
                                                    int64_t total) {
  const int64_t cpr = f >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cpr, c = (i % cpr) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    Vec8<T>::load(x2 + r * ld + c, g);
    Vec8<T>::load(x2 + r * ld + f + c, u);
    Vec8<T>::load(dy + r * f + c, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = sigmoidf_(g[k]);
      const float silu = g[k] * s;
      du[k] = d[k] * silu;
      dg[k] = d[k] * u[k] * s * (1.f + g[k] * (1.f - s));
    }
    Vec8<T>::store(dx2 + r * 2 * f + c, dg);
    Vec8<T>::store(dx2 + r * 2 * f + f + c, du);
  }
}

void swiglu_fwd(const void* x2, void* y, int64_t n, int64_t f, int64_t ld, int dtype, hipStream_t stream) {
  const int64_t total = n * (f / 8);
  if (total == 0) return;
  const int grid = stream_grid(total, 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(swiglu_fwd_k<bf16>, dim3(grid), dim3(256), 0, stream, (const bf16*)x2, (bf16*)y, n, f, ld,
                       total);
  else
    hipLaunchKernelGGL(swiglu_fwd_k<float>, dim3(grid), dim3(256), 0, stream, (const float*)x2, (float*)y, n, f, ld,
                       total);
}

void swiglu_bwd(const void* dy, const void* x2, void* dx2, int64_t n, int64_t f, int64_t ld, int dtype,
                hipStream_t stream) {
  const int64_t total = n * (f / 8);
  if (total == 0) return;
  const int grid = stream_grid(total, 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(swiglu_bwd_k<bf16>, dim3(grid), dim3(256), 0, stream, (const bf16*)dy, (const bf16*)x2,
                       (bf16*)dx2, n, f, ld, total);
  else
    hipLaunchKernelGGL(swiglu_bwd_k<float>, dim3(grid), dim3(256), 0, stream, (const float*)dy, (const float*)x2,
                       (float*)dx2, n, f, ld, total);
}

// ------------------------------------------------------------------------------------------------
// GELU (erf form = nn.GELU(), tanh form = approximate="tanh").
__device__ __forceinline__ float gelu_f(float x, bool tanh_form) {
  if (tanh_form) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
  }
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float gelu_grad_f(float x, bool tanh_form) {
  if (tanh_form) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float inner = k0 * (x + k1 * x * x * x);
    const float t = tanhf(inner);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  }
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

template <typename T, bool TANH>
__global__ __launch_bounds__(256) void gelu_fwd_k(const T* __restrict__ x, T* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<T>::load(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = gelu_f(v[k], TANH);
    Vec8<T>::store(y + i * 8, v);
  }
}
template <typename T, bool TANH>
__global__ __launch_bounds__(256) void gelu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                  T* __restrict__ dx, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8], d[8];
    Vec8<T>::load(x + i * 8, v);
    Vec8<T>::load(dy + i * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = d[k] * gelu_grad_f(v[k], TANH);
    Vec8<T>::store(dx + i * 8, v);
  }
}

void gelu_fwd(const void* x, void* y, int64_t n, int tanh_form, int dtype, hipStream_t stream) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  const int grid = stream_grid(n8, 256);
  if (dtype == kBF16) {
    if (tanh_form) hipLaunchKernelGGL((gelu_fwd_k<bf16, true>), dim3(grid), dim3(256), 0, stream, (const bf16*)x, (bf16*)y, n8);
    else hipLaunchKernelGGL((gelu_fwd_k<bf16, false>), dim3(grid), dim3(256), 0, stream, (const bf16*)x, (bf16*)y, n8);
  } else {
    if (tanh_form) hipLaunchKernelGGL((gelu_fwd_k<float, true>), dim3(grid), dim3(256), 0, stream, (const float*)x, (float*)y, n8);
    else hipLaunchKernelGGL((gelu_fwd_k<float, false>), dim3(grid), dim3(256), 0, stream, (const float*)x, (float*)y, n8);
  }
}
void gelu_bwd(const void* dy, const void* x, void* dx, int64_t n, int tanh_form, int dtype, hipStream_t stream) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  const int grid = stream_grid(n8, 256);
  if (dtype == kBF16) {
    if (tanh_form) hipLaunchKernelGGL((gelu_bwd_k<bf16, true>), dim3(grid), dim3(256), 0, stream, (const bf16*)dy, (const bf16*)x, (bf16*)dx, n8);
    else hipLaunchKernelGGL((gelu_bwd_k<bf16, false>), dim3(grid), dim3(256), 0, stream, (const bf16*)dy, (const bf16*)x, (bf16*)dx, n8);
  } else {
    if (tanh_form) hipLaunchKernelGGL((gelu_bwd_k<float, true>), dim3(grid), dim3(256), 0, stream, (const float*)dy, (const float*)x, (float*)dx, n8);
    else hipLaunchKernelGGL((gelu_bwd_k<float, false>), dim3(grid), dim3(256), 0, stream, (const float*)dy, (const float*)x, (float*)dx, n8);
  }
}

// ------------------------------------------------------------------------------------------------
template <typename S, typename D>
__global__ __launch_bounds__(256) void cast_k(const S* __restrict__ s, D* __restrict__ d, int64_t n8, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<S>::load(s + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= scale;
    Vec8<D>::store(d + i * 8, v);
  }
}
void cast_copy(const void* src, void* dst, int64_t n, int sd, int dd, float scale, hipStream_t stream) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  const int grid = stream_grid(n8, 256);
  if (sd == kBF16 && dd == kF32)
    hipLaunchKernelGGL((cast_k<bf16, float>), dim3(grid), dim3(256), 0, stream, (const bf16*)src, (float*)dst, n8, scale);
  else if (sd == kF32 && dd == kBF16)
    hipLaunchKernelGGL((cast_k<float, bf16>), dim3(grid), dim3(256), 0, stream, (const float*)src, (bf16*)dst, n8, scale);
  else if (sd == kF32)
    hipLaunchKernelGGL((cast_k<float, float>), dim3(grid), dim3(256), 0, stream, (const float*)src, (float*)dst, n8, scale);
  else
    hipLaunchKernelGGL((cast_k<bf16, bf16>), dim3(grid), dim3(256), 0, stream, (const bf16*)src, (bf16*)dst, n8, scale);
}

}  // namespace dph
