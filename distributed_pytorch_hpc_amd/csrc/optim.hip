// Fused optimizer kernels over FLAT buffers (one launch for the whole (sharded) model).
// AdamW reproduces torch.optim.AdamW (decoupled decay, bias corrections, eps after sqrt(v)/sqrt(bc2));
// SGD reproduces torch.optim.SGD (momentum, dampening, nesterov, coupled weight decay).
// Each thread handles 4 consecutive elements per iteration: 16-B fp32 loads/stores for master/m/v,
// 8-B loads for bf16 grads and 8-B stores of the bf16 working copy of the parameter.
// Per element AdamW moves 2 (g) + 12 (p,m,v in) + 12 (out) + 2 (bf16 param) = 28 B: HBM bound.
//
// Graph-capturable form: with `hyper` (device fp32 [lr, step]) the learning rate and the step count are read from
// device memory instead of kernel arguments, so one captured HIP graph replays every optimizer step (the bias
// corrections 1 - beta^step are formed here; the step is incremented on the device by the caller's captured
// add, the learning rate written by the host before each replay -- runtime/graphs.py).
#include <cstdlib>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

template <typename G>
__device__ __forceinline__ void load4(const G* p, float (&o)[4]);
template <>
__device__ __forceinline__ void load4<float>(const float* p, float (&o)[4]) {
  f32x4 v = *reinterpret_cast<const f32x4*>(p);
  o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
}
template <>
__device__ __forceinline__ void load4<bf16>(const bf16* p, float (&o)[4]) {
  bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
}
template <typename G>
__device__ __forceinline__ void store4(G* p, const float (&o)[4]);
template <>
__device__ __forceinline__ void store4<float>(float* p, const float (&o)[4]) {
  f32x4 v = {o[0], o[1], o[2], o[3]};
  *reinterpret_cast<f32x4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<bf16>(bf16* p, const float (&o)[4]) {
  bf16x4 v = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
  *reinterpret_cast<bf16x4*>(p) = v;
}

// Rejected: non-temporal loads / stores on the five streams (4 257 / 4 270 vs 4 352 / 4 334 GB/s at 2^28 parameters,
// 7B 28 330 / 28 282 vs 28 367 / 28 323 tokens/s; profiles/r4/rejected_adamw_nt/).
template <typename G, typename P, bool HAS_OUT>
__global__ __launch_bounds__(256) void adamw_k(float* __restrict__ master, float* __restrict__ m,
                                               float* __restrict__ v, const G* __restrict__ grad,
                                               P* __restrict__ pout, int64_t n, float lr, float b1, float b2,
                                               float eps, float wd, float bc1, float bc2,
                                               const float* __restrict__ gscale, const float* __restrict__ hyper) {
  const float gs = gscale ? *gscale : 1.f;
  if (gs != gs) return;   // NaN scale = skip this update (xGMI health guard, comm/custom_allreduce.py; NaN clip norm)
  if (hyper) {
    lr = hyper[0];
    bc1 = 1.f - powf(b1, hyper[1]);
    bc2 = 1.f - powf(b2, hyper[1]);
  }
  const float decay = 1.f - lr * wd;
  const float step_size = lr / bc1;
  const float inv_bc2_sqrt = 1.f / sqrtf(bc2);
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float p[4], mm[4], vv[4], g[4];
    load4<float>(master + i * 4, p);
    load4<float>(m + i * 4, mm);
    load4<float>(v + i * 4, vv);
    load4<G>(grad + i * 4, g);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = g[k] * gs;
      p[k] *= decay;
      mm[k] = mm[k] + (1.f - b1) * (gk - mm[k]);
      vv[k] = vv[k] * b2 + (1.f - b2) * gk * gk;
      const float denom = sqrtf(vv[k]) * inv_bc2_sqrt + eps;
      p[k] = p[k] - step_size * mm[k] / denom;
    }
    store4<float>(master + i * 4, p);
    store4<float>(m + i * 4, mm);
    store4<float>(v + i * 4, vv);
    if (HAS_OUT) store4<P>(pout + i * 4, p);
  }
  // tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    const float gk = (float)grad[i] * gs;
    float p = master[i] * decay;
    float mm = m[i] + (1.f - b1) * (gk - m[i]);
    float vv = v[i] * b2 + (1.f - b2) * gk * gk;
    p = p - step_size * mm / (sqrtf(vv) * inv_bc2_sqrt + eps);
    master[i] = p; m[i] = mm; v[i] = vv;
    if (HAS_OUT) pout[i] = (P)p;
  }
}

template <typename G, typename P, bool HAS_OUT>
__global__ __launch_bounds__(256) void sgd_k(float* __restrict__ master, float* __restrict__ buf,
                                             const G* __restrict__ grad, P* __restrict__ pout, int64_t n, float lr,
                                             float mom, float damp, float wd, int nesterov, int first,
                                             const float* __restrict__ gscale, const float* __restrict__ hyper) {
  const float gs = gscale ? *gscale : 1.f;
  if (gs != gs) return;   // NaN scale = skip this update (xGMI health guard, comm/custom_allreduce.py; NaN clip norm)
  if (hyper) {
    lr = hyper[0];
    first = hyper[1] == 1.f;
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float p = master[i];
    float d = (float)grad[i] * gs + wd * p;
    if (mom != 0.f) {
      float b = first ? d : buf[i] * mom + (1.f - damp) * d;
      buf[i] = b;
      d = nesterov ? d + mom * b : b;
    }
    p -= lr * d;
    master[i] = p;
    if (HAS_OUT) pout[i] = (P)p;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void sumsq_k(const T* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<T>::load(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k] * v[k];
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const float t = (float)x[n8 * 8 + threadIdx.x];
    s += t * t;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

void adamw_step(float* master, float* m, float* v, const void* grad, void* param_out, int64_t n, float lr,
                float beta1, float beta2, float eps, float wd, float bc1, float bc2, const float* gscale,
                const float* hyper, int grad_dtype, int param_dtype, hipStream_t stream) {
  if (n == 0) return;
  const int grid = stream_grid((n + 3) / 4, 256);
#define AD(G, P, OUT)                                                                                              \
  hipLaunchKernelGGL((adamw_k<G, P, OUT>), dim3(grid), dim3(256), 0, stream, master, m, v, (const G*)grad,        \
                     (P*)param_out, n, lr, beta1, beta2, eps, wd, bc1, bc2, gscale, hyper)
  if (grad_dtype == kBF16) {
    if (!param_out) AD(bf16, bf16, false);
    else if (param_dtype == kBF16) AD(bf16, bf16, true);
    else AD(bf16, float, true);
  } else {
    if (!param_out) AD(float, bf16, false);
    else if (param_dtype == kBF16) AD(float, bf16, true);
    else AD(float, float, true);
  }
#undef AD
}

void sgd_step(float* master, float* buf, const void* grad, void* param_out, int64_t n, float lr, float mom,
              float damp, float wd, int nesterov, int first, const float* gscale, const float* hyper,
              int grad_dtype, int param_dtype, hipStream_t stream) {
  if (n == 0) return;
  const int grid = stream_grid(n, 256);
#define SG(G, P, OUT)                                                                                  \
  hipLaunchKernelGGL((sgd_k<G, P, OUT>), dim3(grid), dim3(256), 0, stream, master, buf, (const G*)grad, \
                     (P*)param_out, n, lr, mom, damp, wd, nesterov, first, gscale, hyper)
  if (grad_dtype == kBF16) {
    if (!param_out) SG(bf16, bf16, false);
    else if (param_dtype == kBF16) SG(bf16, bf16, true);
    else SG(bf16, float, true);
  } else {
    if (!param_out) SG(float, bf16, false);
    else if (param_dtype == kBF16) SG(float, bf16, true);
    else SG(float, float, true);
  }
#undef SG
}

void sumsq(const void* x, int64_t n, float* out, int dtype, hipStream_t stream) {
  if (n == 0) return;
  const int grid = stream_grid((n + 7) / 8, 256);
  if (dtype == kBF16) hipLaunchKernelGGL(sumsq_k<bf16>, dim3(grid), dim3(256), 0, stream, (const bf16*)x, n, out);
  else hipLaunchKernelGGL(sumsq_k<float>, dim3(grid), dim3(256), 0, stream, (const float*)x, n, out);
}

}  // namespace dph
