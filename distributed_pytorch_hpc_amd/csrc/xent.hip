// Fused softmax cross-entropy for [N, V] logits (bf16 or fp32), one 256-thread workgroup per row.
// Pass 1: single-sweep online softmax (running max + rescaled sum) in fp32, 16-B loads.
// Pass 2 (training): the gradient of the MEAN loss is written IN PLACE over the logits
// (softmax - onehot) * (1/count), so the fp32 [N, V] logits tensor of the reference
// (fsdp_tp/llama2_model.py:447 `.float()`) and a separate softmax/grad buffer never exist.
// The row re-read of pass 2 is served from L2 (a 32000-vocab bf16 row is 62.5 KiB).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
  const float mx = fmaxf(m, m2);
  if (mx == -INFINITY) { m = mx; s = 0.f; return; }
  s = s * __expf(m - mx) + s2 * __expf(m2 - mx);
  m = mx;
}

template <typename T>
__global__ __launch_bounds__(256) void xent_k(T* __restrict__ logits, const int64_t* __restrict__ target,
                                              float* __restrict__ loss_rows, float* __restrict__ lse_rows,
                                              const float* __restrict__ inv_count, int64_t V, int64_t ld,
                                              int64_t ignore_index, int grad_inplace, float smoothing, int vec) {
  __shared__ float sm[4], ss[4], sx[4];
  const int64_t row = blockIdx.x;
  T* x = logits + row * ld;
  const int64_t tgt = target[row];
  const bool ignored = (tgt == ignore_index);
  float m = -INFINITY, s = 0.f, sumx = 0.f;
  if (vec) {
    const int64_t n8 = V >> 3;
    for (int64_t i = threadIdx.x; i < n8; i += 256) {
      float v[8];
      Vec8<T>::load(x + i * 8, v);
      float lm = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
      float ls = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) { ls += __expf(v[k] - lm); sumx += v[k]; }
      ms_combine(m, s, lm, ls);
    }
  } else {
    for (int64_t i = threadIdx.x; i < V; i += 256) {
      const float v = (float)x[i];
      sumx += v;
      ms_combine(m, s, v, 1.f);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_combine(m, s, m2, s2);
    sumx += __shfl_xor(sumx, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; sx[w] = sumx; }
  __syncthreads();
  m = sm[0]; s = ss[0]; sumx = sx[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) { ms_combine(m, s, sm[k], ss[k]); sumx += sx[k]; }
  const float lse = m + __logf(s);
  __syncthreads();  // every thread has read tgt-logit below only after all pass-1 reads
  float xt = 0.f;
  if (!ignored) xt = (float)x[tgt];
  if (threadIdx.x == 0) {
    float l = 0.f;
    if (!ignored) l = (1.f - smoothing) * (lse - xt) + smoothing * (lse - sumx / (float)V);
    loss_rows[row] = l;
    if (lse_rows) lse_rows[row] = lse;
  }
  if (!grad_inplace) return;
  __syncthreads();  // the target logit must be read by all threads before it is overwritten
  const float sc = ignored ? 0.f : *inv_count;
  const float off = smoothing / (float)V;
  if (vec) {
    const int64_t n8 = V >> 3;
    for (int64_t i = threadIdx.x; i < n8; i += 256) {
      float v[8];
      Vec8<T>::load(x + i * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t col = i * 8 + k;
        const float p = __expf(v[k] - lse);
        v[k] = (p - off - (col == tgt ? (1.f - smoothing) : 0.f)) * sc;
      }
      Vec8<T>::store(x + i * 8, v);
    }
  } else {
    for (int64_t i = threadIdx.x; i < V; i += 256) {
      const float p = __expf((float)x[i] - lse);
      x[i] = (T)((p - off - (i == tgt ? (1.f - smoothing) : 0.f)) * sc);
    }
  }
}

void cross_entropy_fwd(void* logits, const int64_t* target, float* loss_rows, float* lse_rows, const float* inv_count,
                       int64_t n, int64_t v, int64_t ld, int64_t ignore_index, int grad_inplace, float smoothing,
                       int dtype, hipStream_t stream) {
  if (n == 0) return;
  const int vec = (v % 8 == 0) && (ld % 8 == 0) && ((uintptr_t)logits % 16 == 0);
  if (dtype == kBF16)
    hipLaunchKernelGGL(xent_k<bf16>, dim3((unsigned)n), dim3(256), 0, stream, (bf16*)logits, target, loss_rows,
                       lse_rows, inv_count, v, ld, ignore_index, grad_inplace, smoothing, vec);
  else
    hipLaunchKernelGGL(xent_k<float>, dim3((unsigned)n), dim3(256), 0, stream, (float*)logits, target, loss_rows,
                       lse_rows, inv_count, v, ld, ignore_index, grad_inplace, smoothing, vec);
}

}  // namespace dph
