// LayerNorm forward/backward (nn.LayerNorm semantics, biased variance, fp32 statistics) for the ViT
// (scripts/03_tensor_parallel_tp/tensor_parallel_vit.py:130-148) and the pipeline transformer
// (scripts/04_pipeline_parallel_pp/03_pipeline_training.py:56-65).  Same structure as rmsnorm.hip:
// wave-per-row forward with the row in registers, workgroup-per-row backward with register-resident
// dW/dB partials reduced by a column kernel.
#include "dph_common.h"
#include "kernels.h"

namespace dph {

template <typename T, typename W, int NCH>
__global__ __launch_bounds__(256) void ln_fwd_k(const T* __restrict__ x, const W* __restrict__ w,
                                                const W* __restrict__ b, T* __restrict__ y, float* __restrict__ mean,
                                                float* __restrict__ rstd, int64_t rows, int D, float eps) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wid; r < rows; r += (int64_t)gridDim.x * 4) {
    float v[NCH][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) {
        Vec8<T>::load(x + r * D + idx, v[c]);
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[c][i];
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
      }
    }
    const float mu = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { const float d = v[c][i] - mu; q += d * d; }
      }
    }
    const float rs = rsqrtf(wave_sum(q) / (float)D + eps);
    if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) {
        float wv[8], bv[8], o[8];
        Vec8<W>::load(w + idx, wv);
        Vec8<W>::load(b + idx, bv);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * rs * wv[i] + bv[i];
        Vec8<T>::store(y + r * D + idx, o);
      }
    }
  }
}

template <typename T, typename W, int CPT>
__global__ __launch_bounds__(256) void ln_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                const W* __restrict__ w, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, T* __restrict__ dx,
                                                float* __restrict__ part, int64_t rows, int D) {
  __shared__ float red[2][2][4];
  float wv[CPT][8], dw[CPT][8], db[CPT][8];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = (c * 256 + threadIdx.x) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) { dw[c][i] = 0.f; db[c][i] = 0.f; wv[c][i] = 0.f; }
    if (idx < D) Vec8<W>::load(w + idx, wv[c]);
  }
  int buf = 0;
  const float invD = 1.f / (float)D;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float mu = mean[r], rs = rstd[r];
    float xv[CPT][8], g[CPT][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int idx = (c * 256 + threadIdx.x) * 8;
      if (idx < D) {
        Vec8<T>::load(x + r * D + idx, xv[c]);
        Vec8<T>::load(dy + r * D + idx, g[c]);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) { xv[c][i] = 0.f; g[c][i] = 0.f; }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (xv[c][i] - mu) * rs;
        const float gw = g[c][i] * wv[c][i];
        dw[c][i] += g[c][i] * xh;
        db[c][i] += g[c][i];
        s1 += gw;
        s2 += gw * xh;
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if ((threadIdx.x & 63) == 0) { red[buf][0][threadIdx.x >> 6] = s1; red[buf][1][threadIdx.x >> 6] = s2; }
    __syncthreads();
    const float m1 = (red[buf][0][0] + red[buf][0][1] + red[buf][0][2] + red[buf][0][3]) * invD;
    const float m2 = (red[buf][1][0] + red[buf][1][1] + red[buf][1][2] + red[buf][1][3]) * invD;
    buf ^= 1;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int idx = (c * 256 + threadIdx.x) * 8;
      if (idx < D) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xh = (xv[c][i] - mu) * rs;
          o[i] = rs * (g[c][i] * wv[c][i] - m1 - xh * m2);
        }
        Vec8<T>::store(dx + r * D + idx, o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = (c * 256 + threadIdx.x) * 8;
    if (idx < D) {
      Vec8<float>::store(part + (int64_t)blockIdx.x * 2 * D + idx, dw[c]);
      Vec8<float>::store(part + (int64_t)blockIdx.x * 2 * D + D + idx, db[c]);
    }
  }
}

template <typename W>
__global__ __launch_bounds__(1024) void ln_col_reduce_k(const float* __restrict__ part, W* __restrict__ dw,
                                                        W* __restrict__ db, int nblk, int D) {
  __shared__ float red[2][16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float a = 0.f, c = 0.f;
  if (col < D)
    for (int b = wv; b < nblk; b += 16) {
      a += part[(int64_t)b * 2 * D + col];
      c += part[(int64_t)b * 2 * D + D + col];
    }
  red[0][wv][lane] = a;
  red[1][wv][lane] = c;
  __syncthreads();
  if (wv == 0 && col < D) {
    float ta = 0.f, tc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) { ta += red[0][k][lane]; tc += red[1][k][lane]; }
    dw[col] = (W)ta;
    db[col] = (W)tc;
  }
}

template <typename T, typename W>
static void ln_fwd_d(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                     int D, float eps, hipStream_t st) {
  const int grid = stream_grid(rows, 4);
#define L(N) hipLaunchKernelGGL((ln_fwd_k<T, W, N>), dim3(grid), dim3(256), 0, st, (const T*)x, (const W*)w, \
                                (const W*)b, (T*)y, mean, rstd, rows, D, eps)
  if (D <= 512) L(1);
  else if (D <= 1024) L(2);
  else if (D <= 2048) L(4);
  else if (D <= 4096) L(8);
  else L(16);
#undef L
}
template <typename T, typename W>
static void ln_bwd_d(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
                     float* part, void* dw, void* db, int nblk, int64_t rows, int D, hipStream_t st) {
#define L(N) hipLaunchKernelGGL((ln_bwd_k<T, W, N>), dim3(nblk), dim3(256), 0, st, (const T*)dy, (const T*)x, \
                                (const W*)w, mean, rstd, (T*)dx, part, rows, D)
  if (D <= 2048) L(1);
  else if (D <= 4096) L(2);
  else if (D <= 8192) L(4);
  else L(8);
#undef L
  hipLaunchKernelGGL((ln_col_reduce_k<W>), dim3((int)cdiv(D, 64)), dim3(1024), 0, st, part, (W*)dw, (W*)db, nblk, D);
}

void layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                   int dim, float eps, int xd, int wd, hipStream_t s) {
  if (rows == 0) return;
  if (xd == kBF16) {
    if (wd == kBF16) ln_fwd_d<bf16, bf16>(x, w, b, y, mean, rstd, rows, dim, eps, s);
    else ln_fwd_d<bf16, float>(x, w, b, y, mean, rstd, rows, dim, eps, s);
  } else {
    if (wd == kBF16) ln_fwd_d<float, bf16>(x, w, b, y, mean, rstd, rows, dim, eps, s);
    else ln_fwd_d<float, float>(x, w, b, y, mean, rstd, rows, dim, eps, s);
  }
}
void layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
                   float* part, void* dw, void* db, int nblk, int64_t rows, int dim, int xd, int wd, hipStream_t s) {
  if (xd == kBF16) {
    if (wd == kBF16) ln_bwd_d<bf16, bf16>(dy, x, w, mean, rstd, dx, part, dw, db, nblk, rows, dim, s);
    else ln_bwd_d<bf16, float>(dy, x, w, mean, rstd, dx, part, dw, db, nblk, rows, dim, s);
  } else {
    if (wd == kBF16) ln_bwd_d<float, bf16>(dy, x, w, mean, rstd, dx, part, dw, db, nblk, rows, dim, s);
    else ln_bwd_d<float, float>(dy, x, w, mean, rstd, dx, part, dw, db, nblk, rows, dim, s);
  }
}

}  // namespace dph
