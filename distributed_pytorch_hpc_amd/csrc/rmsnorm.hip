// RMSNorm forward/backward for CDNA4.
// Semantics follow the reference RMSNorm (fsdp_tp/llama2_model.py:115-142): statistics in fp32,
// y = x * rsqrt(mean(x^2) + eps) * w.  Optional fused residual add: h = x + residual, y = norm(h)
// (saves one full read of the residual stream per transformer sub-block).
//
// Forward: one wave per row, the row held in registers (D <= 8192: up to 16 x 16-B chunks per lane),
// wave-shuffle reduction, no LDS, no barrier.  Memory bound: 1 read + 1 write per element.
// Backward: one 256-thread workgroup per row-set (grid-stride over rows); dW partials stay in registers
// across rows and are written once per workgroup, then reduced by a column kernel (deterministic,
// no atomics).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

template <typename T, typename W, int NCH, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_k(const T* __restrict__ x, const W* __restrict__ w,
                                                     const T* __restrict__ res, T* __restrict__ h_out,
                                                     T* __restrict__ y, float* __restrict__ rstd, int64_t rows,
                                                     int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wid; r < rows; r += (int64_t)gridDim.x * 4) {
    const T* xr = x + r * D;
    float v[NCH][8];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) {
        Vec8<T>::load(xr + idx, v[c]);
        if (RES) {
          float rr[8];
          Vec8<T>::load(res + r * D + idx, rr);
#pragma unroll
          for (int i = 0; i < 8; ++i) v[c][i] = (float)(T)(v[c][i] + rr[i]);  // h rounded as stored
          Vec8<T>::store(h_out + r * D + idx, v[c]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
      }
    }
    ss = wave_sum(ss);
    const float rs = rsqrtf(ss / (float)D + eps);
    if (lane == 0 && rstd) rstd[r] = rs;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) {
        float wv[8], o[8];
        Vec8<W>::load(w + idx, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = v[c][i] * rs * wv[i];
        Vec8<T>::store(y + r * D + idx, o);
      }
    }
  }
}

// Generic fallback: D > 8192 (one workgroup per row, two passes through L2).
template <typename T, typename W, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_big_k(const T* __restrict__ x, const W* __restrict__ w,
                                                         const T* __restrict__ res, T* __restrict__ h_out,
                                                         T* __restrict__ y, float* __restrict__ rstd, int64_t rows,
                                                         int D, float eps) {
  __shared__ float red[4];
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const T* xr = RES ? h_out + r * D : x + r * D;
    float ss = 0.f;
    for (int idx = threadIdx.x * 8; idx < D; idx += 256 * 8) {
      float v[8];
      Vec8<T>::load(x + r * D + idx, v);
      if (RES) {
        float rr[8];
        Vec8<T>::load(res + r * D + idx, rr);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)(T)(v[i] + rr[i]);
        Vec8<T>::store(h_out + r * D + idx, v);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    const float rs = rsqrtf(tot / (float)D + eps);
    if (threadIdx.x == 0 && rstd) rstd[r] = rs;
    for (int idx = threadIdx.x * 8; idx < D; idx += 256 * 8) {
      float v[8], wv[8];
      Vec8<T>::load(xr + idx, v);
      Vec8<W>::load(w + idx, wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = v[i] * rs * wv[i];
      Vec8<T>::store(y + r * D + idx, v);
    }
  }
}

// Few rows (decode: one per sequence): one 256-thread workgroup per row instead of one wave, and the weight loads
// issued together with x / residual -- one memory round trip instead of two, 4 waves per row instead of 1.
// CPT = 16-B chunks per thread (D <= CPT * 2048).
template <typename T, typename W, int CPT, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_row_k(const T* __restrict__ x, const W* __restrict__ w,
                                                         const T* __restrict__ res, T* __restrict__ h_out,
                                                         T* __restrict__ y, float* __restrict__ rstd, int D,
                                                         float eps) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  float v[CPT][8], wv[CPT][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = (c * 256 + threadIdx.x) * 8;
    if (idx < D) {
      Vec8<T>::load(x + r * D + idx, v[c]);
      Vec8<W>::load(w + idx, wv[c]);
      if (RES) {
        float rr[8];
        Vec8<T>::load(res + r * D + idx, rr);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = (float)(T)(v[c][i] + rr[i]);   // h rounded as stored
        Vec8<T>::store(h_out + r * D + idx, v[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)D + eps);
  if (threadIdx.x == 0 && rstd) rstd[r] = rs;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = (c * 256 + threadIdx.x) * 8;
    if (idx < D) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[c][i] * rs * wv[c][i];
      Vec8<T>::store(y + r * D + idx, o);
    }
  }
}

// Backward. CPT = 16-B chunks per thread (D <= CPT * 2048).
template <typename T, typename W, int CPT>
__global__ __launch_bounds__(256) void rmsnorm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const W* __restrict__ w, const float* __restrict__ rstd,
                                                     const T* __restrict__ dres, T* __restrict__ dx,
                                                     float* __restrict__ dw_partial, int64_t rows, int D) {
  __shared__ float red[2][4];
  float wv[CPT][8], dwacc[CPT][8];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = (c * 256 + threadIdx.x) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) dwacc[c][i] = 0.f;
    if (idx < D) Vec8<W>::load(w + idx, wv[c]);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) wv[c][i] = 0.f;
    }
  }
  int buf = 0;
  const float invD = 1.f / (float)D;
  // rows are software-pipelined: the next row's x / dy loads are issued before this row's block reduction, so
  // they are in flight across the barrier instead of starting after it
  auto load_row = [&](int64_t r, float (&xv)[CPT][8], float (&g)[CPT][8], float (&d)[CPT][8]) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int idx = (c * 256 + threadIdx.x) * 8;
      if (idx < D) {
        Vec8<T>::load(x + r * D + idx, xv[c]);
        Vec8<T>::load(dy + r * D + idx, g[c]);
        if (dres) Vec8<T>::load(dres + r * D + idx, d[c]);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) { xv[c][i] = 0.f; g[c][i] = 0.f; d[c][i] = 0.f; }
      }
    }
  };
  float xv[CPT][8], g[CPT][8], dr[CPT][8];
  if ((int64_t)blockIdx.x < rows) load_row(blockIdx.x, xv, g, dr);
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float rs = rstd[r];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = xv[c][i] * rs;
        dwacc[c][i] += g[c][i] * xh;
        dot += g[c][i] * wv[c][i] * xh;
      }
    }
    float xn[CPT][8], gn[CPT][8], dn[CPT][8];
    const int64_t rn = r + gridDim.x;
    if (rn < rows) load_row(rn, xn, gn, dn);
    dot = wave_sum(dot);
    if ((threadIdx.x & 63) == 0) red[buf][threadIdx.x >> 6] = dot;
    __syncthreads();
    const float mdot = (red[buf][0] + red[buf][1] + red[buf][2] + red[buf][3]) * invD;
    buf ^= 1;  // double-buffered reduction slot: one barrier per row
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int idx = (c * 256 + threadIdx.x) * 8;
      if (idx < D) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xh = xv[c][i] * rs;
          o[i] = rs * (g[c][i] * wv[c][i] - xh * mdot);
        }
        if (dres) {
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += dr[c][i];
        }
        Vec8<T>::store(dx + r * D + idx, o);
      }
    }
    if (rn < rows) {
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int i = 0; i < 8; ++i) { xv[c][i] = xn[c][i]; g[c][i] = gn[c][i]; dr[c][i] = dn[c][i]; }
    }
  }
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = (c * 256 + threadIdx.x) * 8;
    if (idx < D) Vec8<float>::store(dw_partial + (int64_t)blockIdx.x * D + idx, dwacc[c]);
  }
}

// Column reduction of [nblk, D] fp32 partials -> dw (W dtype): one 1024-thread workgroup per 64 columns,
// each of its 16 waves sums a strided subset of the partial rows (256-B coalesced row segments), then LDS.
template <typename W>
__global__ __launch_bounds__(1024) void col_reduce_k(const float* __restrict__ part, W* __restrict__ out, int nblk,
                                                     int D) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < D)
    for (int b = wv; b < nblk; b += 16) s += part[(int64_t)b * D + col];
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    if (col < D) out[col] = (W)t;
  }
}

template <typename T, typename W>
static void fwd_dispatch(const void* x, const void* w, const void* res, void* h_out, void* y, float* rstd,
                         int64_t rows, int D, float eps, hipStream_t st) {
  const int grid = stream_grid(rows, 4);
  const T* xp = (const T*)x; const W* wp = (const W*)w; const T* rp = (const T*)res;
  T* hp = (T*)h_out; T* yp = (T*)y;
  if (rows <= 1024 && D <= 8192) {   // decode-sized: a workgroup per row
#define ROWL(C)                                                                                                \
  if (res) hipLaunchKernelGGL((rmsnorm_fwd_row_k<T, W, C, true>), dim3((unsigned)rows), dim3(256), 0, st, xp, wp, \
                              rp, hp, yp, rstd, D, eps);                                                       \
  else hipLaunchKernelGGL((rmsnorm_fwd_row_k<T, W, C, false>), dim3((unsigned)rows), dim3(256), 0, st, xp, wp, rp, \
                          hp, yp, rstd, D, eps);
    if (D <= 2048) { ROWL(1) }
    else if (D <= 4096) { ROWL(2) }
    else { ROWL(4) }
#undef ROWL
    return;
  }
#define LAUNCH(N)                                                                                       \
  if (res) hipLaunchKernelGGL((rmsnorm_fwd_k<T, W, N, true>), dim3(grid), dim3(256), 0, st, xp, wp, rp, hp, yp, \
                              rstd, rows, D, eps);                                                      \
  else hipLaunchKernelGGL((rmsnorm_fwd_k<T, W, N, false>), dim3(grid), dim3(256), 0, st, xp, wp, rp, hp, yp,   \
                          rstd, rows, D, eps);
  if (D <= 512) { LAUNCH(1) }
  else if (D <= 1024) { LAUNCH(2) }
  else if (D <= 2048) { LAUNCH(4) }
  else if (D <= 4096) { LAUNCH(8) }
  else if (D <= 8192) { LAUNCH(16) }
  else {
    const int g2 = (int)(rows < 4096 ? rows : 4096);
    if (res) hipLaunchKernelGGL((rmsnorm_fwd_big_k<T, W, true>), dim3(g2), dim3(256), 0, st, xp, wp, rp, hp, yp,
                                rstd, rows, D, eps);
    else hipLaunchKernelGGL((rmsnorm_fwd_big_k<T, W, false>), dim3(g2), dim3(256), 0, st, xp, wp, rp, hp, yp,
                            rstd, rows, D, eps);
  }
#undef LAUNCH
}

void rmsnorm_fwd(const void* x, const void* w, const void* residual, void* h_out, void* y, float* rstd,
                 int64_t rows, int dim, float eps, int x_dtype, int w_dtype, hipStream_t stream) {
  if (rows == 0) return;
  if (x_dtype == kBF16) {
    if (w_dtype == kBF16) fwd_dispatch<bf16, bf16>(x, w, residual, h_out, y, rstd, rows, dim, eps, stream);
    else fwd_dispatch<bf16, float>(x, w, residual, h_out, y, rstd, rows, dim, eps, stream);
  } else {
    if (w_dtype == kBF16) fwd_dispatch<float, bf16>(x, w, residual, h_out, y, rstd, rows, dim, eps, stream);
    else fwd_dispatch<float, float>(x, w, residual, h_out, y, rstd, rows, dim, eps, stream);
  }
}

int rmsnorm_bwd_blocks(int64_t rows) {
  int64_t g = rows < 512 ? rows : 512;
  return (int)(g < 1 ? 1 : g);
}

template <typename T, typename W>
static void bwd_dispatch(const void* dy, const void* x, const void* w, const float* rstd, const void* dres, void* dx,
                         float* part, void* dw, int nblk, int64_t rows, int D, hipStream_t st) {
  const T* dyp = (const T*)dy; const T* xp = (const T*)x; const W* wp = (const W*)w; T* dxp = (T*)dx;
#define LAUNCHB(N) hipLaunchKernelGGL((rmsnorm_bwd_k<T, W, N>), dim3(nblk), dim3(256), 0, st, dyp, xp, wp, rstd, \
                                      (const T*)dres, dxp, part, rows, D);
  if (D <= 2048) { LAUNCHB(1) }
  else if (D <= 4096) { LAUNCHB(2) }
  else if (D <= 8192) { LAUNCHB(4) }
  else if (D <= 16384) { LAUNCHB(8) }
  else { LAUNCHB(16) }
#undef LAUNCHB
  hipLaunchKernelGGL((col_reduce_k<W>), dim3((int)cdiv(D, 64)), dim3(1024), 0, st, part, (W*)dw, nblk, D);
}

void rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dres, void* dx,
                 float* dw_partial, void* dw, int nblk, int64_t rows, int dim, int x_dtype, int w_dtype,
                 hipStream_t stream) {
  if (x_dtype == kBF16) {
    if (w_dtype == kBF16) bwd_dispatch<bf16, bf16>(dy, x, w, rstd, dres, dx, dw_partial, dw, nblk, rows, dim, stream);
    else bwd_dispatch<bf16, float>(dy, x, w, rstd, dres, dx, dw_partial, dw, nblk, rows, dim, stream);
  } else {
    if (w_dtype == kBF16) bwd_dispatch<float, bf16>(dy, x, w, rstd, dres, dx, dw_partial, dw, nblk, rows, dim, stream);
    else bwd_dispatch<float, float>(dy, x, w, rstd, dres, dx, dw_partial, dw, nblk, rows, dim, stream);
  }
}

}  // namespace dph
