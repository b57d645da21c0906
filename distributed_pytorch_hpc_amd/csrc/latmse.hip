// Latitude-weighted MSE of the ERA5 UNet / ViT drivers (reference: scripts/01_data_parallel_ddp/
// multinode_ddp_unet.py:221-229, duplicated in multinode_fsdp_unet.py:119-127 and tensor_parallel_vit.py:209-217):
//   loss = mean_{b,c,h,w} w[h] (pred - target)^2,   w[h] = cos(lat_h) / mean_h cos(lat_h),  lat on a 90..-90 grid.
// The reference materialises w as a [1, 1, H, 1] tensor, the difference, its square and the weighted product
// (four full-size temporaries in fp32).  Here the weight is computed in-kernel from the row index (one cosf per
// 8 elements) and the reduction is one pass: per-workgroup partial sums into a [G] buffer, then a fixed-order
// sum (bit-reproducible).  The backward is one elementwise pass writing d/dpred (and -d/dpred for the target).
// A latitude-sharded field (domain parallelism) passes its global row offset and the global grid size.
// NCHW and channels-last layouts are both read in place: the row of flat element i is (i / step) % H with
// step = W (NCHW) or W*C (NHWC).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int LM_NT = 256;

struct LatGrid {
  int64_t H, W;          // local rows; elements per row step (W for NCHW, W*C for channels-last)
  int64_t lat_offset;    // first local row in the global grid
  float deg_per_row;     // 180 / (n_global - 1)
  float inv_mean_cos;    // 1 / mean(cos(lat)) over the global grid
};

__device__ __forceinline__ float lat_weight(const LatGrid& g, int64_t h) {
  const float lat = 90.f - g.deg_per_row * (float)(h + g.lat_offset);
  return cosf(lat * 0.017453292519943295f) * g.inv_mean_cos;
}

// Vector path: the row step is a multiple of 8, so an 8-element vector never straddles a row.
template <typename T, bool VEC>
__global__ __launch_bounds__(LM_NT) void latmse_fwd_k(const T* __restrict__ p, const T* __restrict__ t,
                                                      float* __restrict__ part, int64_t n, LatGrid g) {
  __shared__ float red[LM_NT / 64];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * LM_NT;
  if (VEC) {
    for (int64_t v = (int64_t)blockIdx.x * LM_NT + threadIdx.x; v < n / 8; v += stride) {
      float a[8], b[8];
      Vec8<T>::load(p + v * 8, a);
      Vec8<T>::load(t + v * 8, b);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = a[i] - b[i];
        s = fmaf(d, d, s);
      }
      acc = fmaf(lat_weight(g, (v * 8 / g.W) % g.H), s, acc);
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * LM_NT + threadIdx.x; i < n; i += stride) {
      const float d = (float)p[i] - (float)t[i];
      acc = fmaf(lat_weight(g, (i / g.W) % g.H), d * d, acc);
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LM_NT / 64; ++i) s += red[i];
    part[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(LM_NT) void latmse_sum_k(const float* __restrict__ part, int G, float inv_n,
                                                      float* __restrict__ out) {
  __shared__ float red[LM_NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < G; i += LM_NT) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < LM_NT / 64; ++i) r += red[i];
    out[0] = r * inv_n;
  }
}

// dpred = gscale * w[h] * (p - t) with gscale = 2 * dloss / n read from device memory (no host sync).
template <typename T, bool VEC, bool DT>
__global__ __launch_bounds__(LM_NT) void latmse_bwd_k(const T* __restrict__ p, const T* __restrict__ t,
                                                      const float* __restrict__ gloss, float two_over_n,
                                                      T* __restrict__ dp, T* __restrict__ dtg, int64_t n, LatGrid g) {
  const float gs = gloss[0] * two_over_n;
  const int64_t stride = (int64_t)gridDim.x * LM_NT;
  if (VEC) {
    for (int64_t v = (int64_t)blockIdx.x * LM_NT + threadIdx.x; v < n / 8; v += stride) {
      float a[8], b[8], o[8];
      Vec8<T>::load(p + v * 8, a);
      Vec8<T>::load(t + v * 8, b);
      const float ws = gs * lat_weight(g, (v * 8 / g.W) % g.H);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = ws * (a[i] - b[i]);
      Vec8<T>::store(dp + v * 8, o);
      if (DT) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = -o[i];
        Vec8<T>::store(dtg + v * 8, o);
      }
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * LM_NT + threadIdx.x; i < n; i += stride) {
      const float o = gs * lat_weight(g, (i / g.W) % g.H) * ((float)p[i] - (float)t[i]);
      dp[i] = (T)o;
      if (DT) dtg[i] = (T)(-o);
    }
  }
}

LatGrid make_grid(int64_t H, int64_t W, int64_t n_global, int64_t lat_offset) {
  LatGrid g;
  g.H = H;
  g.W = W;
  g.lat_offset = lat_offset;
  g.deg_per_row = n_global > 1 ? (float)(180.0 / (double)(n_global - 1)) : 0.f;
  double s = 0.0;
  for (int64_t i = 0; i < n_global; ++i) {
    const double lat = 90.0 - (n_global > 1 ? 180.0 * (double)i / (double)(n_global - 1) : 0.0);
    s += cos(lat * 3.141592653589793 / 180.0);
  }
  const double mean = s / (double)(n_global > 0 ? n_global : 1);
  g.inv_mean_cos = mean != 0.0 ? (float)(1.0 / mean) : 0.f;
  return g;
}

}  // namespace

int latmse_partial_blocks(int64_t n) { return stream_grid(n / 8 + 1, LM_NT); }

void latmse_fwd(const void* pred, const void* target, float* partial, float* out, int64_t n, int64_t H, int64_t W,
                int64_t n_global, int64_t lat_offset, int dt, hipStream_t st) {
  const LatGrid g = make_grid(H, W, n_global, lat_offset);   // W = row step
  const int G = latmse_partial_blocks(n);
  const bool vec = (W % 8) == 0;
  DPH_DISPATCH_FLOAT(dt, T, {
    if (vec) hipLaunchKernelGGL((latmse_fwd_k<T, true>), dim3(G), dim3(LM_NT), 0, st, (const T*)pred,
                                (const T*)target, partial, n, g);
    else hipLaunchKernelGGL((latmse_fwd_k<T, false>), dim3(G), dim3(LM_NT), 0, st, (const T*)pred,
                            (const T*)target, partial, n, g);
  });
  hipLaunchKernelGGL(latmse_sum_k, dim3(1), dim3(LM_NT), 0, st, partial, G, 1.f / (float)n, out);
}

void latmse_bwd(const void* pred, const void* target, const float* gloss, void* dpred, void* dtarget, int64_t n,
                int64_t H, int64_t W, int64_t n_global, int64_t lat_offset, int dt, hipStream_t st) {
  const LatGrid g = make_grid(H, W, n_global, lat_offset);
  const dim3 grid(stream_grid(n / 8 + 1, LM_NT));
  const bool vec = (W % 8) == 0;
  const float two_over_n = 2.f / (float)n;
#define DPH_LM_BWD(V_, D_)                                                                                   \
  hipLaunchKernelGGL((latmse_bwd_k<T, V_, D_>), grid, dim3(LM_NT), 0, st, (const T*)pred, (const T*)target, \
                     gloss, two_over_n, (T*)dpred, (T*)dtarget, n, g)
  DPH_DISPATCH_FLOAT(dt, T, {
    if (vec && dtarget) DPH_LM_BWD(true, true);
    else if (vec) DPH_LM_BWD(true, false);
    else if (dtarget) DPH_LM_BWD(false, true);
    else DPH_LM_BWD(false, false);
  });
#undef DPH_LM_BWD
}

}  // namespace dph
