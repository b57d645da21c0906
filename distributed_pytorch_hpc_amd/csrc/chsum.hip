// Per-channel sum of a channels-last activation gradient, out[c] = sum_m dy[m, c] for a row-major [M, C] view
// (M = N*H*W): the bias gradient of a convolution.
//
// ATen computes a channels-last convolution's bias gradient as a reduction over the outer dimension; with an odd
// channel count (the reference SimpleUNet's 65-channel output convolution, multinode_ddp_unet.py:171-214) that
// reduction took 1.9 ms for a 34 MB gradient on an MI355X (profiles/r2s3/rocprof_unet_*).  Here: pass 1 gives each
// workgroup a contiguous slab of rows; its 256 threads form R = 256 / C row lanes x C channel lanes (C <= 256; wider
// C loops over 256-channel chunks with R = 1), so consecutive lanes read consecutive channels of one row
// (coalesced 2- or 4-byte loads), fp32 accumulation, a fixed-order LDS sum over the row lanes and one fp32
// partial per (slab, channel); pass 2 sums the slabs of a channel in order.  Deterministic, no atomics.
#include <algorithm>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int CS_NT = 256;

template <typename T>
__global__ __launch_bounds__(CS_NT) void chsum_partial_k(const T* __restrict__ x, float* __restrict__ part,
                                                         int64_t M, int C, int64_t rows_per_block) {
  __shared__ float sh[CS_NT];
  const int64_t beg = (int64_t)blockIdx.x * rows_per_block, end = min(M, beg + rows_per_block);
  const int R = C <= CS_NT ? CS_NT / C : 1;
  const int lane_r = threadIdx.x / min(C, CS_NT), lane_c = threadIdx.x % min(C, CS_NT);
  const bool active = lane_r < R;
  for (int c0 = 0; c0 < C; c0 += CS_NT) {
    const int c = c0 + lane_c;
    float acc = 0.f;
    if (active && c < C) {
      for (int64_t r = beg + lane_r; r < end; r += R) acc += (float)x[r * C + c];
    }
    sh[threadIdx.x] = acc;
    __syncthreads();
    if (lane_r == 0 && c < C) {
      float s = sh[threadIdx.x];
      for (int k = 1; k < R; ++k) s += sh[k * min(C, CS_NT) + lane_c];
      part[(int64_t)blockIdx.x * C + c] = s;
    }
    __syncthreads();
  }
}

// C % 8 == 0 and C <= 2048 (every UNet convolution but the 65-channel output): a lane owns an 8-channel chunk and
// reads it with one 16-B load per row; 256 / (C / 8) row lanes, then the same fixed-order sum over the row lanes.
template <typename T>
__global__ __launch_bounds__(CS_NT) void chsum_partial_vec_k(const T* __restrict__ x, float* __restrict__ part,
                                                             int64_t M, int C, int64_t rows_per_block) {
  __shared__ float sh[CS_NT * 8];
  const int ch8 = C / 8, R = CS_NT / ch8;
  const int lane_r = threadIdx.x / ch8, lane_c = threadIdx.x % ch8;
  const int64_t beg = (int64_t)blockIdx.x * rows_per_block, end = min(M, beg + rows_per_block);
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  for (int64_t r = beg + lane_r; r < end; r += R) {
    float v[8];
    Vec8<T>::load(x + r * C + lane_c * 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += v[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) sh[threadIdx.x * 8 + i] = acc[i];
  __syncthreads();
  if (lane_r == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float t = sh[threadIdx.x * 8 + i];
      for (int k = 1; k < R; ++k) t += sh[(k * ch8 + lane_c) * 8 + i];
      part[(int64_t)blockIdx.x * C + lane_c * 8 + i] = t;
    }
  }
}

// one workgroup per channel: threads stride over the slabs, then a fixed-order LDS tree
template <typename OT>
__global__ __launch_bounds__(CS_NT) void chsum_final_k(const float* __restrict__ part, OT* __restrict__ out, int G,
                                                      int C) {
  __shared__ float sh[CS_NT];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int g = threadIdx.x; g < G; g += CS_NT) s += part[(int64_t)g * C + c];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int h = CS_NT / 2; h > 0; h >>= 1) {
    if (threadIdx.x < h) sh[threadIdx.x] += sh[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[c] = (OT)sh[0];
}

}  // namespace

int chsum_partial_blocks(int64_t M, int64_t C) {
  // >= ~16 KB of input per workgroup, at most 1024 workgroups (4 per CU)
  const int64_t min_rows = std::max<int64_t>(16, 8192 / std::max<int64_t>(C, 1));
  int64_t g = std::min<int64_t>(1024, (M + min_rows - 1) / min_rows);
  return (int)std::max<int64_t>(g, 1);
}

void chsum(const void* x, float* part, void* out, int64_t M, int64_t C, int dtype, int out_dtype, hipStream_t st) {
  const int G = chsum_partial_blocks(M, C);
  const int64_t rpb = (M + G - 1) / G;
  const bool vec = C % 8 == 0 && C <= 8 * CS_NT && (CS_NT % (C / 8)) == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0;
  DPH_DISPATCH_FLOAT(dtype, T, {
    if (vec)
      hipLaunchKernelGGL(chsum_partial_vec_k<T>, dim3(G), dim3(CS_NT), 0, st, (const T*)x, part, M, (int)C, rpb);
    else
      hipLaunchKernelGGL(chsum_partial_k<T>, dim3(G), dim3(CS_NT), 0, st, (const T*)x, part, M, (int)C, rpb);
  });
  const dim3 fg((unsigned)C);
  if (out_dtype == kBF16)
    hipLaunchKernelGGL(chsum_final_k<bf16>, fg, dim3(CS_NT), 0, st, (const float*)part, (bf16*)out, G, (int)C);
  else
    hipLaunchKernelGGL(chsum_final_k<float>, fg, dim3(CS_NT), 0, st, (const float*)part, (float*)out, G, (int)C);
}

}  // namespace dph
