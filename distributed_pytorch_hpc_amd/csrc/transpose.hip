// 2-D transpose of a row-major bf16 matrix, dst[C, R] = src[R, C]^T, at HBM bandwidth.
// Used to give hipBLASLt the K-contiguous operand pattern it runs fastest (the input-gradient GEMM
// dX = dY W reads W^T: profiles/gemm_layout_*.json), where torch's strided copy reaches ~1 TB/s.
// 64 x 64 tiles through LDS (row pitch 66 elements: 33 dwords, so the column-wise reads of the store phase
// hit 32 different banks); 16-B vector loads and stores on both global sides.
#include <algorithm>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {
constexpr int TT = 64, PITCH = 66;

// gridDim.z > 1: a batch of transposes, matrix z read at src + (REV ? nz - 1 - z : z) * sz, written at dst + z * dz.
__global__ __launch_bounds__(256) void transpose_k(const bf16* __restrict__ src, bf16* __restrict__ dst, int64_t R,
                                                   int64_t C, int64_t lds_src, int64_t ld_dst, int64_t sz = 0,
                                                   int64_t dz = 0, bool rev = false) {
  __shared__ bf16 tile[TT * PITCH];
  const int z = blockIdx.z, nz = gridDim.z;
  src += (rev ? nz - 1 - z : z) * sz;
  dst += z * dz;
  const int64_t r0 = (int64_t)blockIdx.y * TT, c0 = (int64_t)blockIdx.x * TT;
  const int t = threadIdx.x;
  // load: 64 rows x 8 chunks of 8 elements; 2 chunks per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = t + 256 * i, row = idx >> 3, ch = idx & 7;
    const int64_t gr = r0 + row, gc = c0 + ch * 8;
    bf16x8 v;
    if (gr < R && gc + 8 <= C) {
      v = *reinterpret_cast<const bf16x8*>(src + gr * lds_src + gc);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (gr < R && gc + j < C) ? src[gr * lds_src + gc + j] : (bf16)0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[row * PITCH + ch * 8 + j] = v[j];
  }
  __syncthreads();
  // store: dst row = source column (64 of them) x 8 chunks of 8 source rows
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = t + 256 * i, col = idx >> 3, ch = idx & 7;
    const int64_t gr = c0 + col, gc = r0 + ch * 8;   // dst coordinates
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[(ch * 8 + j) * PITCH + col];
    if (gr < C && gc + 8 <= R) {
      *reinterpret_cast<bf16x8*>(dst + gr * ld_dst + gc) = v;
    } else if (gr < C) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (gc + j < R) dst[gr * ld_dst + gc + j] = v[j];
    }
  }
}

// dst[r, 0:C] = src[r, 0:C], dst[r, C:Cp] = 0: one 16-B output chunk per thread (Cp % 8 == 0), source rows of any
// length and stride (SimpleUNet's 65-channel pixels -> 128-channel rows for the 64-multiple conv kernels).
__global__ __launch_bounds__(256) void pad_cols_k(const bf16* __restrict__ src, bf16* __restrict__ dst, int64_t R,
                                                  int64_t C, int64_t ld_src, int64_t Cp) {
  const int64_t chunks = Cp / 8;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < R * chunks; idx += (int64_t)gridDim.x * 256) {
    const int64_t r = idx / chunks, c = (idx % chunks) * 8;
    const bf16* s = src + r * ld_src + c;
    bf16x8 v;
    if (c + 8 <= C && ((ld_src | c) & 7) == 0) {
      v = *reinterpret_cast<const bf16x8*>(s);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c + j < C ? s[j] : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(dst + r * Cp + c) = v;
  }
}
}  // namespace

void pad_cols(const void* src, void* dst, int64_t R, int64_t C, int64_t ld_src, int64_t Cp, hipStream_t st) {
  if (R == 0) return;
  const int64_t work = R * (Cp / 8);
  const unsigned blocks = (unsigned)std::min<int64_t>((work + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(pad_cols_k, dim3(blocks), dim3(256), 0, st, (const bf16*)src, (bf16*)dst, R, C, ld_src, Cp);
}

void transpose2d(const void* src, void* dst, int64_t R, int64_t C, int64_t ld_src, int64_t ld_dst, hipStream_t st) {
  if (R == 0 || C == 0) return;
  const dim3 grid((unsigned)((C + TT - 1) / TT), (unsigned)((R + TT - 1) / TT));
  hipLaunchKernelGGL(transpose_k, grid, dim3(256), 0, st, (const bf16*)src, (bf16*)dst, R, C, ld_src, ld_dst,
                     (int64_t)0, (int64_t)0, false);
}

void conv3x3_dgrad_weight(const void* w, void* out, int64_t cout, int64_t cin, hipStream_t st) {
  // w: channels-last [cout][3][3][cin]; out[c][t][co] = w[co][8 - t][c] -- nine [cout, cin] transposes, taps reversed
  if (cout == 0 || cin == 0) return;
  const dim3 grid((unsigned)((cin + TT - 1) / TT), (unsigned)((cout + TT - 1) / TT), 9u);
  hipLaunchKernelGGL(transpose_k, grid, dim3(256), 0, st, (const bf16*)w, (bf16*)out, cout, cin, 9 * cin, 9 * cout,
                     cin, cout, true);
}

}  // namespace dph
