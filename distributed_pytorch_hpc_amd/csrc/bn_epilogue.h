// BatchNorm backward reduction in a convolution's input-gradient epilogue (kernels.h BnRed), shared by the 1x1
// (conv1x1.hip ts_nt_k) and 3x3 (conv3x3.hip conv3_k) kernels.
//
// The epilogue stores the bf16 output tile as 16-B row segments; a thread's column chunk is fixed for the whole store
// loop (the loop stride is a multiple of the chunks per row), so each thread keeps the 8 channels' mean / invstd /
// mask coefficients in registers, reads the BatchNorm input x (and the mask byte) at the segment it stores, and
// accumulates sum dz and sum dz * xhat of the values it stores.  Then lanes of one chunk meet by xor shuffles, the
// waves through LDS in a fixed order, and the tile writes one [2][BN] row of partials per 128-row block (no atomics:
// the BatchNorm's finalize kernel sums the rows in a fixed order, so the result is deterministic).
#pragma once

#include "dph_common.h"
#include "kernels.h"

namespace dph {

template <int MODE>   // 1: ReLU mask from x * scale + shift (BatchNorm without residual), 2: the forward's mask bits
struct BnRedAcc {
  float mu[8], is[8], sc[8], sf[8], sd[8], sdx[8];

  __device__ __forceinline__ void init(const BnRed& r, int c0, int C) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mu[i] = r.mean[c0 + i];
      is[i] = r.invstd[c0 + i];
      sc[i] = MODE == 1 ? r.ss[c0 + i] : 0.f;
      sf[i] = MODE == 1 ? r.ss[C + c0 + i] : 0.f;
      sd[i] = 0.f;
      sdx[i] = 0.f;
    }
  }

  // x / the mask byte of row `row`, channels c0 .. c0 + 7 (x and the mask bits are [M, C]): the kernels fetch them
  // a few store iterations ahead (their latency would otherwise be exposed once per iteration)
  __device__ static __forceinline__ bf16x8 load_x(const BnRed& r, int64_t row, int C, int c0) {
    return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(r.x) + row * C + c0);
  }
  __device__ static __forceinline__ unsigned load_m(const BnRed& r, int64_t row, int C, int c0) {
    return MODE == 2 ? (unsigned)r.bits[row * (C >> 3) + (c0 >> 3)] : 0u;
  }

  // g: the 8 stored (bf16) gradient values at those positions
  __device__ __forceinline__ void add(const bf16x8& xv, unsigned mb, const bf16x8& g) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float x = (float)xv[i];
      const bool on = MODE == 2 ? ((mb >> i) & 1u) != 0u : fmaf(x, sc[i], sf[i]) > 0.f;
      const float dz = on ? (float)g[i] : 0.f;
      sd[i] += dz;
      sdx[i] = fmaf(dz, (x - mu[i]) * is[i], sdx[i]);
    }
  }

  // Block reduction into part row g (columns n0 .. n0 + 8 cpr of [2][C]).  Called by every thread of the workgroup
  // after a barrier that ends all reads of `lds` (>= nwv * cpr * 64 bytes); cpr = chunks per row (power of two <= 64).
  __device__ __forceinline__ void finish(float* lds, int cpr, int nwv, int64_t g, int C, int n0, float* part) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int off = cpr; off < 64; off <<= 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sd[i] += __shfl_xor(sd[i], off);
        sdx[i] += __shfl_xor(sdx[i], off);
      }
    }
    if (lane < cpr) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        lds[(wid * cpr + lane) * 16 + i] = sd[i];
        lds[(wid * cpr + lane) * 16 + 8 + i] = sdx[i];
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < cpr * 8; col += nwv * 64) {
      const int ch = col >> 3, i = col & 7;
      float a = 0.f, b = 0.f;
      for (int w = 0; w < nwv; ++w) {
        a += lds[(w * cpr + ch) * 16 + i];
        b += lds[(w * cpr + ch) * 16 + 8 + i];
      }
      part[g * 2 * C + n0 + col] = a;
      part[g * 2 * C + C + n0 + col] = b;
    }
  }
};

}  // namespace dph
