// Stride-2 max pooling on channels-last (NHWC) activations: 3x3 / padding 1 (the ResNet stem's MaxPool2d, torchvision
// layout of scripts/main.py's resnet50: conv1 7x7/2 -> bn1 -> relu -> maxpool 3x3/2/1) and 2x2 / padding 0 (the
// SimpleUNet encoder's MaxPool2d(2), multinode_ddp_unet.py:171-214; floor mode, so an odd last row / column is
// dropped as in ATen).
//
// ATen's NHWC max_pool backward scatters through 64-bit indices and took 0.67 ms of a ResNet-50 B=256 step
// (profiles/rocprof_resnet50_fsdp_bf16_r2_summary.txt) for a 411 MB input gradient.  Here:
//   forward : one thread = one output pixel x 8 channels; the K*K taps are 16-B loads; the window position of the
//             max (0..K*K-1) is kept as one byte per element (8 B per thread, one store) instead of an int64 flat
//             index; ties and NaNs resolve exactly like ATen (scan kh-major, take v > max or NaN).
//   backward: a GATHER per input pixel (no atomics, deterministic): input row iy is covered by the output rows oy
//             with 2 oy - P <= iy <= 2 oy - P + K - 1 (3x3/1: at most 2, 2x2/0: one) and receives dy of each window
//             whose stored tap is its own (fp32 sum, one rounding).  dx is written exactly once, so no zero-fill
//             pass (rows / columns outside every window get 0).
// Traffic: forward reads x (the 9-fold reuse stays in L2) and writes y + 1 byte/elem; backward reads dy + taps
// (each about 2.25x, L2) and writes dx: both run near a device copy of x.
#include "bn_epilogue.h"
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int PNT = 256;

template <typename T, int K, int P>
__global__ __launch_bounds__(PNT) void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                     uint8_t* __restrict__ tap, int H, int W, int Ho, int Wo, int C,
                                                     int64_t total) {
  const int cv = C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * PNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * PNT) {
    const int c8 = (int)(i % cv);
    const int64_t p = i / cv;                       // output pixel n * Ho * Wo + oy * Wo + ox
    const int ox = (int)(p % Wo);
    const int64_t q = p / Wo;
    const int oy = (int)(q % Ho);
    const int64_t n = q / Ho;
    float mx[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { mx[k] = -__builtin_inff(); arg[k] = 0; }
    // a window of all -inf keeps its first in-image tap
    const int ih0 = 2 * oy - P, iw0 = 2 * ox - P;
    const int kh0 = ih0 < 0 ? -ih0 : 0, kw0 = iw0 < 0 ? -iw0 : 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) arg[k] = kh0 * K + kw0;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ih = ih0 + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int iw = iw0 + kw;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        Vec8<T>::load(x + ((n * H + ih) * W + iw) * C + c8 * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (v[k] > mx[k] || __builtin_isnan(v[k])) {
            mx[k] = v[k];
            arg[k] = kh * K + kw;
          }
        }
      }
    }
    Vec8<T>::store(y + p * C + c8 * 8, mx);
    uint64_t packed = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) packed |= (uint64_t)arg[k] << (8 * k);
    *reinterpret_cast<uint64_t*>(tap + p * C + c8 * 8) = packed;
  }
}

// BRED (bf16, the input is a BatchNorm + ReLU output -- the ResNet stem, the SimpleUNet encoder blocks): also the
// BatchNorm backward's reduction over the written gradient (kernels.h BnRed, mask from x; one partial row per block).
// The grid stride is a multiple of C / 8 (PNT % (C / 8) == 0, host-checked), so a thread's channel chunk is fixed.
// ADD: the input's other gradient (SimpleUNet: the skip connection's slice of d(concat), row stride lda) is added
// before the store -- the sum autograd would otherwise form with a separate kernel.
template <typename T, int K, int P, bool BRED = false, bool ADD = false>
__global__ __launch_bounds__(PNT) void maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ tap,
                                                     T* __restrict__ dx, int H, int W, int Ho, int Wo, int C,
                                                     int64_t total, BnRed bnr, const T* __restrict__ add,
                                                     int64_t lda) {
  const int cv = C >> 3;
  [[maybe_unused]] BnRedAcc<1> bra;
  if constexpr (BRED) bra.init(bnr, (int)(((int64_t)blockIdx.x * PNT + threadIdx.x) % cv) * 8, C);
  for (int64_t i = (int64_t)blockIdx.x * PNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * PNT) {
    const int c8 = (int)(i % cv);
    const int64_t p = i / cv;                       // input pixel n * H * W + iy * W + ix
    const int ix = (int)(p % W);
    const int64_t q = p / W;
    const int iy = (int)(q % H);
    const int64_t n = q / H;
    // output windows covering iy: oy with 2 oy - P <= iy <= 2 oy - P + K - 1
    const int oy_lo = max(0, (iy + P - K + 2) >> 1), oy_hi = min((iy + P) >> 1, Ho - 1);
    const int ox_lo = max(0, (ix + P - K + 2) >> 1), ox_hi = min((ix + P) >> 1, Wo - 1);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      const int kh = iy - 2 * oy + P;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int kw = ix - 2 * ox + P;
        const int me = kh * K + kw;
        const int64_t o = ((n * Ho + oy) * Wo + ox) * C + c8 * 8;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(tap + o);
        float g[8];
        Vec8<T>::load(dy + o, g);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if ((int)((packed >> (8 * k)) & 0xff) == me) acc[k] += g[k];
      }
    }
    if constexpr (ADD) {
      float a[8];
      Vec8<T>::load(add + p * lda + c8 * 8, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = (float)(T)acc[k] + a[k];   // = the bf16 sum of the two rounded gradients
    }
    Vec8<T>::store(dx + p * C + c8 * 8, acc);
    if constexpr (BRED) {
      bf16x8 g;
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = (bf16)acc[k];
      bra.add(BnRedAcc<1>::load_x(bnr, p, C, c8 * 8), 0u, g);
    }
  }
  if constexpr (BRED) {
    __shared__ float red[(PNT / 64) * 64 * 16];   // finish(): nwv * cpr * 16 floats, cpr = C / 8 <= 64
    bra.finish(red, cv, PNT / 64, blockIdx.x, C, 0, bnr.part);
  }
}

}  // namespace

#define DPH_POOL_KP(k, ...)                                                      \
  do {                                                                           \
    if (k == 3) { constexpr int K = 3, P = 1; __VA_ARGS__; }                     \
    else { constexpr int K = 2, P = 0; __VA_ARGS__; }                            \
  } while (0)

void maxpool_s2_fwd(const void* x, void* y, uint8_t* tap, int64_t N, int64_t H, int64_t W, int64_t C, int k,
                    int dtype, hipStream_t st) {
  const int64_t Ho = maxpool_s2_out(H, k), Wo = maxpool_s2_out(W, k);
  const int64_t total = N * Ho * Wo * (C / 8);
  if (total <= 0) return;
  const dim3 grid(stream_grid(total, PNT));
  DPH_DISPATCH_FLOAT(dtype, T, {
    DPH_POOL_KP(k, hipLaunchKernelGGL((maxpool_fwd_k<T, K, P>), grid, dim3(PNT), 0, st, (const T*)x, (T*)y, tap,
                                      (int)H, (int)W, (int)Ho, (int)Wo, (int)C, total));
  });
}

void maxpool_s2_bwd(const void* dy, const uint8_t* tap, void* dx, int64_t N, int64_t H, int64_t W, int64_t C, int k,
                    int dtype, hipStream_t st, const void* add, int64_t lda) {
  const int64_t Ho = maxpool_s2_out(H, k), Wo = maxpool_s2_out(W, k);
  const int64_t total = N * H * W * (C / 8);
  if (total <= 0) return;
  const dim3 grid(stream_grid(total, PNT));
  DPH_DISPATCH_FLOAT(dtype, T, {
    if (add) {
      DPH_POOL_KP(k, hipLaunchKernelGGL((maxpool_bwd_k<T, K, P, false, true>), grid, dim3(PNT), 0, st, (const T*)dy,
                                        tap, (T*)dx, (int)H, (int)W, (int)Ho, (int)Wo, (int)C, total, BnRed{},
                                        (const T*)add, lda));
    } else {
      DPH_POOL_KP(k, hipLaunchKernelGGL((maxpool_bwd_k<T, K, P>), grid, dim3(PNT), 0, st, (const T*)dy, tap, (T*)dx,
                                        (int)H, (int)W, (int)Ho, (int)Wo, (int)C, total, BnRed{}, (const T*)nullptr,
                                        (int64_t)0));
    }
  });
}

int maxpool_s2_bwd_bnred_blocks(int64_t N, int64_t H, int64_t W, int64_t C) {
  return stream_grid(N * H * W * (C / 8), PNT);
}

void maxpool_s2_bwd_bnred(const void* dy, const uint8_t* tap, void* dx, int64_t N, int64_t H, int64_t W, int64_t C,
                          int k, const BnRed& r, hipStream_t st, const void* add, int64_t lda) {
  const int64_t Ho = maxpool_s2_out(H, k), Wo = maxpool_s2_out(W, k);
  const int64_t total = N * H * W * (C / 8);
  if (total <= 0) return;
  const dim3 grid(stream_grid(total, PNT));
  if (add) {
    DPH_POOL_KP(k, hipLaunchKernelGGL((maxpool_bwd_k<bf16, K, P, true, true>), grid, dim3(PNT), 0, st,
                                      (const bf16*)dy, tap, (bf16*)dx, (int)H, (int)W, (int)Ho, (int)Wo, (int)C, total,
                                      r, (const bf16*)add, lda));
  } else {
    DPH_POOL_KP(k, hipLaunchKernelGGL((maxpool_bwd_k<bf16, K, P, true>), grid, dim3(PNT), 0, st, (const bf16*)dy, tap,
                                      (bf16*)dx, (int)H, (int)W, (int)Ho, (int)Wo, (int)C, total, r,
                                      (const bf16*)nullptr, (int64_t)0));
  }
}
#undef DPH_POOL_KP

}  // namespace dph
