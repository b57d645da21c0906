// SimpleUNet up-path (multinode_ddp_unet.py:180-188, 205-213): ConvTranspose2d(k = 2, s = 2) -> bilinear resize to
// the skip connection's size -> torch.cat([up, skip], channel dim), as ONE copy kernel behind one library GEMM.
//
// A 2x2 / stride-2 transposed convolution has no overlapping taps: on channels-last activations it is the GEMM
//   Y'[n h w, (i j co)] = X[n h w, ci] * Wr[ci, (i j co)],   Wr = weight[Cin, Cout, 2, 2] permuted to (ci, i, j, co),
// whose row (n, h, w) holds the 2x2 output block (2h + i, 2w + j).  ops/upsample.py runs that GEMM on hipBLASLt and
// hands Y' to these kernels, which never materialise the up-sampled map:
//
//   forward : one thread = one pixel of the concatenated output x 8 channels.  Channels [0, Co): the bilinear
//             sample (align_corners = False, ATen's source-index and lambda arithmetic in fp32) of the VIRTUAL
//             2H x 2W map, each of its <= 4 taps read from Y' through the pixel-shuffle index + the bias, blended
//             in fp32, rounded once.  Channels [Co, Co + Cs): the skip tensor, copied.  A dimension whose size is
//             unchanged (2W == Wo on every ERA5 level, 2H == Ho on the middle one) takes a single tap.
//   backward: a GATHER per element of dY' (pixel-unshuffled bilinear adjoint; no atomics, deterministic):
//             up-sampled row u receives from the output rows o whose source interval holds it, found from the
//             inverse of ATen's source-index map and confirmed by recomputing the forward lambdas exactly; and the
//             skip gradient sliced out of d(cat) as a dense channels-last tensor in the same launch.
//
// Replaces, per up level: MIOpen's transposed convolution + bias, ATen's upsample_bilinear2d (which autocast runs in
// fp32, so two dtype conversions around it) and the cat (fp32 under autocast, promoted by the resize) -- forward and
// backward.  Each kernel is one pass at copy bandwidth over Y' + skip -> cat (or its adjoint).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int UNT = 256;

struct UpCatDims {
  int H, W;          // transposed-convolution input (the up-sampled map is 2H x 2W)
  int Ho, Wo;        // skip / output spatial size
  int Co, Cs;        // up-path and skip channels
  float sh, sw;      // ATen's area_pixel_compute_scale: (2H) / Ho, (2W) / Wo
};

// ATen upsample_bilinear2d (align_corners = False): source index, lower tap, tap step (0 at the last row), lambda
__device__ __forceinline__ void src_tap(float scale, int o, int in_size, int& i0, int& step, float& l1) {
  float s = scale * ((float)o + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  step = i0 < in_size - 1 ? 1 : 0;
  l1 = s - (float)i0;
}

template <typename T>
__global__ __launch_bounds__(UNT) void upcat_fwd_k(const T* __restrict__ y, const float* __restrict__ bias,
                                                   const T* __restrict__ skip, T* __restrict__ out, UpCatDims d,
                                                   int64_t total) {
  const int Ct = d.Co + d.Cs, cv = Ct >> 3;
  const int Hu = 2 * d.H, Wu = 2 * d.W;
  const int64_t ldy = 4 * (int64_t)d.Co;
  for (int64_t i = (int64_t)blockIdx.x * UNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * UNT) {
    const int c = (int)(i % cv) * 8;
    const int64_t p = i / cv;                      // output pixel n * Ho * Wo + oh * Wo + ow
    const int ow = (int)(p % d.Wo);
    const int64_t q = p / d.Wo;
    const int oh = (int)(q % d.Ho);
    const int n = (int)(q / d.Ho);
    float v[8];
    if (c >= d.Co) {
      Vec8<T>::load(skip + p * d.Cs + (c - d.Co), v);
    } else {
      int h0, hs, w0, ws;
      float lh, lw;
      if (Hu == d.Ho) { h0 = oh; hs = 0; lh = 0.f; } else { src_tap(d.sh, oh, Hu, h0, hs, lh); }
      if (Wu == d.Wo) { w0 = ow; ws = 0; lw = 0.f; } else { src_tap(d.sw, ow, Wu, w0, ws, lw); }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = 0.f;
      // taps (uh, uw) of the virtual map -> Y' row (n, uh / 2, uw / 2), column block (uh & 1, uw & 1)
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int uh = h0 + a * hs;
        const float wh = a ? lh : (hs ? 1.f - lh : 1.f);   // last row: both ATen taps coincide
        if (a && hs == 0) break;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int uw = w0 + b * ws;
          const float ww = b ? lw : (ws ? 1.f - lw : 1.f);
          if (b && ws == 0) break;
          const int64_t row = ((int64_t)n * d.H + (uh >> 1)) * d.W + (uw >> 1);
          float t[8];
          Vec8<T>::load(y + row * ldy + (((uh & 1) << 1) | (uw & 1)) * d.Co + c, t);
          const float wgt = wh * ww;
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += wgt * t[k];
        }
      }
      if (bias) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += bias[c + k];
      }
    }
    Vec8<T>::store(out + p * Ct + c, v);
  }
}

// weight with which output index o reads up-sampled index u along one axis (0 if it does not)
__device__ __forceinline__ float tap_weight(float scale, int o, int u, int in_size) {
  int i0, st;
  float l1;
  src_tap(scale, o, in_size, i0, st, l1);
  float w = 0.f;
  if (i0 == u) w += 1.f - l1;
  if (i0 + st == u) w += l1;
  return w;
}

template <typename T>
__global__ __launch_bounds__(UNT) void upcat_bwd_k(const T* __restrict__ dcat, T* __restrict__ dy,
                                                   T* __restrict__ dskip, UpCatDims d, int64_t total_y,
                                                   int64_t total) {
  const int Ct = d.Co + d.Cs;
  const int Hu = 2 * d.H, Wu = 2 * d.W;
  const int cvo = d.Co >> 3, cvs = d.Cs >> 3;
  for (int64_t i = (int64_t)blockIdx.x * UNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * UNT) {
    if (i >= total_y) {                            // skip gradient: dense channels-last slice of d(cat)
      const int64_t j = i - total_y;
      const int c = (int)(j % cvs) * 8;
      const int64_t p = j / cvs;
      float v[8];
      Vec8<T>::load(dcat + p * Ct + d.Co + c, v);
      Vec8<T>::store(dskip + p * d.Cs + c, v);
      continue;
    }
    // dY' element: row (n, h, w), block ij = (i, j), channels c..c+7  (the GEMM's output layout, written in order)
    const int c = (int)(i % cvo) * 8;
    const int64_t q = i / cvo;
    const int ij = (int)(q & 3);
    const int64_t row = q >> 2;
    const int w = (int)(row % d.W);
    const int64_t r2 = row / d.W;
    const int h = (int)(r2 % d.H);
    const int n = (int)(r2 / d.H);
    const int uh = 2 * h + (ij >> 1), uw = 2 * w + (ij & 1);
    // candidate output rows: o with floor(max(scale (o + 0.5) - 0.5, 0)) in {u - 1, u}, widened by one each side
    // and confirmed by tap_weight (identical arithmetic to the forward)
    int oh_lo, oh_hi, ow_lo, ow_hi;
    if (Hu == d.Ho) { oh_lo = oh_hi = uh; } else {
      oh_lo = max(0, (int)floorf(((float)uh - 0.5f) / d.sh - 0.5f) - 1);
      oh_hi = min(d.Ho - 1, (int)ceilf(((float)uh + 1.5f) / d.sh - 0.5f) + 1);
    }
    if (Wu == d.Wo) { ow_lo = ow_hi = uw; } else {
      ow_lo = max(0, (int)floorf(((float)uw - 0.5f) / d.sw - 0.5f) - 1);
      ow_hi = min(d.Wo - 1, (int)ceilf(((float)uw + 1.5f) / d.sw - 0.5f) + 1);
    }
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const float wh = Hu == d.Ho ? 1.f : tap_weight(d.sh, oh, uh, Hu);
      if (wh == 0.f) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const float ww = Wu == d.Wo ? 1.f : tap_weight(d.sw, ow, uw, Wu);
        if (ww == 0.f) continue;
        float g[8];
        Vec8<T>::load(dcat + (((int64_t)n * d.Ho + oh) * d.Wo + ow) * Ct + c, g);
        const float wgt = wh * ww;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += wgt * g[k];
      }
    }
    Vec8<T>::store(dy + i * 8, acc);
  }
}

UpCatDims make_dims(int64_t H, int64_t W, int64_t Co, int64_t Ho, int64_t Wo, int64_t Cs) {
  UpCatDims d;
  d.H = (int)H; d.W = (int)W; d.Ho = (int)Ho; d.Wo = (int)Wo; d.Co = (int)Co; d.Cs = (int)Cs;
  d.sh = (float)(2 * H) / (float)Ho;   // ATen: static_cast<float>(input_size) / output_size
  d.sw = (float)(2 * W) / (float)Wo;
  return d;
}

}  // namespace

void upcat_fwd(const void* y, const float* bias, const void* skip, void* out, int64_t N, int64_t H, int64_t W,
               int64_t Co, int64_t Ho, int64_t Wo, int64_t Cs, int dtype, hipStream_t st) {
  const int64_t total = N * Ho * Wo * ((Co + Cs) / 8);
  if (total <= 0) return;
  const UpCatDims d = make_dims(H, W, Co, Ho, Wo, Cs);
  DPH_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL((upcat_fwd_k<T>), dim3(stream_grid(total, UNT)), dim3(UNT), 0, st, (const T*)y, bias,
                       (const T*)skip, (T*)out, d, total);
  });
}

void upcat_bwd(const void* dcat, void* dy, void* dskip, int64_t N, int64_t H, int64_t W, int64_t Co, int64_t Ho,
               int64_t Wo, int64_t Cs, int dtype, hipStream_t st) {
  const int64_t total_y = N * H * W * 4 * (Co / 8);
  const int64_t total = total_y + (dskip ? N * Ho * Wo * (Cs / 8) : 0);
  if (total <= 0) return;
  const UpCatDims d = make_dims(H, W, Co, Ho, Wo, Cs);
  DPH_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL((upcat_bwd_k<T>), dim3(stream_grid(total, UNT)), dim3(UNT), 0, st, (const T*)dcat, (T*)dy,
                       (T*)dskip, d, total_y, total);
  });
}

}  // namespace dph
