// On-device image batch assembly for small-image datasets held resident in HBM (CIFAR-10: 60,000 x 32 x 32 x 3 uint8
// = 184 MB, nothing next to 288 GB).  One launch per batch gathers the sampled images by index and applies the
// reference's train transform (scripts/02_fully_sharded_fsdp/resnet_fsdp_training.py:45-87: RandomCrop(32, padding=4),
// RandomHorizontalFlip, ToTensor, Normalize(mean, std)) -- crop offsets and flips come in as a per-sample int32 table
// drawn by the caller's generator, so the batch is reproducible and the kernel is a pure gather:
//   out[b, c, y, x] = (P(b, y + dy_b - pad, xs - pad, c) / 255 - mean[c]) / std[c],  xs = flip_b ? W-1-x+dx_b : x+dx_b
// with P = 0 outside the image (zero padding happens before the normalisation, as in torchvision).  The output is
// NCHW-contiguous or channels-last (NHWC storage); one thread per output pixel writes its C channels (NHWC: one
// 8/16-byte vector store; NCHW: C strided stores that are coalesced across the 64 lanes of a row).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int AUG_NT = 256;

template <typename OutT, int C, bool NHWC>
__global__ __launch_bounds__(AUG_NT) void augment_k(const uint8_t* __restrict__ images, const int64_t* __restrict__ idx,
                                                  const int* __restrict__ params, const float* __restrict__ mean,
                                                  const float* __restrict__ inv_std, OutT* __restrict__ out, int B,
                                                  int H, int W, int pad) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t t = (int64_t)blockIdx.x * AUG_NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * AUG_NT) {
    const int x = (int)(t % W);
    const int y = (int)((t / W) % H);
    const int b = (int)(t / ((int64_t)H * W));
    const int dy = params ? params[3 * b] : pad, dx = params ? params[3 * b + 1] : pad;
    const int flip = params ? params[3 * b + 2] : 0;
    const int sy = y + dy - pad;
    const int sx = (flip ? W - 1 - x : x) + dx - pad;
    const bool inside = sy >= 0 && sy < H && sx >= 0 && sx < W;
    const uint8_t* src = images + (idx[b] * H * W + (int64_t)(inside ? sy * W + sx : 0)) * C;
    float v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = ((inside ? (float)src[c] : 0.f) * (1.f / 255.f) - mean[c]) * inv_std[c];
    if (NHWC) {
      OutT* o = out + t * C;
#pragma unroll
      for (int c = 0; c < C; ++c) o[c] = (OutT)v[c];
    } else {
      const int64_t plane = (int64_t)H * W;
      OutT* o = out + (int64_t)b * C * plane + (int64_t)y * W + x;
#pragma unroll
      for (int c = 0; c < C; ++c) o[c * plane] = (OutT)v[c];
    }
  }
}

}  // namespace

void image_augment(const uint8_t* images, const int64_t* idx, const int* params, const float* mean,
                   const float* inv_std, void* out, int64_t B, int64_t H, int64_t W, int64_t C, int64_t pad,
                   bool nhwc, int out_dtype, hipStream_t st) {
  if (B == 0) return;
  const dim3 grid(stream_grid(B * H * W, AUG_NT));
#define DPH_AUG(T, CC, NH)                                                                                      \
  hipLaunchKernelGGL((augment_k<T, CC, NH>), grid, dim3(AUG_NT), 0, st, images, idx, params, mean, inv_std,     \
                     (T*)out, (int)B, (int)H, (int)W, (int)pad)
#define DPH_AUG_C(T, NH) \
  do { if (C == 3) DPH_AUG(T, 3, NH); else DPH_AUG(T, 1, NH); } while (0)
  if (out_dtype == kBF16) {
    if (nhwc) DPH_AUG_C(bf16, true);
    else DPH_AUG_C(bf16, false);
  } else {
    if (nhwc) DPH_AUG_C(float, true);
    else DPH_AUG_C(float, false);
  }
#undef DPH_AUG_C
#undef DPH_AUG
}

}  // namespace dph
