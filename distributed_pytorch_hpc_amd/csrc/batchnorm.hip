// Fused BatchNorm (training statistics) + optional residual add + ReLU for channels-last (NHWC) activations.
// Replaces the MIOpen BN kernels (mean/var, norm, dscale/dbias, dx) plus the separate ReLU / residual-add
// passes of a ResNet block (torchvision-style resnet in scripts/main.py; SimpleUNet conv blocks), which cost more
// than the convolutions themselves in a bf16 channels-last step (profiles/rocprof_resnet50_*).
//
// x is viewed as [M, C] rows (M = N*H*W), C a power of two in [8, 2048] so a 256-thread block tiles rows x
// 8-channel chunks exactly.  Passes over the activation (A = its size):
//   forward : stats (read x)  +  apply (read x [+ residual], write y)            = 3A (+A)
//   backward: reduce (read dy, y, x) + dx (read dy, y, x, write dx [+ dres])      = 7A (+A)
//             (the reduce pass disappears when the convolution that produced dy ran it in its epilogue: pre_part)
//             ReLU without residual: the mask [x * scale + shift > 0] is recomputed from x with the forward's
//             own fp32 scale / shift (bit-identical to y > 0), so y is not read:  5A
//             ReLU with residual: the forward's apply pass also writes the mask [y > 0] as one BIT per element
//             (A / 16 bytes) and both backward passes read it instead of y:  5A + A / 8
// Statistics are accumulated with a per-thread shift (the thread's first value) and merged across threads and
// blocks with Chan's parallel-variance formula, so large-mean channels do not lose the variance to fp32
// cancellation; all reductions go through fixed-order partial buffers (deterministic).
#include <algorithm>
#include <cstdlib>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int BN_NT = 256;

struct Stat {   // count, mean, M2 (sum of squared deviations)
  float n, mean, m2;
};

__device__ __forceinline__ Stat chan_merge(Stat a, Stat b) {
  if (a.n == 0.f) return b;
  if (b.n == 0.f) return a;
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  const float f = b.n / n;
  return {n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}

// A wave's lanes hold (row group lane >> 3, channel lane & 7): merge its 8 row groups per channel by an xor butterfly
// (fixed order: deterministic), no LDS round trip or barrier.
__device__ __forceinline__ Stat wave_merge_groups(Stat a) {
  for (int off = 8; off < 64; off <<= 1) a = chan_merge(a, {__shfl_xor(a.n, off), __shfl_xor(a.mean, off),
                                                            __shfl_xor(a.m2, off)});
  return a;
}

__device__ __forceinline__ float wave_sum_groups(float v) {
  for (int off = 8; off < 64; off <<= 1) v += __shfl_xor(v, off);
  return v;
}

// Per-block statistics: block b covers rows [b*rows_per_block, ...).  Partials: mean/m2 [G][C], n [G].
template <typename T>
__global__ __launch_bounds__(BN_NT) void bn_stats_k(const T* __restrict__ x, float* __restrict__ pmean,
                                                    float* __restrict__ pm2, float* __restrict__ pn, int64_t M,
                                                    int C, int64_t rows_per_block) {
  extern __shared__ float sh[];   // [3][BN_NT][8]
  const int ch8 = C / 8, rpi = BN_NT / ch8;
  const int cc = threadIdx.x % ch8, r0 = threadIdx.x / ch8;
  const int64_t beg = (int64_t)blockIdx.x * rows_per_block, end = min(M, beg + rows_per_block);
  float k[8], s[8], ss[8], n = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) { k[i] = 0.f; s[i] = 0.f; ss[i] = 0.f; }
  int64_t r = beg + r0;
  if (r < end) {
    Vec8<T>::load(x + r * C + cc * 8, k);   // shift = first value
    n = 1.f;
    r += rpi;
  }
  for (; r < end; r += rpi) {
    float v[8];
    Vec8<T>::load(x + r * C + cc * 8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = v[i] - k[i];
      s[i] += d;
      ss[i] = fmaf(d, d, ss[i]);
    }
    n += 1.f;
  }
  float* shn = sh;
  float* shm = sh + BN_NT * 8;
  float* shq = sh + 2 * BN_NT * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float mean_d = n > 0.f ? s[i] / n : 0.f;
    shn[threadIdx.x * 8 + i] = n;
    shm[threadIdx.x * 8 + i] = k[i] + mean_d;
    shq[threadIdx.x * 8 + i] = n > 0.f ? fmaxf(ss[i] - s[i] * mean_d, 0.f) : 0.f;
  }
  __syncthreads();
  // log2(rpi) merge rounds with every row lane of the lower half active (rpi is a power of two), instead of
  // rpi - 1 serial merges by the ch8 lanes of row group 0 (rpi = 32 at C = 64)
  for (int half = rpi >> 1; half > 0; half >>= 1) {
    if (r0 < half) {
      const int t = (r0 + half) * ch8 + cc;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const Stat a = {shn[threadIdx.x * 8 + i], shm[threadIdx.x * 8 + i], shq[threadIdx.x * 8 + i]};
        const Stat m = chan_merge(a, {shn[t * 8 + i], shm[t * 8 + i], shq[t * 8 + i]});
        shn[threadIdx.x * 8 + i] = m.n;
        shm[threadIdx.x * 8 + i] = m.mean;
        shq[threadIdx.x * 8 + i] = m.m2;
      }
    }
    __syncthreads();
  }
  if (r0 == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      pmean[(int64_t)blockIdx.x * C + cc * 8 + i] = shm[threadIdx.x * 8 + i];
      pm2[(int64_t)blockIdx.x * C + cc * 8 + i] = shq[threadIdx.x * 8 + i];
    }
    if (cc == 0) pn[blockIdx.x] = (float)(end > beg ? end - beg : 0);
  }
}

// Merge G partials per channel; produce mean / invstd, the apply coefficients and the running-stat update.
// One block per 8-channel chunk: 32 row-groups of 8 lanes each merge a strided slice of the partials (loads
// issued FIN_UNROLL at a time so the chain is not one memory latency per partial), then a fixed-order LDS tree.
// 1024 threads = 128 row groups of 8 channel lanes per 8-channel chunk: at C = 64 only 8 workgroups exist, so the
// merge of up to 1024 partials is latency-bound; more groups per workgroup = fewer load rounds per thread.
constexpr int FIN_NT = 1024;   // 16 waves: the shuffle trees below assume it (16 x 8 = 2 x 64 LDS entries)
constexpr int FIN_GROUPS = FIN_NT / 8;
// Partials loaded per group before they are merged: the chain over G <= 1024 partials is latency-bound (a finalize
// ran ~10 us, most of it load rounds); 8 per round halves the rounds.  Merge order per thread is unchanged.
constexpr int FIN_UNROLL = 8;

template <typename PT, typename RT>
__global__ __launch_bounds__(FIN_NT) void bn_finalize_k(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                       const float* __restrict__ pn, int G, int C,
                                                       const PT* __restrict__ w, const PT* __restrict__ b,
                                                       RT* __restrict__ rmean, RT* __restrict__ rvar, float momentum,
                                                       float eps, float* __restrict__ mean_out,
                                                       float* __restrict__ invstd_out, float* __restrict__ scale,
                                                       float* __restrict__ shift, int64_t* __restrict__ nbt) {
  __shared__ float sh[3][FIN_NT];
  const int c = blockIdx.x * 8 + (threadIdx.x & 7), grp = threadIdx.x >> 3;
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;   // num_batches_tracked, one launch fewer
  Stat acc = {0.f, 0.f, 0.f};
  for (int g0 = grp; g0 < G; g0 += FIN_UNROLL * FIN_GROUPS) {
    Stat st[FIN_UNROLL];
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const int g = g0 + u * FIN_GROUPS;
      st[u] = g < G ? Stat{pn[g], pmean[(int64_t)g * C + c], pm2[(int64_t)g * C + c]} : Stat{0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) acc = chan_merge(acc, st[u]);
  }
  // the 128 row groups: 8 per wave by shuffles, then the 16 waves' results through LDS (one barrier) into wave 0
  acc = wave_merge_groups(acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < 8) {
    sh[0][wid * 8 + lane] = acc.n;
    sh[1][wid * 8 + lane] = acc.mean;
    sh[2][wid * 8 + lane] = acc.m2;
  }
  __syncthreads();
  if (wid != 0) return;
  acc = chan_merge({sh[0][lane], sh[1][lane], sh[2][lane]}, {sh[0][64 + lane], sh[1][64 + lane], sh[2][64 + lane]});
  acc = wave_merge_groups(acc);
  if (grp != 0) return;
  const float var = acc.n > 0.f ? acc.m2 / acc.n : 0.f;
  const float inv = rsqrtf(var + eps);
  mean_out[c] = acc.mean;
  invstd_out[c] = inv;
  const float gw = w ? (float)w[c] : 1.f, gb = b ? (float)b[c] : 0.f;
  scale[c] = gw * inv;
  shift[c] = gb - acc.mean * gw * inv;
  if (rmean) {
    const float unb = acc.n > 1.f ? acc.m2 / (acc.n - 1.f) : var;
    rmean[c] = (RT)((1.f - momentum) * (float)rmean[c] + momentum * acc.mean);
    rvar[c] = (RT)((1.f - momentum) * (float)rvar[c] + momentum * unb);
  }
}

// Merge G (large) statistics partials into gridDim.y segment partials: block (channel chunk, segment s) Chan-merges
// partials [s*G/S, (s+1)*G/S) of its 8 channels (32 thread groups, then an LDS tree), so bn_finalize_k sees few
// partials.  Used when the partials come per 128-row block from the 1x1 convolution epilogue (thousands of them).
__global__ __launch_bounds__(FIN_NT) void bn_merge_k(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                    const float* __restrict__ pn, int G, int C,
                                                    float* __restrict__ omean, float* __restrict__ om2,
                                                    float* __restrict__ on) {
  __shared__ float sh[3][FIN_NT];
  const int c = blockIdx.x * 8 + (threadIdx.x & 7), grp = threadIdx.x >> 3;
  const int S = gridDim.y, sgm = blockIdx.y;
  const int g_beg = (int)((int64_t)G * sgm / S), g_end = (int)((int64_t)G * (sgm + 1) / S);
  Stat acc = {0.f, 0.f, 0.f};
  for (int g = g_beg + grp; g < g_end; g += FIN_GROUPS)
    acc = chan_merge(acc, Stat{pn[g], pmean[(int64_t)g * C + c], pm2[(int64_t)g * C + c]});
  // the 128 row groups: 8 per wave by shuffles, then the 16 waves' results through LDS (one barrier) into wave 0
  acc = wave_merge_groups(acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < 8) {
    sh[0][wid * 8 + lane] = acc.n;
    sh[1][wid * 8 + lane] = acc.mean;
    sh[2][wid * 8 + lane] = acc.m2;
  }
  __syncthreads();
  if (wid != 0) return;
  acc = chan_merge({sh[0][lane], sh[1][lane], sh[2][lane]}, {sh[0][64 + lane], sh[1][64 + lane], sh[2][64 + lane]});
  acc = wave_merge_groups(acc);
  if (grp != 0) return;
  omean[(int64_t)sgm * C + c] = acc.mean;
  om2[(int64_t)sgm * C + c] = acc.m2;
  if (c == 0) on[sgm] = acc.n;
}

// y = act(x * scale + shift [+ res]).  The grid stride (gridDim.x * 256 vectors) is a multiple of ch8 = C / 8 (a
// power of two <= 256), so a thread's channel chunk never changes: its 8 scales / shifts are loaded once, into
// registers, instead of per element from L1.  MASK: also store [y > 0] of the vector's 8 elements as one byte.
// RESBN: the residual is itself a BatchNorm output, applied here -- res = round(z * rscale + rshift) from the raw z
// (rss = its [scale | shift]) -- so a projection shortcut's normalised activation is never written (bitwise the
// unfused pair: the same fmaf and the same rounding to T before the add).
template <typename T, bool RES, bool RELU, bool MASK = false, bool RESBN = false>
__global__ __launch_bounds__(BN_NT) void bn_apply_k(const T* __restrict__ x, const T* __restrict__ res,
                                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                                    T* __restrict__ y, int64_t nvec, int ch8,
                                                    uint8_t* __restrict__ mask = nullptr,
                                                    const float* __restrict__ rss = nullptr) {
  const int64_t v0 = (int64_t)blockIdx.x * BN_NT + threadIdx.x;
  const int c0 = (int)(v0 % ch8) * 8;
  float sc[8], sf[8], rsc[8], rsf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[c0 + i];
    sf[i] = shift[c0 + i];
    rsc[i] = RESBN ? rss[c0 + i] : 0.f;
    rsf[i] = RESBN ? rss[ch8 * 8 + c0 + i] : 0.f;
  }
  for (int64_t v = v0; v < nvec; v += (int64_t)gridDim.x * BN_NT) {
    float a[8], rr[8];
    Vec8<T>::load(x + v * 8, a);
    if (RES) Vec8<T>::load(res + v * 8, rr);
    if constexpr (RESBN) {
#pragma unroll
      for (int i = 0; i < 8; ++i) rr[i] = (float)from_f32<T>(fmaf(rr[i], rsc[i], rsf[i]));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float t = fmaf(a[i], sc[i], sf[i]);
      if (RES) t += rr[i];
      a[i] = RELU ? fmaxf(t, 0.f) : t;
    }
    Vec8<T>::store(y + v * 8, a);
    if constexpr (MASK) {   // from the stored (rounded) values: the same test the backward applied to y
      unsigned m = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) m |= ((float)from_f32<T>(a[i]) > 0.f ? 1u : 0u) << i;
      mask[v] = (uint8_t)m;
    }
  }
}

// Backward reduction: per channel sum(dz) and sum(dz * xhat), dz = dy * [y > 0 when RELU].
// XMASK: the ReLU mask comes from x * scale + shift (ss = [scale | shift], the forward's values) instead of y.
// BMASK: the ReLU mask comes from the forward's bit mask (one byte per 8-channel vector) instead of y.
template <typename T, bool RELU, bool XMASK, bool BMASK = false>
__global__ __launch_bounds__(BN_NT) void bn_bwd_reduce_k(const T* __restrict__ dy, const T* __restrict__ y,
                                                         const T* __restrict__ x, const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ ss, float* __restrict__ part,
                                                         int64_t M, int C, int64_t rows_per_block,
                                                         const uint8_t* __restrict__ bmask = nullptr) {
  extern __shared__ float sh[];   // [2][BN_NT][8]
  const int ch8 = C / 8, rpi = BN_NT / ch8;
  const int cc = threadIdx.x % ch8, r0 = threadIdx.x / ch8;
  const int64_t beg = (int64_t)blockIdx.x * rows_per_block, end = min(M, beg + rows_per_block);
  float mu[8], is[8], sd[8], sdx[8], xs[8], xb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = mean[cc * 8 + i];
    is[i] = invstd[cc * 8 + i];
    xs[i] = XMASK ? ss[cc * 8 + i] : 0.f;
    xb[i] = XMASK ? ss[C + cc * 8 + i] : 0.f;
    sd[i] = 0.f;
    sdx[i] = 0.f;
  }
  for (int64_t r = beg + r0; r < end; r += rpi) {
    float g[8], xv[8], yv[8];
    Vec8<T>::load(dy + r * C + cc * 8, g);
    Vec8<T>::load(x + r * C + cc * 8, xv);
    if (RELU && !XMASK && !BMASK) Vec8<T>::load(y + r * C + cc * 8, yv);
    const unsigned mb = BMASK ? bmask[r * ch8 + cc] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool on = BMASK ? ((mb >> i) & 1u) != 0u
                            : (XMASK ? fmaf(xv[i], xs[i], xb[i]) > 0.f : (!RELU || yv[i] > 0.f));
      const float dz = on ? g[i] : 0.f;
      sd[i] += dz;
      sdx[i] = fmaf(dz, (xv[i] - mu[i]) * is[i], sdx[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sh[threadIdx.x * 8 + i] = sd[i];
    sh[BN_NT * 8 + threadIdx.x * 8 + i] = sdx[i];
  }
  __syncthreads();
  if (r0 == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float a = 0.f, b = 0.f;
      for (int gq = 0; gq < rpi; ++gq) {
        const int t = gq * ch8 + cc;
        a += sh[t * 8 + i];
        b += sh[BN_NT * 8 + t * 8 + i];
      }
      part[(int64_t)blockIdx.x * 2 * C + cc * 8 + i] = a;
      part[(int64_t)blockIdx.x * 2 * C + C + cc * 8 + i] = b;
    }
  }
}

// Sum the G partials (same block shape as bn_finalize_k); dgamma = sum(dz xhat), dbeta = sum(dz); dx coefficients.
template <typename PT>
__global__ __launch_bounds__(FIN_NT) void bn_bwd_finalize_k(const float* __restrict__ part, int G, int C, float count,
                                                           const PT* __restrict__ w, const float* __restrict__ invstd,
                                                           PT* __restrict__ dw, PT* __restrict__ db,
                                                           float* __restrict__ coef) {
  __shared__ float sh[2][FIN_NT];
  const int c = blockIdx.x * 8 + (threadIdx.x & 7), grp = threadIdx.x >> 3;
  float a = 0.f, b = 0.f;
  for (int g0 = grp; g0 < G; g0 += FIN_UNROLL * FIN_GROUPS) {
    float pa[FIN_UNROLL], pb[FIN_UNROLL];
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      const int g = g0 + u * FIN_GROUPS;
      pa[u] = g < G ? part[(int64_t)g * 2 * C + c] : 0.f;
      pb[u] = g < G ? part[(int64_t)g * 2 * C + C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < FIN_UNROLL; ++u) {
      a += pa[u];
      b += pb[u];
    }
  }
  // the 128 row groups: 8 per wave by shuffles, then the 16 waves' sums through LDS (one barrier) into wave 0
  a = wave_sum_groups(a);
  b = wave_sum_groups(b);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < 8) {
    sh[0][wid * 8 + lane] = a;
    sh[1][wid * 8 + lane] = b;
  }
  __syncthreads();
  if (wid != 0) return;
  a = wave_sum_groups(sh[0][lane] + sh[0][64 + lane]);
  b = wave_sum_groups(sh[1][lane] + sh[1][64 + lane]);
  if (grp != 0) return;
  if (dw) dw[c] = (PT)b;
  if (db) db[c] = (PT)a;
  const float gw = w ? (float)w[c] : 1.f;
  coef[c] = gw * invstd[c];           // dx = coef * (dz - sum_dz / M - xhat * sum_dzx / M)
  coef[C + c] = a / count;
  coef[2 * C + c] = b / count;
}

// Sum G (thousands of) backward partials [G][2C] into gridDim.y segment rows [S][2C] (block = 8 channels x one
// segment; 128 thread groups, then an LDS tree): the convolution-epilogue partials come one per 128-row tile, and
// bn_bwd_finalize_k alone is latency-bound on them (8 blocks at C = 64 walking 6 272 rows: ~10 us per BatchNorm).
__global__ __launch_bounds__(FIN_NT) void bn_bwd_merge_k(const float* __restrict__ part, int G, int C,
                                                        float* __restrict__ out) {
  __shared__ float sh[2][FIN_NT];
  const int c = blockIdx.x * 8 + (threadIdx.x & 7), grp = threadIdx.x >> 3;
  const int S = gridDim.y, sgm = blockIdx.y;
  const int g_beg = (int)((int64_t)G * sgm / S), g_end = (int)((int64_t)G * (sgm + 1) / S);
  float a = 0.f, b = 0.f;
  for (int g = g_beg + grp; g < g_end; g += FIN_GROUPS) {
    a += part[(int64_t)g * 2 * C + c];
    b += part[(int64_t)g * 2 * C + C + c];
  }
  // the 128 row groups: 8 per wave by shuffles, then the 16 waves' sums through LDS (one barrier) into wave 0
  a = wave_sum_groups(a);
  b = wave_sum_groups(b);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < 8) {
    sh[0][wid * 8 + lane] = a;
    sh[1][wid * 8 + lane] = b;
  }
  __syncthreads();
  if (wid != 0) return;
  a = wave_sum_groups(sh[0][lane] + sh[0][64 + lane]);
  b = wave_sum_groups(sh[1][lane] + sh[1][64 + lane]);
  if (grp != 0) return;
  out[(int64_t)sgm * 2 * C + c] = a;
  out[(int64_t)sgm * 2 * C + C + c] = b;
}

template <typename T, bool RELU, bool DRES, bool XMASK, bool BMASK = false>
__global__ __launch_bounds__(BN_NT) void bn_bwd_dx_k(const T* __restrict__ dy, const T* __restrict__ y,
                                                     const T* __restrict__ x, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd, const float* __restrict__ coef,
                                                     const float* __restrict__ ss, T* __restrict__ dx,
                                                     T* __restrict__ dres, int64_t nvec, int ch8,
                                                     const uint8_t* __restrict__ bmask = nullptr) {
  const int C = ch8 * 8;
  // the thread's channel chunk is fixed (grid stride % ch8 == 0, see bn_apply_k): per-channel values in registers
  const int64_t v0 = (int64_t)blockIdx.x * BN_NT + threadIdx.x;
  const int c0 = (int)(v0 % ch8) * 8;
  float mu[8], is[8], k0[8], k1[8], k2[8], ms[8], mb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = c0 + i;
    mu[i] = mean[c];
    is[i] = invstd[c];
    k0[i] = coef[c];
    k1[i] = coef[C + c];
    k2[i] = coef[2 * C + c];
    ms[i] = XMASK ? ss[c] : 0.f;
    mb[i] = XMASK ? ss[C + c] : 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * BN_NT;
  auto one = [&](int64_t v, float (&g)[8], const float (&xv)[8], const float (&yv)[8], unsigned bits) {
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool on = BMASK ? ((bits >> i) & 1u) != 0u
                            : (XMASK ? fmaf(xv[i], ms[i], mb[i]) > 0.f : (!RELU || yv[i] > 0.f));
      const float dz = on ? g[i] : 0.f;
      const float xh = (xv[i] - mu[i]) * is[i];
      o[i] = k0[i] * (dz - k1[i] - xh * k2[i]);
      g[i] = dz;
    }
    Vec8<T>::store(dx + v * 8, o);
    if (DRES) Vec8<T>::store(dres + v * 8, g);
  };
  // two vectors per iteration, both loads issued before either is used: twice the 16-B loads in flight per thread.
  // Backward with the ReLU mask from x 5.66-5.75 -> 5.47-5.52 ms per ResNet-50 step of BN layers, the residual form
  // unchanged (benchmarks/bn_bench.py, profiles/r5/bn_unroll3/); four vectors, and unrolling the apply and reduce
  // passes the same way, measured no better or worse (profiles/r5/bn_unroll/, bn_unroll2/).
  int64_t v = v0;
  for (; v + stride < nvec; v += 2 * stride) {
    float g[2][8], xv[2][8], yv[2][8];
    unsigned bits[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t w = v + u * stride;
      Vec8<T>::load(dy + w * 8, g[u]);
      Vec8<T>::load(x + w * 8, xv[u]);
      if (RELU && !XMASK && !BMASK) Vec8<T>::load(y + w * 8, yv[u]);
      bits[u] = BMASK ? bmask[w] : 0u;
    }
    one(v, g[0], xv[0], yv[0], bits[0]);
    one(v + stride, g[1], xv[1], yv[1], bits[1]);
  }
  if (v < nvec) {
    float g[8], xv[8], yv[8];
    Vec8<T>::load(dy + v * 8, g);
    Vec8<T>::load(x + v * 8, xv);
    if (RELU && !XMASK && !BMASK) Vec8<T>::load(y + v * 8, yv);
    one(v, g, xv, yv, BMASK ? bmask[v] : 0u);
  }
}

// Two BatchNorms behind one residual add + ReLU (the projection shortcut: relu(bn_a(x) + bn_b(z)), _BNDualActFn):
// both see the same output gradient dz = dy * bit, so one pass reads dy, the bits, x and z and writes both input
// gradients -- the two single passes read dy and the bits once each.  Same per-element arithmetic as bn_bwd_dx_k.
template <typename T>
__global__ __launch_bounds__(BN_NT) void bn_bwd_dx2_k(const T* __restrict__ dy, const uint8_t* __restrict__ bmask,
                                                      const T* __restrict__ x, const T* __restrict__ z,
                                                      const float* __restrict__ mean_a,
                                                      const float* __restrict__ invstd_a,
                                                      const float* __restrict__ coef_a,
                                                      const float* __restrict__ mean_b,
                                                      const float* __restrict__ invstd_b,
                                                      const float* __restrict__ coef_b, T* __restrict__ dx,
                                                      T* __restrict__ dz_out, int64_t nvec, int ch8) {
  const int C = ch8 * 8;
  const int64_t v0 = (int64_t)blockIdx.x * BN_NT + threadIdx.x;
  const int c0 = (int)(v0 % ch8) * 8;
  float mua[8], isa[8], ka0[8], ka1[8], ka2[8], mub[8], isb[8], kb0[8], kb1[8], kb2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = c0 + i;
    mua[i] = mean_a[c];
    isa[i] = invstd_a[c];
    ka0[i] = coef_a[c];
    ka1[i] = coef_a[C + c];
    ka2[i] = coef_a[2 * C + c];
    mub[i] = mean_b[c];
    isb[i] = invstd_b[c];
    kb0[i] = coef_b[c];
    kb1[i] = coef_b[C + c];
    kb2[i] = coef_b[2 * C + c];
  }
  const int64_t stride = (int64_t)gridDim.x * BN_NT;
  for (int64_t v = v0; v < nvec; v += stride) {
    float g[8], xv[8], zv[8], oa[8], ob[8];
    Vec8<T>::load(dy + v * 8, g);
    Vec8<T>::load(x + v * 8, xv);
    Vec8<T>::load(z + v * 8, zv);
    const unsigned bits = bmask[v];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float dz = ((bits >> i) & 1u) != 0u ? g[i] : 0.f;
      const float xa = (xv[i] - mua[i]) * isa[i];
      const float xb = (zv[i] - mub[i]) * isb[i];
      oa[i] = ka0[i] * (dz - ka1[i] - xa * ka2[i]);
      ob[i] = kb0[i] * (dz - kb1[i] - xb * kb2[i]);
    }
    Vec8<T>::store(dx + v * 8, oa);
    Vec8<T>::store(dz_out + v * 8, ob);
  }
}

// The statistics kernel merges its row-lane partials as an LDS tree (25.0 -> 19.7 ms of bn_stats_k over
// benchmarks/bn_bench.py against a serial merge by row group 0, profiles/r2s3/ab_bn_tree/).  The backward
// reduction's plain sums gained nothing from the same tree (16.1 / 14.7 vs 16.3 / 14.8 ms) and stay serial.

int stats_grid(int64_t M, int C, int64_t* rows_per_block) {
  const int rpi = BN_NT / (C / 8);
  // ~4 row-iterations per thread minimum, at most 1024 blocks
  int64_t rpb = std::max<int64_t>((int64_t)rpi * 16, (M + 1023) / 1024);
  rpb = (rpb + rpi - 1) / rpi * rpi;
  *rows_per_block = rpb;
  return (int)((M + rpb - 1) / rpb);
}

}  // namespace

bool bn_nhwc_supported(int64_t C) { return C >= 8 && C <= 2048 && (C & (C - 1)) == 0; }

int bn_partial_blocks(int64_t M, int64_t C) {
  int64_t rpb;
  return stats_grid(M, (int)C, &rpb);
}

void bn_fwd_train(const void* x, const void* res, void* y, const void* w, const void* b, void* rmean, void* rvar,
                  float* mean, float* invstd, float* scale, float* shift, float* workspace, int64_t M, int64_t C,
                  float momentum, float eps, bool relu, int dt, int pdt, int rdt, hipStream_t st,
                  const float* pre_stats, int pre_groups, int64_t* nbt, uint8_t* relu_mask) {
  int64_t rpb;
  int G = stats_grid(M, (int)C, &rpb);
  const float* pmean = workspace;
  const float* pm2 = workspace + (int64_t)G * C;
  const float* pn = workspace + 2 * (int64_t)G * C;
  if (pre_stats) {   // partials from the producing convolution's epilogue (one per 128-row block)
    // Merged first into S segments of >= 4 partials per thread (FIN_GROUPS row groups per block); with a few hundred
    // partials or fewer bn_finalize_k takes them directly.  (S = 64 for every shape -- up to 16 384 mostly idle
    // 1024-thread blocks at 2048 channels -- measured 16 us per merge.)
    const int S = std::min(std::min(G, 64), (pre_groups + 4 * FIN_GROUPS - 1) / (4 * FIN_GROUPS));
    if (S <= 1) {
      G = pre_groups;
      pmean = pre_stats;
      pm2 = pre_stats + (int64_t)pre_groups * C;
      pn = pre_stats + 2 * (int64_t)pre_groups * C;
    } else {
      float* om = workspace;
      float* o2 = workspace + (int64_t)S * C;
      float* on = workspace + 2 * (int64_t)S * C;
      hipLaunchKernelGGL(bn_merge_k, dim3((unsigned)(C / 8), (unsigned)S), dim3(FIN_NT), 0, st, pre_stats,
                         pre_stats + (int64_t)pre_groups * C, pre_stats + 2 * (int64_t)pre_groups * C, pre_groups,
                         (int)C, om, o2, on);
      G = S;
      pmean = om;
      pm2 = o2;
      pn = on;
    }
  } else {
    const size_t shs = 3 * BN_NT * 8 * sizeof(float);
    DPH_DISPATCH_FLOAT(dt, T, {
      hipLaunchKernelGGL((bn_stats_k<T>), dim3(G), dim3(BN_NT), shs, st, (const T*)x, workspace,
                         workspace + (int64_t)G * C, workspace + 2 * (int64_t)G * C, M, (int)C, rpb);
    });
  }
  const dim3 fg((unsigned)(C / 8));
#define DPH_BN_FIN(PT_, RT_)                                                                                    \
  hipLaunchKernelGGL((bn_finalize_k<PT_, RT_>), fg, dim3(FIN_NT), 0, st, pmean, pm2, pn, G, (int)C, (const PT_*)w, \
                     (const PT_*)b, (RT_*)rmean, (RT_*)rvar, momentum, eps, mean, invstd, scale, shift, nbt)
  if (pdt == kBF16 && rdt == kBF16) DPH_BN_FIN(bf16, bf16);
  else if (pdt == kBF16) DPH_BN_FIN(bf16, float);
  else if (rdt == kBF16) DPH_BN_FIN(float, bf16);
  else DPH_BN_FIN(float, float);
#undef DPH_BN_FIN
  if (y != nullptr) bn_apply(x, res, scale, shift, y, M, C, relu, dt, st, relu_mask);   // null: folded into the consumer
}

void bn_apply(const void* x, const void* res, const float* scale, const float* shift, void* y, int64_t M, int64_t C,
              bool relu, int dt, hipStream_t st, uint8_t* relu_mask) {
  const int64_t nvec = M * C / 8;
  const dim3 grid(stream_grid(nvec, BN_NT));
  DPH_DISPATCH_FLOAT(dt, T, {
    if (res && relu && relu_mask)
      hipLaunchKernelGGL((bn_apply_k<T, true, true, true>), grid, dim3(BN_NT), 0, st, (const T*)x, (const T*)res,
                         scale, shift, (T*)y, nvec, (int)(C / 8), relu_mask);
    else if (res && relu) hipLaunchKernelGGL((bn_apply_k<T, true, true>), grid, dim3(BN_NT), 0, st, (const T*)x,
                                             (const T*)res, scale, shift, (T*)y, nvec, (int)(C / 8), nullptr);
    else if (res) hipLaunchKernelGGL((bn_apply_k<T, true, false>), grid, dim3(BN_NT), 0, st, (const T*)x,
                                     (const T*)res, scale, shift, (T*)y, nvec, (int)(C / 8), nullptr);
    else if (relu) hipLaunchKernelGGL((bn_apply_k<T, false, true>), grid, dim3(BN_NT), 0, st, (const T*)x,
                                      (const T*)nullptr, scale, shift, (T*)y, nvec, (int)(C / 8), nullptr);
    else hipLaunchKernelGGL((bn_apply_k<T, false, false>), grid, dim3(BN_NT), 0, st, (const T*)x, (const T*)nullptr,
                            scale, shift, (T*)y, nvec, (int)(C / 8), nullptr);
  });
}

void bn_apply_resbn(const void* x, const void* z, const float* ss, const float* zss, void* y, uint8_t* relu_mask,
                    int64_t M, int64_t C, int dt, hipStream_t st) {
  const int64_t nvec = M * C / 8;
  const dim3 grid(stream_grid(nvec, BN_NT));
  DPH_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL((bn_apply_k<T, true, true, true, true>), grid, dim3(BN_NT), 0, st, (const T*)x, (const T*)z,
                       ss, ss + C, (T*)y, nvec, (int)(C / 8), relu_mask, zss);
  });
}

// The backward's reduction (or the producer's partials, merged) and finalize: dgamma / dbeta and the dx coefficients
// [3C] in the workspace; returns the coefficients.
static float* bwd_coef(const void* dy, const void* y, const void* x, const float* mean, const float* invstd,
                       const void* w, void* dw, void* db, float* workspace, int64_t M, int64_t C, bool relu, int dt,
                       int pdt, hipStream_t st, const float* xmask_ss, const uint8_t* relu_mask,
                       const float* pre_part, int pre_groups) {
  const bool bm = relu && relu_mask != nullptr;
  const bool xm = relu && !bm && xmask_ss != nullptr;
  int64_t rpb;
  int G = stats_grid(M, (int)C, &rpb);
  const float* part = workspace;                 // [G][2C]
  float* coef = workspace + 2 * (int64_t)G * C;  // [3C]
  const size_t shs = 2 * BN_NT * 8 * sizeof(float);
  if (pre_part != nullptr) {   // reduced by the input-gradient epilogue that produced dy (kernels.h BnRed)
    // thousands of per-tile rows: merged first into S segment rows (>= 4 rows per thread, as bn_fwd_train does
    // with the forward's epilogue statistics) in the reduction pass's workspace (G >= S rows of 2C)
    const int S = std::min(std::min(G, 64), (pre_groups + 4 * FIN_GROUPS - 1) / (4 * FIN_GROUPS));
    if (S > 1) {
      hipLaunchKernelGGL(bn_bwd_merge_k, dim3((unsigned)(C / 8), (unsigned)S), dim3(FIN_NT), 0, st, pre_part,
                         pre_groups, (int)C, workspace);
      G = S;
    } else {
      part = pre_part;
      G = pre_groups;
    }
  } else {
#define DPH_BN_RED(R_, X_, B_)                                                                                     \
  hipLaunchKernelGGL((bn_bwd_reduce_k<T, R_, X_, B_>), dim3(G), dim3(BN_NT), shs, st, (const T*)dy, (const T*)y,  \
                     (const T*)x, mean, invstd, xmask_ss, workspace, M, (int)C, rpb, relu_mask)
  DPH_DISPATCH_FLOAT(dt, T, {
    if (bm) DPH_BN_RED(true, false, true);
    else if (xm) DPH_BN_RED(true, true, false);
    else if (relu) DPH_BN_RED(true, false, false);
    else DPH_BN_RED(false, false, false);
  });
#undef DPH_BN_RED
  }
  const dim3 fg((unsigned)(C / 8));
  if (pdt == kBF16) {
    hipLaunchKernelGGL((bn_bwd_finalize_k<bf16>), fg, dim3(FIN_NT), 0, st, part, G, (int)C, (float)M, (const bf16*)w,
                       invstd, (bf16*)dw, (bf16*)db, coef);
  } else {
    hipLaunchKernelGGL((bn_bwd_finalize_k<float>), fg, dim3(FIN_NT), 0, st, part, G, (int)C, (float)M,
                       (const float*)w, invstd, (float*)dw, (float*)db, coef);
  }
  return coef;
}

void bn_bwd(const void* dy, const void* y, const void* x, const float* mean, const float* invstd, const void* w,
            void* dx, void* dres, void* dw, void* db, float* workspace, int64_t M, int64_t C, bool relu, int dt,
            int pdt, hipStream_t st, const float* xmask_ss, const uint8_t* relu_mask, const float* pre_part,
            int pre_groups) {
  const bool bm = relu && relu_mask != nullptr;
  const bool xm = relu && !bm && xmask_ss != nullptr;
  const float* coef = bwd_coef(dy, y, x, mean, invstd, w, dw, db, workspace, M, C, relu, dt, pdt, st, xmask_ss,
                               relu_mask, pre_part, pre_groups);
  const int64_t nvec = M * C / 8;
  const dim3 grid(stream_grid(nvec, BN_NT));
#define DPH_BN_DX(R_, D_, X_, B_)                                                                                 \
  hipLaunchKernelGGL((bn_bwd_dx_k<T, R_, D_, X_, B_>), grid, dim3(BN_NT), 0, st, (const T*)dy, (const T*)y,       \
                     (const T*)x, mean, invstd, coef, xmask_ss, (T*)dx, (T*)dres, nvec, (int)(C / 8), relu_mask)
  DPH_DISPATCH_FLOAT(dt, T, {
    if (bm && dres) DPH_BN_DX(true, true, false, true);
    else if (bm) DPH_BN_DX(true, false, false, true);
    else if (xm && dres) DPH_BN_DX(true, true, true, false);
    else if (xm) DPH_BN_DX(true, false, true, false);
    else if (relu && dres) DPH_BN_DX(true, true, false, false);
    else if (relu) DPH_BN_DX(true, false, false, false);
    else if (dres) DPH_BN_DX(false, true, false, false);
    else DPH_BN_DX(false, false, false, false);
  });
#undef DPH_BN_DX
}

void bn_bwd_dual(const void* dy, const uint8_t* relu_mask, const void* x, const void* z, const float* mean_a,
                 const float* invstd_a, const void* w_a, const float* mean_b, const float* invstd_b, const void* w_b,
                 void* dx, void* dz, void* dw_a, void* db_a, void* dw_b, void* db_b, float* ws_a, float* ws_b,
                 int64_t M, int64_t C, int dt, int pdt, hipStream_t st, const float* pre_part_a, int pre_groups_a) {
  const float* ca = bwd_coef(dy, x, x, mean_a, invstd_a, w_a, dw_a, db_a, ws_a, M, C, true, dt, pdt, st, nullptr,
                             relu_mask, pre_part_a, pre_groups_a);
  const float* cb = bwd_coef(dy, z, z, mean_b, invstd_b, w_b, dw_b, db_b, ws_b, M, C, true, dt, pdt, st, nullptr,
                             relu_mask, nullptr, 0);
  const int64_t nvec = M * C / 8;
  const dim3 grid(stream_grid(nvec, BN_NT));
  DPH_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL((bn_bwd_dx2_k<T>), grid, dim3(BN_NT), 0, st, (const T*)dy, relu_mask, (const T*)x,
                       (const T*)z, mean_a, invstd_a, ca, mean_b, invstd_b, cb, (T*)dx, (T*)dz, nvec, (int)(C / 8));
  });
}

}  // namespace dph
