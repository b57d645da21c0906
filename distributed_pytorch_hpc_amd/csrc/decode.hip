// Serving path of the Llama decoder (models/llama2.py KVCache, inference/generator.py): the KV-cache append and the
// single-token decode attention.  Decode attention is a memory-bound stream over the cache (512 B of K+V per key and
// KV head at head_dim 128), so it is built for bytes in flight, not for MFMA:
//
//   kv_append_k      : RoPE of q (in place in the fused QKV GEMM output) and of k, k and v written into the cache at
//                      position pos[b] + s.  Positions are read from device memory, so a captured HIP-graph decode
//                      step replays correctly with the cache advancing between replays.
//   decode_attn_k    : split-KV ("flash-decoding") -- one wave per 64-key chunk of one (batch, KV head), all G query
//                      heads of that KV head's group at once (GQA: the K/V rows are read once per chunk).  16 lanes
//                      per 256-B key row (head_dim 128), 4 keys per wave instruction; every K and V row of the
//                      chunk is loaded up front (16 + 16 KiB per wave in flight) and scores, softmax and P.V stay in
//                      registers -- no LDS, no barriers.  Writes the chunk's unnormalised o and its (max, sum).
//                      Opt-in FP8 caches (OCP e4m3 x a per-cache scale) halve the bytes: 8-B rows per lane,
//                      widened by v_cvt_pk_f32_fp8.
//   decode_combine_k : one wave per (batch, query head) merges the chunks of the sequence (log-sum-exp rescaling)
//                      and writes bf16 o straight into the [B, Hq * D] input of the output projection.
// Keys past a sequence's length re-read its last valid row (finite data) and get probability 0, so the cache never
// needs clearing and every load stays inside the written region.
#include <cstdio>
#include <cstdlib>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

__global__ __launch_bounds__(256) void kv_append_k(KVAppendParams p) {
  const int CH = p.D / 8, NH = p.Hq + 2 * p.Hkv;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)p.B * p.S * NH * CH;
  if (i >= total) return;
  const int c = (int)(i % CH);
  int64_t r = i / CH;
  const int h = (int)(r % NH);
  r /= NH;
  const int s = (int)(r % p.S);
  const int b = (int)(r / p.S);
  const int t = p.pos[b] + s;
  if (t >= p.Smax) return;   // the host checks capacity; never write past the cache
  bf16* src = (bf16*)p.qkv + (int64_t)b * p.qkv_sb + (int64_t)s * p.qkv_ss + (int64_t)h * p.D + c * 8;
  float v[8];
  Vec8<bf16>::load(src, v);
  if (h < p.Hq + p.Hkv) {   // interleaved-pair rotation, pair index 4c + j, angle table row t
    const float* cs = p.cos + (int64_t)t * (p.D / 2) + c * 4;
    const float* sn = p.sin + (int64_t)t * (p.D / 2) + c * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = v[2 * j], bb = v[2 * j + 1], co = cs[j], si = sn[j];
      v[2 * j] = a * co - bb * si;
      v[2 * j + 1] = a * si + bb * co;
    }
  }
  if (h < p.Hq) {
    Vec8<bf16>::store(src, v);
  } else {
    const bool is_k = h < p.Hq + p.Hkv;
    const int hk = is_k ? h - p.Hq : h - p.Hq - p.Hkv;
    const int64_t off = (int64_t)b * p.c_sb + (int64_t)t * p.c_ss + (int64_t)hk * p.c_sh + c * 8;
    if (p.kv_fp8) {   // key / value rounded to bf16 first (what the bf16 cache would hold), then to e4m3
      const float inv = 1.f / p.kv_scale;
      float q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = __builtin_amdgcn_fmed3f((float)(bf16)v[j] * inv, 448.f, -448.f);
      uint2 o;
      o.x = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false),
                                                      true);
      o.y = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], 0, false),
                                                      true);
      *reinterpret_cast<uint2*>((uint8_t*)(is_k ? p.kc : p.vc) + off) = o;
    } else {
      Vec8<bf16>::store((bf16*)(is_k ? p.kc : p.vc) + off, v);
    }
  }
}

// 8 cache elements of one key / value row -> fp32 (bf16 or OCP e4m3 x scale)
template <bool FP8>
struct KVRow;
template <>
struct KVRow<false> {
  typedef bf16x8 raw;
  static __device__ __forceinline__ raw load(const void* base, int64_t off) {
    return *reinterpret_cast<const bf16x8*>((const bf16*)base + off);
  }
  static __device__ __forceinline__ void unpack(const raw& r, float (&o)[8], float) {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (float)r[e];
  }
};
template <>
struct KVRow<true> {
  typedef uint2 raw;
  static __device__ __forceinline__ raw load(const void* base, int64_t off) {
    return *reinterpret_cast<const uint2*>((const uint8_t*)base + off);
  }
  static __device__ __forceinline__ void unpack(const raw& r, float (&o)[8], float sc) {
    const auto a = __builtin_amdgcn_cvt_pk_f32_fp8((int)r.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)r.x, true);
    const auto c = __builtin_amdgcn_cvt_pk_f32_fp8((int)r.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)r.y, true);
    o[0] = a[0] * sc; o[1] = a[1] * sc; o[2] = b[0] * sc; o[3] = b[1] * sc;
    o[4] = c[0] * sc; o[5] = c[1] * sc; o[6] = d[0] * sc; o[7] = d[1] * sc;
  }
};

template <int N>
__device__ __forceinline__ float group_sum(float v) {   // sum over aligned groups of N lanes
#pragma unroll
  for (int o = N / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int FROM>
__device__ __forceinline__ float across_groups_max(float v) {   // max over lanes congruent mod FROM
#pragma unroll
  for (int o = FROM; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int FROM>
__device__ __forceinline__ float across_groups_sum(float v) {
#pragma unroll
  for (int o = FROM; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int HD, int G, bool FP8>
__global__ __launch_bounds__(256) void decode_attn_k(DecodeParams p) {
  using KV = KVRow<FP8>;
  constexpr int TPK = HD / 8;     // lanes per key row (8 bf16 = 16 B each)
  constexpr int KPI = 64 / TPK;   // keys per wave instruction
  constexpr int NIT = 64 / KPI;   // instructions per 64-key chunk
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = lane % TPK, j = lane / TPK;
  const int b = blockIdx.z, hg = blockIdx.y;
  const int chunk = blockIdx.x * 4 + wave;
  const int len = min(p.pos[b] + p.len_add, p.Smax);
  const int k0 = chunk * 64;
  if (chunk >= p.nch || k0 >= len) return;   // no barriers below: a finished wave may leave
  const int hq0 = hg * G;
  const int hkv = hq0 / (p.Hq / p.Hkv);

  const float sl2 = p.scale * 1.4426950408889634f;
  float qf[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    Vec8<bf16>::load((const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)(hq0 + g) * p.q_sh + t * 8, qf[g]);
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[g][e] *= sl2;
  }

  const int64_t hoff = (int64_t)b * p.c_sb + (int64_t)hkv * p.c_sh + t * 8;
  const float ksc = p.kv_scale;
  typename KV::raw kr[NIT], vr[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int row = min(k0 + it * KPI + j, len - 1);
    kr[it] = KV::load(p.kc, hoff + (int64_t)row * p.c_ss);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int row = min(k0 + it * KPI + j, len - 1);
    vr[it] = KV::load(p.vc, hoff + (int64_t)row * p.c_ss);
  }

  // scores (log2 units): s[g][it] is key k0 + it * KPI + j, identical in the TPK lanes of group j
  float s[G][NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const bool valid = k0 + it * KPI + j < len;
    float kf[8];
    KV::unpack(kr[it], kf, ksc);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qf[g][e], kf[e], d);
      d = group_sum<TPK>(d);
      s[g][it] = valid ? d : -INFINITY;
    }
  }
  float m[G], l[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float mx = s[g][0];
#pragma unroll
    for (int it = 1; it < NIT; ++it) mx = fmaxf(mx, s[g][it]);
    m[g] = across_groups_max<TPK>(mx);   // finite: key k0 < len is valid
    float sum = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      s[g][it] = exp2f(s[g][it] - m[g]);
      sum += s[g][it];
    }
    l[g] = across_groups_sum<TPK>(sum);
  }

  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float vf[8];
    KV::unpack(vr[it], vf, ksc);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(s[g][it], vf[e], acc[g][e]);
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = across_groups_sum<TPK>(acc[g][e]);

  if (j == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t slot = ((int64_t)b * p.Hq + hq0 + g) * p.nch + chunk;
      Vec8<float>::store(p.opart + slot * HD + t * 8, acc[g]);
      if (t == 0) {
        p.mlpart[2 * slot] = m[g];
        p.mlpart[2 * slot + 1] = l[g];
      }
    }
  }
}

// one wave per (b, hq); lane d-slice of EPL = max(HD / 64, 1) elements (HD 32: lanes >= 32 idle)
template <int HD>
__global__ __launch_bounds__(256) void decode_combine_k(DecodeParams p) {
  constexpr int EPL = HD >= 64 ? HD / 64 : 1;
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= p.B * p.Hq) return;
  const int b = w / p.Hq, hq = w % p.Hq;
  const int len = min(p.pos[b] + p.len_add, p.Smax);
  const int n = min((len + 63) / 64, p.nch);
  const float* ml = p.mlpart + (int64_t)w * p.nch * 2;
  const float* op = p.opart + (int64_t)w * p.nch * HD;
  float M = -INFINITY;
  for (int c = lane; c < n; c += 64) M = fmaxf(M, ml[2 * c]);
  M = wave_max(M);
  float L = 0.f, acc[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
  const bool active = lane * EPL < HD;
#pragma unroll 4
  for (int c = 0; c < n; ++c) {
    const float wgt = exp2f(ml[2 * c] - M);
    L = fmaf(wgt, ml[2 * c + 1], L);
    if (active) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] = fmaf(wgt, op[(int64_t)c * HD + lane * EPL + e], acc[e]);
    }
  }
  if (active && n > 0) {
    const float inv = 1.f / L;
    bf16* out = (bf16*)p.out + (int64_t)b * p.out_sb + (int64_t)hq * HD + lane * EPL;
#pragma unroll
    for (int e = 0; e < EPL; ++e) out[e] = (bf16)(acc[e] * inv);
  }
}

}  // namespace

void kv_append(const KVAppendParams& p, hipStream_t st) {
  const int64_t total = (int64_t)p.B * p.S * (p.Hq + 2 * p.Hkv) * (p.D / 8);
  if (total == 0) return;
  hipLaunchKernelGGL(kv_append_k, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, p);
}

// Query heads per wave: the largest of 4 / 2 / 1 dividing the GQA group (K/V rows are read once per head group).
int decode_heads_per_wave(int Hq, int Hkv) {
  const int rep = Hq / Hkv;
  return rep % 4 == 0 ? 4 : (rep % 2 == 0 ? 2 : 1);
}

void decode_attention(const DecodeParams& p, hipStream_t st) {
  const int G = decode_heads_per_wave(p.Hq, p.Hkv);
  const dim3 grid((unsigned)cdiv(p.nch, 4), (unsigned)(p.Hq / G), (unsigned)p.B);
#define DPH_DEC(HD_, G_)                                                                     \
  do {                                                                                       \
    if (p.kv_fp8) hipLaunchKernelGGL((decode_attn_k<HD_, G_, true>), grid, dim3(256), 0, st, p); \
    else hipLaunchKernelGGL((decode_attn_k<HD_, G_, false>), grid, dim3(256), 0, st, p);       \
  } while (0)
#define DPH_DEC_G(HD_)          \
  do {                          \
    if (G == 4) DPH_DEC(HD_, 4); \
    else if (G == 2) DPH_DEC(HD_, 2); \
    else DPH_DEC(HD_, 1);       \
  } while (0)
  if (p.D == 128) DPH_DEC_G(128);
  else if (p.D == 64) DPH_DEC_G(64);
  else DPH_DEC_G(32);
#undef DPH_DEC_G
#undef DPH_DEC
  const dim3 cgrid((unsigned)cdiv((int64_t)p.B * p.Hq, 4));
  if (p.D == 128) hipLaunchKernelGGL(decode_combine_k<128>, cgrid, dim3(256), 0, st, p);
  else if (p.D == 64) hipLaunchKernelGGL(decode_combine_k<64>, cgrid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL(decode_combine_k<32>, cgrid, dim3(256), 0, st, p);
}

// ==================================================================================================
// Skinny GEMM for decode: y[M, N] = x[M, K] W[N, K]^T with M <= 64 (one token per sequence), bf16, fp32 accumulate.
// Pure weight streaming (2 N K bytes read once, x re-read from L2): hipBLASLt's small-M tiles ran the Llama-2-7B
// decode projections at 2.6-3.7 TB/s (profiles/serving/).  One workgroup = 16 output rows (n) x all M, SG_WAVES waves
// splitting K; each 16-row W tile goes straight from HBM into the A operand of v_mfma_f32_16x16x32_bf16 (lane l: row
// l & 15, k 8 (l >> 4) .. +7 -- 64 contiguous bytes per row per instruction), x^T is the B operand, so the matrix
// core does the k reduction and no shuffles are needed.  U unrolled k-steps keep U x 1 KiB of W in flight per wave;
// the per-wave partial tiles are summed through LDS.
// ==================================================================================================
namespace {

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// default K split (workgroup = SG_WAVES waves) and unroll: the best of the (waves x unroll) sweep on every 7B
// decode projection (profiles/serving/skinny_sweep/)
constexpr int SG_WAVES = 4, SG_UNROLL = 4;

template <int MT, int U, int NWV = SG_WAVES>
__global__ __launch_bounds__(64 * NWV) void skinny_gemm_k(const bf16* __restrict__ x, int64_t ldx,
                                                         const bf16* __restrict__ w, int64_t ldw,
                                                         bf16* __restrict__ y, int64_t ldy, int M, int K) {
  __shared__ f32x4 red[NWV][MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kq = K / NWV;
  const int kbeg = wave * kq;
  const bf16* wp = w + (int64_t)(n0 + r) * ldw + kbeg + 8 * g;
  const bf16* xp[MT];
  bool xv[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    xv[mt] = m < M;
    xp[mt] = x + (int64_t)(xv[mt] ? m : 0) * ldx + kbeg + 8 * g;
  }
  const bf16x8 z = {};
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // software pipeline over groups of U k-steps: the W tiles and x slices (B operands, L2) of group g+1 are requested
  // before group g's MFMAs, which only read registers loaded one group earlier -- whatever order hipcc issues the
  // loads in, the counted vmcnt in front of the MFMAs leaves the prefetch in flight.  The last group re-reads its
  // own slices (no branch: a conditional prefetch makes hipcc pick one conservative count for both paths).  Lanes
  // past M load row 0 and select zero.
  const int ng = kq / (32 * U);
  bf16x8 a[U], b[MT][U];
  if (ng > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = *reinterpret_cast<const bf16x8*>(wp + 32 * u);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[mt][u] = *reinterpret_cast<const bf16x8*>(xp[mt] + 32 * u);
    }
  }
  for (int gi = 0; gi < ng; ++gi) {
    const int kn = (gi + 1 < ng ? gi + 1 : gi) * 32 * U;
    bf16x8 an[U], bn[MT][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      an[u] = *reinterpret_cast<const bf16x8*>(wp + kn + 32 * u);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) bn[mt][u] = *reinterpret_cast<const bf16x8*>(xp[mt] + kn + 32 * u);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the whole prefetch ahead of this group's MFMAs
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16(a[u], xv[mt] ? b[mt][u] : z, acc[mt]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = an[u];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[mt][u] = bn[mt][u];
    }
  }
  for (int k = ng * 32 * U; k < kq; k += 32) {
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(wp + k);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(xp[mt] + k);
      acc[mt] = mfma16(a1, xv[mt] ? b1 : z, acc[mt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = acc[mt];
  __syncthreads();
  // wave w sums m-tiles w, w + NWV, ...: C[n = 4 g + i][m = mt * 16 + r] (fewer waves than m-tiles is legal)
  for (int mt = wave; mt < MT; mt += NWV) {
    f32x4 s = red[0][mt][lane];
#pragma unroll
    for (int v = 1; v < NWV; ++v) s += red[v][mt][lane];
    const int m = mt * 16 + r;
    if (m < M) {
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (bf16)s[i];
      *reinterpret_cast<bf16x4*>(y + (int64_t)m * ldy + n0 + 4 * g) = o;
    }
  }
}

// GEMV form for M <= 2 (batch-1/2 decode): the MFMA form above spends 15/16 of its x operand on padding there.
// A workgroup owns 8 rows of W; its waves split K in slices of C = 2 chunks of 512 (lane: 8 consecutive k per
// chunk, so one wave instruction reads 1 KiB of one row); every lane issues all R x C = 16 W loads up front (16 KiB
// per wave in flight, counted waits as the FMAs consume them; <= 128 VGPRs so 4 waves / SIMD stay resident), keeps
// its 8 x values per chunk and m packed in registers, then each row's partial is reduced over the lanes and over
// the waves through LDS.  K <= 16 waves x 1024.
//
// The x operand can be PRODUCED in the kernel while the W loads are in flight (decode is launch-latency bound at
// batch 1, ~4 us per small kernel): XM = GX_SWIGLU reads the fused [gate | up] w13 output and forms silu(g) * u
// (the w2 input), XM = GX_NORM forms RMSNorm(x + res) * g (the wqkv / w13 / LM-head input; the sum of squares is
// reduced over the workgroup's waves, every workgroup recomputes it from L2) and workgroup 0 writes h = x + res
// for the residual stream.  Both round to bf16 where the separate kernels store, so the fused and unfused paths
// agree to the rounding of the sum-of-squares order.
enum { GX_PLAIN = 0, GX_SWIGLU = 1, GX_NORM = 2 };

template <int M, int XM>
__global__ __launch_bounds__(1024) void gemv_k(GemvArgs a) {
  constexpr int R = 8, C = 2;
  __shared__ float red[16][R * M];
  __shared__ float nred[16][M];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int n0 = blockIdx.x * R;
  const int K = a.K;
  int kc[C];
  bool cv[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int k = (wave * C + c) * 512 + lane * 8;
    cv[c] = k < K;
    kc[c] = cv[c] ? k : 0;   // out-of-range lanes read column 0 and contribute zero
  }
  const bf16* w = (const bf16*)a.w;
  bf16x8 wr[R][C];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) wr[r][c] = *reinterpret_cast<const bf16x8*>(w + (int64_t)(n0 + r) * a.ldw + kc[c]);

  const bf16* x = (const bf16*)a.x;
  bf16x8 xs[C][M];
  if constexpr (XM == GX_PLAIN) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int m = 0; m < M; ++m) xs[c][m] = *reinterpret_cast<const bf16x8*>(x + (int64_t)m * a.ldx + kc[c]);
  } else if constexpr (XM == GX_SWIGLU) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float g[8], u[8];
        Vec8<bf16>::load(x + (int64_t)m * a.ldx + kc[c], g);
        Vec8<bf16>::load(x + (int64_t)m * a.ldx + K + kc[c], u);
#pragma unroll
        for (int e = 0; e < 8; ++e) xs[c][m][e] = (bf16)(g[e] * (1.f / (1.f + __expf(-g[e]))) * u[e]);
      }
  } else {
    const bf16* res = (const bf16*)a.res;
    float hv[C][M][8], ss[M];
#pragma unroll
    for (int m = 0; m < M; ++m) ss[m] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int m = 0; m < M; ++m) {
        Vec8<bf16>::load(x + (int64_t)m * a.ldx + kc[c], hv[c][m]);
        if (res) {
          float rr[8];
          Vec8<bf16>::load(res + (int64_t)m * a.ldres + kc[c], rr);
#pragma unroll
          for (int e = 0; e < 8; ++e) hv[c][m][e] = (float)(bf16)(hv[c][m][e] + rr[e]);   // h rounded as stored
          if (a.h_out && blockIdx.x == 0 && cv[c]) Vec8<bf16>::store((bf16*)a.h_out + (int64_t)m * a.ldh + kc[c], hv[c][m]);
        }
        if (cv[c]) {
#pragma unroll
          for (int e = 0; e < 8; ++e) ss[m] += hv[c][m][e] * hv[c][m][e];
        }
      }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v = wave_sum(ss[m]);
      if (lane == 0) nred[wave][m] = v;
    }
    __syncthreads();
    const bf16* gw = (const bf16*)a.g;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float gv[8];
      Vec8<bf16>::load(gw + kc[c], gv);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float tot = 0.f;
        for (int v = 0; v < nw; ++v) tot += nred[v][m];
        const float rs = rsqrtf(tot / (float)K + a.eps);
#pragma unroll
        for (int e = 0; e < 8; ++e) xs[c][m][e] = (bf16)(hv[c][m][e] * rs * gv[e]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
    if (!cv[c]) {
#pragma unroll
      for (int m = 0; m < M; ++m) xs[c][m] = bf16x8{};
    }

  float acc[R][M];
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float wv = (float)wr[r][c][e];
#pragma unroll
        for (int m = 0; m < M; ++m) acc[r][m] = fmaf(wv, (float)xs[c][m][e], acc[r][m]);
      }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v = wave_sum(acc[r][m]);
      if (lane == 0) red[wave][r * M + m] = v;
    }
  __syncthreads();
  if ((int)threadIdx.x < R * M) {
    float sum = 0.f;
    for (int v = 0; v < nw; ++v) sum += red[v][threadIdx.x];
    const int r = threadIdx.x / M, m = threadIdx.x % M;
    ((bf16*)a.y)[(int64_t)m * a.ldy + n0 + r] = (bf16)sum;
  }
}

}  // namespace

constexpr int GEMV_MAX_M = 2, GEMV_MAX_K = 16 * 1024, GEMV_ROWS = 8;

bool gemv_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 1 && M <= GEMV_MAX_M && N > 0 && N % GEMV_ROWS == 0 && K > 0 && K <= GEMV_MAX_K && K % 8 == 0;
}

void gemv(const GemvArgs& a, int xmode, hipStream_t st) {
  const dim3 grid((unsigned)(a.N / GEMV_ROWS)), block((unsigned)(64 * cdiv(a.K, 1024)));   // a wave per 1024 of K
#define DPH_GEMV(M_, XM_) hipLaunchKernelGGL((gemv_k<M_, XM_>), grid, block, 0, st, a)
#define DPH_GEMV_M(XM_)          \
  do {                           \
    if (a.M == 1) DPH_GEMV(1, XM_); \
    else DPH_GEMV(2, XM_);       \
  } while (0)
  if (xmode == GX_SWIGLU) DPH_GEMV_M(GX_SWIGLU);
  else if (xmode == GX_NORM) DPH_GEMV(1, GX_NORM);   // one row only (two rows spill; callers check)
  else DPH_GEMV_M(GX_PLAIN);
#undef DPH_GEMV_M
#undef DPH_GEMV
}

bool skinny_gemm_supported(int64_t M, int64_t N, int64_t K) {
  if (M < 1 || M > 64 || N <= 0 || K <= 0) return false;
  if (M <= GEMV_MAX_M && K <= GEMV_MAX_K && K % 8 == 0) return N % GEMV_ROWS == 0;
  return N % 16 == 0 && K % (32 * SG_WAVES) == 0;
}

void skinny_gemm(const void* x, int64_t ldx, const void* w, int64_t ldw, void* y, int64_t ldy, int M, int N, int K,
                 hipStream_t st) {
  const dim3 grid((unsigned)(N / 16)), block(64 * SG_WAVES);
  const bf16* xb = (const bf16*)x;
  const bf16* wb = (const bf16*)w;
  bf16* yb = (bf16*)y;
  if (M <= GEMV_MAX_M && K <= GEMV_MAX_K && K % 8 == 0) {
    GemvArgs a{};
    a.x = x; a.ldx = ldx; a.w = w; a.ldw = ldw; a.y = y; a.ldy = ldy; a.M = M; a.N = N; a.K = K;
    gemv(a, GX_PLAIN, st);
    return;
  }
  // (waves, unroll) sweeps of benchmarks/skinny_gemm_bench.py picked SG_WAVES / SG_UNROLL (profiles/r3/skinny_*)
  const int mt = (M + 15) / 16;
  switch (mt) {
    case 1: hipLaunchKernelGGL((skinny_gemm_k<1, SG_UNROLL>), grid, block, 0, st, xb, ldx, wb, ldw, yb, ldy, M, K); break;
    case 2: hipLaunchKernelGGL((skinny_gemm_k<2, SG_UNROLL>), grid, block, 0, st, xb, ldx, wb, ldw, yb, ldy, M, K); break;
    case 3: hipLaunchKernelGGL((skinny_gemm_k<3, 4>), grid, block, 0, st, xb, ldx, wb, ldw, yb, ldy, M, K); break;
    default: hipLaunchKernelGGL((skinny_gemm_k<4, 4>), grid, block, 0, st, xb, ldx, wb, ldw, yb, ldy, M, K); break;
  }
}

}  // namespace dph
