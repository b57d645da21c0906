// Flash attention forward + backward for CDNA4 (gfx950), bf16 in / fp32 accumulate, MFMA 32x32x16.
// Replaces the reference's F.scaled_dot_product_attention(q, k, v, is_causal=True)
// (fsdp_tp/llama2_model.py:223) and the explicit softmax(QK^T)V of the ViT
// (scripts/03_tensor_parallel_tp/tensor_parallel_vit.py:120-122).
//
// Forward ("swapped" product, cdna_hip_programming.md App. B): one workgroup = 4 waves = 128 query rows,
// one wave = 32 query rows.  S^T = K Q^T puts ONE query per lane (lane & 31) with 16 of the tile's keys
// per half-wave, so the online-softmax state (m, l) and the O^T accumulator rescale are lane-local and
// a row reduction is 31 VALU ops + one permlane32_swap.  O^T = V^T P^T consumes the S^T accumulator
// directly as the B operand (no LDS round trip for P); V^T fragments come from ds_read_b64_tr_b16
// transposed LDS reads.  K/V tiles (64 keys) are register-staged into a double-buffered, XOR-swizzled
// LDS image (conflict-free for both ds_read_b128 row reads and tr reads), one barrier per tile.
//
// Backward: one workgroup = 4 waves (one per SIMD) = 128 keys of one (batch, kv-head); each wave owns 32 keys and keeps
// dK^T and dV^T in registers while the workgroup sweeps all query heads of the GQA group x 32-row query
// tiles.  S and dP are computed with the key on the lane, so P and dS are directly the B operands of
// dV^T += dO^T P and dK^T += Q^T dS; dS crosses LDS once (a [key][q] image) for dQ = dS K, which
// waves 0..D/32-1 compute for one 32-column d-tile each over all 128 keys and add to an fp32 dQ
// accumulator with 256-B-per-instruction global atomics (1/320 atomic byte per FLOP).
#include "dph_common.h"
#include "kernels.h"

namespace dph {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__device__ __forceinline__ float exp2_(float x) { return __builtin_amdgcn_exp2f(x); }

// Byte offset of 16-B chunk `ch` of row `row` in an LDS image whose rows hold NC 16-B chunks.
// Rows are packed into 256-B lines; chunk slots are XOR-permuted per line so that (a) 32 lanes reading
// the same chunk of 32 consecutive rows with ds_read_b128 and (b) ds_read_b64_tr_b16 reads of 4
// consecutive rows x 4 consecutive chunks hit distinct bank slots.
template <int NC>
__device__ __forceinline__ int img_off(int row, int ch) {
  const int F = row * NC + ch;
  const int line = F >> 4, c = F & 15;
  const int f = ((line & 3) << 2) | ((line >> 2) & 3);
  return (line << 8) + ((c ^ f) << 4);
}

__device__ __forceinline__ bf16x8 lds_b128(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}
// Two transposed 4x16 reads -> one 8-element MFMA operand.
__device__ __forceinline__ bf16x8 lds_tr2(const char* base, int off_lo, int off_hi) {
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off_lo));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off_hi));
  bf16x4 a = __builtin_bit_cast(bf16x4, lo), b = __builtin_bit_cast(bf16x4, hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Both half-waves end up with the max / sum over the 32 keys of their shared query.
__device__ __forceinline__ float half_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Accumulator register r of a 32x32 MFMA tile holds row (r&3) + 8*(r>>2) + 4*h of column lane&31.
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}

// ==================================================================================================
// Forward
// ==================================================================================================
template <int HD, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(AttnParams p) {
  constexpr int BM = 128, BN = 64, NC = HD / 8, KS = HD / 16, DT = HD / 32;
  constexpr int TILE = BN * HD * 2;          // bytes of one K (or V) tile image
  constexpr int CPT = (BN * NC) / 256;       // 16-B chunks per thread per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (p.Sq + BM - 1) / BM;
  const int qb = CAUSAL ? nqb - 1 - (int)blockIdx.x : (int)blockIdx.x;  // heaviest causal blocks first
  const int hq = blockIdx.y, b = blockIdx.z;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qb * BM;
  const int myq = q0 + wid * 32 + l32;
  const int off = p.Sk - p.Sq;

  const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[myq][16*kk + 8h .. +7].
  bf16x8 qf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
    qf[kk] = (myq < p.Sq) ? *reinterpret_cast<const bf16x8*>(qp + (int64_t)myq * p.q_ss + kk * 16 + 8 * h) : zero8();

  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + off);
  const int ntiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m = -INFINITY, lsum = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;

  bf16x8 stk[CPT], stv[CPT];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int F = threadIdx.x + 256 * i;
      const int key = t * BN + F / NC, ch = F % NC;
      if (key < p.Sk) {
        stk[i] = *reinterpret_cast<const bf16x8*>(kp + (int64_t)key * p.k_ss + ch * 8);
        stv[i] = *reinterpret_cast<const bf16x8*>(vp + (int64_t)key * p.v_ss + ch * 8);
      } else {
        stk[i] = zero8();
        stv[i] = zero8();
      }
    }
  };
  auto swrite = [&](int buf) {
    char* Kl = smem + buf * 2 * TILE;
    char* Vl = Kl + TILE;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int F = threadIdx.x + 256 * i;
      const int o_ = img_off<NC>(F / NC, F % NC);
      *reinterpret_cast<bf16x8*>(Kl + o_) = stk[i];
      *reinterpret_cast<bf16x8*>(Vl + o_) = stv[i];
    }
  };

  if (ntiles > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();

  // per-lane constant parts of the tr-read addresses (A = V^T operand)
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) gload(t + 1);
    const char* Kl = smem + buf * 2 * TILE;
    const char* Vl = Kl + TILE;

    // ---- S^T = K Q^T for two 32-key sub-tiles ----
    f32x16 s[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[sub][r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const bf16x8 a = lds_b128(Kl, img_off<NC>(sub * 32 + l32, kk * 2 + h));
        s[sub] = mfma32(a, qf[kk], s[sub]);
      }
    }
    // ---- scale, mask, online softmax (lane-local per query) ----
    const int k0 = t * BN;
    const bool need_mask = (k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0 + wid * 32 + off));
    float mx = -INFINITY;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = s[sub][r] * sl2;
        if (need_mask) {
          const int key = k0 + sub * 32 + acc_row(r, h);
          if (key >= p.Sk || (CAUSAL && key > myq + off)) v = -INFINITY;
        }
        s[sub][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = half_max(mx);
    const float m_new = fmaxf(m, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2_(m - m_use);
    float ls = 0.f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = exp2_(s[sub][r] - m_use);
        s[sub][r] = e;
        ls += e;
      }
    ls = half_sum(ls);
    lsum = lsum * alpha + ls;
    m = m_new;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;

    // ---- P^T as B operand: k-step ks covers keys 16*ks .. 16*ks+15 of the tile ----
    bf16x8 pf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[ks][j] = (bf16)s[ks >> 1][8 * (ks & 1) + j];

    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int krow = ks * 16 + 4 * (g >> 1) + tq;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int ch = dt * 4 + 2 * (g & 1) + (tp >> 1);
        const int bo = 8 * (tp & 1);
        const bf16x8 a = lds_tr2(Vl, img_off<NC>(krow, ch) + bo, img_off<NC>(krow + 8, ch) + bo);
        o[dt] = mfma32(a, pf[ks], o[dt]);
      }
    }
    if (t + 1 < ntiles) swrite(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: O = O^T / l, lse ----
  if (myq < p.Sq) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* op = (bf16*)p.o + (int64_t)b * p.o_sb + (int64_t)myq * p.o_ss + (int64_t)hq * p.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (bf16)(o[dt][4 * gg + j] * inv);
        *reinterpret_cast<bf16x4*>(op + dt * 32 + 8 * gg + 4 * h) = w;
      }
    if (h == 0 && p.lse)
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + myq] =
          lsum > 0.f ? (m + __log2f(lsum)) * 0.6931471805599453f : -INFINITY;
  }
}

// ==================================================================================================
// Backward
// ==================================================================================================
// delta[b, h, q] = sum_d dO[b,q,h,d] * O[b,q,h,d]   (one wave per row, fp32)
__global__ __launch_bounds__(256) void attn_delta_k(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                    float* __restrict__ delta, int B, int S, int H, int D,
                                                    int64_t o_sb, int64_t o_ss, int64_t o_sh, int64_t d_sb,
                                                    int64_t d_ss, int64_t d_sh) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = (int64_t)B * H * S;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
    const int q = (int)(r % S);
    const int64_t bh = r / S;
    const int hh = (int)(bh % H), bb = (int)(bh / H);
    const bf16* a = o + bb * o_sb + (int64_t)q * o_ss + hh * o_sh;
    const bf16* c = dout + bb * d_sb + (int64_t)q * d_ss + hh * d_sh;
    float s = 0.f;
    for (int d = lane * 8; d < D; d += 512) {
      float x[8], y[8];
      Vec8<bf16>::load(a + d, x);
      Vec8<bf16>::load(c + d, y);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += x[k] * y[k];
    }
    s = wave_sum(s);
    if (lane == 0) delta[r] = s;
  }
}

// dq (bf16, [B,Sq,Hq,D] contiguous) = scale * dq_accum
__global__ __launch_bounds__(256) void attn_dq_convert_k(const float* __restrict__ acc, bf16* __restrict__ dq,
                                                         int64_t n8, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<float>::load(acc + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= scale;
    Vec8<bf16>::store(dq + i * 8, v);
  }
}

template <int HD, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_bwd_k(AttnBwdParams P) {
  constexpr int NT = 256;                   // 4 waves, one per SIMD: the whole 512-entry register file per wave
  constexpr int BNK = 128, BMQ = 32, NC = HD / 8, KS = HD / 16, DT = HD / 32;
  constexpr int KIMG = BNK * HD * 2;        // K image [128 keys][HD]
  constexpr int QIMG = BMQ * HD * 2;        // Q / dO tile image [32 q][HD]
  constexpr int SIMG = BNK * BMQ * 2;       // dS image [128 keys][32 q]
  // smem: K | Q0 | dO0 | Q1 | dO1 | dS | lse[2][32] | delta[2][32]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kimg = smem;
  char* Qbuf = smem + KIMG;                  // Q buf b at Qbuf + b*2*QIMG, dO at +QIMG
  char* Simg = Qbuf + 4 * QIMG;
  float* lse_s = reinterpret_cast<float*>(Simg + SIMG);
  float* del_s = lse_s + 2 * BMQ;

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int kb0 = blockIdx.x * BNK;
  const int hk = blockIdx.y, b = blockIdx.z;
  const int grp = p.Hq / p.Hkv;
  const int off = p.Sk - p.Sq;
  const int mykey = kb0 + wid * 32 + l32;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  // K image (all BNK keys) in LDS; V^T fragments of this wave's 32 keys in registers.
#pragma unroll
  for (int i = 0; i < (BNK * NC) / NT; ++i) {
    const int F = threadIdx.x + NT * i;
    const int key = kb0 + F / NC, ch = F % NC;
    bf16x8 v = key < p.Sk ? *reinterpret_cast<const bf16x8*>(kp + (int64_t)key * p.k_ss + ch * 8) : zero8();
    *reinterpret_cast<bf16x8*>(Kimg + img_off<NC>(F / NC, ch)) = v;
  }
  bf16x8 vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
    vf[kk] = mykey < p.Sk ? *reinterpret_cast<const bf16x8*>(vp + (int64_t)mykey * p.v_ss + kk * 16 + 8 * h) : zero8();

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

  // query tiles: causal -> only queries q with q + off >= kb0 can see any key of this block
  int qstart = 0;
  if (CAUSAL) qstart = max(0, kb0 - off) / BMQ * BMQ;
  const int nqt_head = qstart < p.Sq ? (p.Sq - qstart + BMQ - 1) / BMQ : 0;
  const int total = nqt_head * grp;

  // staging registers for the next Q / dO tile (one 16-B chunk each per thread when HD = 128)
  constexpr int QCPT = (BMQ * NC + NT - 1) / NT;
  bf16x8 stq[QCPT], sto[QCPT];
  float st_lse = 0.f, st_del = 0.f;
  auto gload = [&](int it) {
    const int hq = hk * grp + it / nqt_head;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
    const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
#pragma unroll
    for (int i = 0; i < QCPT; ++i) {
      const int F = threadIdx.x + NT * i;
      const int q = qt0 + F / NC, ch = F % NC;
      if (F < BMQ * NC && q < p.Sq) {
        stq[i] = *reinterpret_cast<const bf16x8*>(qp + (int64_t)q * p.q_ss + ch * 8);
        sto[i] = *reinterpret_cast<const bf16x8*>(dop + (int64_t)q * P.do_ss + ch * 8);
      } else {
        stq[i] = zero8();
        sto[i] = zero8();
      }
    }
    if (threadIdx.x < BMQ) {
      const int q = qt0 + threadIdx.x;
      const int64_t idx = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      st_lse = q < p.Sq ? p.lse[idx] * 1.4426950408889634f : 0.f;  // log2 units
      st_del = q < p.Sq ? P.delta[idx] : 0.f;
    }
  };
  auto swrite = [&](int buf) {
    char* Ql = Qbuf + buf * 2 * QIMG;
    char* Ol = Ql + QIMG;
#pragma unroll
    for (int i = 0; i < QCPT; ++i) {
      const int F = threadIdx.x + NT * i;
      if (F < BMQ * NC) {
        const int o_ = img_off<NC>(F / NC, F % NC);
        *reinterpret_cast<bf16x8*>(Ql + o_) = stq[i];
        *reinterpret_cast<bf16x8*>(Ol + o_) = sto[i];
      }
    }
    if (threadIdx.x < BMQ) {
      lse_s[buf * BMQ + threadIdx.x] = st_lse;
      del_s[buf * BMQ + threadIdx.x] = st_del;
    }
  };

  if (total > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const int hq = hk * grp + it / nqt_head;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    if (it + 1 < total) gload(it + 1);
    const char* Ql = Qbuf + buf * 2 * QIMG;
    const char* Ol = Ql + QIMG;

    // S = Q K^T and dP = dO V^T with the key on the lane: A = Q / dO rows (LDS), B = K^T / V^T.
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const bf16x8 kf = lds_b128(Kimg, img_off<NC>(wid * 32 + l32, kk * 2 + h));
      const bf16x8 qa = lds_b128(Ql, img_off<NC>(l32, kk * 2 + h));
      const bf16x8 oa = lds_b128(Ol, img_off<NC>(l32, kk * 2 + h));
      s = mfma32(qa, kf, s);
      dp = mfma32(oa, vf[kk], dp);
    }
    // P = exp2(S * c - lse), dS = P (dP - delta); rows = queries
    const bool need_mask = CAUSAL && (kb0 + wid * 32 + 31 > qt0 + off);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = acc_row(r, h);
      float pv = exp2_(s[r] * sl2 - lse_s[buf * BMQ + qr]);
      if (qt0 + qr >= p.Sq || mykey >= p.Sk) pv = 0.f;
      if (need_mask && mykey > qt0 + qr + off) pv = 0.f;
      s[r] = pv;
      dp[r] = pv * (dp[r] - del_s[buf * BMQ + qr]);
    }
    bf16x8 pb[2], sb[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pb[ks][j] = (bf16)s[8 * ks + j];
        sb[ks][j] = (bf16)dp[8 * ks + j];
      }
    // dV^T += dO^T P ; dK^T += Q^T dS   (A via transposed reads, k-order matching the accumulator)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int qrow = ks * 16 + 4 * (g >> 1) + tq;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int ch = dt * 4 + 2 * (g & 1) + (tp >> 1);
        const int bo = 8 * (tp & 1);
        const bf16x8 oa = lds_tr2(Ol, img_off<NC>(qrow, ch) + bo, img_off<NC>(qrow + 8, ch) + bo);
        dv[dt] = mfma32(oa, pb[ks], dv[dt]);
        const bf16x8 qa = lds_tr2(Ql, img_off<NC>(qrow, ch) + bo, img_off<NC>(qrow + 8, ch) + bo);
        dk[dt] = mfma32(qa, sb[ks], dk[dt]);
      }
    }
    // dS -> LDS as a [key][q] image (64-B rows): lane writes 4 consecutive q per group
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      bf16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (bf16)dp[4 * gg + j];
      *reinterpret_cast<bf16x4*>(Simg + (wid * 32 + l32) * (BMQ * 2) + (8 * gg + 4 * h) * 2) = w;
    }
    __syncthreads();
    // dQ[q][d] += sum_key dS[q][key] K[key][d] for d-tile `wid` (waves 0..DT-1)
    if (wid < DT) {
      f32x16 dq;
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[r] = 0.f;
#pragma unroll 4
      for (int kstep = 0; kstep < BNK / 16; ++kstep) {
        // A = dS [q x key]: lane (q = l32) needs keys 16*kstep + 8h + 0..7 -> tr reads of the [key][q] image
        const int krow = kstep * 16 + 8 * h + tq;
        const int qcol = 16 * (g & 1) + 4 * tp;
        const bf16x8 a = lds_tr2(Simg, krow * (BMQ * 2) + qcol * 2, (krow + 4) * (BMQ * 2) + qcol * 2);
        // B = K [key x d]: lane (d = l32) needs keys 16*kstep + 8h + 0..7 -> tr reads of the K image
        const int ch = wid * 4 + 2 * (g & 1) + (tp >> 1);
        const int bo = 8 * (tp & 1);
        const bf16x8 kb = lds_tr2(Kimg, img_off<NC>(krow, ch) + bo, img_off<NC>(krow + 4, ch) + bo);
        dq = mfma32(a, kb, dq);
      }
      float* dqp = P.dq_accum + ((int64_t)b * p.Sq) * p.Hq * HD + (int64_t)hq * HD + wid * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qt0 + acc_row(r, h);
        if (q < p.Sq) atomicAdd(dqp + (int64_t)q * p.Hq * HD, dq[r]);
      }
    }
    if (it + 1 < total) swrite(buf ^ 1);
    __syncthreads();
  }

  // epilogue: dK = scale * dK^T^T, dV ; per-kv-head complete (all query heads of the group swept)
  if (mykey < p.Sk) {
    bf16* dkp = (bf16*)P.dk + (((int64_t)b * p.Sk + mykey) * p.Hkv + hk) * HD;
    bf16* dvp = (bf16*)P.dv + (((int64_t)b * p.Sk + mykey) * p.Hkv + hk) * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 wk, wv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wk[j] = (bf16)(dk[dt][4 * gg + j] * p.scale);
          wv[j] = (bf16)dv[dt][4 * gg + j];
        }
        *reinterpret_cast<bf16x4*>(dkp + dt * 32 + 8 * gg + 4 * h) = wk;
        *reinterpret_cast<bf16x4*>(dvp + dt * 32 + 8 * gg + 4 * h) = wv;
      }
  }
}

// ==================================================================================================
template <int HD>
static void fwd_launch(const AttnParams& p, hipStream_t st) {
  const dim3 grid((p.Sq + 127) / 128, p.Hq, p.B);
  const size_t lds = 2 * 2 * 64 * HD * 2;
  if (p.causal) hipLaunchKernelGGL((attn_fwd_k<HD, true>), grid, dim3(256), lds, st, p);
  else hipLaunchKernelGGL((attn_fwd_k<HD, false>), grid, dim3(256), lds, st, p);
}

void flash_attn_fwd(const AttnParams& p, hipStream_t st) {
  if (p.B == 0 || p.Sq == 0) return;
  switch (p.D) {
    case 32: fwd_launch<32>(p, st); break;
    case 64: fwd_launch<64>(p, st); break;
    case 128: fwd_launch<128>(p, st); break;
    default: break;  // rejected by the host op before launch
  }
}

template <int HD>
static void bwd_launch(const AttnBwdParams& P, hipStream_t st) {
  const AttnParams& p = P.f;
  const size_t lds = 128 * HD * 2 + 4 * 32 * HD * 2 + 128 * 32 * 2 + 4 * 32 * 4;
  static bool attr_set[2] = {false, false};
  if (!attr_set[p.causal ? 1 : 0]) {
    if (p.causal) hipFuncSetAttribute((const void*)attn_bwd_k<HD, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    else hipFuncSetAttribute((const void*)attn_bwd_k<HD, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set[p.causal ? 1 : 0] = true;
  }
  const dim3 grid((p.Sk + 127) / 128, p.Hkv, p.B);
  if (p.causal) hipLaunchKernelGGL((attn_bwd_k<HD, true>), grid, dim3(256), lds, st, P);
  else hipLaunchKernelGGL((attn_bwd_k<HD, false>), grid, dim3(256), lds, st, P);
}

void flash_attn_bwd(const AttnBwdParams& P, hipStream_t st) {
  const AttnParams& p = P.f;
  if (p.B == 0 || p.Sq == 0) return;
  // delta = rowsum(dO * O)
  const int64_t rows = (int64_t)p.B * p.Hq * p.Sq;
  hipLaunchKernelGGL(attn_delta_k, dim3(stream_grid(rows, 4)), dim3(256), 0, st, (const bf16*)p.o,
                     (const bf16*)P.dout, P.delta, p.B, p.Sq, p.Hq, p.D, p.o_sb, p.o_ss, p.o_sh, P.do_sb, P.do_ss,
                     P.do_sh);
  const int64_t nq = (int64_t)p.B * p.Sq * p.Hq * p.D;
  hipMemsetAsync(P.dq_accum, 0, nq * sizeof(float), st);
  switch (p.D) {
    case 32: bwd_launch<32>(P, st); break;
    case 64: bwd_launch<64>(P, st); break;
    case 128: bwd_launch<128>(P, st); break;
    default: break;
  }
  hipLaunchKernelGGL(attn_dq_convert_k, dim3(stream_grid(nq / 8, 256)), dim3(256), 0, st, P.dq_accum, (bf16*)P.dq,
                     nq / 8, p.scale);
}

}  // namespace dph
