// Flash attention forward for CDNA4 (gfx950): the kernel and its launcher.  Design notes for the whole attention
// family (forward, backward, dropout) are at the top of attention_common.h.
#include <type_traits>

#include "attention_common.h"

namespace dph {

// ==================================================================================================
// Forward
// ==================================================================================================
// Online softmax in log2 units with the 1/sqrt(d) scale folded into one FMA per score:
//   p = exp2(s * scale*log2e - m).  The running max m is only raised (and O, l rescaled) when some lane's
// tile max exceeds it by more than RESCALE_THR (FA4-style lazy rescaling): p is then bounded by 2^THR,
// harmless for the bf16 P operand and the fp32 accumulators, and the exact result is recovered by the
// final 1/l.  The rescale branch is wave-uniform (ballot), so steady-state tiles skip 16*DT multiplies.
// Rejected round-4/5 variants of this kernel (evidence kept under profiles/): 8-wave workgroups (819-822 vs 834-838
// TFLOP/s), waves 4..7 staggered one barrier behind (809-814), issue priority over the MFMA chains (within noise),
// a software-pipelined body that overlaps each wave's softmax with its own next QK^T (754-788 vs 831-833,
// profiles/r5/attn_fwd_pipe/), and one wave per SIMD with 64 query rows per wave, every K / V fragment feeding two
// 32-row blocks, the whole 512-entry file (256 VGPR + 256 AGPR, no scratch): 629-630 vs 819 TFLOP/s, the compiler's
// AGPR form adds ~350 v_accvgpr moves per tile and no second wave hides the barrier (profiles/r5/attn_q2/).
template <int HD, bool CAUSAL, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(AttnParams p) {
  constexpr int NW = 4;
  using Plan = KVTilePlan<HD, 64 * NW>;
  constexpr int BM = 32 * NW, BN = Plan::BN, KS = Plan::KS, DT = Plan::DT, TILE = Plan::TILE;
  constexpr float RESCALE_THR = 8.f;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (p.Sq + BM - 1) / BM;
  int bx, hq, b;
  xcd_block(nqb, p.Hq, bx, hq, b, nqb * p.Hq * p.B);
  const int qb = CAUSAL ? nqb - 1 - bx : bx;  // heaviest causal blocks first
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int myq = q0w + l32;
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
  const int wtiles = wave_tile_count<CAUSAL>(ntiles, q0w, off);

  Plan plan;
  plan.init(lane, p.k_ss);
  plan.init_async();
  const unsigned lds_w = lds_addr(smem + (threadIdx.x >> 6) * 64 * 16);

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  const f32x16 zacc = {};
  float m = -INFINITY, lsum = 0.f;  // m: running max of s*sl2; lsum: this half-wave's partial row sum
  const float sl2 = p.scale * 1.4426950408889634f;
  const unsigned drk = DROP ? attn_row_key(p.drop_seed, (unsigned)(b * p.Hq + hq), (unsigned)myq) : 0u;
  const unsigned dthr = DROP ? attn_drop_thr(p.drop_p) : 0u;

  if (ntiles > 0) plan.stage_async(lds_w, kp, vp, p.k_ss, p.v_ss, 0, p.Sk);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  auto tile = [&](const char* Kl, const char* Vl, int k0, bool need_mask) {
    // ---- S^T = K Q^T for two 32-key sub-tiles ----
    // all 2 x KS K fragments are read before the MFMA chains (counted lgkmcnt waits): read one, wait, multiply
    // exposed a full LDS round trip per MFMA
    bf16x8 kf[2][KS];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) kf[sub][kk] = lds_b128(Kl, plan.row(sub, kk));
    f32x16 s[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      s[sub] = mfma32(kf[sub][0], qf[0], zacc);
#pragma unroll
      for (int kk = 1; kk < KS; ++kk) s[sub] = mfma32(kf[sub][kk], qf[kk], s[sub]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * KS, 0);   // the DS reads first ...
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * KS, 0);   // ... then the MFMAs
    // phase fences keep the scheduler from hoisting the next phase's LDS reads into this one's live range
    __builtin_amdgcn_sched_barrier(0);
    if (need_mask) {  // wave-uniform: only diagonal / ragged tiles pay for the selects
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + sub * 32 + acc_row(r, h);
          s[sub][r] = (key >= p.Sk || (CAUSAL && key > myq + off)) ? -INFINITY : s[sub][r];
        }
    }
    float mx = fmaxf(s[0][0], s[1][0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
    mx = half_max(mx) * sl2;
    if (__ballot(mx > m + RESCALE_THR)) {
      const float mn = fmaxf(m, mx);
      const float alpha = mn == -INFINITY ? 1.f : exp2_(m - mn);
      lsum *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      m = mn;
    }
    const float mneg = m == -INFINITY ? 0.f : -m;
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[0][r] = exp2_(fmaf(s[0][r], sl2, mneg));
      s[1][r] = exp2_(fmaf(s[1][r], sl2, mneg));
      ls0 += s[0][r];
      ls1 += s[1][r];
    }
    lsum += ls0 + ls1;
    if constexpr (DROP) {   // after the row sum: the normaliser is the undropped softmax's
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (!attn_keep(drk, (unsigned)(k0 + sub * 32 + acc_row(r, h)), dthr)) s[sub][r] = 0.f;
    }

    // ---- P^T as B operand: k-step ks covers keys 16*ks .. 16*ks+15 of the tile ----
    bf16x8 pf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[ks][j] = (bf16)s[ks >> 1][8 * (ks & 1) + j];
    // no fence before the PV MFMAs: the compiler overlaps the first PV k-steps with the tail of the exp / convert work
    // (+2 % forward TFLOP/s at B 8, H 32, S 4096, D 128; the backward kernels keep their fences: -2 % without them)

    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        o[dt] = mfma32(lds_tr2(Vl, plan.tr(ks, dt, 0), plan.tr(ks, dt, 1)), pf[ks], o[dt]);
  };

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) plan.stage_async(lds_w + (buf ^ 1) * 2 * TILE, kp, vp, p.k_ss, p.v_ss, (t + 1) * BN, p.Sk);
    const char* Kl = smem + buf * 2 * TILE;
    if (t < wtiles) {
      const int k0 = t * BN;
      tile(Kl, Kl + TILE, k0, (k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0w + off)));
    }
    wait_vmcnt<0>();   // this wave's share of tile t+1 has landed ...
    __builtin_amdgcn_s_barrier();   // ... and every wave's, and nobody reads tile t's images any more
  }

  // ---- epilogue: O = O^T / l, lse ----
  lsum = half_sum(lsum);
  if (myq < p.Sq && p.acc_o) {
    // ring merge into the fp32 accumulators (both half-waves read the old lse before half 0 writes the new one:
    // one instruction stream, loads issued first)
    const float inv = lsum > 0.f ? (DROP ? 1.f / (1.f - p.drop_p) : 1.f) / lsum : 0.f;
    const float lse_b = lsum > 0.f ? (m + __log2f(lsum)) * 0.6931471805599453f : -INFINITY;
    float* al = p.acc_lse + (int64_t)b * p.al_sb + (int64_t)hq * p.al_sh + myq;
    const float old = *al;
    const float mx = fmaxf(old, lse_b);
    float w1 = 0.f, w2 = 0.f, nl = -INFINITY;
    if (mx != -INFINITY) {
      const float e1 = __expf(old - mx), e2 = __expf(lse_b - mx), sum = e1 + e2;
      nl = mx + __logf(sum);
      w1 = e1 / sum;
      w2 = e2 / sum * inv;
    }
    float* ao = p.acc_o + (int64_t)b * p.ao_sb + (int64_t)myq * p.ao_ss + (int64_t)hq * p.ao_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        f32x4* ptr = reinterpret_cast<f32x4*>(ao + dt * 32 + 8 * gg + 4 * h);
        f32x4 cur = *ptr;
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = cur[j] * w1 + o[dt][4 * gg + j] * w2;
        *ptr = cur;
      }
    if (h == 0) *al = nl;
  } else if (!p.acc_o) {
    // O = O^T / l through this wave's LDS slab (the K/V images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= 4 * TILE, "epilogue slabs exceed the forward kernel's LDS");
    const float inv = lsum > 0.f ? (DROP ? 1.f / (1.f - p.drop_p) : 1.f) / lsum : 0.f;
    bf16* o0 = (bf16*)p.o + (int64_t)b * p.o_sb + (int64_t)q0w * p.o_ss + (int64_t)hq * p.o_sh;
    store_rows_lds<DT>(smem + wid * (32 * HD * 2), o0, p.o_ss, min(32, p.Sq - q0w), o, inv, h, l32, 0, nullptr,
                       nullptr, 0);
    if (myq < p.Sq && h == 0 && p.lse)
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + myq] =
          lsum > 0.f ? (m + __log2f(lsum)) * 0.6931471805599453f : -INFINITY;
  }
}

// ==================================================================================================
// Forward on v_mfma_f32_16x16x32_bf16 (head dim 128, no dropout, no ring merge): the structure above as 16x16 tiles.
// A wave owns 32 queries = two 16-query column blocks qb; per 64-key tile:
//   S^T[kb][qb] = K Q^T      A = K rows (x16 image, b128), B = Q^T fragments (registers)      32 MFMAs
//   online softmax with the query on the lane: a lane holds 16 of the tile's keys per query (4 per key block), the
//   row max / sum finish with two lane swaps (permlane16 / permlane32), lazy rescale as above
//   O^T[db][qb] += V^T P^T   A = x16_tr(V image), B = the P^T pair of key blocks (2 ks, 2 ks + 1)   32 MFMAs
__device__ __forceinline__ float quad_max(float x) {   // max over lanes l, l ^ 16, l ^ 32, l ^ 48
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(c[0]), __uint_as_float(c[1]));
}
__device__ __forceinline__ float quad_sum(float x) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(c[0]) + __uint_as_float(c[1]);
}

template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd16_k(AttnParams p) {
  constexpr int HD = 128, NW = 4, NT = 64 * NW, BM = 32 * NW, BN = 64;
  constexpr int TILE = BN * HD * 2;   // one 64-row x16 image; buffer = K | V
  constexpr float RESCALE_THR = 8.f;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int nqb = (p.Sq + BM - 1) / BM;
  int bx, hq, b;
  xcd_block(nqb, p.Hq, bx, hq, b, nqb * p.Hq * p.B);
  const int qblk = CAUSAL ? nqb - 1 - bx : bx;  // heaviest causal blocks first
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qblk * BM, q0w = q0 + wid * 32;
  const int off = p.Sk - p.Sq;

  const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  bf16x8 qf[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = q0w + qb * 16 + i16;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      qf[qb][kk] = q < p.Sq ? *reinterpret_cast<const bf16x8*>(qp + (int64_t)q * p.q_ss + kk * 32 + 8 * g) : zero8();
  }
  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + off);
  const int ntiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;
  const int wtiles = wave_tile_count<CAUSAL>(ntiles, q0w, off);

  X16Stage<BN, NT> st;
  st.init(p.k_ss);
  X16Reads rd;
  rd.init(lane, lds_addr(smem));
  const unsigned lds_w = lds_addr(smem + wid * 1024);

  f32x4 o[8][2];
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[db][qb][r] = 0.f;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};   // per query block: running max (log2 units), partial sum
  const float sl2 = p.scale * 1.4426950408889634f;

  if (ntiles > 0) {
    st.stage(lds_w, kp, p.k_ss, 0, p.Sk);
    st.stage(lds_w + TILE, vp, p.v_ss, 0, p.Sk);
  }
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  // one instantiation of the tile body per image buffer: every LDS read is a per-lane address plus an immediate
  auto tile = [&](auto BUFC, int t) {
    constexpr int buf = decltype(BUFC)::value;
    constexpr unsigned KL = buf * 2 * TILE, VL = KL + TILE;
    if (t + 1 < ntiles) {
      const unsigned nb = lds_w + (buf ^ 1) * 2 * TILE;
      st.stage(nb, kp, p.k_ss, (t + 1) * BN, p.Sk);
      st.stage(nb + TILE, vp, p.v_ss, (t + 1) * BN, p.Sk);
    }
    if (t < wtiles) {
      const int k0 = t * BN;
      f32x4 s[4][2];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) s[kb][qb] = z4;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bf16x8 kf[4];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) kf[kb] = ldsa_b128(rd.row[kk] + KL + (kb << 12));
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          s[kb][0] = mfma16(kf[kb], qf[0][kk], s[kb][0]);
          s[kb][1] = mfma16(kf[kb], qf[1][kk], s[kb][1]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if ((k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0w + off))) {   // wave-uniform
        asm volatile("" ::: "memory");   // a real branch: no if-converted selects on every tile
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = k0 + kb * 16 + 4 * g + r, q = q0w + qb * 16 + i16;
              s[kb][qb][r] = (key >= p.Sk || (CAUSAL && key > q + off)) ? -INFINITY : s[kb][qb][r];
            }
      }
      bf16x8 pf[2][2];   // [ks][qb]
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float mx = fmaxf(s[0][qb][0], s[1][qb][0]);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kb][qb][r]);
        mx = quad_max(mx) * sl2;
        if (__ballot(mx > m[qb] + RESCALE_THR)) {
          const float mn = fmaxf(m[qb], mx);
          const float alpha = mn == -INFINITY ? 1.f : exp2_(m[qb] - mn);
          lsum[qb] *= alpha;
#pragma unroll
          for (int db = 0; db < 8; ++db)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[db][qb][r] *= alpha;
          m[qb] = mn;
        }
        const float mneg = m[qb] == -INFINITY ? 0.f : -m[qb];
        float ls = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[kb][qb][r] = exp2_(fmaf(s[kb][qb][r], sl2, mneg));
            ls += s[kb][qb][r];
          }
        lsum[qb] += ls;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) pf[ks][qb] = acc_pair_b(s[2 * ks][qb], s[2 * ks + 1][qb]);
      }
      // O^T += V^T P^T
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int db = 0; db < 8; ++db) {
          const bf16x8 vt = ldsa_tr(rd.tr[db] + VL + ((ks * 32) << 8));
          o[db][0] = mfma16(vt, pf[ks][0], o[db][0]);
          o[db][1] = mfma16(vt, pf[ks][1], o[db][1]);
        }
    }
    wait_vmcnt<0>();   // this wave's share of tile t+1 has landed ...
    __builtin_amdgcn_s_barrier();   // ... and every wave's, and nobody reads tile t's images any more
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t + 1);
  }

  // ---- epilogue: O = O^T / l, lse ----
  float inv[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    lsum[qb] = quad_sum(lsum[qb]);
    inv[qb] = lsum[qb] > 0.f ? 1.f / lsum[qb] : 0.f;
#pragma unroll
    for (int db = 0; db < 8; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[db][qb][r] *= inv[qb];
  }
  bf16* o0 = (bf16*)p.o + (int64_t)b * p.o_sb + (int64_t)q0w * p.o_ss + (int64_t)hq * p.o_sh;
  store_rows16(smem + wid * (32 * HD * 2), o0, p.o_ss, min(32, p.Sq - q0w), o, 1.f, lane, q0w, nullptr, nullptr, 0);
  if (g == 0 && p.lse) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int q = q0w + qb * 16 + i16;
      if (q < p.Sq)
        p.lse[((int64_t)b * p.Hq + hq) * p.Sq + q] =
            lsum[qb] > 0.f ? (m[qb] + __log2f(lsum[qb])) * 0.6931471805599453f : -INFINITY;
    }
  }
}

// ==================================================================================================
// One geometry for every kernel: 4 waves = 128 query rows (or keys) per workgroup, two workgroups per CU.
template <int HD>
static void fwd_launch(const AttnParams& p, hipStream_t st) {
  const dim3 grid((unsigned)((p.Sq + 127) / 128 * p.Hq * p.B));   // 1-D: xcd_block() maps it
  const size_t lds = 2 * 2 * 64 * HD * 2;
  if (p.drop_p > 0.f) {
    if (p.causal) hipLaunchKernelGGL((attn_fwd_k<HD, true, true>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((attn_fwd_k<HD, false, true>), grid, dim3(256), lds, st, p);
  } else if (HD == 128 && !p.acc_o && attn_get_variant() == 2) {
    if (p.causal) hipLaunchKernelGGL((attn_fwd16_k<true>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((attn_fwd16_k<false>), grid, dim3(256), lds, st, p);
  } else {
    if (p.causal) hipLaunchKernelGGL((attn_fwd_k<HD, true>), grid, dim3(256), lds, st, p);
    else hipLaunchKernelGGL((attn_fwd_k<HD, false>), grid, dim3(256), lds, st, p);
  }
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

}  // namespace dph
