// Flash attention backward for CDNA4 (gfx950): the Q-stationary dQ kernel (which also forms delta = rowsum(dO * O)),
// the KV-stationary dK/dV kernel and their launcher.  Design notes at the top of attention_common.h.
#include <type_traits>

#include "attention_common.h"

namespace dph {

// ==================================================================================================
// Backward
// ==================================================================================================
// ---- dK / dV: KV-stationary.  One workgroup = 4 waves = 128 keys of one (batch, kv head); one wave =
// 32 keys whose K^T / V^T B-operand fragments stay in registers.  The workgroup sweeps every query head
// of the GQA group x 32-row query tiles (double-buffered Q / dO LDS images, one barrier per tile).
// S and dP are computed with the key on the lane, so P and dS are directly the B operands of
// dV^T += dO^T P and dK^T += Q^T dS: no LDS round trip, no atomics.
// The dV / dK transposed reads are software-pipelined one step ahead (the first step issued before the softmax), and a
// wave runs at issue priority 1 while in its MFMA chains (S / dP, then dV / dK) and 0 in its softmax, so the partner
// wave on the SIMD (the other workgroup's) fills the chains' gaps with its softmax instead of competing for issue
// (round 3/4 A/B: +2 % and +1 %; row constants as the initial S / dP accumulators measured -2 % and were removed).
template <int HD, bool CAUSAL, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_k(AttnBwdParams P) {
  constexpr int NW = 4;
  constexpr int NT = 64 * NW, BNK = 32 * NW, BMQ = 32, NC = HD / 8, KS = HD / 16, DT = HD / 32;
  constexpr bool RINIT = false;
  constexpr bool TRPIPE = true;
  constexpr int QIMG = BMQ * HD * 2;        // Q / dO tile image [32 q][HD]
  constexpr int KIMG = BNK * HD * 2;        // K image [128 keys][HD] (B operand of S = Q K^T)
  // img_off's line permutation repeats every 16 lines.  For NC >= 8, rows r and r + 32 are a multiple of 16
  // lines apart, so the wave's K rows reuse the Q-image offsets plus a constant.
  constexpr bool KSHARE = NC >= 8;
  constexpr bool TRADD = NC >= 16;          // +16 rows is a pure byte offset for the transposed reads
  // smem: K | Q0 | dO0 | Q1 | dO1 | -lse2[2][32] | delta[2][32] | dropout row keys[2][32]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kimg = smem;
  char* Qbuf = smem + KIMG;
  float* lse_s = reinterpret_cast<float*>(Qbuf + 4 * QIMG);
  float* del_s = lse_s + 2 * BMQ;
  unsigned* rk_s = reinterpret_cast<unsigned*>(del_s + 2 * BMQ);

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int nkb = (p.Sk + BNK - 1) / BNK;
  int kbx, hk, b;
  xcd_block(nkb, p.Hkv, kbx, hk, b, nkb * p.Hkv * p.B);
  const int kb0 = kbx * BNK;   // ascending = heaviest causal key blocks first
  const int grp = p.Hq / p.Hkv;
  const int off = p.Sk - p.Sq;
  const int key0 = kb0 + wid * 32;
  const int mykey = key0 + l32;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;
  glds_stage<NC, BNK, NT>(Kimg, kp, p.k_ss, kb0, p.Sk);
  bf16x8 vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
    vf[kk] = mykey < p.Sk ? *reinterpret_cast<const bf16x8*>(vp + (int64_t)mykey * p.v_ss + kk * 16 + 8 * h)
                          : zero8();
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }
  const f32x16 zacc = {};

  // hoisted per-lane LDS offsets
  int qro[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) qro[kk] = img_off<NC>(l32, kk * 2 + h);
  auto kofs = [&](int kk) {
    return KSHARE ? qro[kk] + wid * 32 * NC * 16 : img_off<NC>(wid * 32 + l32, kk * 2 + h);
  };
  int tro[TRADD ? 1 : 2][DT][2];
#pragma unroll
  for (int ks = 0; ks < (TRADD ? 1 : 2); ++ks)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi)
        tro[ks][dt][hi] = img_off<NC>(ks * 16 + 4 * (g >> 1) + tq + 8 * hi, dt * 4 + 2 * (g & 1) + (tp >> 1)) +
                          8 * (tp & 1);
  auto trofs = [&](int ks, int dt, int hi) {
    return TRADD ? tro[0][dt][hi] + ks * 16 * NC * 16 : tro[ks][dt][hi];
  };

  int qstart = 0;
  if (CAUSAL) qstart = max(0, kb0 - off) / BMQ * BMQ;
  const int nqt_head = qstart < p.Sq ? (p.Sq - qstart + BMQ - 1) / BMQ : 0;
  const int total = nqt_head * grp;

  // Q / dO tiles are prefetched by inline-asm LDS-DMA (RowStagePlan), retired by the explicit wait_vmcnt<0>() ahead
  // of the end-of-tile barrier: with the compiler-visible builtin, hipcc drained the whole prefetch (vmcnt(0))
  // before the transposed reads of the CURRENT tile.  The lse / delta row scalars are loaded raw and only scaled
  // when written to LDS at the end of the tile, so their loads are not waited for (and, vmcnt retiring in order,
  // the DMA behind them with it) at the top of the tile either.
  RowStagePlan<NC, BMQ, NT> qplan;
  qplan.init();
  const unsigned lds_q = lds_addr(Qbuf + wid * 64 * 16);
  float st_lse = 0.f, st_del = 0.f;
  unsigned st_rk = 0u;
  const unsigned dthr = DROP ? attn_drop_thr(p.drop_p) : 0u;
  const float drs = DROP ? 1.f / (1.f - p.drop_p) : 1.f;
  auto stage = [&](int it, int buf) {
    const int hq = hk * grp + it / nqt_head;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
    const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
    const unsigned ql = lds_q + buf * 2 * QIMG;
    qplan.stage(ql, qp, p.q_ss, qt0, p.Sq);
    qplan.stage(ql + QIMG, dop, P.do_ss, qt0, p.Sq);
    if (threadIdx.x < BMQ) {
      const int q = min(qt0 + (int)threadIdx.x, p.Sq - 1);   // rows past Sq: finite, masked by the caller
      const int64_t idx = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      st_lse = p.lse[idx];
      st_del = P.delta[idx];
      if constexpr (DROP) st_rk = attn_row_key(p.drop_seed, (unsigned)(b * p.Hq + hq), (unsigned)(qt0 + threadIdx.x));
    }
  };
  // Row constants: without dropout they become the INITIAL accumulators of the S and dP chains (S' = Q K^T - lse/scale,
  // dP' = dO V^T - delta), so p = exp2(S' scale log2e) and dS = p dP' need no per-element row reads after the chains
  // (cdna_hip_programming.md 'Row constants as the initial accumulator'); dropout keeps the explicit form.
  const float inv_scale = 1.f / p.scale;
  auto stage_scalars = [&](int buf) {
    if (threadIdx.x < BMQ) {
      if constexpr (!RINIT) {
        lse_s[buf * BMQ + threadIdx.x] = -st_lse * 1.4426950408889634f;  // -lse in log2 units
        del_s[buf * BMQ + threadIdx.x] = st_del;
        if constexpr (DROP) rk_s[buf * BMQ + threadIdx.x] = st_rk;
      } else {
        lse_s[buf * BMQ + threadIdx.x] = -st_lse * inv_scale;
        del_s[buf * BMQ + threadIdx.x] = -st_del;
      }
    }
  };
  // accumulator register r holds query row acc_row(r, h) = (r & 3) + 8 (r >> 2) + 4 h: four 16-B row reads
  auto row_init = [&](const float* rows) {
    f32x16 a;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(rows + 8 * j + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[4 * j + i] = v[i];
    }
    return a;
  };

  if (total > 0) {
    stage(0, 0);
    stage_scalars(0);
  }
  wait_vmcnt<0>();
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    if (it + 1 < total) stage(it + 1, buf ^ 1);
    const char* Ql = Qbuf + buf * 2 * QIMG;
    const char* Ol = Ql + QIMG;
    // a wave whose 32 keys are all hidden from this query tile by the causal mask skips the tile
    if (!(CAUSAL && key0 > qt0 + BMQ - 1 + off)) {
      const float* ls = lse_s + buf * BMQ;
      const float* ds = del_s + buf * BMQ;
      __builtin_amdgcn_s_setprio(1);
      f32x16 s = mfma32(lds_b128(Ql, qro[0]), lds_b128(Kimg, kofs(0)), RINIT ? row_init(ls) : zacc);
      f32x16 dp = mfma32(lds_b128(Ol, qro[0]), vf[0], RINIT ? row_init(ds) : zacc);
#pragma unroll
      for (int kk = 1; kk < KS; ++kk) {
        s = mfma32(lds_b128(Ql, qro[kk]), lds_b128(Kimg, kofs(kk)), s);
        dp = mfma32(lds_b128(Ol, qro[kk]), vf[kk], dp);
      }
      __builtin_amdgcn_s_setprio(0);
      // wave-uniform: only diagonal / ragged tiles pay for the selects (masked scores -> -inf -> P = 0)
      if ((qt0 + BMQ > p.Sq) || (key0 + 32 > p.Sk) || (CAUSAL && key0 + 31 > qt0 + off)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = qt0 + acc_row(r, h);
          s[r] = (q >= p.Sq || mykey >= p.Sk || (CAUSAL && mykey > q + off)) ? -INFINITY : s[r];
        }
      }
      // TRPIPE: the first dV / dK step's transposed operands are read now, their latency covered by the softmax
      bf16x8 tro_o[2], tro_q[2];
      if constexpr (TRPIPE) {
        tro_o[0] = lds_tr2(Ol, trofs(0, 0, 0), trofs(0, 0, 1));
        tro_q[0] = lds_tr2(Ql, trofs(0, 0, 0), trofs(0, 0, 1));
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if constexpr (RINIT) {
          const float pv = exp2_(s[r] * sl2);
          s[r] = pv;
          dp[r] = pv * dp[r];
        } else if constexpr (DROP) {   // dV from the dropped, rescaled P; dS = P (Z dP / (1-p) - delta)
          const int qr = acc_row(r, h);
          const float pv = exp2_(fmaf(s[r], sl2, ls[qr]));
          const bool keep = attn_keep(rk_s[buf * BMQ + qr], (unsigned)mykey, dthr);
          s[r] = keep ? pv * drs : 0.f;
          dp[r] = pv * ((keep ? dp[r] * drs : 0.f) - ds[qr]);
        } else {
          const int qr = acc_row(r, h);
          const float pv = exp2_(fmaf(s[r], sl2, ls[qr]));
          s[r] = pv;
          dp[r] = pv * (dp[r] - ds[qr]);
        }
      }
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[ks][j] = (bf16)s[8 * ks + j];
          sb[ks][j] = (bf16)dp[8 * ks + j];
        }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (TRPIPE) {
        // step i = (ks, dt): its operands were read one step earlier; each step issues the next step's 4 reads
        // ahead of its own 2 MFMAs
#pragma unroll
        for (int i = 0; i < 2 * DT; ++i) {
          const int ks = i / DT, dt = i % DT;
          if (i + 1 < 2 * DT) {
            const int k2 = (i + 1) / DT, d2 = (i + 1) % DT;
            tro_o[(i + 1) & 1] = lds_tr2(Ol, trofs(k2, d2, 0), trofs(k2, d2, 1));
            tro_q[(i + 1) & 1] = lds_tr2(Ql, trofs(k2, d2, 0), trofs(k2, d2, 1));
          }
          dv[dt] = mfma32(tro_o[i & 1], pb[ks], dv[dt]);
          dk[dt] = mfma32(tro_q[i & 1], sb[ks], dk[dt]);
          if (i + 1 < 2 * DT) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int o0 = trofs(ks, dt, 0), o1 = trofs(ks, dt, 1);
            dv[dt] = mfma32(lds_tr2(Ol, o0, o1), pb[ks], dv[dt]);
            dk[dt] = mfma32(lds_tr2(Ql, o0, o1), sb[ks], dk[dt]);
          }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (it + 1 < total) stage_scalars(buf ^ 1);
    wait_vmcnt<0>();
    __syncthreads();
  }

  {   // dK then dV through this wave's LDS slab (the K and Q / dO images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= KIMG + 4 * QIMG, "epilogue slabs exceed the dK/dV kernel's LDS");
    const int nvalid = min(32, p.Sk - key0);
    bf16* dk0 = (bf16*)P.dk + (int64_t)b * P.dk_sb + (int64_t)key0 * P.dk_ss + (int64_t)hk * P.dk_sh;
    bf16* dv0 = (bf16*)P.dv + (int64_t)b * P.dv_sb + (int64_t)key0 * P.dv_ss + (int64_t)hk * P.dv_sh;
    char* slab = smem + wid * (32 * HD * 2);
    store_rows_lds<DT>(slab, dk0, P.dk_ss, nvalid, dk, p.scale, h, l32, mykey, P.rope_cos, P.rope_sin, P.rope_off);
    store_rows_lds<DT>(slab, dv0, P.dv_ss, nvalid, dv, 1.f, h, l32, mykey, nullptr, nullptr, 0);
  }
}

// ---- dQ: Q-stationary, the forward's structure.  One workgroup = 4 waves = 128 queries; a lane owns one
// query (lane & 31).  Per 64-key tile: S^T = K Q^T and dP^T = V dO^T (A = K / V rows from LDS, B = Q^T / dO^T
// fragments in registers), P^T = exp2(S^T c - lse) and dS^T = P^T (dP^T - delta) lane-locally (lse and delta
// are one scalar per lane), then dQ^T += K^T dS^T with dS^T consumed straight from the accumulator.
// K / V fragments are read a quarter sub-tile ahead of their MFMAs (KQ = 4: no register spills; the half-sub-tile form
// spilled 3 registers).  Rejected A/B variants (profiles/r4/attn_dq/, attn_prio/): the dQ product's transposed K reads
// software-pipelined one MFMA ahead, and issue priority over the MFMA chains.
template <int HD, bool CAUSAL, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_k(AttnBwdParams P) {
  constexpr int NW = 4, KQ = 4;
  constexpr bool PF = false, PRIO = false;
  using Plan = KVTilePlan<HD, 64 * NW>;
  constexpr int BM = 32 * NW, BN = Plan::BN, KS = Plan::KS, DT = Plan::DT, TILE = Plan::TILE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (p.Sq + BM - 1) / BM;
  int bx, hq, b;
  xcd_block(nqb, p.Hq, bx, hq, b, nqb * p.Hq * p.B);
  const int qb = CAUSAL ? nqb - 1 - bx : bx;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qb * BM, q0w = q0 + wid * 32;
  const int myq = q0w + l32;
  const int off = p.Sk - p.Sq;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  bf16x8 qf[KS], df[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const bool ok = myq < p.Sq;
    qf[kk] = ok ? *reinterpret_cast<const bf16x8*>(qp + (int64_t)myq * p.q_ss + kk * 16 + 8 * h) : zero8();
    df[kk] = ok ? *reinterpret_cast<const bf16x8*>(dop + (int64_t)myq * P.do_ss + kk * 16 + 8 * h) : zero8();
  }
  // delta = rowsum(dO * O) of this lane's query, formed here from the dO fragments already in registers plus the same
  // slice of O (the two half-waves hold complementary halves of the row), and written out for the dK/dV kernel, which
  // runs after this one: no separate delta pass over dO and O
  float nlse2 = 0.f, delta = 0.f;  // -lse in log2 units
  {
    const bf16* opp = (const bf16*)p.o + (int64_t)b * p.o_sb + (int64_t)hq * p.o_sh;
    float part = 0.f;
    if (myq < p.Sq) {
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(opp + (int64_t)myq * p.o_ss + kk * 16 + 8 * h);
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)df[kk][j] * (float)ov[j];
      }
    }
    delta = half_sum(part);
    if (myq < p.Sq) {
      const int64_t idx = ((int64_t)b * p.Hq + hq) * p.Sq + myq;
      nlse2 = -p.lse[idx] * 1.4426950408889634f;
      if (h == 0) P.delta[idx] = delta;
    }
  }

  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + off);
  const int ntiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;
  const int wtiles = wave_tile_count<CAUSAL>(ntiles, q0w, off);
  const unsigned drk = DROP ? attn_row_key(p.drop_seed, (unsigned)(b * p.Hq + hq), (unsigned)myq) : 0u;
  const unsigned dthr = DROP ? attn_drop_thr(p.drop_p) : 0u;
  const float drs = DROP ? 1.f / (1.f - p.drop_p) : 1.f;

  Plan plan;
  plan.init(lane, p.k_ss);
  plan.init_async();
  const unsigned lds_w = lds_addr(smem + (threadIdx.x >> 6) * 64 * 16);

  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;
  const f32x16 zacc = {};

  if (ntiles > 0) plan.template stage_async<true>(lds_w, kp, vp, p.k_ss, p.v_ss, 0, p.Sk);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  auto tile = [&](const char* Kl, const char* Vl, int k0, bool need_mask) {
    bf16x8 sf[4];
    bf16x8 tk[2];   // PF: ring of transposed K operands, step i = (ks, dt) = (i / DT, i % DT)
    auto tk_read = [&](int i) { return lds_tr2(Kl, plan.tr(i / DT, i % DT, 0), plan.tr(i / DT, i % DT, 1)); };
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      // K and V fragments are read a half sub-tile (KH k-steps) ahead of their MFMAs with counted lgkmcnt waits
      // (one read + wait + multiply at a time exposed an LDS round trip per MFMA; all KS at once spills)
      constexpr int NQ = KS >= KQ ? KQ : KS, KH = KS / NQ;
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      f32x16 s = zacc, dp = zacc;
#pragma unroll
      for (int half = 0; half < NQ; ++half) {
        bf16x8 kf[KH], vf[KH];
#pragma unroll
        for (int j = 0; j < KH; ++j) {
          kf[j] = lds_b128(Kl, plan.row(sub, half * KH + j));
          vf[j] = lds_b128(Vl, plan.row(sub, half * KH + j));
        }
#pragma unroll
        for (int j = 0; j < KH; ++j) {
          s = mfma32(kf[j], qf[half * KH + j], s);
          dp = mfma32(vf[j], df[half * KH + j], dp);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * KH, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * KH, 0);
      }
      if constexpr (PF) {
        if (sub == 1) {
          tk[0] = tk_read(0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      if (need_mask) {  // wave-uniform; masked scores -> -inf -> p = 0
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + sub * 32 + acc_row(r, h);
          s[r] = (key >= p.Sk || (CAUSAL && key > myq + off)) ? -INFINITY : s[r];
        }
      }
      if constexpr (DROP) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool keep = attn_keep(drk, (unsigned)(k0 + sub * 32 + acc_row(r, h)), dthr);
          s[r] = exp2_(fmaf(s[r], sl2, nlse2)) * ((keep ? dp[r] * drs : 0.f) - delta);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = exp2_(fmaf(s[r], sl2, nlse2)) * (dp[r] - delta);
      }
#pragma unroll
      for (int half = 0; half < 2; ++half)
#pragma unroll
        for (int j = 0; j < 8; ++j) sf[sub * 2 + half][j] = (bf16)s[8 * half + j];
      __builtin_amdgcn_sched_barrier(0);
    }
    // dQ^T += K^T dS^T
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < 4 * DT; ++i) {
        if (i + 1 < 4 * DT) tk[(i + 1) & 1] = tk_read(i + 1);
        dq[i % DT] = mfma32(tk[i & 1], sf[i / DT], dq[i % DT]);
        if (i + 1 < 4 * DT) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          dq[dt] = mfma32(lds_tr2(Kl, plan.tr(ks, dt, 0), plan.tr(ks, dt, 1)), sf[ks], dq[dt]);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles)
      plan.template stage_async<true>(lds_w + (buf ^ 1) * 2 * TILE, kp, vp, p.k_ss, p.v_ss, (t + 1) * BN, p.Sk);
    const char* Kl = smem + buf * 2 * TILE;
    if (t < wtiles) {
      const int k0 = t * BN;
      tile(Kl, Kl + TILE, k0, (k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0w + off)));
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  }

  {   // dQ through this wave's LDS slab (the K / V images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= 4 * TILE, "epilogue slabs exceed the dQ kernel's LDS");
    bf16* dq0 = (bf16*)P.dq + (int64_t)b * P.dq_sb + (int64_t)q0w * P.dq_ss + (int64_t)hq * P.dq_sh;
    store_rows_lds<DT>(smem + wid * (32 * HD * 2), dq0, P.dq_ss, min(32, p.Sq - q0w), dq, p.scale, h, l32, myq,
                       P.rope_cos, P.rope_sin, P.rope_off);
  }
}

// ---- dK / dV on v_mfma_f32_16x16x32_bf16 (head dim 128, no dropout): the KV-stationary structure above with every
// product a set of 16x16 tiles.  A wave owns 32 keys = two 16-key column blocks kb; per 32-query tile:
//   S[qb][kb]  = Q K^T   A = Q rows (x16 image, b128), B = K^T (K image rows, b128)        16 MFMAs
//   dP[qb][kb] = dO V^T  A = dO rows,                  B = V^T (registers, loaded once)     16 MFMAs
//   dV^T[db][kb] += dO^T P,  dK^T[db][kb] += Q^T dS:  A = x16_tr (transposed image reads), B = the S / dP accumulator
//   pair of the key block (acc_pair_b: no lane movement)                                   32 MFMAs
// The key is on the lane of S / dP (col = lane & 15), so P and dS are B operands as they stand.  LDS traffic per MFMA
// FLOP is that of the 32x32x16 kernel; the x16 image makes every read conflict-free.
// OPT bits (measured, profiles/r6/attn16/README.md): bit 0 = -delta as the dP chain's initial accumulator, bit 1 = one
// tile-body instance per image buffer (immediate LDS offsets), bit 2 = no compiler fence in the mask branch.  Per-kernel
// times under --kernel-trace on one box, dK/dV + dQ per call: OPT 0 2.32 + 1.65 ms, 4 2.29 + 1.63, 3 2.19 + 1.60,
// 7 2.20 + 1.60; the round-5 32x32x16 kernels 2.23 + 1.65.  Default 3.
template <bool CAUSAL, int OPT = 3>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv16_k(AttnBwdParams P) {
  constexpr bool RINIT = OPT & 1, UNROLL = OPT & 2;
  constexpr int HD = 128, NW = 4, NT = 64 * NW, BNK = 32 * NW, BMQ = 32;
  constexpr int QIMG = BMQ * HD * 2;        // Q / dO tile image [32 q][128]
  constexpr int KIMG = BNK * HD * 2;        // K image [128 keys][128]
  // smem: K | Q0 | dO0 | Q1 | dO1 | -lse2[2][32] | delta[2][32]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kimg = smem;
  char* Qbuf = smem + KIMG;
  float* lse_s = reinterpret_cast<float*>(Qbuf + 4 * QIMG);
  float* del_s = lse_s + 2 * BMQ;

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int nkb = (p.Sk + BNK - 1) / BNK;
  int kbx, hk, b;
  xcd_block(nkb, p.Hkv, kbx, hk, b, nkb * p.Hkv * p.B);
  const int kb0 = kbx * BNK;   // ascending = heaviest causal key blocks first
  const int grp = p.Hq / p.Hkv;
  const int off = p.Sk - p.Sq;
  const int key0 = kb0 + wid * 32;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;
  {
    X16Stage<BNK, NT> kst;
    kst.init(p.k_ss);
    kst.stage(lds_addr(Kimg + wid * 1024), kp, p.k_ss, kb0, p.Sk);
  }
  // V^T B fragments of dP = dO V^T: lane (key i, g) holds V[key][32 kk + 8 g .. + 7]
  bf16x8 vf[2][4];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = key0 + kb * 16 + i16;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      vf[kb][kk] = key < p.Sk ? *reinterpret_cast<const bf16x8*>(vp + (int64_t)key * p.v_ss + kk * 32 + 8 * g)
                              : zero8();
  }
  f32x4 dk[8][2], dv[8][2];
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) { dk[db][kb][r] = 0.f; dv[db][kb][r] = 0.f; }
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  X16Reads rd;
  rd.init(lane, lds_addr(smem));
  // image bases relative to smem (immediates in every read): K | Q0 | dO0 | Q1 | dO1
  const unsigned kro = (wid * 32) << 8;   // this wave's K rows

  int qstart = 0;
  if (CAUSAL) qstart = max(0, kb0 - off) / BMQ * BMQ;
  const int nqt_head = qstart < p.Sq ? (p.Sq - qstart + BMQ - 1) / BMQ : 0;
  const int total = nqt_head * grp;

  X16Stage<BMQ, NT> qst, ost;   // one plan per row stride (Q is often a view of the packed QKV projection, dO is not)
  qst.init(p.q_ss);
  ost.init(P.do_ss);
  const unsigned lds_q = lds_addr(Qbuf + wid * 1024);
  float st_lse = 0.f, st_del = 0.f;
  auto stage = [&](int it, int buf) {
    const int hq = hk * grp + it / nqt_head;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
    const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
    const unsigned ql = lds_q + buf * 2 * QIMG;
    qst.stage(ql, qp, p.q_ss, qt0, p.Sq);
    ost.stage(ql + QIMG, dop, P.do_ss, qt0, p.Sq);
    if (threadIdx.x < BMQ) {
      const int q = min(qt0 + (int)threadIdx.x, p.Sq - 1);   // rows past Sq: finite, masked below
      const int64_t idx = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      st_lse = p.lse[idx];
      st_del = P.delta[idx];
    }
  };
  auto stage_scalars = [&](int buf) {
    if (threadIdx.x < BMQ) {
      lse_s[buf * BMQ + threadIdx.x] = -st_lse * 1.4426950408889634f;  // -lse in log2 units
      del_s[buf * BMQ + threadIdx.x] = RINIT ? -st_del : st_del;   // -delta: the dP chain's initial accumulator
    }
  };

  if (total > 0) {
    stage(0, 0);
    stage_scalars(0);
  }
  wait_vmcnt<0>();
  __syncthreads();

  // The tile body is instantiated once per image buffer (even / odd tiles), so every LDS address is a per-lane offset
  // plus an immediate: no per-read address arithmetic on the vector ALU, which this body is bound by.
  auto tile = [&](auto BUFC, int it) {
    const int buf = BUFC;
    const int qt0 = qstart + (it % nqt_head) * BMQ;
    if (it + 1 < total) stage(it + 1, buf ^ 1);
    const unsigned QL = KIMG + buf * 2 * QIMG, OL = QL + QIMG;
    if (!(CAUSAL && key0 > qt0 + BMQ - 1 + off)) {   // some of this wave's keys are visible to the tile
      const float* ls = lse_s + buf * BMQ;
      const float* ds = del_s + buf * BMQ;
      // row constants: -delta is the dP chain's initial accumulator (dS = P dP' needs no subtraction afterwards)
      f32x4 nl[2], ndl[2], s[2][2], dp[2][2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        nl[qb] = *reinterpret_cast<const f32x4*>(ls + qb * 16 + 4 * g);
        const f32x4 nd = *reinterpret_cast<const f32x4*>(ds + qb * 16 + 4 * g);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) { s[qb][kb] = z4; dp[qb][kb] = RINIT ? nd : z4; }
        ndl[qb] = nd;
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const unsigned ka = rd.row[kk] + kro;
        const bf16x8 k0f = ldsa_b128(ka), k1f = ldsa_b128(ka + 4096);
        const bf16x8 q0f = ldsa_b128(rd.row[kk] + QL), q1f = ldsa_b128(rd.row[kk] + QL + 4096);
        const bf16x8 o0f = ldsa_b128(rd.row[kk] + OL), o1f = ldsa_b128(rd.row[kk] + OL + 4096);
        s[0][0] = mfma16(q0f, k0f, s[0][0]);
        s[0][1] = mfma16(q0f, k1f, s[0][1]);
        s[1][0] = mfma16(q1f, k0f, s[1][0]);
        s[1][1] = mfma16(q1f, k1f, s[1][1]);
        dp[0][0] = mfma16(o0f, vf[0][kk], dp[0][0]);
        dp[0][1] = mfma16(o0f, vf[1][kk], dp[0][1]);
        dp[1][0] = mfma16(o1f, vf[0][kk], dp[1][0]);
        dp[1][1] = mfma16(o1f, vf[1][kk], dp[1][1]);
      }
      __builtin_amdgcn_s_setprio(0);
      // wave-uniform: only diagonal / ragged tiles pay for the selects (masked scores -> -inf -> P = 0); the empty asm
      // keeps the compiler from if-converting the block into selects that every tile would execute
      if ((qt0 + BMQ > p.Sq) || (key0 + 32 > p.Sk) || (CAUSAL && key0 + 31 > qt0 + off)) {
        if constexpr (!(OPT & 4)) asm volatile("" ::: "memory");
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int q = qt0 + qb * 16 + 4 * g + r, key = key0 + kb * 16 + i16;
              s[qb][kb][r] = (q >= p.Sq || key >= p.Sk || (CAUSAL && key > q + off)) ? -INFINITY : s[qb][kb][r];
            }
      }
      // the first dV / dK step's transposed operands are read now, their latency covered by the softmax
      bf16x8 tro_o[2], tro_q[2];
      tro_o[0] = ldsa_tr(rd.tr[0] + OL);
      tro_q[0] = ldsa_tr(rd.tr[0] + QL);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pv = exp2_(fmaf(s[qb][kb][r], sl2, nl[qb][r]));
            s[qb][kb][r] = pv;
            dp[qb][kb][r] = RINIT ? pv * dp[qb][kb][r] : pv * (dp[qb][kb][r] - ndl[qb][r]);
          }
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        pb[kb] = acc_pair_b(s[0][kb], s[1][kb]);
        sb[kb] = acc_pair_b(dp[0][kb], dp[1][kb]);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      // step db: its operands were read one step earlier; each step issues the next step's 4 reads ahead of its MFMAs
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        if (db + 1 < 8) {
          tro_o[(db + 1) & 1] = ldsa_tr(rd.tr[db + 1] + OL);
          tro_q[(db + 1) & 1] = ldsa_tr(rd.tr[db + 1] + QL);
        }
        dv[db][0] = mfma16(tro_o[db & 1], pb[0], dv[db][0]);
        dv[db][1] = mfma16(tro_o[db & 1], pb[1], dv[db][1]);
        dk[db][0] = mfma16(tro_q[db & 1], sb[0], dk[db][0]);
        dk[db][1] = mfma16(tro_q[db & 1], sb[1], dk[db][1]);
        if (db + 1 < 8) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (it + 1 < total) stage_scalars(buf ^ 1);
    wait_vmcnt<0>();
    __syncthreads();
  };
  if constexpr (UNROLL) {
    for (int it = 0; it < total; it += 2) {
      tile(std::integral_constant<int, 0>{}, it);
      if (it + 1 < total) tile(std::integral_constant<int, 1>{}, it + 1);
    }
  } else {
    for (int it = 0; it < total; ++it) tile(it & 1, it);
  }

  {   // dK then dV through this wave's 8-KiB LDS slab (the images are free after the loop's last barrier)
    static_assert(NW * 32 * HD * 2 <= KIMG + 4 * QIMG, "epilogue slabs exceed the dK/dV kernel's LDS");
    const int nvalid = min(32, p.Sk - key0);
    bf16* dk0 = (bf16*)P.dk + (int64_t)b * P.dk_sb + (int64_t)key0 * P.dk_ss + (int64_t)hk * P.dk_sh;
    bf16* dv0 = (bf16*)P.dv + (int64_t)b * P.dv_sb + (int64_t)key0 * P.dv_ss + (int64_t)hk * P.dv_sh;
    char* slab = smem + wid * (32 * HD * 2);
    store_rows16(slab, dk0, P.dk_ss, nvalid, dk, p.scale, lane, key0, P.rope_cos, P.rope_sin, P.rope_off);
    store_rows16(slab, dv0, P.dv_ss, nvalid, dv, 1.f, lane, key0, nullptr, nullptr, 0);
  }
}

// ---- dQ on v_mfma_f32_16x16x32_bf16 (head dim 128, no dropout): the Q-stationary structure above as 16x16 tiles.
// A wave owns 32 queries = two 16-query column blocks qb (Q^T / dO^T B fragments in registers); per 64-key tile, in
// two 32-key halves h (register budget: one half's S^T / dP^T accumulators live at a time):
//   S^T[kb][qb] = K Q^T, dP^T[kb][qb] = V dO^T   A = K / V rows (x16 images, b128)          2 x 16 MFMAs
//   dS^T = P^T (dP^T - delta), P^T = exp2(S^T c - lse): the query is on the lane, row constants are lane scalars
//   dQ^T[db][qb] += K^T dS^T                       A = x16_tr(K image), B = the half's dS^T pair   16 MFMAs
// and it forms delta = rowsum(dO * O) for its queries first (written for the dK/dV kernel, which runs after it).
template <bool CAUSAL, int OPT = 3>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq16_k(AttnBwdParams P) {
  constexpr bool RINIT = OPT & 1, UNROLL = OPT & 2;
  constexpr int HD = 128, NW = 4, NT = 64 * NW, BM = 32 * NW, BN = 64;
  constexpr int TILE = BN * HD * 2;   // one 64-row x16 image (16 KiB); buffer = K | V
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const AttnParams& p = P.f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
  const int nqb = (p.Sq + BM - 1) / BM;
  int bx, hq, b;
  xcd_block(nqb, p.Hq, bx, hq, b, nqb * p.Hq * p.B);
  const int qblk = CAUSAL ? nqb - 1 - bx : bx;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q0 = qblk * BM, q0w = q0 + wid * 32;
  const int off = p.Sk - p.Sq;
  const float sl2 = p.scale * 1.4426950408889634f;

  const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_sb + (int64_t)hq * p.q_sh;
  const bf16* dop = (const bf16*)P.dout + (int64_t)b * P.do_sb + (int64_t)hq * P.do_sh;
  const bf16* opp = (const bf16*)p.o + (int64_t)b * p.o_sb + (int64_t)hq * p.o_sh;
  const bf16* kp = (const bf16*)p.k + (int64_t)b * p.k_sb + (int64_t)hk * p.k_sh;
  const bf16* vp = (const bf16*)p.v + (int64_t)b * p.v_sb + (int64_t)hk * p.v_sh;

  // Q^T / dO^T B fragments: lane (query i, g) holds row q0w + 16 qb + i, columns 32 kk + 8 g .. + 7
  bf16x8 qf[2][4], df[2][4];
  float nlse2[2], delta[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = q0w + qb * 16 + i16;
    const bool ok = q < p.Sq;
    float part = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int64_t c = kk * 32 + 8 * g;
      qf[qb][kk] = ok ? *reinterpret_cast<const bf16x8*>(qp + (int64_t)q * p.q_ss + c) : zero8();
      df[qb][kk] = ok ? *reinterpret_cast<const bf16x8*>(dop + (int64_t)q * P.do_ss + c) : zero8();
      if (ok) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(opp + (int64_t)q * p.o_ss + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)df[qb][kk][j] * (float)ov[j];
      }
    }
    // the four lane groups hold complementary column slices of the row
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    delta[qb] = part;
    nlse2[qb] = 0.f;
    if (ok) {
      const int64_t idx = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      nlse2[qb] = -p.lse[idx] * 1.4426950408889634f;
      if (g == 0) P.delta[idx] = part;
    }
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

  f32x4 dq[8][2];
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int r = 0; r < 4; ++r) dq[db][qb][r] = 0.f;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  if (ntiles > 0) {
    st.stage(lds_w, kp, p.k_ss, 0, p.Sk);
    st.stage(lds_w + TILE, vp, p.v_ss, 0, p.Sk);
  }
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  // one instantiation of the tile body per image buffer: every LDS read is a per-lane address plus an immediate
  f32x4 nd[2];   // -delta of this lane's queries: the dP^T chain's initial accumulator (dS^T = P^T dP^T')
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int r = 0; r < 4; ++r) nd[qb][r] = -delta[qb];
  auto tile = [&](auto BUFC, int t) {
    const int buf = BUFC;
    const unsigned KL = buf * 2 * TILE, VL = KL + TILE;
    if (t + 1 < ntiles) {
      const unsigned nb = lds_w + (buf ^ 1) * 2 * TILE;
      st.stage(nb, kp, p.k_ss, (t + 1) * BN, p.Sk);
      st.stage(nb + TILE, vp, p.v_ss, (t + 1) * BN, p.Sk);
    }
    if (t < wtiles) {
      const int k0 = t * BN;
      const bool need_mask = (k0 + BN > p.Sk) || (CAUSAL && (k0 + BN - 1 > q0w + off));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const unsigned R0 = (unsigned)(h * 32) << 8;
        f32x4 sa[2][2], pa[2][2];   // [kb within the half][qb]
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) { sa[a][qb] = z4; pa[a][qb] = RINIT ? nd[qb] : z4; }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const bf16x8 k0f = ldsa_b128(rd.row[kk] + KL + R0), k1f = ldsa_b128(rd.row[kk] + KL + R0 + 4096);
          const bf16x8 v0f = ldsa_b128(rd.row[kk] + VL + R0), v1f = ldsa_b128(rd.row[kk] + VL + R0 + 4096);
          sa[0][0] = mfma16(k0f, qf[0][kk], sa[0][0]);
          sa[0][1] = mfma16(k0f, qf[1][kk], sa[0][1]);
          sa[1][0] = mfma16(k1f, qf[0][kk], sa[1][0]);
          sa[1][1] = mfma16(k1f, qf[1][kk], sa[1][1]);
          pa[0][0] = mfma16(v0f, df[0][kk], pa[0][0]);
          pa[0][1] = mfma16(v0f, df[1][kk], pa[0][1]);
          pa[1][0] = mfma16(v1f, df[0][kk], pa[1][0]);
          pa[1][1] = mfma16(v1f, df[1][kk], pa[1][1]);
        }
        // wave-uniform; masked scores -> -inf -> p = 0.  The empty asm keeps hipcc from if-converting the block into
        // selects that every tile would execute.
        if (need_mask) {
          if constexpr (!(OPT & 4)) asm volatile("" ::: "memory");
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int key = k0 + h * 32 + a * 16 + 4 * g + r, q = q0w + qb * 16 + i16;
                sa[a][qb][r] = (key >= p.Sk || (CAUSAL && key > q + off)) ? -INFINITY : sa[a][qb][r];
              }
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              sa[a][qb][r] = exp2_(fmaf(sa[a][qb][r], sl2, nlse2[qb])) * (RINIT ? pa[a][qb][r] : pa[a][qb][r] - delta[qb]);
        bf16x8 dsb[2];
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) dsb[qb] = acc_pair_b(sa[0][qb], sa[1][qb]);
        __builtin_amdgcn_sched_barrier(0);
        // dQ^T += K^T dS^T over this half's 32 keys
#pragma unroll
        for (int db = 0; db < 8; ++db) {
          const bf16x8 kt = ldsa_tr(rd.tr[db] + KL + R0);
          dq[db][0] = mfma16(kt, dsb[0], dq[db][0]);
          dq[db][1] = mfma16(kt, dsb[1], dq[db][1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  };
  if constexpr (UNROLL) {
    for (int t = 0; t < ntiles; t += 2) {
      tile(std::integral_constant<int, 0>{}, t);
      if (t + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t + 1);
    }
  } else {
    for (int t = 0; t < ntiles; ++t) tile(t & 1, t);
  }

  {   // dQ through this wave's 8-KiB LDS slab (the K / V images are free after the loop's last barrier)
    bf16* dq0 = (bf16*)P.dq + (int64_t)b * P.dq_sb + (int64_t)q0w * P.dq_ss + (int64_t)hq * P.dq_sh;
    store_rows16(smem + wid * (32 * HD * 2), dq0, P.dq_ss, min(32, p.Sq - q0w), dq, p.scale, lane, q0w,
                 P.rope_cos, P.rope_sin, P.rope_off);
  }
}

// Which flash-attention kernels run for head dim 128 (process-wide, set by the attn_variant op; not read from the
// environment): 0 (default) = the 32x32x16 kernels, 2 = the 16x16x32 kernels (attn_fwd16_k / attn_bwd_dq16_k /
// attn_bwd_dkdv16_k).  In isolation the 16x16x32 forms are 1-4 % faster (they hold a 6-11 % higher clock), but in
// the 7B training step, where the package power limit sets the clock for every kernel, they lose that clock and keep
// their lower MFMA busy share: 28 650 / 28 507 / 28 706 vs 28 756 / 28 757 / 28 782 tokens/s interleaved on one box,
// 28 845 / 28 755 vs 29 150 / 29 079 on another (profiles/r6/attn16/README.md).  So the 32x32x16 kernels stay the
// default.
static int g_attn_variant = 0;
int attn_set_variant(int v) {
  const int old = g_attn_variant;
  g_attn_variant = v;
  return old;
}
int attn_get_variant() { return g_attn_variant; }

template <int HD, bool DROP>
static void bwd_launch_t(const AttnBwdParams& P, hipStream_t st) {
  const AttnParams& p = P.f;
  // dQ first: it forms delta = rowsum(dO * O) for its rows and writes it for the dK/dV kernel
  const size_t lds_q = 2 * 2 * 64 * HD * 2;
  const dim3 grid_q((unsigned)((p.Sq + 127) / 128 * p.Hq * p.B));
  if (HD == 128 && !DROP && g_attn_variant == 2) {
    if (p.causal) hipLaunchKernelGGL((attn_bwd_dq16_k<true>), grid_q, dim3(256), lds_q, st, P);
    else hipLaunchKernelGGL((attn_bwd_dq16_k<false>), grid_q, dim3(256), lds_q, st, P);
  } else if (p.causal) hipLaunchKernelGGL((attn_bwd_dq_k<HD, true, DROP>), grid_q, dim3(256), lds_q, st, P);
  else hipLaunchKernelGGL((attn_bwd_dq_k<HD, false, DROP>), grid_q, dim3(256), lds_q, st, P);
  const size_t lds_kv = 128 * HD * 2 + 4 * 32 * HD * 2 + 6 * 32 * 4;
  const dim3 grid_kv((unsigned)((p.Sk + 127) / 128 * p.Hkv * p.B));
  if (HD == 128 && !DROP && g_attn_variant == 2) {
    if (p.causal) hipLaunchKernelGGL((attn_bwd_dkdv16_k<true>), grid_kv, dim3(256), lds_kv, st, P);
    else hipLaunchKernelGGL((attn_bwd_dkdv16_k<false>), grid_kv, dim3(256), lds_kv, st, P);
    return;
  }
  if (p.causal) hipLaunchKernelGGL((attn_bwd_dkdv_k<HD, true, DROP>), grid_kv, dim3(256), lds_kv, st, P);
  else hipLaunchKernelGGL((attn_bwd_dkdv_k<HD, false, DROP>), grid_kv, dim3(256), lds_kv, st, P);
}

template <int HD>
static void bwd_launch(const AttnBwdParams& P, hipStream_t st) {
  if (P.f.drop_p > 0.f) bwd_launch_t<HD, true>(P, st);
  else bwd_launch_t<HD, false>(P, st);
}

void flash_attn_bwd(const AttnBwdParams& P, hipStream_t st) {
  const AttnParams& p = P.f;
  if (p.B == 0 || p.Sq == 0) return;
  switch (p.D) {
    case 32: bwd_launch<32>(P, st); break;
    case 64: bwd_launch<64>(P, st); break;
    case 128: bwd_launch<128>(P, st); break;
    default: break;
  }
}

}  // namespace dph
