// Forward / input-gradient GEMM for CDNA4 (gfx950):  C[M, N] = A[M, K] B[N, K]^T, both operands K-contiguous
// (token-major activations x [out, in] weights: y = x W^T; the input gradient dX = dY W runs on the same kernel
// with a transposed weight copy), with fusable epilogues:
//   * STORE   -- plain bf16 C;
//   * SWIGLU  -- the fused w13 projection of the Llama FFN: B = [W1; W3] ([2H, K]); one 256-column tile holds the
//                gate AND up columns of 128 hidden units, so h = silu(gate) * up is formed in registers and the
//                kernel writes x13 = [gate | up] (saved for backward) and h (the next GEMM's input) -- the separate
//                swiglu_fwd pass (read 2H, write H per token) disappears;
//   * DSWIGLU -- the input gradient of w2 (dh = dY W2) followed by the SwiGLU backward: the epilogue reads the
//                saved gate / up values and writes d13 = [dgate | dup] straight away (no dh round trip);
//   * ROPE    -- the fused wqkv projection with the rotary embedding of the q / k columns applied to the fp32
//                accumulators (one rounding instead of GEMM-round + rope-round, no separate rope pass).
//
// Structure (cdna_hip_programming.md §5 "256^2 8-phase template", designed for this layout):
//   * 256 x 256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), wave tile 128 tokens x 64 features,
//     v_mfma_f32_16x16x32_bf16 with the weight rows as the MFMA A operand and the token rows as B, so a lane ends
//     with 4 CONSECUTIVE features of one token (8-byte stores; RoPE pairs and gate/up pairs are lane-local);
//   * K-tiles of 64, staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B / lane, full 128-B rows,
//     XOR-swizzled 16-B chunks: slot = chunk ^ ((row >> 1) & 7), conflict-free ds_read_b128 fragment reads);
//   * each K-tile is four "quarter" images (16 KB each): Q_A0 / Q_A1 = the first / second 64 token rows of every
//     wave row-group, Q_B0 / Q_B1 = the first / second 32 feature rows of every wave column-group.  A K-tile
//     runs as 4 phases, one quadrant of the wave tile each: (A0,B0) (A0,B1) (A1,B1) (A1,B0), so phase 1 reads
//     A0+B0 fragments, phase 2 B1, phase 3 A1, phase 4 nothing;
//   * every phase issues ONE quarter of a future K-tile (Q_B1 / Q_A1 of t+1, Q_A0 / Q_B0 of t+2, each region
//     >= 2 phases after its last read) and waits vmcnt(8): four quarters (64 KB per CU) stay in flight across
//     the barriers and the wait retires exactly what the next phase reads;
//   * the second half of the waves (4..7) runs one barrier behind the first (stagger): on every SIMD one wave
//     issues its MFMAs while its partner reads fragments / issues DMA -- the matrix pipe ping-pongs;
//   * workgroups are remapped XCD-aware and grouped GROUP_M tiles tall (as gemm.hip) for L2 reuse.
// Requirements (host-checked): M % 256, N % 256 (SWIGLU: H % 128), K % 64, leading dims % 8, 16-B aligned bases.
#include <type_traits>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int NBM = 256, NBN = 256, NBK = 64, NNT = 512;
constexpr int QB = 16384;       // one quarter image: 128 rows x 128 B
constexpr int BUFB = 4 * QB;    // one K-tile: Q_A0 | Q_A1 | Q_B0 | Q_B1
constexpr int NGROUP_M = 8;

enum : int { Q_A0 = 0, Q_A1 = 1, Q_B0 = 2, Q_B1 = 3 };

__device__ __forceinline__ void nt_grouped_tile(int lin, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int first_m = lin / (NGROUP_M * tiles_n) * NGROUP_M;
  const int gsz = min(tiles_m - first_m, NGROUP_M);
  const int in_group = lin % (NGROUP_M * tiles_n);
  tm = first_m + in_group % gsz;
  tn = in_group / gsz;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float nt_sigmoid(float x) { return 1.f / (1.f + __expf(-x)); }

// LOOK = 1: phase 1 reads only the A0 fragments; the next K-tile's B0 fragments are read inside phase 4's MFMA
// segment (interleaved with its MFMAs) into the B register set phase 4 does not use, so the four read segments
// carry 8 / 4 / 8 / 0 ds_read_b128 instead of 12 / 4 / 8 / 0.  Reading in an MFMA segment needs the data retired one
// phase earlier under the stagger, so three quarters stay in flight (vmcnt(6)) instead of four.
// LEPI (every mode): the epilogue goes through LDS -- dh / C rounded to bf16 into a 256 x 256 image (16-B chunks
// XOR-swizzled by the row, conflict-free 8-B writes from the accumulators), then whole 16-B row segments: one vector
// load per operand and one store per output (DSWIGLU: x13's gate / up in, d13's dgate / dup out) instead of 8-B
// accesses at 16 rows per instruction.  Same rounding and math as the register epilogue, so bitwise-equal output.
// RAG (LEPI only): ragged N / H and K as in gemm_nt32_k below -- clamped weight rows, a zero-filled partial last K-tile
// by range-checked buffer DMA, epilogue stores masked to whole 8-column segments below N.
template <int MODE, int LOOK, bool LEPI = false, bool RAG = false>
__global__ __launch_bounds__(NNT, 1) void gemm_nt_k(GemmNtParams p) {
  static_assert(!RAG || LEPI, "ragged edges need the LDS epilogue");
  constexpr int VMC = LOOK ? 6 : 8;
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUFB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int r16 = lane & 15, kq = lane >> 4;

  // ---- tile of this workgroup (XCD-aware, grouped) ----
  const int tiles_m = p.M / NBM, tiles_n = p.tiles_n;
  int tm, tn;
  nt_grouped_tile(xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * NBM;
  // first global weight row of Q_B0's / Q_B1's image row 0, and the image-row -> weight-row map:
  //   STORE / DSWIGLU / ROPE: rho -> n0 + 64 (rho >> 5) + (rho & 31) (+ 32 for Q_B1)   (wave wn: 64 rows)
  //   SWIGLU:                 rho -> 128 tn + rho (gate) / H + 128 tn + rho (up)      (wave wn: 32 units)
  int64_t nbase0, nbase1;
  if constexpr (MODE == kNtSwiglu) {
    nbase0 = (int64_t)tn * 128;
    nbase1 = (int64_t)p.H + (int64_t)tn * 128;
  } else {
    nbase0 = (int64_t)tn * NBN;
    nbase1 = nbase0 + 32;
  }

  // ---- per-lane LDS-DMA source offsets (bytes, relative to the quarter's row-0 pointer at k-tile 0) ----
  const int nk = RAG ? (p.K + NBK - 1) / NBK : p.K / NBK;
  unsigned voff[4][2], vtail[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = i * NNT + tid, rho = c >> 3, kc = (c & 7) ^ ((rho >> 1) & 7);
      int64_t row;
      if (q < 2) row = 128 * (rho >> 6) + (rho & 63);            // Q_A1's base pointer carries the +64
      else if (MODE == kNtSwiglu) row = rho;
      else row = 64 * (rho >> 5) + (rho & 31);                    // Q_B1's base pointer carries the +32
      if constexpr (RAG) {   // weight quarters: absolute rows from the operand's base, clamped to the last valid one
        if (q >= 2) {
          const int64_t nb = q == Q_B0 ? nbase0 : nbase1;
          int64_t lim;
          if constexpr (MODE == kNtSwiglu) lim = q == Q_B0 ? p.H : 2 * (int64_t)p.H;
          else lim = p.N;
          row = min(nb + row, lim - 1);
        }
      }
      const int64_t ld = q < 2 ? p.lda : p.ldb;
      voff[q][i] = (unsigned)(row * ld * 2 + kc * 16);
      vtail[q][i] = ((nk - 1) * NBK + kc * 8 < p.K) ? voff[q][i] : 0x80000000u;
    }
  const char* qptr[4];
  const bf16* Ap = reinterpret_cast<const bf16*>(p.A);
  const bf16* Bp = reinterpret_cast<const bf16*>(p.B);
  qptr[Q_A0] = reinterpret_cast<const char*>(Ap + (int64_t)m0 * p.lda);
  qptr[Q_A1] = reinterpret_cast<const char*>(Ap + (int64_t)(m0 + 64) * p.lda);
  qptr[Q_B0] = reinterpret_cast<const char*>(RAG ? Bp : Bp + nbase0 * p.ldb);
  qptr[Q_B1] = reinterpret_cast<const char*>(RAG ? Bp : Bp + nbase1 * p.ldb);
  const unsigned lds_w = lds_addr(lds + wid * 1024);
  const bool ktail = RAG && (p.K % NBK) != 0;

  auto dma = [&](auto QI, int kt, auto BI) {
    constexpr int Q = decltype(QI)::value, BUF = decltype(BI)::value;
    const int ktc = min(kt, nk - 1);   // past the end: re-load the last tile into a slot nobody reads again
    const char* src = qptr[Q] + (int64_t)ktc * (NBK * 2);
    const unsigned d = lds_w + BUF * BUFB + Q * QB;
    if (RAG && ktail && ktc == nk - 1) {   // wave-uniform: the partial last K-tile, zero-filled past K
      const dph_rsrc rs = make_rsrc(src, 0x7fffffffu);
      lds_dma16_buf(rs, vtail[Q][0], d);
      lds_dma16_buf(rs, vtail[Q][1], d + NNT * 16);
    } else {
      lds_dma16(src, voff[Q][0], d);
      lds_dma16(src, voff[Q][1], d + NNT * 16);
    }
  };

  // ---- per-lane fragment read offsets: row r16 of a 16-row block, logical chunk 4 s + kq ----
  const int xsw = (r16 >> 1) & 7;
  const int off_s0 = r16 * 128 + ((kq ^ xsw) << 4);
  const int off_s1 = r16 * 128 + (((4 + kq) ^ xsw) << 4);
  const char* a_img = lds + wm * 8192;    // + Q * QB + buf * BUFB, + mb * 2048
  const char* b_img = lds + wn * 4096;    // + Q * QB + buf * BUFB, + nb * 2048

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read_a = [&](auto QI, auto BI) {
    constexpr int Q = decltype(QI)::value, BUF = decltype(BI)::value;
    const char* base = a_img + BUF * BUFB + Q * QB;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      fa[mb][0] = *reinterpret_cast<const bf16x8*>(base + mb * 2048 + off_s0);
      fa[mb][1] = *reinterpret_cast<const bf16x8*>(base + mb * 2048 + off_s1);
    }
  };
  auto read_b = [&](auto QI, auto BI, bf16x8 (&fb)[2][2]) {
    constexpr int Q = decltype(QI)::value, BUF = decltype(BI)::value;
    const char* base = b_img + BUF * BUFB + Q * QB;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      fb[nb][0] = *reinterpret_cast<const bf16x8*>(base + nb * 2048 + off_s0);
      fb[nb][1] = *reinterpret_cast<const bf16x8*>(base + nb * 2048 + off_s1);
    }
  };
  // quadrant (a-half AH, b-half BH): 4 token blocks x 2 feature blocks x 2 k-steps of 32
  auto mma = [&](auto AHI, auto BHI, const bf16x8 (&fb)[2][2]) {
    constexpr int AH = decltype(AHI)::value, BH = decltype(BHI)::value;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[4 * AH + mb][2 * BH + nb] = mfma16(fb[nb][s], fa[mb][s], acc[4 * AH + mb][2 * BH + nb]);
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using IA0 = std::integral_constant<int, Q_A0>;
  using IA1 = std::integral_constant<int, Q_A1>;
  using IB0 = std::integral_constant<int, Q_B0>;
  using IB1 = std::integral_constant<int, Q_B1>;

  // One phase P (0..3) of K-tile kt held in buffer CUR:
  //   reads (covered by the previous phase's wait + barrier) -> one quarter of DMA -> vmcnt -> barrier ->
  //   16 MFMAs (LOOK: + the next tile's B0 reads in phase 4) -> barrier.
  // B register sets: without LOOK fb0 = B0, fb1 = B1 always; with LOOK they swap roles every K-tile (B0 of tile t
  // lives in fb0 for even t, fb1 for odd t), so the lookahead read of phase 4 lands in the set phase 4 leaves idle.
  auto phase = [&](auto PI, auto CI, int kt) {
    constexpr int P = decltype(PI)::value, CUR = decltype(CI)::value;
    using ICUR = std::integral_constant<int, CUR>;
    using INXT = std::integral_constant<int, CUR ^ 1>;
    constexpr bool SW = LOOK && CUR == 1;          // swapped B roles in odd tiles
    auto& fB0 = SW ? fb1 : fb0;
    auto& fB1 = SW ? fb0 : fb1;
    if constexpr (P == 0) {
      if constexpr (!LOOK) read_b(IB0{}, ICUR{}, fB0);
      read_a(IA0{}, ICUR{});
    }
    if constexpr (P == 1) read_b(IB1{}, ICUR{}, fB1);
    if constexpr (P == 2) read_a(IA1{}, ICUR{});
    if constexpr (P == 0) dma(IB1{}, kt + 1, INXT{});
    if constexpr (P == 1) dma(IA1{}, kt + 1, INXT{});
    if constexpr (P == 2) dma(IA0{}, kt + 2, ICUR{});
    if constexpr (P == 3) dma(IB0{}, kt + 2, ICUR{});
    wait_vmcnt<VMC>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (P == 0) mma(I0{}, I0{}, fB0);
    if constexpr (P == 1) mma(I0{}, I1{}, fB1);
    if constexpr (P == 2) mma(I1{}, I1{}, fB1);
    if constexpr (P == 3) {
      mma(I1{}, I0{}, fB0);
      if constexpr (LOOK) {   // next tile's B0 (retired by phase 3's wait) into the idle set, between the MFMAs
        read_b(IB0{}, INXT{}, fB1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // 3 MFMAs
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: Q_A0(0) Q_B0(0) Q_B1(0) Q_A1(0) Q_A0(1) Q_B0(1), as if phases of tiles -2 / -1 had run ----
  dma(IA0{}, 0, I0{});
  dma(IB0{}, 0, I0{});
  dma(IB1{}, 0, I0{});
  dma(IA1{}, 0, I0{});
  dma(IA0{}, 1, I1{});
  dma(IB0{}, 1, I1{});
  wait_vmcnt<8>();   // Q_A0(0), Q_B0(0) landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if constexpr (LOOK) read_b(IB0{}, I0{}, fb0);   // tile 0's B0 (phase 4 of tile -1 would have read it)
  // stagger: waves 4..7 run one barrier behind waves 0..3 (uniform per wave: wid is wave-uniform)
  const bool late = __builtin_amdgcn_readfirstlane(wid) >= 4;
  if (late) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    phase(I0{}, I0{}, kt);
    phase(I1{}, I0{}, kt);
    phase(std::integral_constant<int, 2>{}, I0{}, kt);
    phase(std::integral_constant<int, 3>{}, I0{}, kt);
    phase(I0{}, I1{}, kt + 1);
    phase(I1{}, I1{}, kt + 1);
    phase(std::integral_constant<int, 2>{}, I1{}, kt + 1);
    phase(std::integral_constant<int, 3>{}, I1{}, kt + 1);
  }
  if (kt < nk) {   // odd number of K-tiles: the last one sits in buffer 0
    phase(I0{}, I0{}, kt);
    phase(I1{}, I0{}, kt);
    phase(std::integral_constant<int, 2>{}, I0{}, kt);
    phase(std::integral_constant<int, 3>{}, I0{}, kt);
  }
  if (!late) __builtin_amdgcn_s_barrier();   // balance the stagger
  wait_vmcnt<0>();                            // the clamped tail DMAs must land before the workgroup exits

  // ---- epilogue: acc[mb][nb][j] = C[token m0 + 128 wm + 16 mb + r16][feature col(nb) + 4 kq + j] ----
  if constexpr (LEPI && MODE == kNtSwiglu) {
    // the tile's 128 gate units | their 128 up units, as image columns 0..127 | 128..255
    __syncthreads();
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int row = 128 * wm + 16 * mb + r16, col = (nb >> 1) * 128 + 32 * wn + 16 * (nb & 1) + 4 * kq;
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)acc[mb][nb][j];
        *reinterpret_cast<bf16x4*>(lds + row * 512 + (((col >> 3) ^ (row & 15)) << 4) + (col & 7) * 2) = o;
      }
    __syncthreads();
    const int c = tid & 15;                       // gate chunk c (units 8c ..) and its up chunk 16 + c
    const int64_t u0 = (int64_t)tn * 128 + c * 8;
    if (RAG && u0 >= p.H) return;                 // whole 8-unit segment past H (H % 8 == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int row = (tid >> 4) + 32 * k;
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(lds + row * 512 + ((c ^ (row & 15)) << 4));
      const bf16x8 up = *reinterpret_cast<const bf16x8*>(lds + row * 512 + (((16 + c) ^ (row & 15)) << 4));
      bf16x8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gf = (float)g[j];   // exactly swiglu_fwd_k's math on the rounded gate / up
        hv[j] = (bf16)(gf * nt_sigmoid(gf) * (float)up[j]);
      }
      const int64_t t = (int64_t)m0 + row;
      *reinterpret_cast<bf16x8*>((bf16*)p.C + t * p.ldc + u0) = g;
      *reinterpret_cast<bf16x8*>((bf16*)p.C + t * p.ldc + p.H + u0) = up;
      *reinterpret_cast<bf16x8*>((bf16*)p.C2 + t * p.ldc2 + u0) = hv;
    }
    return;
  }
  if constexpr (LEPI && (MODE == kNtStore || MODE == kNtDswiglu || MODE == kNtRope)) {
    __syncthreads();   // every wave is past its last fragment read
    // image byte offset of (row, 16-B chunk c, byte b): row * 512 + ((c ^ (row & 15)) << 4) + b
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int row = 128 * wm + 16 * mb + r16, col = 64 * wn + 16 * nb + 4 * kq;
        f32x4 v = acc[mb][nb];
        if constexpr (MODE == kNtRope) {   // rotated on the fp32 accumulators (one rounding), as the register path
          const int n = tn * NBN + col;
          if (n < p.n_rot) {
            const int64_t t = (int64_t)m0 + row;
            const int pos = (int)(t % p.S) + p.pos_off, i0 = (n % p.hd) >> 1;
            const float* ct = p.rope_cos + (int64_t)pos * (p.hd >> 1) + i0;
            const float* st = p.rope_sin + (int64_t)pos * (p.hd >> 1) + i0;
            const float c0 = ct[0], c1 = ct[1], s0 = st[0], s1 = st[1];
            const float a0 = v[0], b0 = v[1], a1 = v[2], b1 = v[3];
            v[0] = a0 * c0 - b0 * s0;
            v[1] = a0 * s0 + b0 * c0;
            v[2] = a1 * c1 - b1 * s1;
            v[3] = a1 * s1 + b1 * c1;
          }
        }
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
        *reinterpret_cast<bf16x4*>(lds + row * 512 + (((col >> 3) ^ (row & 15)) << 4) + (col & 7) * 2) = o;
      }
    __syncthreads();
    const int c = tid & 31;                       // this thread's 16-B column chunk (512 threads, 32 per row)
    const int64_t n0c = (int64_t)tn * NBN + c * 8;
    if (RAG && n0c >= p.N) return;
    constexpr int BATCH = 4;
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += BATCH) {      // rows tid / 32 + 16 k
      bf16x8 dh[BATCH], gv[BATCH], uv[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int row = (tid >> 5) + 16 * (k0 + k);
        dh[k] = *reinterpret_cast<const bf16x8*>(lds + row * 512 + ((c ^ (row & 15)) << 4));
        if constexpr (MODE == kNtDswiglu) {
          const int64_t t = (int64_t)m0 + row;
          gv[k] = *reinterpret_cast<const bf16x8*>((const bf16*)p.X + t * p.ldx + n0c);
          uv[k] = *reinterpret_cast<const bf16x8*>((const bf16*)p.X + t * p.ldx + p.H + n0c);
        }
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int64_t t = (int64_t)m0 + (tid >> 5) + 16 * (k0 + k);
        bf16* out = (bf16*)p.C + t * p.ldc + n0c;
        if constexpr (MODE == kNtDswiglu) {
          bf16x8 dg, du;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = (float)dh[k][j];
            const float g = (float)gv[k][j], u = (float)uv[k][j];
            const float sg = nt_sigmoid(g);
            du[j] = (bf16)(d * (g * sg));
            dg[j] = (bf16)(d * u * sg * (1.f + g * (1.f - sg)));
          }
          *reinterpret_cast<bf16x8*>(out) = dg;
          *reinterpret_cast<bf16x8*>(out + p.H) = du;
        } else {
          *reinterpret_cast<bf16x8*>(out) = dh[k];
        }
      }
    }
    return;
  }
  const int64_t tok0 = (int64_t)m0 + 128 * wm + r16;
  if constexpr (MODE == kNtSwiglu) {
    // gate units u = 128 tn + 32 wn + 16 nb + 4 kq + j (nb < 2); acc[.][nb + 2] holds the matching up values
    bf16* x13 = (bf16*)p.C;
    bf16* hout = (bf16*)p.C2;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      const int64_t t = tok0 + 16 * mb;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int64_t u = (int64_t)tn * 128 + 32 * wn + 16 * nb + 4 * kq;
        bf16x4 g, up, hv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          g[j] = (bf16)acc[mb][nb][j];
          up[j] = (bf16)acc[mb][nb + 2][j];
          const float gf = (float)g[j];   // exactly swiglu_fwd_k's math on the rounded gate / up
          hv[j] = (bf16)(gf * nt_sigmoid(gf) * (float)up[j]);
        }
        *reinterpret_cast<bf16x4*>(x13 + t * p.ldc + u) = g;
        *reinterpret_cast<bf16x4*>(x13 + t * p.ldc + p.H + u) = up;
        *reinterpret_cast<bf16x4*>(hout + t * p.ldc2 + u) = hv;
      }
    }
  } else if constexpr (MODE == kNtDswiglu) {
    // dh for hidden units u = n0 + 64 wn + 16 nb + 4 kq + j; x13 = saved [gate | up], d13 = [dgate | dup]
    const bf16* x13 = (const bf16*)p.X;
    bf16* d13 = (bf16*)p.C;
    const int64_t ubase = (int64_t)tn * NBN + 64 * wn + 4 * kq;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      const int64_t t = tok0 + 16 * mb;
      bf16x4 gv[4], uv[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {   // issue all 8 loads of the row before any math
        gv[nb] = *reinterpret_cast<const bf16x4*>(x13 + t * p.ldx + ubase + 16 * nb);
        uv[nb] = *reinterpret_cast<const bf16x4*>(x13 + t * p.ldx + p.H + ubase + 16 * nb);
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        bf16x4 dg, du;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = (float)(bf16)acc[mb][nb][j];   // dh rounded like the unfused GEMM output
          const float g = (float)gv[nb][j], u = (float)uv[nb][j];
          const float s = nt_sigmoid(g);
          du[j] = (bf16)(d * (g * s));
          dg[j] = (bf16)(d * u * s * (1.f + g * (1.f - s)));
        }
        *reinterpret_cast<bf16x4*>(d13 + t * p.ldc + ubase + 16 * nb) = dg;
        *reinterpret_cast<bf16x4*>(d13 + t * p.ldc + p.H + ubase + 16 * nb) = du;
      }
    }
  } else {
    bf16* C = (bf16*)p.C;
    const int n_base = tn * NBN + 64 * wn + 4 * kq;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      const int64_t t = tok0 + 16 * mb;
      int pos = 0;
      if constexpr (MODE == kNtRope) pos = (int)(t % p.S) + p.pos_off;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int n = n_base + 16 * nb;
        f32x4 v = acc[mb][nb];
        if constexpr (MODE == kNtRope) {
          if (n < p.n_rot) {   // interleaved pairs (n, n+1), (n+2, n+3) of head column d = n % hd
            const int i0 = (n % p.hd) >> 1;
            const float* ct = p.rope_cos + (int64_t)pos * (p.hd >> 1) + i0;
            const float* st = p.rope_sin + (int64_t)pos * (p.hd >> 1) + i0;
            const float c0 = ct[0], c1 = ct[1], s0 = st[0], s1 = st[1];
            const float a0 = v[0], b0 = v[1], a1 = v[2], b1 = v[3];
            v[0] = a0 * c0 - b0 * s0;
            v[1] = a0 * s0 + b0 * c0;
            v[2] = a1 * c1 - b1 * s1;
            v[3] = a1 * s1 + b1 * c1;
          }
        }
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
        *reinterpret_cast<bf16x4*>(C + t * p.ldc + n) = o;
      }
    }
  }
}

// ==================================================================================================
// gemm_nt4_k: the STORE GEMM in hipBLASLt's workgroup shape -- 4 waves (2 M x 2 N), each owning a 128-token x 128-
// feature wave tile in 256 ACCUMULATOR registers (one wave per SIMD, the whole 512-entry register file), so a K-step
// reads 16 fragments for 64 MFMAs (0.25 ds_read_b128 per MFMA, 0.375 in gemm_nt_k's 128 x 64 wave tile).  hipcc
// keeps 256 accumulators in AGPRs cleanly only when every MFMA names them as asm "+a" operands (the plain-C++ form
// leaves hundreds of v_accvgpr moves and scratch in the loop: docs/guide/performance.md, round 2 wgrad note), so the
// MFMAs are inline asm and the compiler only allocates.  Same K-tile images, swizzle and quarter DMA schedule as
// gemm_nt_k (a quarter = 4 DMA instructions per lane at 256 threads); wave row-group wm owns token rows 128 wm..,
// wave column-group wn feature rows 128 wn..; Q_B0 / Q_B1 hold the first / second 64 feature rows of each group.
// Hazards the asm statements need (cdna_hip_programming.md §5.7 item 2): an MFMA chain on one accumulator needs no
// wait states; the accumulators are zeroed before the prologue's DMA waits (far more than 2 states before the first
// MFMA) and read only after an explicit 16-state pad behind the last MFMA.
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

constexpr int N4T = 256;

// PIPE = 1: every fragment a phase needs is read during the PREVIOUS phase's MFMAs (one ds_read between every 2-4
// MFMAs), so a phase's MFMAs start on registers that are already loaded and the LDS latency hides behind the matrix
// pipe -- with one wave per SIMD nothing else would hide it.  That needs two A register sets (A0 of tile t+1 is read
// while phase 4 still multiplies A1 of tile t) and every quarter retired one phase earlier: the wait before phase P's
// barrier retires what phase P's MFMA section reads (4 quarters stay in flight).  PIPE = 0: the reads before the
// barrier of the phase that uses them (gemm_nt_k's order without the stagger).
template <int PIPE>
__global__ __launch_bounds__(N4T, 1) void gemm_nt4_k(GemmNtParams p) {
  constexpr int QI = 4;                    // DMA instructions per quarter and lane
  constexpr int VMC = 4 * QI;
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUFB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int r16 = lane & 15, kq = lane >> 4;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "=a"(acc[i][j]) : "0"(z));
    }

  const int tiles_m = p.M / NBM, tiles_n = p.tiles_n;
  int tm, tn;
  nt_grouped_tile(xcd_remap(blockIdx.x, tiles_m * tiles_n), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * NBM;
  const int64_t n0 = (int64_t)tn * NBN;
  const int nk = p.K / NBK;

  // per-lane DMA source offsets: instruction i of a quarter copies chunk c = i * 256 + tid -> image row rho = c >> 3
  // (operand row 128 (rho >> 6) + (rho & 63) relative to the quarter's base row), 16-B chunk kc (source-side swizzle)
  unsigned voffA[QI], voffB[QI];
#pragma unroll
  for (int i = 0; i < QI; ++i) {
    const int c = i * N4T + tid, rho = c >> 3, kc = (c & 7) ^ ((rho >> 1) & 7);
    const int64_t row = 128 * (rho >> 6) + (rho & 63);
    voffA[i] = (unsigned)(row * p.lda * 2 + kc * 16);
    voffB[i] = (unsigned)(row * p.ldb * 2 + kc * 16);
  }
  const bf16* Ap = reinterpret_cast<const bf16*>(p.A);
  const bf16* Bp = reinterpret_cast<const bf16*>(p.B);
  const char* qptr[4];
  qptr[Q_A0] = reinterpret_cast<const char*>(Ap + (int64_t)m0 * p.lda);
  qptr[Q_A1] = reinterpret_cast<const char*>(Ap + (int64_t)(m0 + 64) * p.lda);
  qptr[Q_B0] = reinterpret_cast<const char*>(Bp + n0 * p.ldb);
  qptr[Q_B1] = reinterpret_cast<const char*>(Bp + (n0 + 64) * p.ldb);
  const unsigned lds_w = lds_addr(lds + wid * 1024);

  auto dma = [&](auto QIc, int kt, auto BI) {
    constexpr int Q = decltype(QIc)::value, BUF = decltype(BI)::value;
    const int ktc = min(kt, nk - 1);   // past the end: re-load the last tile into a slot nobody reads again
    const char* src = uniform_ptr(qptr[Q] + (int64_t)ktc * (NBK * 2));
    const unsigned d = lds_w + BUF * BUFB + Q * QB;
#pragma unroll
    for (int i = 0; i < QI; ++i) lds_dma16(src, Q < 2 ? voffA[i] : voffB[i], d + i * N4T * 16);
  };
  // instruction i of a quarter's DMA (PIPE 2 spreads a quarter over a phase's MFMA section)
  auto dma1 = [&](int Q, int kt, int BUF, int i) {
    const int ktc = min(kt, nk - 1);
    const char* src = uniform_ptr(qptr[Q] + (int64_t)ktc * (NBK * 2));
    lds_dma16(src, Q < 2 ? voffA[i] : voffB[i], lds_w + BUF * BUFB + Q * QB + i * N4T * 16);
  };

  // fragment reads: row r16 of a 16-row block, logical chunk 4 s + kq (image rows 64 w + 16 b + r16)
  const int xsw = (r16 >> 1) & 7;
  const int off_s0 = r16 * 128 + ((kq ^ xsw) << 4);
  const int off_s1 = r16 * 128 + (((4 + kq) ^ xsw) << 4);
  const char* a_img = lds + wm * 8192;
  const char* b_img = lds + wn * 8192;
  bf16x8 fa0[4][2], fa1[4][2], fb0[4][2], fb1[4][2];
  auto read4 = [&](const char* img, auto QIc, auto BI, bf16x8 (&f)[4][2]) {
    constexpr int Q = decltype(QIc)::value, BUF = decltype(BI)::value;
    const char* base = img + BUF * BUFB + Q * QB;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      f[b][0] = *reinterpret_cast<const bf16x8*>(base + b * 2048 + off_s0);
      f[b][1] = *reinterpret_cast<const bf16x8*>(base + b * 2048 + off_s1);
    }
  };
  // quadrant (AH, BH): 4 token blocks x 4 feature blocks x 2 k-steps of 32 = 32 MFMAs; `rd(r)` issues the r-th of R
  // fragment reads for the next phase, one after every 32 / R MFMAs (pinned there by scheduling fences)
  auto mma = [&](auto AHI, auto BHI, const bf16x8 (&fA)[4][2], const bf16x8 (&fB)[4][2], auto RI, auto&& rd,
                 auto&& dq) {
    constexpr int AH = decltype(AHI)::value, BH = decltype(BHI)::value, R = decltype(RI)::value;
    // 8 reads go out after MFMAs 2, 5, .., 23 (front-loaded: their latency is hidden before the phase ends); 16 reads
    // after every other MFMA
    constexpr int EVERY = R == 8 ? 3 : (R ? 32 / (R ? R : 1) : 64);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int s = i >> 4, mb = (i >> 2) & 3, nb = i & 3;
      mfma_acc(acc[4 * AH + mb][4 * BH + nb], fB[nb][s], fA[mb][s]);
      if constexpr (R > 0) {
        if (i % EVERY == EVERY - 1 && i / EVERY < R) {
          __builtin_amdgcn_sched_barrier(0);
          rd(i / EVERY);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (i % 8 == 4) {   // PIPE 2: one DMA instruction of the next phase's quarter every 8 MFMAs
        __builtin_amdgcn_sched_barrier(0);
        dq(i / 8);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // one fragment read: r < 8 -> block r / 2, k-step r % 2 of image img (quarter Q, buffer BUF) into f
  auto rd1 = [&](const char* img, int Q, int BUF, bf16x8 (&f)[4][2], int r) {
    const char* base = img + BUF * BUFB + Q * QB + (r >> 1) * 2048;
    f[r >> 1][r & 1] = *reinterpret_cast<const bf16x8*>(base + ((r & 1) ? off_s1 : off_s0));
  };
  auto none = [](int) {};
  auto nodma = [](int) {};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using IA0 = std::integral_constant<int, Q_A0>;
  using IA1 = std::integral_constant<int, Q_A1>;
  using IB0 = std::integral_constant<int, Q_B0>;
  using IB1 = std::integral_constant<int, Q_B1>;

  auto phase = [&](auto PI, auto CI, int kt) {
    constexpr int P = decltype(PI)::value, CUR = decltype(CI)::value;
    using ICUR = std::integral_constant<int, CUR>;
    using INXT = std::integral_constant<int, CUR ^ 1>;
    using R0 = std::integral_constant<int, 0>;
    using R8 = std::integral_constant<int, 8>;
    using R16 = std::integral_constant<int, 16>;
    constexpr bool SW = CUR == 1;            // B0 of tile t lives in fb0 for even t, fb1 for odd t
    auto& fB0 = SW ? fb1 : fb0;
    auto& fB1 = SW ? fb0 : fb1;
    if constexpr (!PIPE) {
      if constexpr (P == 0) {
        read4(b_img, IB0{}, ICUR{}, fB0);
        read4(a_img, IA0{}, ICUR{}, fa0);
      }
      if constexpr (P == 1) read4(b_img, IB1{}, ICUR{}, fB1);
      if constexpr (P == 2) read4(a_img, IA1{}, ICUR{}, fa1);
    }
    if constexpr (PIPE < 2) {
      if constexpr (P == 0) dma(IB1{}, kt + 1, INXT{});
      if constexpr (P == 1) dma(IA1{}, kt + 1, INXT{});
      if constexpr (P == 2) dma(IA0{}, kt + 2, ICUR{});
      if constexpr (P == 3) dma(IB0{}, kt + 2, ICUR{});
    }
    wait_vmcnt<VMC>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // PIPE 2: the quarter gemm_nt_k issues at the start of phase P + 1 goes out during phase P's MFMAs instead (same
    // issue order, so the same vmcnt retires the same quarters; every overwritten region was last read >= 2 phases
    // before and the barrier bounds the skew to one phase)
    auto dq = [&](int i) {
      if constexpr (PIPE == 2) {
        if constexpr (P == 0) dma1(Q_A1, kt + 1, CUR ^ 1, i);
        if constexpr (P == 1) dma1(Q_A0, kt + 2, CUR, i);
        if constexpr (P == 2) dma1(Q_B0, kt + 2, CUR, i);
        if constexpr (P == 3) dma1(Q_B1, kt + 2, CUR, i);
      }
    };
    if constexpr (!PIPE) {
      if constexpr (P == 0) mma(I0{}, I0{}, fa0, fB0, R0{}, none, nodma);
      if constexpr (P == 1) mma(I0{}, I1{}, fa0, fB1, R0{}, none, nodma);
      if constexpr (P == 2) mma(I1{}, I1{}, fa1, fB1, R0{}, none, nodma);
      if constexpr (P == 3) mma(I1{}, I0{}, fa1, fB0, R0{}, none, nodma);
    } else {
      // P0 reads B1(t) for P1, P1 reads A1(t) for P2, P3 reads A0(t+1) and B0(t+1) (into the B set P3 leaves idle)
      if constexpr (P == 0) mma(I0{}, I0{}, fa0, fB0, R8{}, [&](int r) { rd1(b_img, Q_B1, CUR, fB1, r); }, dq);
      if constexpr (P == 1) mma(I0{}, I1{}, fa0, fB1, R8{}, [&](int r) { rd1(a_img, Q_A1, CUR, fa1, r); }, dq);
      if constexpr (PIPE == 1) {
        if constexpr (P == 2) mma(I1{}, I1{}, fa1, fB1, R0{}, none, dq);
        if constexpr (P == 3)
          mma(I1{}, I0{}, fa1, fB0, R16{}, [&](int r) {
            if (r < 8) rd1(a_img, Q_A0, CUR ^ 1, fa0, r);
            else rd1(b_img, Q_B0, CUR ^ 1, fB1, r - 8);
          }, dq);
      } else {   // PIPE 2: A0(t+1) is retired one phase earlier here, so P2 reads it and P3 only B0(t+1)
        if constexpr (P == 2) mma(I1{}, I1{}, fa1, fB1, R8{}, [&](int r) { rd1(a_img, Q_A0, CUR ^ 1, fa0, r); }, dq);
        if constexpr (P == 3) mma(I1{}, I0{}, fa1, fB0, R8{}, [&](int r) { rd1(b_img, Q_B0, CUR ^ 1, fB1, r); }, dq);
      }
    }
    // One barrier per phase is enough under PIPE: every region a DMA overwrites was last read >= 3 phases earlier
    // and one barrier bounds the skew between waves to one phase; PIPE = 0 keeps the template's second barrier
    // (its reads sit right before the barrier of the phase that uses them).
    if constexpr (!PIPE) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  if constexpr (PIPE == 3) {
    // PIPE 3: two phases per K-tile (64 MFMAs each, one barrier each: half of PIPE 2's barriers).  H0 = A0 x (B0,
    // B1), H1 = A1 x (B1, B0).  Every fragment is read during the phase before its first use (B1(t) in H0(t)'s first
    // half, A1(t) in H0(t), A0(t+1) in H1(t), B0(t+1) in H1(t)'s second half into the B set H1's first half is done
    // with, so the two B sets swap roles every K-tile); a phase's two DMA quarters are the ones the phase after next
    // reads (issued two phases ahead, 2 quarters in flight at every barrier: vmcnt(8)).  Every DMA target was last
    // read >= 2 phases before its issue and one barrier per phase bounds the skew between waves to one phase.
    auto hphase = [&](auto HI, auto CI, int kt) {
      constexpr int H = decltype(HI)::value, CUR = decltype(CI)::value;
      constexpr bool SW = CUR == 1;
      auto& fB0 = SW ? fb1 : fb0;   // B0 of tile kt
      auto& fB1 = SW ? fb0 : fb1;   // B1 of tile kt (and B0 of tile kt + 1 after H1's first half)
      wait_vmcnt<2 * QI>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const int s = (i >> 4) & 1, mb = (i >> 2) & 3, nb = i & 3;
        if constexpr (H == 0) {
          if (i < 32) mfma_acc(acc[mb][nb], fB0[nb][s], fa0[mb][s]);
          else mfma_acc(acc[mb][4 + nb], fB1[nb][s], fa0[mb][s]);
        } else {
          if (i < 32) mfma_acc(acc[4 + mb][4 + nb], fB1[nb][s], fa1[mb][s]);
          else mfma_acc(acc[4 + mb][nb], fB0[nb][s], fa1[mb][s]);
        }
        if (i % 2 == 0 && i < 48 && (i < 16 || i >= 32 || H == 0)) {
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (H == 0) {   // B1(t) first (used by this phase's second half), then A1(t)
            if (i < 16) rd1(b_img, Q_B1, CUR, fB1, i / 2);
            else if (i < 32) rd1(a_img, Q_A1, CUR, fa1, (i - 16) / 2);
          } else {                  // A0(t+1), then B0(t+1) once the first half no longer reads fB1
            if (i < 16) rd1(a_img, Q_A0, CUR ^ 1, fa0, i / 2);
            else if (i >= 32) rd1(b_img, Q_B0, CUR ^ 1, fB1, (i - 32) / 2);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (i % 8 == 5) {   // 2 quarters = 8 DMA instructions per phase (front-loading them measured 0.6 % slower)
          __builtin_amdgcn_sched_barrier(0);
          const int j = i / 8;
          if constexpr (H == 0) dma1(j < 4 ? Q_A1 : Q_B1, kt + 1, CUR ^ 1, j & 3);
          else dma1(j < 4 ? Q_A0 : Q_B0, kt + 2, CUR, j & 3);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    // prologue: A0(0) B0(0) A1(0) B1(0) A0(1) B0(1); tile 0's A0 / B0 into registers
    dma(IA0{}, 0, I0{});
    dma(IB0{}, 0, I0{});
    dma(IA1{}, 0, I0{});
    dma(IB1{}, 0, I0{});
    dma(IA0{}, 1, I1{});
    dma(IB0{}, 1, I1{});
    wait_vmcnt<4 * QI>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    read4(a_img, IA0{}, I0{}, fa0);
    read4(b_img, IB0{}, I0{}, fb0);
    __builtin_amdgcn_sched_barrier(0);
    int kt = 0;
    for (; kt + 2 <= nk; kt += 2) {
      hphase(I0{}, I0{}, kt);
      hphase(I1{}, I0{}, kt);
      hphase(I0{}, I1{}, kt + 1);
      hphase(I1{}, I1{}, kt + 1);
    }
    if (kt < nk) {
      hphase(I0{}, I0{}, kt);
      hphase(I1{}, I0{}, kt);
    }
  } else {
    // prologue: Q_A0(0) Q_B0(0) Q_B1(0) Q_A1(0) Q_A0(1) Q_B0(1)
    dma(IA0{}, 0, I0{});
    dma(IB0{}, 0, I0{});
    dma(IB1{}, 0, I0{});
    dma(IA1{}, 0, I0{});
    dma(IA0{}, 1, I1{});
    dma(IB0{}, 1, I1{});
    wait_vmcnt<4 * QI>();   // Q_A0(0), Q_B0(0) landed
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    if constexpr (PIPE) {   // tile 0's A0 / B0, as phase 4 of tile -1 would have read them
      read4(a_img, IA0{}, I0{}, fa0);
      read4(b_img, IB0{}, I0{}, fb0);
    }
    if constexpr (PIPE == 2) dma(IB1{}, 1, I1{});   // the quarter phase 4 of tile -1 would have issued
    __builtin_amdgcn_sched_barrier(0);

    int kt = 0;
    for (; kt + 2 <= nk; kt += 2) {
      phase(I0{}, I0{}, kt);
      phase(I1{}, I0{}, kt);
      phase(std::integral_constant<int, 2>{}, I0{}, kt);
      phase(std::integral_constant<int, 3>{}, I0{}, kt);
      phase(I0{}, I1{}, kt + 1);
      phase(I1{}, I1{}, kt + 1);
      phase(std::integral_constant<int, 2>{}, I1{}, kt + 1);
      phase(std::integral_constant<int, 3>{}, I1{}, kt + 1);
    }
    if (kt < nk) {
      phase(I0{}, I0{}, kt);
      phase(I1{}, I0{}, kt);
      phase(std::integral_constant<int, 2>{}, I0{}, kt);
      phase(std::integral_constant<int, 3>{}, I0{}, kt);
    }
  }
  wait_vmcnt<0>();                                  // the clamped tail DMAs land before the images are reused
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // MFMA results -> accumulator reads
  __syncthreads();

  // epilogue through LDS: acc[mb][nb][j] = C[token m0 + 128 wm + 16 mb + r16][feature n0 + 128 wn + 16 nb + 4 kq + j]
  // rounded to bf16 into a 256 x 256 image (16-B chunks XOR-swizzled by the row), then whole 16-B row segments
#pragma unroll
  for (int mb = 0; mb < 8; ++mb)
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const int row = 128 * wm + 16 * mb + r16, col = 128 * wn + 16 * nb + 4 * kq;
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)acc[mb][nb][j];
      *reinterpret_cast<bf16x4*>(lds + row * 512 + (((col >> 3) ^ (row & 15)) << 4) + (col & 7) * 2) = o;
    }
  __syncthreads();
  const int c = tid & 31;
  bf16* C = (bf16*)p.C;
#pragma unroll 4
  for (int k = 0; k < 32; ++k) {
    const int row = (tid >> 5) + 8 * k;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + row * 512 + ((c ^ (row & 15)) << 4));
    *reinterpret_cast<bf16x8*>(C + (int64_t)(m0 + row) * p.ldc + n0 + c * 8) = v;
  }
}

// Rejected in round 5 (profiles/r5/nt16_slots/): STORE mode on the weight-gradient kernel's lockstep slot pipeline
// (32-k slots in a 5-region ring, DMA three slots ahead, one ds_read_b128 per fragment): 1221-1275 TFLOP/s against
// 1482-1515 for this kernel and 1439-1601 for hipBLASLt on the 7B shapes -- a 32-k slot of a K-contiguous operand is a
// 64-B piece of every row, half a cache line per DMA lane.
// Rejected variants (code removed; evidence kept): the same pipeline on v_mfma_f32_32x32x16_bf16 (0.86-0.96x this
// kernel, profiles/r4/nt_mfma32/; at the 1400 W package limit it delivers 0.98-1.00 TFLOP/J against 1.06-1.09 here
// and 1.10-1.14 for hipBLASLt, profiles/r5/gemm_power/), the two-phase form without the B0 look-ahead (LOOK = 0,
// profiles/r3/rejected/gemm_nt_2phase_*) and the register epilogue (bitwise equal, slower: profiles/r3/ab_fused_mlp_fwd_lds/).

}  // namespace

bool gemm_nt_supported(int mode, int64_t M, int64_t N, int64_t K) {
  // ragged N / K run on the 32x32x16 kernel's edge tiles; offsets stay 32-bit (weights < 2 GB per operand)
  if (M <= 0 || N <= 0 || K <= 0 || M % NBM || K % 8 || N % 8) return false;
  return (mode == kNtSwiglu ? 2 * N : N) * K * 2 < (int64_t)1 << 31;
}

bool gemm_nt_ragged(int mode, int64_t N, int64_t K) {
  return K % NBK != 0 || (mode == kNtSwiglu ? N % 128 : N % NBN) != 0;
}

// A/B of the plain-store GEMM forms (gemm_nt_variant op): 0 = gemm_nt_k (8 waves), 4 / 5 / 6 / 7 = gemm_nt4_k (PIPE 0 / 1 / 2 / 3)
static int g_nt_variant = 0;
int gemm_nt_set_variant(int v) {
  const int old = g_nt_variant;
  g_nt_variant = v;
  return old;
}

void gemm_nt(int mode, const GemmNtParams& prm, hipStream_t st) {
  GemmNtParams p = prm;
  p.tiles_n = mode == kNtSwiglu ? (p.N + 127) / 128 : (p.N + NBN - 1) / NBN;
  const dim3 grid((unsigned)((p.M / NBM) * p.tiles_n)), block(NNT);
  const bool rag = gemm_nt_ragged(mode, p.N, p.K);
  if (mode == kNtStore && !rag && g_nt_variant >= 4 && g_nt_variant <= 7) {
    if (g_nt_variant == 4) hipLaunchKernelGGL((gemm_nt4_k<0>), grid, dim3(N4T), 0, st, p);
    else if (g_nt_variant == 5) hipLaunchKernelGGL((gemm_nt4_k<1>), grid, dim3(N4T), 0, st, p);
    else if (g_nt_variant == 6) hipLaunchKernelGGL((gemm_nt4_k<2>), grid, dim3(N4T), 0, st, p);
    else hipLaunchKernelGGL((gemm_nt4_k<3>), grid, dim3(N4T), 0, st, p);
    return;
  }
#define DPH_NT_LAUNCH(MD)                                                                    \
  do {                                                                                       \
    if (rag) hipLaunchKernelGGL((gemm_nt_k<MD, 1, true, true>), grid, block, 0, st, p);      \
    else hipLaunchKernelGGL((gemm_nt_k<MD, 1, true>), grid, block, 0, st, p);                \
  } while (0)
  switch (mode) {
    case kNtSwiglu: DPH_NT_LAUNCH(kNtSwiglu); break;
    case kNtDswiglu: DPH_NT_LAUNCH(kNtDswiglu); break;
    case kNtRope: DPH_NT_LAUNCH(kNtRope); break;
    default: DPH_NT_LAUNCH(kNtStore); break;
  }
#undef DPH_NT_LAUNCH
}

}  // namespace dph
