// Single-node all-reduce over peer-mapped IPC buffers (xGMI), for the latency-bound messages of tensor-parallel
// layers and small data-parallel buckets (SURVEY.md §2.10 "comm/xgmi_allreduce"; reference call sites C1/C11:
// the DDP gradient all-reduce and the Rowwise TP output all-reduce, which the reference leaves to NCCL rings).
//
// Why not a ring: xGMI on an MI355X node is a full mesh of point-to-point links, so a ring uses one link per step
// and pays (2N-2) latency hops.  Here every rank reads its peers' buffers directly, all links at once:
//   one-shot : each rank reads the whole message from every peer and reduces it          (1 barrier + data)
//   two-shot : rank r reduces slice r from every peer (reduce-scatter), then every rank gathers the N reduced
//              slices (all-gather)                                                        (2 barriers + data)
// The caller's input is copied into this rank's IPC staging area by the same kernel (no separate memcpy); peers
// only ever read staging memory, so the output may alias the input.  Sums are accumulated in fp32 in rank order
// 0..N-1 on every rank, so all ranks get bit-identical results (replicas never drift).
//
// Memory: one uncached (fine-grained, MTYPE UC) allocation per rank = [signals | staging A | staging B], exported
// with hipIpcGetMemHandle and mapped by every peer.  Uncached memory keeps peer reads coherent without cache
// maintenance; flags use system-scope release/acquire atomics.
//
// Synchronisation is per workgroup: block b of every rank touches the same element positions in every phase, so
// block b only waits for block b of its peers.  Every barrier has a wall-clock timeout: a missing peer makes the
// kernel count an error (car_status) and exit instead of hanging the GPU.  The per-block epoch counters live in
// device memory and are advanced by the kernel itself, so the op can be captured in a HIP graph.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <stdexcept>
#include <string>

#include "dph_common.h"
#include "kernels.h"

namespace dph {

namespace {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_BLOCKS = 256;
constexpr int CAR_NT = 512;

struct CarSignal {
  uint32_t flag[3][CAR_MAX_BLOCKS][CAR_MAX_RANKS];   // [start | mid | end][block][from-rank]
  uint32_t epoch[CAR_MAX_BLOCKS];                    // this rank's per-block call counter
  uint32_t err;                                      // barrier timeouts
};
constexpr size_t CAR_SIG_BYTES = (sizeof(CarSignal) + 4095) / 4096 * 4096;

struct CarPeers {
  char* base[CAR_MAX_RANKS];
  uint32_t* err_host;   // device view of a pinned, host-mapped word: the host reads timeouts without a device sync
};

#define DPH_HIP_OK(expr)                                                                          \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("dph custom all-reduce: ") + #expr + \
                                                   " failed: " + hipGetErrorString(e_));          \
  } while (0)

__device__ __forceinline__ CarSignal* sig(const CarPeers& p, int r) { return reinterpret_cast<CarSignal*>(p.base[r]); }

// Block-level barrier among the same block index of all ranks.  Every thread first makes its own prior stores
// visible at system scope; then lane r < world posts `epoch` into rank r's slot for us and waits for rank r's.
template <int WHICH>
__device__ __forceinline__ void car_barrier(const CarPeers& p, int rank, int world, uint32_t epoch,
                                            uint64_t timeout_ticks) {
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world) {
    const int r = threadIdx.x;
    __hip_atomic_store(&sig(p, r)->flag[WHICH][blockIdx.x][rank], epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = &sig(p, rank)->flag[WHICH][blockIdx.x][r];
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (wall_clock64() - t0 > timeout_ticks) {
        __hip_atomic_fetch_add(&sig(p, rank)->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t car_begin(const CarPeers& p, int rank) {
  __shared__ uint32_t ep;
  if (threadIdx.x == 0) ep = sig(p, rank)->epoch[blockIdx.x] + 1;
  __syncthreads();
  return ep;
}

__device__ __forceinline__ void car_finish(const CarPeers& p, int rank, uint32_t ep) {
  if (threadIdx.x == 0) sig(p, rank)->epoch[blockIdx.x] = ep;
}

// 16-byte vector <-> 8 (bf16) or 4 (fp32) fp32 lanes.
template <typename T> struct V16;
template <> struct V16<bf16> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void add(const u32x4& v, float (&a)[8]) {
    const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += (float)b[i];
  }
  static __device__ __forceinline__ u32x4 pack(const float (&a)[8]) {
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (bf16)a[i];
    return __builtin_bit_cast(u32x4, b);
  }
};
template <> struct V16<float> {
  static constexpr int N = 4;
  static __device__ __forceinline__ void add(const u32x4& v, float (&a)[4]) {
    const f32x4 b = __builtin_bit_cast(f32x4, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] += b[i];
  }
  static __device__ __forceinline__ u32x4 pack(const float (&a)[4]) {
    f32x4 b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = a[i];
    return __builtin_bit_cast(u32x4, b);
  }
};

// Sum of vector v over all NR ranks' buffers at byte offset `off`, in rank order; scaled, packed.
template <typename T, int NR>
__device__ __forceinline__ u32x4 reduce_vec(const CarPeers& p, size_t off, int64_t v, float scale) {
  u32x4 in[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) in[r] = reinterpret_cast<const u32x4*>(p.base[r] + off)[v];
  float a[V16<T>::N];
#pragma unroll
  for (int i = 0; i < V16<T>::N; ++i) a[i] = 0.f;
#pragma unroll
  for (int r = 0; r < NR; ++r) V16<T>::add(in[r], a);
#pragma unroll
  for (int i = 0; i < V16<T>::N; ++i) a[i] *= scale;
  return V16<T>::pack(a);
}

// Element range [lo, hi) of rank r's slice when nvec vectors are split N ways.
__device__ __forceinline__ void slice_of(int64_t nvec, int world, int r, int64_t& lo, int64_t& hi) {
  const int64_t per = (nvec + world - 1) / world;
  lo = min(nvec, per * r);
  hi = min(nvec, lo + per);
}

template <typename T, int NR>
__global__ __launch_bounds__(CAR_NT) void car_oneshot_k(CarPeers p, int rank, const u32x4* in,
                                                        u32x4* out, int64_t nvec, float scale,
                                                        uint64_t timeout_ticks) {
  const uint32_t ep = car_begin(p, rank);
  u32x4* stage = reinterpret_cast<u32x4*>(p.base[rank] + CAR_SIG_BYTES);
  const int64_t stride = (int64_t)gridDim.x * CAR_NT;
  for (int64_t v = (int64_t)blockIdx.x * CAR_NT + threadIdx.x; v < nvec; v += stride) stage[v] = in[v];
  car_barrier<0>(p, rank, NR, ep, timeout_ticks);
  for (int64_t v = (int64_t)blockIdx.x * CAR_NT + threadIdx.x; v < nvec; v += stride)
    out[v] = reduce_vec<T, NR>(p, CAR_SIG_BYTES, v, scale);
  car_barrier<2>(p, rank, NR, ep, timeout_ticks);   // peers are done reading our staging
  car_finish(p, rank, ep);
}

template <typename T, int NR>
__global__ __launch_bounds__(CAR_NT) void car_twoshot_k(CarPeers p, int rank, const u32x4* in,
                                                        u32x4* out, int64_t nvec, size_t b_off,
                                                        float scale, uint64_t timeout_ticks) {
  const uint32_t ep = car_begin(p, rank);
  u32x4* stage_a = reinterpret_cast<u32x4*>(p.base[rank] + CAR_SIG_BYTES);
  u32x4* stage_b = reinterpret_cast<u32x4*>(p.base[rank] + b_off);
  const int64_t stride = (int64_t)gridDim.x * CAR_NT, t0 = (int64_t)blockIdx.x * CAR_NT + threadIdx.x;
  // copy-in, slice by slice, with the same block->position map the reduce phase of each owner uses
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    int64_t lo, hi;
    slice_of(nvec, NR, r, lo, hi);
    for (int64_t v = lo + t0; v < hi; v += stride) stage_a[v] = in[v];
  }
  car_barrier<0>(p, rank, NR, ep, timeout_ticks);
  int64_t lo, hi;
  slice_of(nvec, NR, rank, lo, hi);
  for (int64_t v = lo + t0; v < hi; v += stride) {
    const u32x4 s = reduce_vec<T, NR>(p, CAR_SIG_BYTES, v, scale);
    stage_b[v] = s;
    out[v] = s;
  }
  car_barrier<1>(p, rank, NR, ep, timeout_ticks);
#pragma unroll
  for (int r = 1; r < NR; ++r) {   // gather the other ranks' reduced slices, nearest peer first
    const int src = (rank + r) % NR;
    int64_t slo, shi;
    slice_of(nvec, NR, src, slo, shi);
    const u32x4* peer_b = reinterpret_cast<const u32x4*>(p.base[src] + b_off);
    for (int64_t v = slo + t0; v < shi; v += stride) out[v] = peer_b[v];
  }
  car_barrier<2>(p, rank, NR, ep, timeout_ticks);
  car_finish(p, rank, ep);
}

struct CarContext {
  int rank = 0, world = 1, device = 0;
  size_t max_bytes = 0;
  char* local = nullptr;
  uint32_t* err_host = nullptr;   // pinned host memory (mapped into the device's address space)
  CarPeers peers{};
  bool opened[CAR_MAX_RANKS] = {};
  uint64_t timeout_ticks = 0;
};

}  // namespace

int64_t car_create(int rank, int world, int64_t max_bytes, double timeout_s) {
  if (world < 1 || world > CAR_MAX_RANKS || rank < 0 || rank >= world)
    throw std::runtime_error("dph custom all-reduce: world must be in [1, 8]");
  auto* c = new CarContext();
  c->rank = rank;
  c->world = world;
  c->max_bytes = (size_t)((max_bytes + 4095) / 4096 * 4096);
  DPH_HIP_OK(hipGetDevice(&c->device));
  const size_t total = CAR_SIG_BYTES + 2 * c->max_bytes;
  void* p = nullptr;
  DPH_HIP_OK(hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached));
  DPH_HIP_OK(hipMemset(p, 0, CAR_SIG_BYTES));
  DPH_HIP_OK(hipDeviceSynchronize());
  c->local = static_cast<char*>(p);
  c->peers.base[rank] = c->local;
  void* hp = nullptr;
  DPH_HIP_OK(hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
  c->err_host = static_cast<uint32_t*>(hp);
  c->err_host[0] = 0u;   // this rank's barrier timeouts
  c->err_host[1] = 0u;   // the group-agreed verdict of the last guard
  void* dp = nullptr;
  DPH_HIP_OK(hipHostGetDevicePointer(&dp, hp, 0));
  c->peers.err_host = static_cast<uint32_t*>(dp);
  int khz = 0;
  DPH_HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
  c->timeout_ticks = (uint64_t)(timeout_s * (double)khz * 1000.0);
  return reinterpret_cast<int64_t>(c);
}

void car_ipc_handle(int64_t ctx, void* out64) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  hipIpcMemHandle_t h;
  DPH_HIP_OK(hipIpcGetMemHandle(&h, c->local));
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle larger than 64 bytes");
  std::memset(out64, 0, 64);
  std::memcpy(out64, &h, sizeof(h));
}

void car_open(int64_t ctx, const void* handles /* [world][64] */) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank || c->opened[r]) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, static_cast<const char*>(handles) + 64 * r, sizeof(h));
    void* p = nullptr;
    DPH_HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    c->peers.base[r] = static_cast<char*>(p);
    c->opened[r] = true;
  }
}

int64_t car_max_bytes(int64_t ctx) { return (int64_t)reinterpret_cast<CarContext*>(ctx)->max_bytes; }

void car_allreduce(int64_t ctx, const void* in, void* out, int64_t bytes, int dt, int algo, float scale, int max_blocks,
                   hipStream_t st) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  if (bytes % 16 || (size_t)bytes > c->max_bytes)
    throw std::runtime_error("dph custom all-reduce: message must be a multiple of 16 B and fit the staging buffer");
  for (int r = 0; r < c->world; ++r)
    if (!c->peers.base[r]) throw std::runtime_error("dph custom all-reduce: peers not opened (call car_open)");
  const int64_t nvec = bytes / 16;
  if (nvec == 0) return;
  if (algo == 0) algo = (bytes <= (256 << 10) || c->world <= 2) ? 1 : 2;
  const int64_t work = algo == 1 ? nvec : (nvec + c->world - 1) / c->world;
  int blocks = (int)std::min<int64_t>(cdiv(work, CAR_NT), std::min(max_blocks, CAR_MAX_BLOCKS));
  if (blocks < 1) blocks = 1;
  const size_t b_off = CAR_SIG_BYTES + c->max_bytes;
  const u32x4* vin = static_cast<const u32x4*>(in);
  u32x4* vout = static_cast<u32x4*>(out);
#define DPH_CAR_LAUNCH(T_, NR_)                                                                                 \
  do {                                                                                                          \
    if (algo == 1)                                                                                              \
      hipLaunchKernelGGL((car_oneshot_k<T_, NR_>), dim3(blocks), dim3(CAR_NT), 0, st, c->peers, c->rank, vin, \
                         vout, nvec, scale, c->timeout_ticks);                                                  \
    else                                                                                                        \
      hipLaunchKernelGGL((car_twoshot_k<T_, NR_>), dim3(blocks), dim3(CAR_NT), 0, st, c->peers, c->rank, vin, \
                         vout, nvec, b_off, scale, c->timeout_ticks);                                           \
  } while (0)
#define DPH_CAR_WORLD(T_)                                                                                       \
  switch (c->world) {                                                                                           \
    case 1: DPH_CAR_LAUNCH(T_, 1); break;                                                                       \
    case 2: DPH_CAR_LAUNCH(T_, 2); break;                                                                       \
    case 3: DPH_CAR_LAUNCH(T_, 3); break;                                                                       \
    case 4: DPH_CAR_LAUNCH(T_, 4); break;                                                                       \
    case 5: DPH_CAR_LAUNCH(T_, 5); break;                                                                       \
    case 6: DPH_CAR_LAUNCH(T_, 6); break;                                                                       \
    case 7: DPH_CAR_LAUNCH(T_, 7); break;                                                                       \
    default: DPH_CAR_LAUNCH(T_, 8); break;                                                                      \
  }
  if (dt == kBF16) {
    DPH_CAR_WORLD(bf16);
  } else {
    DPH_CAR_WORLD(float);
  }
#undef DPH_CAR_WORLD
#undef DPH_CAR_LAUNCH
}

// ---- stream-ordered health guard (the engines run it between a step's reductions and its optimizer update) ----
// car_flag copies this rank's timeout word into a device int; the caller MAX-all-reduces it over the group (RCCL);
// car_poison then turns the step's gradient scale into NaN when any rank of the group timed out -- the optimizer
// kernels skip their update on a NaN scale (csrc/optim.hip), on every rank alike, so sums that may hold a late peer's
// stale staging data never reach the weights -- and records the agreed verdict in the second host-mapped word, which
// the host reads after the guard's event (comm/custom_allreduce.py check_health): same verdict, same step, every rank.
__global__ void car_flag_k(const uint32_t* err, int* flag) {
  flag[0] = (int)__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void car_poison_k(const int* flag, float* gscale, uint32_t* agreed) {
  if (flag[0] != 0) {
    gscale[0] = __builtin_nanf("");
    __hip_atomic_store(agreed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

void car_flag(int64_t ctx, int* flag_dev, hipStream_t st) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  hipLaunchKernelGGL(car_flag_k, dim3(1), dim3(64), 0, st, c->peers.err_host, flag_dev);
}
void car_poison(int64_t ctx, const int* flag_dev, float* gscale_dev, hipStream_t st) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  hipLaunchKernelGGL(car_poison_k, dim3(1), dim3(64), 0, st, flag_dev, gscale_dev, c->peers.err_host + 1);
}
// The group-agreed verdict of the last guard (0 = healthy); read after the guard's event has completed.
int64_t car_agreed(int64_t ctx) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  return (int64_t)__atomic_load_n(c->err_host + 1, __ATOMIC_ACQUIRE);
}

// Non-zero once any barrier of this rank's kernels timed out.  Reads the host-mapped word the kernel stores to at
// system scope: no device synchronisation, so the training engines can check it every step (a kernel still in
// flight reports on a later check).
int64_t car_status(int64_t ctx) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  return (int64_t)__atomic_load_n(c->err_host, __ATOMIC_ACQUIRE);
}

void car_destroy(int64_t ctx) {
  auto* c = reinterpret_cast<CarContext*>(ctx);
  if (!c) return;
  (void)hipDeviceSynchronize();
  for (int r = 0; r < c->world; ++r)
    if (c->opened[r]) (void)hipIpcCloseMemHandle(c->peers.base[r]);
  if (c->local) (void)hipFree(c->local);
  if (c->err_host) (void)hipHostFree(c->err_host);
  delete c;
}

}  // namespace dph
