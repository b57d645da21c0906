// Token-embedding gather and its backward scatter-add, vocab-shard aware: a rank holding rows
// [vocab_start, vocab_start + vocab_local) of the table writes zeros for ids outside its shard, which
// is what RowwiseParallel does for tok_embeddings in the reference TP plan (fsdp_tp/fsdp_tp_example.py:146-149)
// before its reduce-scatter.  16-B vector copies; backward accumulates fp32 rows with
// global_atomic_add_f32, one 256-B wave-instruction per 64 contiguous floats (the full-rate shape of
// MI355X_MICROARCH.md 'Global float atomics').
#include "dph_common.h"
#include "kernels.h"

namespace dph {

template <typename T>
__global__ __launch_bounds__(256) void emb_fwd_k(const int64_t* __restrict__ ids, const T* __restrict__ table,
                                                 T* __restrict__ out, int64_t n, int64_t dim, int64_t vstart,
                                                 int64_t vlocal) {
  const int64_t cpr = dim >> 3;
  const int64_t total = n * cpr;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cpr, c = (i % cpr) * 8;
    const int64_t id = ids[r] - vstart;
    float v[8];
    if (id >= 0 && id < vlocal) Vec8<T>::load(table + id * dim + c, v);
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = 0.f;
    }
    Vec8<T>::store(out + r * dim + c, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void emb_bwd_k(const int64_t* __restrict__ ids, const T* __restrict__ dout,
                                                 float* __restrict__ dtab, int64_t n, int64_t dim, int64_t vstart,
                                                 int64_t vlocal) {
  const int64_t total = n * dim;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / dim, c = i % dim;
    const int64_t id = ids[r] - vstart;
    if (id >= 0 && id < vlocal) atomicAdd(dtab + id * dim + c, (float)dout[i]);
  }
}

void embedding_fwd(const int64_t* ids, const void* table, void* out, int64_t n, int64_t dim, int64_t vstart,
                   int64_t vlocal, int dtype, hipStream_t stream) {
  if (n == 0) return;
  const int grid = stream_grid(n * (dim / 8), 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(emb_fwd_k<bf16>, dim3(grid), dim3(256), 0, stream, ids, (const bf16*)table, (bf16*)out, n, dim,
                       vstart, vlocal);
  else
    hipLaunchKernelGGL(emb_fwd_k<float>, dim3(grid), dim3(256), 0, stream, ids, (const float*)table, (float*)out, n,
                       dim, vstart, vlocal);
}

void embedding_bwd(const int64_t* ids, const void* dout, float* dtab, int64_t n, int64_t dim, int64_t vstart,
                   int64_t vlocal, int dtype, hipStream_t stream) {
  if (n == 0) return;
  const int grid = stream_grid(n * dim, 256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(emb_bwd_k<bf16>, dim3(grid), dim3(256), 0, stream, ids, (const bf16*)dout, dtab, n, dim, vstart,
                       vlocal);
  else
    hipLaunchKernelGGL(emb_bwd_k<float>, dim3(grid), dim3(256), 0, stream, ids, (const float*)dout, dtab, n, dim,
                       vstart, vlocal);
}

}  // namespace dph
