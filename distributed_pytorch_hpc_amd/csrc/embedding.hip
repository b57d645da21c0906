// Token-embedding gather and its backward scatter-add, vocab-shard aware: a rank holding rows
// [vocab_start, vocab_start + vocab_local) of the table writes zeros for ids outside its shard, which
// is what RowwiseParallel does for tok_embeddings in the reference TP plan (fsdp_tp/fsdp_tp_example.py:146-149)
// before its reduce-scatter.  16-B vector copies; the backward is a deterministic segmented sum over
// stably-sorted ids (no float atomics).
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

// Deterministic backward over ids sorted by a stable sort (sorted ids + the permutation back to token rows):
// workgroup (j, chunk) owns the segment of equal ids that STARTS at sorted position j (other j exit at once) and
// sums that segment's dout rows in sorted order -- no atomics, so the gradient is bit-reproducible run to run
// (SURVEY.md §5.2).  Each thread accumulates 8 contiguous columns in fp32; rows of ids outside this rank's vocab
// shard stay zero.
template <typename T>
__global__ __launch_bounds__(256) void emb_bwd_sorted_k(const int64_t* __restrict__ sids, const int64_t* __restrict__ perm,
                                                        const T* __restrict__ dout, float* __restrict__ dtab, int64_t n,
                                                        int64_t dim, int64_t vstart, int64_t vlocal) {
  const int64_t j = blockIdx.x;
  const int64_t sid = sids[j];
  if (j > 0 && sids[j - 1] == sid) return;
  const int64_t id = sid - vstart;
  if (id < 0 || id >= vlocal) return;
  const int64_t c = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 8;
  if (c >= dim) return;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  for (int64_t k = j; k < n && sids[k] == sid; ++k) {
    float v[8];
    Vec8<T>::load(dout + perm[k] * dim + c, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += v[q];
  }
  Vec8<float>::store(dtab + id * dim + c, acc);
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

void embedding_bwd(const int64_t* sorted_ids, const int64_t* perm, const void* dout, float* dtab, int64_t n,
                   int64_t dim, int64_t vstart, int64_t vlocal, int dtype, hipStream_t stream) {
  if (n == 0) return;
  const dim3 grid((unsigned)n, (unsigned)((dim / 8 + 255) / 256));
  if (dtype == kBF16)
    hipLaunchKernelGGL(emb_bwd_sorted_k<bf16>, grid, dim3(256), 0, stream, sorted_ids, perm, (const bf16*)dout, dtab, n,
                       dim, vstart, vlocal);
  else
    hipLaunchKernelGGL(emb_bwd_sorted_k<float>, grid, dim3(256), 0, stream, sorted_ids, perm, (const float*)dout, dtab,
                       n, dim, vstart, vlocal);
}

}  // namespace dph
