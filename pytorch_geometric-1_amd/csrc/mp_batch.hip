// Device-side collation of a graph list into one block-diagonal batch
// (torch_geometric.data.Batch.from_data_list, PyG 1.4.3 [U8]; caller
// /root/reference/ConvexPruning.py:530 and examples/data_parallel.py:35-49 via
// DataParallel).  The host concatenates each key's raw items once and moves
// them to the replica's device in one copy; these kernels then apply what the
// reference does per graph on the host:
//   * `item + cumsum[key]`: every element of graph g's segment of an index
//     key (edge_index, face) gains the node count of the graphs before it;
//   * `torch.full((n_g,), g)`: the batch vector (and follow_batch vectors).
// Segments are given by their start offsets (starts[G] = n); an element finds
// its graph by binary search, so the work is balanced whatever the graph sizes
// (a few large graphs or thousands of small ones).  Integer work: bit-exact.
#include "mp_common.h"

namespace mp {

// the graph g of element i: the last g with starts[g] <= i (empty graphs,
// starts[g] == starts[g + 1], are never chosen)
__device__ __forceinline__ int64_t seg_of(const int64_t* __restrict__ starts, int64_t G, int64_t i) {
  int64_t lo = 0, hi = G;  // invariant: starts[lo] <= i < starts[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (starts[mid] <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}

// data[r * ld + i] += inc[g(i)] for r < rows, i < n
__global__ void k_segment_offset_i64(int64_t* __restrict__ data, int64_t ld, int32_t rows, int64_t n,
                                     const int64_t* __restrict__ starts, const int64_t* __restrict__ inc,
                                     int64_t G) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t d = inc[seg_of(starts, G, i)];
  for (int r = 0; r < rows; ++r) data[(int64_t)r * ld + i] += d;
}

// ids[i] = g(i)
__global__ void k_segment_ids_i64(int64_t* __restrict__ ids, int64_t n, const int64_t* __restrict__ starts,
                                  int64_t G) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ids[i] = seg_of(starts, G, i);
}

constexpr int kBatchBlock = 256;

}  // namespace mp

using namespace mp;

extern "C" {

int mp_segment_offset_i64(int64_t* data, int64_t ld, int32_t rows, int64_t n, const int64_t* starts,
                          const int64_t* inc, int64_t n_graphs, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n >= 0 && rows >= 0 && n_graphs >= 0, "mp_segment_offset_i64: negative size");
  if (n == 0 || rows == 0) return MP_OK;
  MP_CHECK_ARG(n_graphs > 0, "mp_segment_offset_i64: %lld elements but no graphs", (long long)n);
  MP_CHECK_ARG(data && starts && inc, "mp_segment_offset_i64: null pointer");
  MP_CHECK_ARG(rows == 1 || ld >= n, "mp_segment_offset_i64: ld < n");
  hipLaunchKernelGGL(k_segment_offset_i64, dim3((unsigned)((n + kBatchBlock - 1) / kBatchBlock)), dim3(kBatchBlock),
                     0, as_stream(stream), data, ld, rows, n, starts, inc, n_graphs);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_segment_ids_i64(int64_t* ids, int64_t n, const int64_t* starts, int64_t n_graphs, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n >= 0 && n_graphs >= 0, "mp_segment_ids_i64: negative size");
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(n_graphs > 0, "mp_segment_ids_i64: %lld elements but no graphs", (long long)n);
  MP_CHECK_ARG(ids && starts, "mp_segment_ids_i64: null pointer");
  hipLaunchKernelGGL(k_segment_ids_i64, dim3((unsigned)((n + kBatchBlock - 1) / kBatchBlock)), dim3(kBatchBlock), 0,
                     as_stream(stream), ids, n, starts, n_graphs);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
