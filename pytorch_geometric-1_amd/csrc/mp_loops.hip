// Self-loop rewrites of edge_index on the device (PyG 1.4.3 utils.loop [U4],
// SURVEY a7 / 8f-2): remove_self_loops, add_self_loops and
// add_remaining_self_loops as a stable compaction of the non-loop edges
// (rocPRIM select: original order kept) followed by the N loop edges 0..N-1.
//
// Upstream add_remaining_self_loops sets the loop weights with
// `loop_weight[row[inv_mask]] = edge_weight[inv_mask]`, a sequential
// index_put_ on the CPU: with duplicate self loops of one node the LAST one's
// weight wins.  Here every output edge carries the position of the input edge
// its weight comes from (pos[k]; -1 = fill value), and a node's loop takes
// the largest loop position (atomicMax over int32 positions) -- the same
// choice, deterministic.  Weights are then one gather (mp_gather_fill_f32).
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "mp_common.h"

namespace mp {

// count[0] = self loops; count[1] = self loops (r, r) with r outside [0, n_nodes)
// (upstream's `loop_weight[row[inv_mask]]` raises an IndexError for those)
__global__ void k_loop_count(const int64_t* __restrict__ row, const int64_t* __restrict__ col, int64_t n,
                             int64_t n_nodes, unsigned long long* __restrict__ count) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = e < n ? row[e] : 0;
  const bool loop = e < n && r == col[e];
  const unsigned long long m = __ballot(loop);
  const unsigned long long bad = __ballot(loop && (r < 0 || r >= n_nodes));
  if (lane_id() == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
  if (lane_id() == 0 && bad) atomicAdd(count + 1, (unsigned long long)__popcll(bad));
}

__global__ void k_loop_flags(const int64_t* __restrict__ row, const int64_t* __restrict__ col, int64_t n,
                             int64_t n_nodes, uint8_t* __restrict__ keep, int32_t* __restrict__ last) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t r = row[e];
  const bool loop = r == col[e];
  keep[e] = loop ? 0 : 1;
  // the range guard keeps a bad index from writing outside `last`; the caller has
  // already rejected it through mp_self_loop_count's out-of-range count
  if (loop && last && r >= 0 && r < n_nodes) atomicMax(last + r, (int32_t)e);
}

// out[k] = edge pos[k] for k < n_kept (pos == nullptr: identity), then the
// loops n = 0..N-1 at n_kept + n with pos = last loop of n (or -1)
__global__ void k_loop_emit(const int64_t* __restrict__ row, const int64_t* __restrict__ col, int64_t n_kept,
                            int64_t n_loops, const int32_t* __restrict__ last, int64_t* __restrict__ out_row,
                            int64_t* __restrict__ out_col, int64_t* __restrict__ pos, bool identity) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_kept) {
    const int64_t p = identity ? k : pos[k];
    out_row[k] = row[p];
    out_col[k] = col[p];
    if (identity && pos) pos[k] = k;
  } else if (k < n_kept + n_loops) {
    const int64_t v = k - n_kept;
    out_row[k] = v;
    out_col[k] = v;
    if (pos) pos[k] = last ? (int64_t)last[v] : -1;
  }
}

__global__ void k_gather_fill(const float* __restrict__ src, const int64_t* __restrict__ pos, int64_t n, float fill,
                              float* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int64_t p = pos[k];
  out[k] = p >= 0 ? src[p] : fill;
}

static size_t loop_select_bytes(int64_t n) {
  size_t bytes = 0;
  rocprim::counting_iterator<int64_t> it(0);
  (void)rocprim::select((void*)nullptr, bytes, it, (const uint8_t*)nullptr, (int64_t*)nullptr,
                        (unsigned long long*)nullptr, (size_t)(n > 0 ? n : 1), (hipStream_t)0, false);
  return bytes;
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_self_loop_count(const int64_t* row, const int64_t* col, int64_t n_edges, int64_t n_nodes, int64_t* count_dev,
                       void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && count_dev && (n_edges == 0 || (row && col)),
               "mp_self_loop_count: bad arguments");
  hipStream_t s = as_stream(stream);
  MP_CHECK_HIP(hipMemsetAsync(count_dev, 0, 2 * sizeof(int64_t), s));
  if (n_edges == 0) return MP_OK;
  const int B = 256;
  k_loop_count<<<ceil_div(n_edges, B), B, 0, s>>>(row, col, n_edges, n_nodes,
                                                  reinterpret_cast<unsigned long long*>(count_dev));
  MP_CHECK_LAUNCH();
  return MP_OK;
}

size_t mp_self_loops_workspace(int64_t n_edges, int64_t n_nodes) {
  const size_t e = (size_t)(n_edges > 0 ? n_edges : 1);
  const size_t n = (size_t)(n_nodes > 0 ? n_nodes : 1);
  return align_up(e, 256) + align_up(n * 4, 256) + align_up(8, 256) + align_up(loop_select_bytes(n_edges), 256) + 256;
}

int mp_self_loops(const int64_t* row, const int64_t* col, int64_t n_edges, int64_t n_nodes, int32_t mode,
                  int64_t n_kept, int64_t* out_row, int64_t* out_col, int64_t* out_pos, void* ws, size_t ws_bytes,
                  void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(mode == MP_LOOPS_REMOVE || mode == MP_LOOPS_ADD || mode == MP_LOOPS_ADD_REMAINING,
               "mp_self_loops: unknown mode %d", mode);
  MP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_kept >= 0 && n_kept <= n_edges, "mp_self_loops: bad sizes");
  MP_CHECK_ARG(mode != MP_LOOPS_ADD || n_kept == n_edges, "mp_self_loops: add keeps every edge (n_kept == n_edges)");
  MP_CHECK_ARG(n_edges < (int64_t)INT32_MAX, "mp_self_loops: more than 2^31 edges");
  const int64_t n_loops = mode == MP_LOOPS_REMOVE ? 0 : n_nodes;
  const int64_t n_out = n_kept + n_loops;
  MP_CHECK_ARG(n_out == 0 || (out_row && out_col), "mp_self_loops: null output");
  MP_CHECK_ARG(n_edges == 0 || (row && col), "mp_self_loops: null input");
  MP_CHECK_ARG(mode == MP_LOOPS_ADD || out_pos || n_kept == 0 || n_kept == n_edges,
               "mp_self_loops: out_pos is needed as the compaction buffer");
  MP_CHECK_ARG(ws && ws_bytes >= mp_self_loops_workspace(n_edges, n_nodes), "mp_self_loops: workspace too small");
  hipStream_t s = as_stream(stream);
  if (n_out == 0) return MP_OK;
  char* p = (char*)ws;
  uint8_t* keep = (uint8_t*)p;
  p += align_up((size_t)(n_edges > 0 ? n_edges : 1), 256);
  int32_t* last = (int32_t*)p;
  p += align_up((size_t)(n_nodes > 0 ? n_nodes : 1) * 4, 256);
  unsigned long long* n_sel = (unsigned long long*)p;
  p += align_up(8, 256);
  void* tmp = p;
  const int B = 256;
  const bool remaining = mode == MP_LOOPS_ADD_REMAINING;
  const bool identity = mode == MP_LOOPS_ADD || n_kept == n_edges;
  if (remaining && n_nodes > 0) MP_CHECK_HIP(hipMemsetAsync(last, 0xff, (size_t)n_nodes * 4, s));  // -1
  if (n_edges > 0 && (remaining || !identity)) {
    k_loop_flags<<<ceil_div(n_edges, B), B, 0, s>>>(row, col, n_edges, n_nodes, keep, remaining ? last : nullptr);
    MP_CHECK_LAUNCH();
  }
  if (!identity) {
    size_t sel_bytes = loop_select_bytes(n_edges);
    rocprim::counting_iterator<int64_t> it(0);
    MP_CHECK_HIP(rocprim::select(tmp, sel_bytes, it, keep, out_pos, n_sel, (size_t)n_edges, s, false));
  }
  k_loop_emit<<<ceil_div(n_out, B), B, 0, s>>>(row, col, n_kept, n_loops, remaining ? last : nullptr, out_row,
                                               out_col, out_pos, identity);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gather_fill_f32(const float* src, const int64_t* pos, int64_t n, float fill, float* out, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n >= 0 && (n == 0 || (pos && out)), "mp_gather_fill_f32: bad arguments");
  if (n == 0) return MP_OK;
  hipStream_t s = as_stream(stream);
  const int B = 256;
  k_gather_fill<<<ceil_div(n, B), B, 0, s>>>(src, pos, n, fill, out);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
