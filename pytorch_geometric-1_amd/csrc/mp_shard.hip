// Shard-plan build on the device (SURVEY 8e / 8f-2 "halo maps"): for rank p
// owning the key rows [lo, hi) of a destination-range partition,
//   edge_pos     = positions of the edges whose key lies in [lo, hi), in the
//                  global edge order (rocPRIM stable select),
//   halo_nodes   = the sorted unique remote `other` endpoints of those edges,
//   local ids    = key - lo, and other - lo (owned) or n_own + halo index,
//   recv_counts  = halo nodes per owner rank (halo_nodes are sorted, so they
//                  are grouped by owner).
// No sort: remote endpoints are flagged in an [N] array and an exclusive scan
// of the flags is both the halo index of every node and, read at the cut
// points, the per-owner counts -- O(E + N), deterministic.
// Replaces the torch-op plan of mi355_mp.dist.ShardPlan (nonzero / unique /
// searchsorted) for device edge lists.
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "mp_common.h"

namespace mp {

__global__ void k_plan_flags(const int64_t* __restrict__ key, const int64_t* __restrict__ other, int64_t n,
                             int64_t n_nodes, int64_t lo, int64_t hi, uint8_t* __restrict__ keep,
                             int32_t* __restrict__ flag, int32_t* __restrict__ bad) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t k = key[e];
  const bool mine = k >= lo && k < hi;
  keep[e] = mine ? 1 : 0;
  if (mine) {
    const int64_t o = other[e];
    if (o < 0 || o >= n_nodes) {
      *bad = 1;  // reported through counts[1] = -1
    } else if (o < lo || o >= hi) {
      flag[o] = 1;  // every writer stores the same value
    }
  }
}

__global__ void k_plan_halo(const int32_t* __restrict__ flag, const int32_t* __restrict__ hidx, int64_t n_nodes,
                            int64_t* __restrict__ halo_nodes) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n_nodes && flag[v]) halo_nodes[hidx[v]] = v;
}

// local ids of the selected edges; n_sel is read on the device (the grid
// covers the upper bound n_edges)
__global__ void k_plan_local(const int64_t* __restrict__ key, const int64_t* __restrict__ other,
                             const int64_t* __restrict__ edge_pos, const unsigned long long* __restrict__ n_sel,
                             int64_t n_nodes, int64_t lo, int64_t hi, const int32_t* __restrict__ hidx,
                             int64_t* __restrict__ local_key, int64_t* __restrict__ local_other) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)*n_sel) return;
  const int64_t p = edge_pos[k];
  const int64_t o = other[p];
  local_key[k] = key[p] - lo;
  local_other[k] = (o >= lo && o < hi) ? o - lo : (o >= 0 && o < n_nodes) ? (hi - lo) + (int64_t)hidx[o] : -1;
}

// counts[0] = selected edges, counts[1] = halo nodes (-1: an `other` index of
// a selected edge lies outside [0, n_nodes)), counts[2 + q] = halo nodes owned
// by rank q (cuts[q] <= v < cuts[q + 1])
__global__ void k_plan_counts(const int32_t* __restrict__ flag, const int32_t* __restrict__ hidx, int64_t n_nodes,
                              const int64_t* __restrict__ cuts, int32_t world,
                              const unsigned long long* __restrict__ n_sel, const int32_t* __restrict__ bad,
                              int64_t* __restrict__ counts) {
  const int q = (int)threadIdx.x;
  const int64_t total = n_nodes > 0 ? (int64_t)hidx[n_nodes - 1] + flag[n_nodes - 1] : 0;
  auto before = [&](int64_t c) -> int64_t { return c >= n_nodes ? total : (c <= 0 ? 0 : (int64_t)hidx[c]); };
  if (q == 0) {
    counts[0] = (int64_t)*n_sel;
    counts[1] = *bad ? -1 : total;
  }
  if (q < world) counts[2 + q] = before(cuts[q + 1]) - before(cuts[q]);
}

static size_t plan_select_bytes(int64_t n) {
  size_t bytes = 0;
  rocprim::counting_iterator<int64_t> it(0);
  (void)rocprim::select((void*)nullptr, bytes, it, (const uint8_t*)nullptr, (int64_t*)nullptr,
                        (unsigned long long*)nullptr, (size_t)(n > 0 ? n : 1), (hipStream_t)0, false);
  return bytes;
}

static size_t plan_scan_bytes(int64_t n) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan((void*)nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                                (size_t)(n > 0 ? n : 1), rocprim::plus<int32_t>(), (hipStream_t)0, false);
  return bytes;
}

}  // namespace mp

using namespace mp;

extern "C" {

size_t mp_shard_plan_workspace(int64_t n_edges, int64_t n_nodes) {
  const size_t e = (size_t)(n_edges > 0 ? n_edges : 1);
  const size_t n = (size_t)(n_nodes > 0 ? n_nodes : 1);
  const size_t tmp = std::max(plan_select_bytes(n_edges), plan_scan_bytes(n_nodes));
  return align_up(e, 256) + 2 * align_up(n * 4, 256) + 2 * align_up(8, 256) + align_up(tmp, 256) + 256;
}

int mp_shard_plan(const int64_t* key, const int64_t* other, int64_t n_edges, int64_t n_nodes, const int64_t* cuts,
                  int32_t world, int32_t rank, int64_t lo, int64_t hi, int64_t* edge_pos, int64_t* local_key,
                  int64_t* local_other, int64_t* halo_nodes, int64_t* counts, void* ws, size_t ws_bytes,
                  void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_nodes < (int64_t)INT32_MAX, "mp_shard_plan: bad sizes");
  MP_CHECK_ARG(world >= 1 && world <= 1024 && rank >= 0 && rank < world, "mp_shard_plan: bad rank / world");
  MP_CHECK_ARG(0 <= lo && lo <= hi && hi <= n_nodes, "mp_shard_plan: [lo, hi) outside [0, n_nodes)");
  MP_CHECK_ARG(cuts && counts, "mp_shard_plan: null cuts / counts");
  MP_CHECK_ARG(n_edges == 0 || (key && other && edge_pos && local_key && local_other),
               "mp_shard_plan: null edge array");
  MP_CHECK_ARG(n_nodes == 0 || halo_nodes, "mp_shard_plan: null halo_nodes");
  MP_CHECK_ARG(ws && ws_bytes >= mp_shard_plan_workspace(n_edges, n_nodes), "mp_shard_plan: workspace too small");
  hipStream_t s = as_stream(stream);
  char* p = (char*)ws;
  uint8_t* keep = (uint8_t*)p;
  p += align_up((size_t)(n_edges > 0 ? n_edges : 1), 256);
  int32_t* flag = (int32_t*)p;
  p += align_up((size_t)(n_nodes > 0 ? n_nodes : 1) * 4, 256);
  int32_t* hidx = (int32_t*)p;
  p += align_up((size_t)(n_nodes > 0 ? n_nodes : 1) * 4, 256);
  unsigned long long* n_sel = (unsigned long long*)p;
  p += align_up(8, 256);
  int32_t* bad = (int32_t*)p;
  p += align_up(8, 256);
  void* tmp = p;
  const int B = 256;
  MP_CHECK_HIP(hipMemsetAsync(n_sel, 0, 8, s));
  MP_CHECK_HIP(hipMemsetAsync(bad, 0, 4, s));
  if (n_nodes > 0) MP_CHECK_HIP(hipMemsetAsync(flag, 0, (size_t)n_nodes * 4, s));
  if (n_edges > 0) {
    k_plan_flags<<<ceil_div(n_edges, B), B, 0, s>>>(key, other, n_edges, n_nodes, lo, hi, keep, flag, bad);
    MP_CHECK_LAUNCH();
    size_t sel_bytes = plan_select_bytes(n_edges);
    rocprim::counting_iterator<int64_t> it(0);
    MP_CHECK_HIP(rocprim::select(tmp, sel_bytes, it, keep, edge_pos, n_sel, (size_t)n_edges, s, false));
  }
  if (n_nodes > 0) {
    size_t scan_bytes = plan_scan_bytes(n_nodes);
    MP_CHECK_HIP(rocprim::exclusive_scan(tmp, scan_bytes, flag, hidx, 0, (size_t)n_nodes, rocprim::plus<int32_t>(),
                                         s, false));
    k_plan_halo<<<ceil_div(n_nodes, B), B, 0, s>>>(flag, hidx, n_nodes, halo_nodes);
    MP_CHECK_LAUNCH();
  }
  if (n_edges > 0) {
    k_plan_local<<<ceil_div(n_edges, B), B, 0, s>>>(key, other, edge_pos, n_sel, n_nodes, lo, hi, hidx,
                                                    local_key, local_other);
    MP_CHECK_LAUNCH();
  }
  k_plan_counts<<<1, 1024, 0, s>>>(flag, hidx, n_nodes, cuts, world, n_sel, bad, counts);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
