// CSR build + edge-balanced schedule for the aggregation engine (gfx950).
//
// Upstream torch_scatter 2.0.4 scatter_sum is `out.scatter_add_(dim, index, src)`
// over edges in their original order ([U8]); the CUDA version is one
// atomicAdd per element.  Here the aggregation index is sorted ONCE (stable, so
// each row keeps its edges in original order — the order the CPU oracle sums
// in), and every later aggregation is a deterministic segmented reduction.
#include <stdarg.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "mp_common.h"

namespace mp {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---------------------------------------------------------------------------
// CSR build kernels
// ---------------------------------------------------------------------------

__global__ void k_prepare_keys(const int64_t* __restrict__ key, const int64_t* __restrict__ other,
                               int64_t n_edges, int64_t n_rows, int64_t n_other,
                               uint32_t* __restrict__ keys32, int32_t* __restrict__ vals,
                               int32_t* __restrict__ bad) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int nbad = 0;
  if (e < n_edges) {
    int64_t k = key[e];
    if (k < 0 || k >= n_rows) {
      nbad++;
      k = 0;
    }
    if (other != nullptr) {
      int64_t o = other[e];
      if (o < 0 || o >= n_other) nbad++;
    }
    keys32[e] = (uint32_t)k;
    vals[e] = (int32_t)e;
  }
  // one atomic per wave with a bad index (never in valid input)
  unsigned long long m = __ballot(nbad != 0);
  if (m != 0 && nbad) atomicAdd(bad, nbad);
}

// rowptr[r] = lower_bound(sorted_keys, r), r in [0, n_rows]
__global__ void k_rowptr(const uint32_t* __restrict__ ks, int64_t n_edges, int64_t n_rows,
                         int32_t* __restrict__ rowptr) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n_rows) return;
  int64_t lo = 0, hi = n_edges;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if ((int64_t)ks[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = (int32_t)lo;
}

__global__ void k_gather_col(const int64_t* __restrict__ other, const int32_t* __restrict__ eid,
                             int64_t n_edges, int32_t* __restrict__ col) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_edges) return;
  int32_t e = eid[k];
  col[k] = other ? (int32_t)other[e] : e;
}

static unsigned bits_for(int64_t n_rows) {
  unsigned b = 1;
  while (b < 32 && ((int64_t)1 << b) < n_rows) b++;
  return b;
}

static size_t sort_temp_bytes(int64_t n_edges, int64_t n_rows) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                            (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n_edges, 0,
                            bits_for(n_rows), (hipStream_t)0, false);
  return bytes;
}

// ---------------------------------------------------------------------------
// Schedule kernels
// ---------------------------------------------------------------------------

// Merge-path split: row r's marker sits at merged position P_r = rowptr[r] + r,
// slot k of row r at k + r + 1.  Task w covers positions [w*chunk, (w+1)*chunk):
//   wave_row[w]  = first r with P_r >= w*chunk           (lower_bound over rows)
//   wave_slot[w] = min(w*chunk - wave_row[w], rowptr[wave_row[w]])
// so every task does at most `chunk` units of (row store | edge gather) work,
// whatever the degree distribution (power-law hubs, runs of empty rows).
// Snap: when the boundary falls inside a row of at most `snap` slots, it is
// moved back to that row's marker, so the row is not split (a task then does
// at most chunk + snap units; snap < chunk keeps the starts increasing).
// Only rows longer than `snap` (hubs) are ever cut and need a fix-up.
__global__ void k_wave_row(const int32_t* __restrict__ rowptr, int64_t n_rows, int64_t n_edges,
                           int32_t chunk, int32_t snap, int32_t n_waves, int32_t* __restrict__ wave_row,
                           int32_t* __restrict__ wave_slot) {
  int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w > n_waves) return;
  if (w == n_waves) {
    wave_row[w] = (int32_t)n_rows;
    wave_slot[w] = (int32_t)n_edges;
    return;
  }
  if (w == 0) {
    wave_row[0] = 0;
    wave_slot[0] = 0;
    return;
  }
  int64_t target = w * (int64_t)chunk;
  int64_t lo = 0, hi = n_rows;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if ((int64_t)rowptr[mid] + mid < target) lo = mid + 1;
    else hi = mid;
  }
  int64_t slot = target - lo;
  int64_t rs = rowptr[lo];  // rowptr[n_rows] == n_edges
  if (slot < rs && lo > 0) {  // the boundary cuts row lo-1
    int64_t r0 = rowptr[lo - 1];
    if (rs - r0 <= snap) {
      wave_row[w] = (int32_t)(lo - 1);
      wave_slot[w] = (int32_t)r0;
      return;
    }
  }
  wave_row[w] = (int32_t)lo;
  wave_slot[w] = (int32_t)(slot < rs ? slot : rs);
}

// flag[w] = 1 iff task w carries a continuation of a row owned by an earlier
// task AND it is the last task touching that row (that row needs a fix-up).
__global__ void k_split_flags(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ wave_row,
                              const int32_t* __restrict__ wave_slot, int32_t n_waves,
                              uint8_t* __restrict__ flags) {
  int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_waves) return;
  uint8_t f = 0;
  if (w > 0) {
    int32_t r = wave_row[w];
    bool cont = wave_slot[w] < rowptr[r];
    bool next_same = false;
    if (w + 1 < n_waves) {
      int32_t r1 = wave_row[w + 1];
      next_same = (r1 == r) && (wave_slot[w + 1] < rowptr[r1]);
    }
    f = (cont && !next_same) ? 1 : 0;
  }
  flags[w] = f;
}

static size_t select_temp_bytes(int32_t n_waves) {
  size_t bytes = 0;
  rocprim::counting_iterator<int32_t> it(0);
  (void)rocprim::select((void*)nullptr, bytes, it, (const uint8_t*)nullptr, (int32_t*)nullptr,
                  (int32_t*)nullptr, (size_t)n_waves, (hipStream_t)0, false);
  return bytes;
}

}  // namespace mp

using namespace mp;

extern "C" {

const char* mp_last_error(void) { return mp::g_err; }

int mp_abi_version(void) { return MP_ABI_VERSION; }

size_t mp_csr_build_workspace(int64_t n_edges, int64_t n_rows) {
  size_t e4 = align_up((size_t)(n_edges > 0 ? n_edges : 1) * 4, 256);
  return 3 * e4 + align_up(sort_temp_bytes(n_edges, n_rows), 256) + 256;
}

int mp_csr_build(const int64_t* key, const int64_t* other, int64_t n_edges, int64_t n_rows,
                 int64_t n_other, int32_t* rowptr, int32_t* col, int32_t* eid, int32_t* bad,
                 void* ws, size_t ws_bytes, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_edges >= 0 && n_rows >= 0, "mp_csr_build: negative size");
  MP_CHECK_ARG(n_edges < (int64_t)INT32_MAX && n_rows < (int64_t)INT32_MAX,
               "mp_csr_build: int32 CSR limits exceeded (E=%lld, N=%lld)", (long long)n_edges,
               (long long)n_rows);
  MP_CHECK_ARG(rowptr && bad && (n_edges == 0 || (key && col && eid)), "mp_csr_build: null pointer");
  MP_CHECK_ARG(ws_bytes >= mp_csr_build_workspace(n_edges, n_rows), "mp_csr_build: workspace too small");
  hipStream_t s = as_stream(stream);
  MP_CHECK_HIP(hipMemsetAsync(bad, 0, sizeof(int32_t), s));
  if (n_edges == 0) {
    MP_CHECK_HIP(hipMemsetAsync(rowptr, 0, (size_t)(n_rows + 1) * sizeof(int32_t), s));
    return MP_OK;
  }
  char* p = (char*)ws;
  size_t e4 = align_up((size_t)n_edges * 4, 256);
  uint32_t* keys32 = (uint32_t*)p; p += e4;
  int32_t* vals = (int32_t*)p; p += e4;
  uint32_t* ks = (uint32_t*)p; p += e4;
  size_t sort_bytes = sort_temp_bytes(n_edges, n_rows);
  void* tmp = p;

  const int B = 256;
  k_prepare_keys<<<ceil_div(n_edges, B), B, 0, s>>>(key, other, n_edges, n_rows, n_other, keys32,
                                                    vals, bad);
  MP_CHECK_LAUNCH();
  MP_CHECK_HIP(rocprim::radix_sort_pairs(tmp, sort_bytes, keys32, ks, vals, eid, (size_t)n_edges, 0,
                                         bits_for(n_rows), s, false));
  k_rowptr<<<ceil_div(n_rows + 1, B), B, 0, s>>>(ks, n_edges, n_rows, rowptr);
  MP_CHECK_LAUNCH();
  k_gather_col<<<ceil_div(n_edges, B), B, 0, s>>>(other, eid, n_edges, col);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int32_t mp_schedule_n_waves(int64_t n_rows, int64_t n_edges, int32_t chunk) {
  if (chunk <= 0) return 0;
  int64_t n = ceil_div(n_rows + n_edges, chunk);
  return (int32_t)(n < 1 ? 1 : n);
}

size_t mp_schedule_workspace(int32_t n_waves) {
  return align_up((size_t)(n_waves > 0 ? n_waves : 1), 256) +
         align_up(select_temp_bytes(n_waves), 256) + 256;
}

int mp_schedule_build(const int32_t* rowptr, int64_t n_rows, int64_t n_edges, int32_t chunk,
                      int32_t snap, int32_t* wave_row, int32_t* wave_slot, int32_t* split_waves,
                      int32_t* n_split_dev, void* ws, size_t ws_bytes, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(chunk >= 16 && chunk % 8 == 0, "mp_schedule_build: chunk must be a multiple of 8, >= 16");
  MP_CHECK_ARG(snap >= 0 && snap < chunk - 1, "mp_schedule_build: need 0 <= snap < chunk - 1");
  MP_CHECK_ARG(rowptr && wave_row && wave_slot && split_waves && n_split_dev,
               "mp_schedule_build: null pointer");
  MP_CHECK_ARG(n_rows + n_edges < (int64_t)INT32_MAX, "mp_schedule_build: N+E exceeds int32");
  int32_t n_waves = mp_schedule_n_waves(n_rows, n_edges, chunk);
  MP_CHECK_ARG(ws_bytes >= mp_schedule_workspace(n_waves), "mp_schedule_build: workspace too small");
  hipStream_t s = as_stream(stream);
  const int B = 256;
  k_wave_row<<<ceil_div((int64_t)n_waves + 1, B), B, 0, s>>>(rowptr, n_rows, n_edges, chunk, snap,
                                                             n_waves, wave_row, wave_slot);
  MP_CHECK_LAUNCH();
  uint8_t* flags = (uint8_t*)ws;
  void* tmp = (char*)ws + align_up((size_t)n_waves, 256);
  k_split_flags<<<ceil_div(n_waves, B), B, 0, s>>>(rowptr, wave_row, wave_slot, n_waves, flags);
  MP_CHECK_LAUNCH();
  size_t sel_bytes = select_temp_bytes(n_waves);
  rocprim::counting_iterator<int32_t> it(0);
  MP_CHECK_HIP(rocprim::select(tmp, sel_bytes, it, flags, split_waves, n_split_dev, (size_t)n_waves, s,
                               false));
  return MP_OK;
}

}  // extern "C"
