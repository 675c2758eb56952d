// torch_scatter 2.0.4 reductions for the other dtypes (gfx950): float64,
// float16, bfloat16, int64 (and float32 through the same code, for tests).
//
// torch_scatter reduces any dtype ([U8/U9]: scatter_cpu.cpp dispatches
// AT_DISPATCH_ALL_TYPES_AND(Half, ...); scatter_sum / scatter_mean are Python
// over scatter_add_).  The fp32 hot path is mp_aggregate_f32; this is the
// breadth path: one wave per (row, 64-feature tile), one feature per lane, the
// row's slots walked in CSR (= original edge) order and never split across
// waves, so every row follows the reference's left-to-right order:
//   * float64 / int64: the reference's arithmetic bit for bit (int64 sums wrap
//     like the CPU's two's-complement adds);
//   * float16 / bfloat16: accumulated in fp32 (the reference adds in the half
//     type, rounding after every add), rounded once to the output type.
// max / min: strict compare in edge order (the first edge wins ties), the
// accumulator starts at the type's lowest() / max(), rows that keep it report
// 0 and arg = n_ids (torch_scatter's `out == init -> 0` fix, also for values
// equal to lowest()).  mean: (sum [+ out]) / max(count, 1), integer division
// truncating toward zero (torch 1.4/1.5 div_ on integer tensors).
#include <float.h>

#include "mp_common.h"

namespace mp {

struct bf16_t {
  uint16_t b;
};

template <class T>
struct Ty;

template <>
struct Ty<float> {
  using A = float;
  __device__ static A ld(const float* p) { return *p; }
  __device__ static float st(A a) { return a; }
  __device__ static A lowest() { return -FLT_MAX; }
  __device__ static A highest() { return FLT_MAX; }
  __device__ static A add(A a, A b) { return __fadd_rn(a, b); }
  __device__ static A div(A a, int64_t c) { return __fdiv_rn(a, (float)c); }
};

template <>
struct Ty<double> {
  using A = double;
  __device__ static A ld(const double* p) { return *p; }
  __device__ static double st(A a) { return a; }
  __device__ static A lowest() { return -DBL_MAX; }
  __device__ static A highest() { return DBL_MAX; }
  __device__ static A add(A a, A b) { return __dadd_rn(a, b); }
  __device__ static A div(A a, int64_t c) { return __ddiv_rn(a, (double)c); }
};

template <>
struct Ty<int64_t> {
  using A = int64_t;
  __device__ static A ld(const int64_t* p) { return *p; }
  __device__ static int64_t st(A a) { return a; }
  __device__ static A lowest() { return INT64_MIN; }
  __device__ static A highest() { return INT64_MAX; }
  __device__ static A add(A a, A b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
  __device__ static A div(A a, int64_t c) { return a / c; }  // truncation toward zero
};

template <>
struct Ty<_Float16> {
  using A = float;
  __device__ static A ld(const _Float16* p) { return (float)*p; }
  __device__ static _Float16 st(A a) { return (_Float16)a; }  // round to nearest even
  __device__ static A lowest() { return -65504.f; }
  __device__ static A highest() { return 65504.f; }
  __device__ static A add(A a, A b) { return __fadd_rn(a, b); }
  __device__ static A div(A a, int64_t c) { return __fdiv_rn(a, (float)c); }
};

template <>
struct Ty<bf16_t> {
  using A = float;
  __device__ static A ld(const bf16_t* p) { return __uint_as_float((uint32_t)p->b << 16); }
  __device__ static bf16_t st(A a) {  // round to nearest even, NaN kept quiet (torch's rule)
    uint32_t u = __float_as_uint(a);
    if ((u & 0x7fffffffu) > 0x7f800000u) return bf16_t{(uint16_t)((u >> 16) | 0x40u)};
    u += 0x7fffu + ((u >> 16) & 1u);
    return bf16_t{(uint16_t)(u >> 16)};
  }
  __device__ static A lowest() { return __uint_as_float(0xff7f0000u); }
  __device__ static A highest() { return __uint_as_float(0x7f7f0000u); }
  __device__ static A add(A a, A b) { return __fadd_rn(a, b); }
  __device__ static A div(A a, int64_t c) { return __fdiv_rn(a, (float)c); }
};

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const int lo = readlane((int)(uint32_t)(uint64_t)v, l);
  const int hi = readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

constexpr int kAnyQ = 4;  // row loads in flight per lane

// RED: 0 sum, 1 mean, 2 max, 3 min
template <class T, int RED>
__global__ __launch_bounds__(256) void k_seg_any(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                 const int32_t* __restrict__ eid, int64_t n_rows, int64_t n_ids,
                                                 const T* __restrict__ src, int64_t lds, int32_t F, int32_t flags,
                                                 T* __restrict__ out, int64_t ldo, int64_t* __restrict__ arg) {
  using A = typename Ty<T>::A;
  const int lane = lane_id();
  const int f = blockIdx.y * 64 + lane;
  const bool fv = f < F;
  const int fc = fv ? f : 0;
  const bool init_out = (flags & MP_FLAG_INIT_FROM_OUT) != 0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_rows; r += nw) {
    const int b = rowptr[r], e = rowptr[r + 1];
    A acc;
    if (init_out && fv) acc = Ty<T>::ld(out + r * ldo + f);
    else if (RED == 2) acc = Ty<T>::lowest();
    else if (RED == 3) acc = Ty<T>::highest();
    else acc = (A)0;
    int64_t a = n_ids;
    for (int k0 = b; k0 < e; k0 += 64) {
      const int kk = k0 + lane < e ? k0 + lane : b;
      const int c = col ? col[kk] : kk;
      const int id = eid ? eid[kk] : kk;
      const int n = uni(e - k0 < 64 ? e - k0 : 64);
      for (int i0 = 0; i0 < n; i0 += kAnyQ) {
        A v[kAnyQ];
#pragma unroll
        for (int q = 0; q < kAnyQ; ++q) {
          const int i = i0 + q < n ? i0 + q : i0;
          v[q] = Ty<T>::ld(src + (int64_t)readlane(c, i) * lds + fc);
        }
#pragma unroll
        for (int q = 0; q < kAnyQ; ++q) {
          if (i0 + q < n) {
            if (RED <= 1) {
              acc = Ty<T>::add(acc, v[q]);
            } else if (RED == 2 ? v[q] > acc : v[q] < acc) {
              acc = v[q];
              a = readlane(id, i0 + q);
            }
          }
        }
      }
    }
    if (!fv) continue;
    A res = acc;
    if (RED == 1) {
      const int64_t cnt = e - b;
      res = Ty<T>::div(acc, cnt > 1 ? cnt : 1);
    } else if (RED >= 2) {
      if (!init_out && acc == (RED == 2 ? Ty<T>::lowest() : Ty<T>::highest())) res = (A)0;
      if (flags & MP_FLAG_PYG_MASK) {
        if (RED == 2 && res < (A)-10000) res = (A)0;
        if (RED == 3 && res > (A)10000) res = (A)0;
      }
      if (arg) arg[r * F + f] = a;
    }
    out[r * ldo + f] = Ty<T>::st(res);
  }
}

template <class T>
static int launch_seg(const mp_csr* g, const void* src, int64_t lds, int32_t F, int32_t reduce, int32_t flags, void* out,
                      int64_t ldo, int64_t* arg, hipStream_t s) {
  int64_t bx = ceil_div(g->n_rows, 4);
  if (bx > 65536) bx = 65536;
  dim3 grid((unsigned)bx, (unsigned)ceil_div(F, 64));
  const int64_t n_ids = g->n_ids > 0 ? g->n_ids : g->n_edges;
  const T* x = static_cast<const T*>(src);
  T* o = static_cast<T*>(out);
  switch (reduce) {
    case MP_REDUCE_SUM:
      k_seg_any<T, 0><<<grid, 256, 0, s>>>(g->rowptr, g->col, g->eid, g->n_rows, n_ids, x, lds, F, flags, o, ldo, arg);
      break;
    case MP_REDUCE_MEAN:
      k_seg_any<T, 1><<<grid, 256, 0, s>>>(g->rowptr, g->col, g->eid, g->n_rows, n_ids, x, lds, F, flags, o, ldo, arg);
      break;
    case MP_REDUCE_MAX:
      k_seg_any<T, 2><<<grid, 256, 0, s>>>(g->rowptr, g->col, g->eid, g->n_rows, n_ids, x, lds, F, flags, o, ldo, arg);
      break;
    default:
      k_seg_any<T, 3><<<grid, 256, 0, s>>>(g->rowptr, g->col, g->eid, g->n_rows, n_ids, x, lds, F, flags, o, ldo, arg);
      break;
  }
  MP_CHECK_LAUNCH();
  return MP_OK;
}

// out[k, :] = x[idx[k], :] for rows of `elem` bytes per element (2, 4 or 8)
template <class U>
__global__ __launch_bounds__(256) void k_gather_any(const U* __restrict__ x, int64_t ldx, const int64_t* __restrict__ idx,
                                                    int64_t n, int64_t W, U* __restrict__ out, int64_t ldo) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += nw) {
    const U* xr = x + idx[k] * ldx;
    U* orow = out + k * ldo;
    for (int64_t f = lane; f < W; f += 64) orow[f] = xr[f];
  }
}

// grad[arg[r, f], f] = grad_out[r, f] for arg in [0, n_edges) (ScatterMax
// backward on materialised messages: a plain store, each (e, f) written at most once)
template <class U>
__global__ void k_scatter_arg_any(const U* __restrict__ g, const int64_t* __restrict__ arg, int64_t n_rows, int32_t F,
                                  int64_t n_edges, U* __restrict__ grad, int64_t ldg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows * (int64_t)F) return;
  const int64_t e = arg[i];
  if (e < 0 || e >= n_edges) return;
  grad[e * ldg + (i % F)] = g[i];
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_segment_reduce(const mp_csr* g, int32_t dtype, const void* src, int64_t lds, int32_t F, int32_t reduce,
                      int32_t flags, void* out, int64_t ldo, int64_t* arg_out, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(g && g->rowptr && g->n_rows >= 0 && g->n_edges >= 0 && F >= 0, "mp_segment_reduce: bad graph");
  MP_CHECK_ARG(reduce >= MP_REDUCE_SUM && reduce <= MP_REDUCE_MIN, "mp_segment_reduce: unknown reduce %d", reduce);
  MP_CHECK_ARG(dtype >= MP_DTYPE_F32 && dtype <= MP_DTYPE_I64, "mp_segment_reduce: unknown dtype %d", dtype);
  if (g->n_rows == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(out && ldo >= F, "mp_segment_reduce: bad output");
  MP_CHECK_ARG(g->n_edges == 0 || (src && lds >= F), "mp_segment_reduce: bad source");
  MP_CHECK_ARG(g->col == nullptr || g->n_cols > 0, "mp_segment_reduce: n_cols required with col");
  const bool is_arg = reduce == MP_REDUCE_MAX || reduce == MP_REDUCE_MIN;
  MP_CHECK_ARG(!is_arg || arg_out, "mp_segment_reduce: max/min need arg_out");
  MP_CHECK_ARG(!is_arg || g->eid || g->n_edges == 0, "mp_segment_reduce: max/min need eid");
  hipStream_t s = as_stream(stream);
  int64_t* arg = is_arg ? arg_out : nullptr;
  switch (dtype) {
    case MP_DTYPE_F32: return launch_seg<float>(g, src, lds, F, reduce, flags, out, ldo, arg, s);
    case MP_DTYPE_F64: return launch_seg<double>(g, src, lds, F, reduce, flags, out, ldo, arg, s);
    case MP_DTYPE_F16: return launch_seg<_Float16>(g, src, lds, F, reduce, flags, out, ldo, arg, s);
    case MP_DTYPE_BF16: return launch_seg<bf16_t>(g, src, lds, F, reduce, flags, out, ldo, arg, s);
    default: return launch_seg<int64_t>(g, src, lds, F, reduce, flags, out, ldo, arg, s);
  }
}

int mp_gather_rows_any(int32_t elem_bytes, const void* x, int64_t ldx, const int64_t* idx, int64_t n, int32_t F,
                       void* out, int64_t ldo, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8, "mp_gather_rows_any: element size %d", elem_bytes);
  MP_CHECK_ARG(n >= 0 && F >= 0, "mp_gather_rows_any: negative size");
  if (n == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(x && idx && out && ldx >= F && ldo >= F, "mp_gather_rows_any: bad argument");
  int64_t blocks = ceil_div(n, 4);
  if (blocks > 16384) blocks = 16384;
  hipStream_t s = as_stream(stream);
  if (elem_bytes == 2)
    k_gather_any<uint16_t><<<(unsigned)blocks, 256, 0, s>>>((const uint16_t*)x, ldx, idx, n, F, (uint16_t*)out, ldo);
  else if (elem_bytes == 4)
    k_gather_any<uint32_t><<<(unsigned)blocks, 256, 0, s>>>((const uint32_t*)x, ldx, idx, n, F, (uint32_t*)out, ldo);
  else
    k_gather_any<uint64_t><<<(unsigned)blocks, 256, 0, s>>>((const uint64_t*)x, ldx, idx, n, F, (uint64_t*)out, ldo);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_scatter_arg_any(int32_t elem_bytes, const void* grad_out, const int64_t* arg, int64_t n_rows, int32_t F,
                       int64_t n_edges, void* grad, int64_t ldg, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8, "mp_scatter_arg_any: element size %d", elem_bytes);
  if (n_rows == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(grad_out && arg && grad && ldg >= F, "mp_scatter_arg_any: bad argument");
  const int64_t total = n_rows * (int64_t)F;
  hipStream_t s = as_stream(stream);
  const unsigned blocks = (unsigned)ceil_div(total, 256);
  if (elem_bytes == 2)
    k_scatter_arg_any<uint16_t><<<blocks, 256, 0, s>>>((const uint16_t*)grad_out, arg, n_rows, F, n_edges,
                                                       (uint16_t*)grad, ldg);
  else if (elem_bytes == 4)
    k_scatter_arg_any<uint32_t><<<blocks, 256, 0, s>>>((const uint32_t*)grad_out, arg, n_rows, F, n_edges,
                                                       (uint32_t*)grad, ldg);
  else
    k_scatter_arg_any<uint64_t><<<blocks, 256, 0, s>>>((const uint64_t*)grad_out, arg, n_rows, F, n_edges,
                                                       (uint64_t*)grad, ldg);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
