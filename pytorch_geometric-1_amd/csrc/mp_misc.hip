// Row gather, permutation, ScatterMax backward, GCN normalisation and the GAT
// node-score GEMV: the small kernels around the fused aggregation (gfx950).
#include <float.h>

#include "mp_common.h"

namespace mp {

// out[k,:] = x[idx[k],:]; one wave per row, VEC features per lane, grid-stride.
template <int VEC>
__global__ __launch_bounds__(256) void k_gather_rows(const float* __restrict__ x, int64_t ldx,
                                                      const int64_t* __restrict__ idx, int64_t n,
                                                      int32_t F, float* __restrict__ out, int64_t ldo) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += nw) {
    const int64_t src = idx[k];
    const float* xr = x + src * ldx;
    float* orow = out + k * ldo;
    for (int f = lane * VEC; f < F; f += 64 * VEC) store_frag<VEC>(orow + f, load_frag<VEC>(xr + f));
  }
}

__global__ void k_permute(const float* __restrict__ src, const int32_t* __restrict__ perm, int64_t n,
                          float* __restrict__ dst) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) dst[k] = src[perm[k]];
}

// torch_scatter ScatterMax.backward [U8] on materialised message rows:
//   grad_src = zeros(E+1, F).scatter_(0, arg, grad_out)[:E]
// Message row e belongs to exactly one output row, so each (e, f) is stored by
// at most one (r, f): plain stores, no atomics, deterministic.  (A fused
// message w_e * x_j has the CSR form: mp_scatter_arg_backward_csr_f32.)
__global__ void k_scatter_arg_backward(const float* __restrict__ grad_out, const int64_t* __restrict__ arg,
                                       int64_t n_rows, int32_t F, int64_t n_edges, float* __restrict__ grad,
                                       int64_t ldg) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows * (int64_t)F) return;
  const int64_t e = arg[i];
  if (e < 0 || e >= n_edges) return;
  const int f = (int)(i % F);
  grad[e * ldg + f] = grad_out[i];
}

// GCNConv.norm [U5], step 1: deg = scatter_add(edge_weight, row)
__global__ void k_gcn_degree(const int64_t* __restrict__ row, const float* __restrict__ w, int64_t n_edges,
                             float* __restrict__ deg) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n_edges) atomicAdd(deg + row[e], w ? w[e] : 1.f);
}

// Correctly rounded fp32 sqrt and reciprocal, exact on any hardware sqrt / div
// accuracy: a double-precision estimate rounded to float, then checked against
// the rounding midpoints with products that are exact in double (a 26-bit
// midpoint squared, or times a 24-bit float, fits 53 bits) and moved by one ulp
// if needed.  (gfx950's fp32 __fsqrt_rn is not correctly rounded: 426 of 3000
// real-valued degrees came out one ulp off torch's CPU pow(-0.5).)
__device__ __forceinline__ float f_next(float v) { return __int_as_float(__float_as_int(v) + 1); }
__device__ __forceinline__ float f_prev(float v) { return __int_as_float(__float_as_int(v) - 1); }
// half the distance to the next float above / below a positive normal v
__device__ __forceinline__ double half_ulp_up(float v) {
  const int e = (__float_as_int(v) >> 23) & 0xff;
  return ldexp(1.0, (e ? e : 1) - 127 - 24);
}
__device__ __forceinline__ double half_ulp_down(float v) {
  const int b = __float_as_int(v);
  const int e = (b >> 23) & 0xff;
  return ldexp(1.0, (e ? e : 1) - 127 - 24 - ((b & 0x7fffff) == 0 && e > 1 ? 1 : 0));
}

__device__ float sqrt_rn_exact(float x) {
  if (!(x > 0.f) || isinf(x)) return sqrtf(x);  // 0, negative, NaN, inf: the IEEE special cases
  const double xd = x;
  float s = (float)sqrt(xd);
  for (int it = 0; it < 3; ++it) {
    const double sd = s, lo = sd - half_ulp_down(s), hi = sd + half_ulp_up(s);
    if (lo * lo > xd) s = f_prev(s);
    else if (hi * hi < xd) s = f_next(s);
    else break;
  }
  return s;
}

__device__ float rcp_rn_exact(float s) {
  if (!(s > 0.f) || isinf(s)) return 1.f / s;  // 0 -> inf, inf -> 0, NaN, negatives (not a degree)
  const double sd = s;
  float q = (float)(1.0 / sd);
  for (int it = 0; it < 3; ++it) {
    const double qd = q, lo = qd - half_ulp_down(q), hi = qd + half_ulp_up(q);
    if (lo * sd > 1.0) q = f_prev(q);
    else if (hi * sd < 1.0) q = f_next(q);
    else break;
  }
  return q;
}

// step 2: deg^-0.5 as torch's CPU pow(-0.5) computes it, 1 / sqrt(deg) with a
// correctly rounded sqrt, then a correctly rounded division; inf -> 0.
__global__ void k_gcn_dinv(float* __restrict__ deg, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float d = rcp_rn_exact(sqrt_rn_exact(deg[i]));
  deg[i] = isinf(d) ? 0.f : d;
}

// step 3: norm = dinv[row] * w * dinv[col] (left to right, as written upstream)
__global__ void k_gcn_norm(const int64_t* __restrict__ row, const int64_t* __restrict__ col,
                           const float* __restrict__ w, int64_t n_edges, const float* __restrict__ dinv,
                           float* __restrict__ norm) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_edges) return;
  float v = __fmul_rn(dinv[row[e]], w ? w[e] : 1.f);
  norm[e] = __fmul_rn(v, dinv[col[e]]);
}

// a_dst[n,h] = sum_c xw[n,h,c]*att[h,c]; a_src[n,h] = sum_c xw[n,h,c]*att[h,C+c]
// one thread per (n,h); the att row of a head is wave-shared (L1/LDS-served).
__global__ void k_gat_node_scores(const float* __restrict__ xw, int64_t n_nodes, int32_t H, int32_t C,
                                  const float* __restrict__ att, float* __restrict__ a_src,
                                  float* __restrict__ a_dst) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes * (int64_t)H) return;
  const int h = (int)(i % H);
  const float* xr = xw + i * C;  // [n, h, :] is contiguous
  const float* ai = att + (int64_t)h * 2 * C;
  float sd = 0.f, ss = 0.f;
  for (int c = 0; c < C; ++c) {
    float v = xr[c];
    sd += v * ai[c];
    ss += v * ai[C + c];
  }
  a_dst[i] = sd;
  a_src[i] = ss;
}

// Wave-per-node form (C % 4 == 0, G = C/4 lanes per head a power of two
// <= 64): one coalesced 1 KiB pass per 256 features, per-lane partial dot
// products, then a shuffle-xor reduction inside each G-lane head group.
__global__ __launch_bounds__(256) void k_gat_node_scores_wave(const float* __restrict__ xw, int64_t n_nodes,
                                                               int32_t H, int32_t C, int32_t G,
                                                               const float* __restrict__ att,
                                                               float* __restrict__ a_src,
                                                               float* __restrict__ a_dst) {
  const int lane = lane_id();
  const int64_t HC = (int64_t)H * C;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); n < n_nodes; n += nw) {
    for (int64_t base = 0; base < HC; base += 256) {
      const int64_t f = base + lane * 4;
      float sd = 0.f, ss = 0.f;
      int h = 0;
      if (f < HC) {
        h = (int)(f / C);
        const int c = (int)(f % C);
        f32x4 v = *reinterpret_cast<const f32x4*>(xw + n * HC + f);
        f32x4 ad = *reinterpret_cast<const f32x4*>(att + (int64_t)h * 2 * C + c);
        f32x4 as = *reinterpret_cast<const f32x4*>(att + (int64_t)h * 2 * C + C + c);
        sd = v.x * ad.x + v.y * ad.y + v.z * ad.z + v.w * ad.w;
        ss = v.x * as.x + v.y * as.y + v.z * as.z + v.w * as.w;
      }
      // the reduction GatRed<4, true>::own_as repeats per gathered row (bitwise)
      sd = group_sum(sd, G);
      ss = group_sum(ss, G);
      if (f < HC && (lane & (G - 1)) == 0) {
        a_dst[n * H + h] = sd;
        a_src[n * H + h] = ss;
      }
    }
  }
}

// alpha[e,h] = exp(leaky(a_src[j,h]+a_dst[i,h]) - max_i,h) / (den_i,h)
__global__ void k_gat_alpha(const int64_t* __restrict__ src_idx, const int64_t* __restrict__ dst_idx,
                            int64_t n_edges, int32_t H, const float* __restrict__ a_src,
                            const float* __restrict__ a_dst, float slope, const float* __restrict__ stats,
                            float* __restrict__ alpha) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_edges * (int64_t)H) return;
  const int64_t e = i / H;
  const int h = (int)(i % H);
  const int64_t j = src_idx[e], d = dst_idx[e];
  float a = a_src[j * H + h] + a_dst[d * H + h];
  a = a > 0.f ? a : a * slope;
  const float m = stats[(d * H + h) * 2];
  const float den = stats[(d * H + h) * 2 + 1];
  alpha[i] = expf(a - m) / den;
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_gather_rows_f32(const float* x, int64_t ldx, const int64_t* idx, int64_t n, int32_t F, float* out,
                       int64_t ldo, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n >= 0 && F >= 0, "mp_gather_rows_f32: negative size");
  if (n == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(x && idx && out, "mp_gather_rows_f32: null pointer");
  MP_CHECK_ARG(ldx >= F && ldo >= F, "mp_gather_rows_f32: leading dimension < F");
  hipStream_t s = as_stream(stream);
  int64_t blocks = ceil_div(n, 4);
  if (blocks > 8192) blocks = 8192;
  bool a4 = F % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)out % 16 == 0;
  if (a4) k_gather_rows<4><<<(unsigned)blocks, 256, 0, s>>>(x, ldx, idx, n, F, out, ldo);
  else k_gather_rows<1><<<(unsigned)blocks, 256, 0, s>>>(x, ldx, idx, n, F, out, ldo);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_permute_f32(const float* src, const int32_t* perm, int64_t n, float* dst, void* stream) {
  MP_DEVICE_GUARD(stream);
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(src && perm && dst && n > 0, "mp_permute_f32: bad argument");
  k_permute<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(src, perm, n, dst);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_scatter_arg_backward_f32(const float* grad_out, const int64_t* arg, int64_t n_rows, int32_t F,
                                int64_t n_edges, float* grad, int64_t ldg, void* stream) {
  MP_DEVICE_GUARD(stream);
  if (n_rows == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(grad_out && arg && grad, "mp_scatter_arg_backward_f32: null pointer");
  MP_CHECK_ARG(ldg >= F, "mp_scatter_arg_backward_f32: ldg < F");
  int64_t total = n_rows * (int64_t)F;
  k_scatter_arg_backward<<<(unsigned)ceil_div(total, 256), 256, 0, as_stream(stream)>>>(grad_out, arg, n_rows, F,
                                                                                          n_edges, grad, ldg);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gcn_norm_f32(const int64_t* row, const int64_t* col, const float* w, int64_t n_edges, int64_t n_nodes,
                    float* deg_ws, float* norm, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0, "mp_gcn_norm_f32: negative size");
  MP_CHECK_ARG(deg_ws && (n_edges == 0 || (row && col && norm)), "mp_gcn_norm_f32: null pointer");
  hipStream_t s = as_stream(stream);
  if (n_nodes > 0) MP_CHECK_HIP(hipMemsetAsync(deg_ws, 0, (size_t)n_nodes * sizeof(float), s));
  if (n_edges > 0) {
    k_gcn_degree<<<(unsigned)ceil_div(n_edges, 256), 256, 0, s>>>(row, w, n_edges, deg_ws);
    MP_CHECK_LAUNCH();
  }
  if (n_nodes > 0) {
    k_gcn_dinv<<<(unsigned)ceil_div(n_nodes, 256), 256, 0, s>>>(deg_ws, n_nodes);
    MP_CHECK_LAUNCH();
  }
  if (n_edges > 0) {
    k_gcn_norm<<<(unsigned)ceil_div(n_edges, 256), 256, 0, s>>>(row, col, w, n_edges, deg_ws, norm);
    MP_CHECK_LAUNCH();
  }
  return MP_OK;
}

int mp_gcn_norm_from_deg_f32(const int64_t* row, const int64_t* col, const float* w, int64_t n_edges,
                             int64_t n_nodes, float* deg, float* norm, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0, "mp_gcn_norm_from_deg_f32: negative size");
  MP_CHECK_ARG((n_nodes == 0 || deg) && (n_edges == 0 || (row && col && norm)), "mp_gcn_norm_from_deg_f32: null pointer");
  hipStream_t s = as_stream(stream);
  if (n_nodes > 0) {
    k_gcn_dinv<<<(unsigned)ceil_div(n_nodes, 256), 256, 0, s>>>(deg, n_nodes);
    MP_CHECK_LAUNCH();
  }
  if (n_edges > 0) {
    k_gcn_norm<<<(unsigned)ceil_div(n_edges, 256), 256, 0, s>>>(row, col, w, n_edges, deg, norm);
    MP_CHECK_LAUNCH();
  }
  return MP_OK;
}

int mp_gat_node_scores_f32(const float* xw, int64_t n_nodes, int32_t H, int32_t C, const float* att,
                           float* a_src, float* a_dst, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(H > 0 && C > 0 && n_nodes >= 0, "mp_gat_node_scores_f32: bad sizes");
  if (n_nodes == 0) return MP_OK;
  MP_CHECK_ARG(xw && att && a_src && a_dst, "mp_gat_node_scores_f32: null pointer");
  const int G = C / 4;
  const bool wave_form = C % 4 == 0 && G <= 64 && (G & (G - 1)) == 0 && (uintptr_t)xw % 16 == 0 &&
                         (uintptr_t)att % 16 == 0;
  if (wave_form) {
    int64_t blocks = ceil_div(n_nodes, 4);
    if (blocks > 16384) blocks = 16384;
    k_gat_node_scores_wave<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(xw, n_nodes, H, C, G, att, a_src,
                                                                            a_dst);
  } else if (C % 4 == 0 && (uintptr_t)xw % 16 == 0 && (uintptr_t)att % 16 == 0) {
    // heads of any other width: one wave per node, 256-feature chunks (mp_gat_wide.hip)
    return mp_gat_node_scores_wide_f32(xw, n_nodes, H, C, att, a_src, a_dst, stream);
  } else {
    int64_t total = n_nodes * (int64_t)H;
    k_gat_node_scores<<<(unsigned)ceil_div(total, 256), 256, 0, as_stream(stream)>>>(xw, n_nodes, H, C, att,
                                                                                     a_src, a_dst);
  }
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_alpha_f32(const int64_t* src_idx, const int64_t* dst_idx, int64_t n_edges, int32_t H,
                     const float* a_src, const float* a_dst, float slope, const float* row_stats, float* alpha,
                     void* stream) {
  MP_DEVICE_GUARD(stream);
  if (n_edges == 0) return MP_OK;
  MP_CHECK_ARG(src_idx && dst_idx && a_src && a_dst && row_stats && alpha && H > 0,
               "mp_gat_alpha_f32: bad argument");
  int64_t total = n_edges * (int64_t)H;
  k_gat_alpha<<<(unsigned)ceil_div(total, 256), 256, 0, as_stream(stream)>>>(src_idx, dst_idx, n_edges, H, a_src,
                                                                             a_dst, slope, row_stats, alpha);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
