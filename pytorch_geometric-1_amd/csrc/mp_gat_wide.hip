// Node-wise kernels of the GATConv path for heads of any width (C % 4 == 0, a
// head possibly wider than one 256-feature tile, H * C any size): the shapes
// the reference's own GAT stacks use (ConvexPruning.py:209-214: heads = 1,
// out_channels drawn at random by ContractionLayerCoefficients, :106-114).
// The per-head dot products are taken per node here, so the edge passes
// (GatRed non-own forward, GatBwdWideRed backward in mp_aggregate.hip) need no
// cross-lane reduction per slot.  One wave per node; a head is walked in
// 256-feature chunks (lane = 4 features), each lane keeps its running partial
// across the chunks (separately rounded, chunk order), then one 64-lane
// shuffle-xor tree (group_sum) per head.
#include "mp_common.h"

namespace mp {

constexpr int kWideWaves = 4;  // waves per block

// sum over a head's features [h*C, h*C + C) of a[.] * (b[.] - sub[.]) for row
// pointers a, b (sub optional: b holds out = agg + bias, sub the bias; lane
// partials in chunk order, then the wave tree); every lane gets the sum
__device__ __forceinline__ float head_dot(const float* __restrict__ a, const float* __restrict__ b, int C,
                                         int lane, const float* __restrict__ sub = nullptr) {
  float t = 0.f;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int c = c0 + 4 * lane;
    if (c < C) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(a + c);
      f32x4 y = *reinterpret_cast<const f32x4*>(b + c);
      if (sub) {
        const f32x4 d = *reinterpret_cast<const f32x4*>(sub + c);
        y.x = __fsub_rn(y.x, d.x);
        y.y = __fsub_rn(y.y, d.y);
        y.z = __fsub_rn(y.z, d.z);
        y.w = __fsub_rn(y.w, d.w);
      }
      t = __builtin_fmaf(x.x, y.x, t);
      t = __builtin_fmaf(x.y, y.y, t);
      t = __builtin_fmaf(x.z, y.z, t);
      t = __builtin_fmaf(x.w, y.w, t);
    }
  }
  return group_sum(t, 64);
}

// a_dst[n,h] = <xw[n,h,:], att[h, 0:C]>,  a_src[n,h] = <xw[n,h,:], att[h, C:2C]>
__global__ __launch_bounds__(64 * kWideWaves) void k_gat_node_scores_wide(const float* __restrict__ xw,
                                                                         int64_t n_nodes, int32_t H, int32_t C,
                                                                         const float* __restrict__ att,
                                                                         float* __restrict__ a_src,
                                                                         float* __restrict__ a_dst) {
  const int lane = lane_id();
  const int64_t HC = (int64_t)H * C;
  const int64_t nw = (int64_t)gridDim.x * kWideWaves;
  for (int64_t n = (int64_t)blockIdx.x * kWideWaves + (threadIdx.x >> 6); n < n_nodes; n += nw) {
    for (int h = 0; h < H; ++h) {
      const float* row = xw + n * HC + (int64_t)h * C;
      const float* at = att + (int64_t)h * 2 * C;
      const float sd = head_dot(row, at, C, lane);
      const float ss = head_dot(row, at + C, C, lane);
      if (lane == 0) {
        a_dst[n * H + h] = sd;
        a_src[n * H + h] = ss;
      }
    }
  }
}

// Backward prologue after the training forward, per (node n, head h):
//   rs = <g[n,h,:], agg[n,h,:]>,  pack[n,h] = (a_dst, m, 1/den, rs),
//   (bias != nullptr: agg holds out = agg + bias, rs over out - bias)
//   grad_a_dst[n,h] = <g[n,h,:], agg2[n,h,:]> - rs * row_s2[n,h]
__global__ __launch_bounds__(64 * kWideWaves) void k_gat_bwd_prep_wide(
    const float* __restrict__ g, int64_t ldg, const float* __restrict__ agg, int64_t lda,
    const float* __restrict__ bias, const float* __restrict__ agg2, const float* __restrict__ s2,
    const float* __restrict__ a_dst,
    const float* __restrict__ stats, int64_t n, int32_t H, int32_t C, float* __restrict__ pack,
    float* __restrict__ ga_dst) {
  const int lane = lane_id();
  const int64_t HC = (int64_t)H * C;
  const int64_t nw = (int64_t)gridDim.x * kWideWaves;
  for (int64_t r = (int64_t)blockIdx.x * kWideWaves + (threadIdx.x >> 6); r < n; r += nw) {
    for (int h = 0; h < H; ++h) {
      const int64_t o = (int64_t)h * C;
      const float rs = head_dot(g + r * ldg + o, agg + r * lda + o, C, lane, bias ? bias + o : nullptr);
      const float t2 = head_dot(g + r * ldg + o, agg2 + r * HC + o, C, lane);
      if (lane == 0) {
        const int64_t q = r * H + h;
        f32x4 v = {a_dst[q], stats[2 * q], 1.f / stats[2 * q + 1], rs};
        *reinterpret_cast<f32x4*>(pack + 4 * q) = v;
        ga_dst[q] = stats[2 * q + 1] == 1.f ? 0.f : __builtin_fmaf(-rs, s2[q], t2);  // one-hot row: 0
      }
    }
  }
}

// Backward epilogue after GatBwdWideRed, per (node j, head h):
//   ga_src[j,h] = <acc2[j,h,:], xw[j,h,:]> - sc[j,h]      (sc in, ga_src out, in place)
//   gx[j,h,:]  += ga_src[j,h] att[h, C:2C] + ga_dst[j,h] att[h, 0:C]
__global__ __launch_bounds__(64 * kWideWaves) void k_gat_bwd_epilogue_wide(
    float* __restrict__ gx, const float* __restrict__ acc2, const float* __restrict__ xw,
    const float* __restrict__ att, const float* __restrict__ ga_dst, float* __restrict__ sc_ga_src, int64_t n,
    int32_t H, int32_t C) {
  const int lane = lane_id();
  const int64_t HC = (int64_t)H * C;
  const int64_t nw = (int64_t)gridDim.x * kWideWaves;
  for (int64_t j = (int64_t)blockIdx.x * kWideWaves + (threadIdx.x >> 6); j < n; j += nw) {
    for (int h = 0; h < H; ++h) {
      const int64_t o = j * HC + (int64_t)h * C;
      const int64_t q = j * H + h;
      const float gs = head_dot(acc2 + o, xw + o, C, lane) - sc_ga_src[q];
      const float gd = ga_dst[q];
      const float* at = att + (int64_t)h * 2 * C;
      for (int c = 4 * lane; c < C; c += 256) {
        f32x4 v = *reinterpret_cast<f32x4*>(gx + o + c);
        const f32x4 ad = *reinterpret_cast<const f32x4*>(at + c);
        const f32x4 as = *reinterpret_cast<const f32x4*>(at + C + c);
        v.x = __builtin_fmaf(gd, ad.x, __builtin_fmaf(gs, as.x, v.x));
        v.y = __builtin_fmaf(gd, ad.y, __builtin_fmaf(gs, as.y, v.y));
        v.z = __builtin_fmaf(gd, ad.z, __builtin_fmaf(gs, as.z, v.z));
        v.w = __builtin_fmaf(gd, ad.w, __builtin_fmaf(gs, as.w, v.w));
        *reinterpret_cast<f32x4*>(gx + o + c) = v;
      }
      __builtin_amdgcn_wave_barrier();  // every lane has read sc before lane 0 overwrites it
      if (lane == 0) sc_ga_src[q] = gs;
    }
  }
}

static unsigned wide_blocks(int64_t n) {
  int64_t b = (n + kWideWaves - 1) / kWideWaves;
  if (b > 16384) b = 16384;
  return (unsigned)(b < 1 ? 1 : b);
}

static bool al16(const void* p) { return (uintptr_t)p % 16 == 0; }

}  // namespace mp

using namespace mp;

extern "C" {

int mp_gat_wide_ok(int32_t H, int32_t C) { return H > 0 && C > 0 && C % 4 == 0 ? 1 : 0; }

int mp_gat_node_scores_wide_f32(const float* xw, int64_t n_nodes, int32_t H, int32_t C, const float* att,
                                float* a_src, float* a_dst, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(mp_gat_wide_ok(H, C) && n_nodes >= 0, "mp_gat_node_scores_wide_f32: needs C %% 4 == 0");
  if (n_nodes == 0) return MP_OK;
  MP_CHECK_ARG(xw && att && a_src && a_dst, "mp_gat_node_scores_wide_f32: null pointer");
  MP_CHECK_ARG(al16(xw) && al16(att), "mp_gat_node_scores_wide_f32: xw and att must be 16-byte aligned");
  k_gat_node_scores_wide<<<wide_blocks(n_nodes), 64 * kWideWaves, 0, as_stream(stream)>>>(xw, n_nodes, H, C, att,
                                                                                          a_src, a_dst);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_backward_prep_wide_f32(const float* grad_out, int64_t ldg, const float* agg, int64_t lda,
                                  const float* bias, const float* agg2, const float* row_s2, const float* a_dst, const float* row_stats,
                                  int64_t n, int32_t H, int32_t C, float* pack, size_t pack_bytes,
                                  float* grad_a_dst, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(mp_gat_wide_ok(H, C) && n >= 0, "mp_gat_backward_prep_wide_f32: needs C %% 4 == 0");
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(grad_out && agg && agg2 && row_s2 && a_dst && row_stats && pack && grad_a_dst,
               "mp_gat_backward_prep_wide_f32: null pointer");
  MP_CHECK_EXTENT("mp_gat_backward_prep_wide_f32", "pack", pack_bytes, (size_t)n * H * 16);
  const int64_t F = (int64_t)H * C;
  MP_CHECK_ARG(ldg >= F && lda >= F && ldg % 4 == 0 && lda % 4 == 0, "mp_gat_backward_prep_wide_f32: bad ld");
  MP_CHECK_ARG(al16(grad_out) && al16(agg) && al16(agg2) && al16(pack) && al16(bias),
               "mp_gat_backward_prep_wide_f32: 16-byte alignment required");
  k_gat_bwd_prep_wide<<<wide_blocks(n), 64 * kWideWaves, 0, as_stream(stream)>>>(
      grad_out, ldg, agg, lda, bias, agg2, row_s2, a_dst, row_stats, n, H, C, pack, grad_a_dst);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_backward_epilogue_wide_f32(float* grad_xw, const float* acc2, const float* xw, const float* att,
                                      const float* grad_a_dst, float* sc_grad_a_src, int64_t n, int32_t H,
                                      int32_t C, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(mp_gat_wide_ok(H, C) && n >= 0, "mp_gat_backward_epilogue_wide_f32: needs C %% 4 == 0");
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(grad_xw && acc2 && xw && att && grad_a_dst && sc_grad_a_src,
               "mp_gat_backward_epilogue_wide_f32: null pointer");
  MP_CHECK_ARG(al16(grad_xw) && al16(acc2) && al16(xw) && al16(att),
               "mp_gat_backward_epilogue_wide_f32: 16-byte alignment required");
  k_gat_bwd_epilogue_wide<<<wide_blocks(n), 64 * kWideWaves, 0, as_stream(stream)>>>(
      grad_xw, acc2, xw, att, grad_a_dst, sc_grad_a_src, n, H, C);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
