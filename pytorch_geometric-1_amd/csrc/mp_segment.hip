// Deterministic, edge-ordered reductions keyed on the SOURCE side (gfx950):
//   * the weighted GCN degree   deg[j] = sum_{e: row[e] = j} w[e]       (GCNConv.norm [U5])
//   * the ScatterMax / ScatterMin backward of a fused message w_e * x[src_e]
//       d x[j, f] = sum_{e: src(e) = j, arg[dst(e), f] = e} w_e * g[dst(e), f]
//     ([U8] ScatterMax.backward = zeros(E+1, F).scatter_(0, arg, g)[:E], then
//     the message's backward and index_select's backward, an index_add_ by source
//     in edge order).
// Both walk the TRANSPOSED CSR (rows = source nodes, slots = out-edges in
// original edge order), one wave per row, and add in slot order -- the
// reference's left-to-right order, so the results are bit-identical to the
// serial CPU loop and independent of scheduling (no float atomics).
#include "mp_common.h"

namespace mp {

// ---------------------------------------------------------------------------
// serial segment sum: out[r] = ((0 + v[id(k0)]) + v[id(k0+1)]) + ...
// One wave per row: 64 slots are loaded coalesced (the next 64 in flight),
// then added left to right through v_readlane (one VALU add per slot).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_segment_sum_serial(const int32_t* __restrict__ rowptr,
                                                            const int32_t* __restrict__ eid,
                                                            const float* __restrict__ v, int64_t n_rows,
                                                            float* __restrict__ out) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_rows; r += nw) {
    const int b = rowptr[r], e = rowptr[r + 1];
    float acc = 0.f;
    int k = b + lane;
    float cur = 0.f;
    if (k < e) cur = v[eid ? eid[k] : k];
    for (int k0 = b; k0 < e; k0 += 64) {
      const int kn = k0 + 64 + lane;
      float nxt = 0.f;
      if (kn < e) nxt = v[eid ? eid[kn] : kn];
      const int n = uni(e - k0 < 64 ? e - k0 : 64);
      for (int i = 0; i < n; ++i) acc = __fadd_rn(acc, readlane(cur, i));
      cur = nxt;
    }
    if (lane == 0) out[r] = acc;
  }
}

// inv[eid[k]] = k: the slot of every edge in this CSR
__global__ void k_csr_inverse(const int32_t* __restrict__ eid, int64_t n, int32_t* __restrict__ inv) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) inv[eid[k]] = (int32_t)k;
}

// winner mask in transposed-CSR slot order: bit f of mask[inv[e], :] is set when
// edge e is the argmax of (its destination row, feature f).  Integer atomics
// (the result is a set of bits: order-independent).
__global__ void k_arg_mask(const int64_t* __restrict__ arg, int64_t n_rows, int32_t F, int64_t n_edges,
                           const int32_t* __restrict__ inv, uint32_t* __restrict__ mask, int32_t W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows * (int64_t)F) return;
  const int64_t e = arg[i];
  if (e < 0 || e >= n_edges) return;
  const int f = (int)(i % F);
  atomicOr(mask + (int64_t)inv[e] * W + (f >> 5), 1u << (f & 31));
}

// d x rows over the transposed CSR: block (x: 4 rows, y: 64-feature tile t).
// Lane l owns feature t*64 + l; a batch of 64 slots loads each slot's two mask
// words of this tile, a ballot picks the slots that won any feature of the tile,
// and those are added in slot order, four gathers in flight.
constexpr int kArgBwdQ = 4;

__global__ __launch_bounds__(256) void k_arg_bwd_csr(const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const int32_t* __restrict__ eid, int64_t n_rows,
                                                     const uint32_t* __restrict__ mask, int32_t W,
                                                     const float* __restrict__ g, int64_t ldg, int32_t F,
                                                     const float* __restrict__ w, float* __restrict__ gx,
                                                     int64_t ldgx) {
  const int lane = lane_id();
  const int t = blockIdx.y;
  const int f = t * 64 + lane;
  const bool hi = lane >= 32;
  const uint32_t bit = 1u << (lane & 31);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_rows; r += nw) {
    const int b = rowptr[r], e = rowptr[r + 1];
    float acc = 0.f;
    for (int k0 = b; k0 < e; k0 += 64) {
      const int k = k0 + lane;
      const bool valid = k < e;
      const int kk = valid ? k : b;
      const int c = col[kk];
      float wv = 1.f;
      if (w) wv = w[eid[kk]];
      const uint2 m2 = *reinterpret_cast<const uint2*>(mask + (int64_t)kk * W + 2 * t);
      const bool any = valid && (m2.x | m2.y) != 0u;
      uint64_t act = __ballot(any);
      while (act) {
        int s[kArgBwdQ];
        int n = 0;
#pragma unroll
        for (int q = 0; q < kArgBwdQ; ++q) {
          s[q] = 0;
          if (act) {
            s[q] = __builtin_ctzll(act);
            act &= act - 1;
            n = q + 1;
          }
        }
        float val[kArgBwdQ];
        bool on[kArgBwdQ];
#pragma unroll
        for (int q = 0; q < kArgBwdQ; ++q) {
          const uint32_t lo_w = (uint32_t)readlane((int)m2.x, s[q]);
          const uint32_t hi_w = (uint32_t)readlane((int)m2.y, s[q]);
          on[q] = q < n && ((hi ? hi_w : lo_w) & bit) != 0u && f < F;
          const int rr = readlane(c, s[q]);
          val[q] = on[q] ? g[(int64_t)rr * ldg + f] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < kArgBwdQ; ++q) {
          if (on[q]) {
            const float term = w ? __fmul_rn(val[q], readlane(wv, s[q])) : val[q];
            acc = __fadd_rn(acc, term);
          }
        }
      }
    }
    if (f < F) gx[r * ldgx + f] = acc;
  }
}

// d w_e = sum over the features f that edge e won of g[dst_e, f] * x[src_e, f]
// (the weight's share of the message's backward; wave reduction in a fixed tree).
// One wave per 64 consecutive edges; edges that won nothing get 0.
__global__ __launch_bounds__(256) void k_arg_grad_w(const int64_t* __restrict__ src_map,
                                                    const int64_t* __restrict__ dst_map, int64_t n_edges,
                                                    const int32_t* __restrict__ inv,
                                                    const uint32_t* __restrict__ mask, int32_t W,
                                                    const float* __restrict__ g, int64_t ldg,
                                                    const float* __restrict__ x, int64_t ldx, int32_t F,
                                                    float* __restrict__ gw) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t e0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; e0 < n_edges; e0 += nw * 64) {
    const int64_t e = e0 + lane;
    const bool valid = e < n_edges;
    int k = 0;
    uint32_t any_w = 0;
    if (valid) {
      k = inv[e];
      for (int q = 0; q < W; ++q) any_w |= mask[(int64_t)k * W + q];
    }
    uint64_t act = __ballot(any_w != 0u);
    if (valid && any_w == 0u) gw[e] = 0.f;
    while (act) {
      const int s = __builtin_ctzll(act);
      act &= act - 1;
      const int64_t es = e0 + s;
      const int ks = readlane(k, s);
      const int64_t j = src_map[es], r = dst_map[es];
      float sum = 0.f;
      for (int f = lane; f < F; f += 64) {
        const uint32_t word = mask[(int64_t)ks * W + (f >> 5)];
        if (word & (1u << (f & 31))) sum = __fadd_rn(sum, __fmul_rn(g[r * ldg + f], x[j * ldx + f]));
      }
      sum = group_sum(sum, 64);
      if (lane == 0) gw[es] = sum;
    }
  }
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_segment_sum_serial_f32(const int32_t* rowptr, const int32_t* eid, const float* v, int64_t n_rows,
                              float* out, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_rows >= 0, "mp_segment_sum_serial_f32: negative size");
  if (n_rows == 0) return MP_OK;
  MP_CHECK_ARG(rowptr && out, "mp_segment_sum_serial_f32: null pointer");
  int64_t blocks = ceil_div(n_rows, 4);
  if (blocks > 65536) blocks = 65536;
  k_segment_sum_serial<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(rowptr, eid, v, n_rows, out);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_csr_inverse_eid(const mp_csr* g, int32_t* inv, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(g && inv, "mp_csr_inverse_eid: null pointer");
  if (g->n_edges == 0) return MP_OK;
  MP_CHECK_ARG(g->eid, "mp_csr_inverse_eid: the CSR has no eid array");
  k_csr_inverse<<<(unsigned)ceil_div(g->n_edges, 256), 256, 0, as_stream(stream)>>>(g->eid, g->n_edges, inv);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int32_t mp_arg_mask_words(int32_t F) { return F > 0 ? 2 * (int32_t)ceil_div(F, 64) : 0; }

int mp_arg_winner_mask(const int64_t* arg, int64_t n_rows, int32_t F, int64_t n_edges, const int32_t* inv,
                       uint32_t* mask, size_t mask_bytes, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_rows >= 0 && F >= 0 && n_edges >= 0, "mp_arg_winner_mask: negative size");
  const int32_t W = mp_arg_mask_words(F);
  hipStream_t s = as_stream(stream);
  if (n_edges == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(mask && inv && (n_rows == 0 || arg), "mp_arg_winner_mask: null pointer");
  MP_CHECK_EXTENT("mp_arg_winner_mask", "mask", mask_bytes, (size_t)n_edges * W * 4);
  MP_CHECK_HIP(hipMemsetAsync(mask, 0, (size_t)n_edges * W * sizeof(uint32_t), s));
  const int64_t total = n_rows * (int64_t)F;
  if (total == 0) return MP_OK;
  k_arg_mask<<<(unsigned)ceil_div(total, 256), 256, 0, s>>>(arg, n_rows, F, n_edges, inv, mask, W);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_scatter_arg_backward_csr_f32(const mp_csr* gt, const uint32_t* mask, size_t mask_bytes,
                                    const float* grad_out, int64_t ldg, int32_t F, const float* w, float* grad,
                                    int64_t ldgx, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(gt && F >= 0, "mp_scatter_arg_backward_csr_f32: bad arguments");
  if (gt->n_rows == 0 || F == 0) return MP_OK;
  MP_CHECK_ARG(grad && gt->rowptr && (gt->n_edges == 0 || (gt->col && gt->eid && mask && grad_out)),
               "mp_scatter_arg_backward_csr_f32: null pointer");
  MP_CHECK_ARG(ldg >= F && ldgx >= F, "mp_scatter_arg_backward_csr_f32: leading dimension < F");
  MP_CHECK_ARG((uintptr_t)mask % 8 == 0, "mp_scatter_arg_backward_csr_f32: mask must be 8-byte aligned");
  const int32_t W = mp_arg_mask_words(F);
  MP_CHECK_EXTENT("mp_scatter_arg_backward_csr_f32", "mask", mask_bytes, (size_t)gt->n_edges * W * 4);
  int64_t bx = ceil_div(gt->n_rows, 4);
  if (bx > 65536) bx = 65536;
  dim3 grid((unsigned)bx, (unsigned)(W / 2));
  k_arg_bwd_csr<<<grid, 256, 0, as_stream(stream)>>>(gt->rowptr, gt->col, gt->eid, gt->n_rows, mask, W, grad_out,
                                                      ldg, F, w, grad, ldgx);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_scatter_arg_grad_w_f32(const int64_t* src_map, const int64_t* dst_map, int64_t n_edges, const int32_t* inv,
                              const uint32_t* mask, size_t mask_bytes, int32_t F, const float* grad_out, int64_t ldg,
                              const float* x, int64_t ldx, float* grad_w, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_edges >= 0 && F >= 0, "mp_scatter_arg_grad_w_f32: negative size");
  if (n_edges == 0) return MP_OK;
  MP_CHECK_ARG(src_map && dst_map && inv && grad_w && (F == 0 || (mask && grad_out && x)),
               "mp_scatter_arg_grad_w_f32: null pointer");
  MP_CHECK_ARG(ldg >= F && ldx >= F, "mp_scatter_arg_grad_w_f32: leading dimension < F");
  const int32_t W = mp_arg_mask_words(F);
  MP_CHECK_EXTENT("mp_scatter_arg_grad_w_f32", "mask", mask_bytes, (size_t)n_edges * W * 4);
  if (F == 0) {
    MP_CHECK_HIP(hipMemsetAsync(grad_w, 0, (size_t)n_edges * sizeof(float), as_stream(stream)));
    return MP_OK;
  }
  int64_t blocks = ceil_div(ceil_div(n_edges, 64), 4);
  if (blocks > 65536) blocks = 65536;
  k_arg_grad_w<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(src_map, dst_map, n_edges, inv, mask, W, grad_out,
                                                                 ldg, x, ldx, F, grad_w);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
