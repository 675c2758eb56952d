// Merge of GAT softmax partials: the receiving side of a sharded GATConv over
// the hybrid halo cover (mi355_mp.dist.GatHaloCover).
//
// A destination row i of rank p sums its in-edges in two kinds of pieces: the
// local piece (its own and pulled sources, aggregated on p by the fused GAT
// kernel: out_loc = acc/den normalised, stats (m, den)), and one partial per
// peer q that pushed its sum over q's own sources of i's in-edges (the same
// kernel on q's send graph, with a_dst[i] sent over beforehand).  Each piece is
// an online-softmax state; per head
//     M = max(m_loc, m_1, ..),   w_k = den_k e^(m_k - M),   tot = sum_k w_k
//     out[i] = sum_k (w_k / tot) out_k + bias     (local piece first, then the
//                                                 partials in peer order)
// -- the rescaling rule GatRed::merge applies to task partials.  A row with no
// partial keeps out_loc + bias bit for bit (the single-GPU kernel's finish).
// One wave per row, 4 features per lane (C % 4 == 0: a lane's features share a
// head), rows of any width in 256-feature chunks.  A head may span two chunks
// (C > 256, or C not dividing 256: PPI's conv3 pads 121 -> 124 features per
// head), so the row's stats are read in the first sweep over the chunks and
// written back only in a second sweep, by each head's first lane -- every
// chunk of the row merges with the local piece's own (m, den).
#include "mp_common.h"

namespace mp {

// (M, tot, c_loc) of head h of a row: the merged max, the merged denominator
// and the local piece's weight in the merged row; false when every piece of
// the head is empty (M = -inf: the row keeps its local piece).
__device__ __forceinline__ bool merge_head(float m_loc, float d_loc, int k0, int k1, const int32_t* __restrict__ pidx,
                                           const float* __restrict__ pst, int32_t H, int h, float& M, float& tot,
                                           float& c_loc) {
  M = m_loc;
  for (int k = k0; k < k1; ++k) M = fmaxf(M, pst[2 * ((int64_t)pidx[k] * H + h)]);
  if (M == -INFINITY) return false;
  const float w_loc = m_loc == -INFINITY ? 0.f : d_loc * expf(m_loc - M);
  tot = w_loc;
  for (int k = k0; k < k1; ++k) {
    const int64_t pq = (int64_t)pidx[k] * H + h;
    const float mk = pst[2 * pq];
    if (mk != -INFINITY) tot = tot + pst[2 * pq + 1] * expf(mk - M);
  }
  c_loc = w_loc / tot;
  return true;
}

__global__ __launch_bounds__(256) void k_gat_merge_partials(int64_t n, int32_t H, int32_t C,
                                                            const int32_t* __restrict__ pptr,
                                                            const int32_t* __restrict__ pidx,
                                                            const float* __restrict__ pout, int64_t ldp,
                                                            const float* __restrict__ pst,
                                                            const float* __restrict__ bias, float* __restrict__ out,
                                                            int64_t ldo, float* __restrict__ st,
                                                            float* __restrict__ agg2, float* __restrict__ s2) {
  const int lane = lane_id();
  const int64_t F = (int64_t)H * C;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += nw) {
    const int k0 = pptr[r], k1 = pptr[r + 1];
    // sweep 1: the merged features (st is only read here)
    for (int64_t f0 = 0; f0 < F; f0 += 256) {
      const int64_t f = f0 + 4 * lane;
      if (f >= F) continue;
      const int h = (int)(f / C);
      const int64_t q = r * H + h;
      Frag<4> o = load_frag<4>(out + r * ldo + f);
      float c_loc = 1.f, M, tot;
      if (k1 > k0 && merge_head(st[2 * q], st[2 * q + 1], k0, k1, pidx, pst, H, h, M, tot, c_loc)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = o.v[j] * c_loc;
        for (int k = k0; k < k1; ++k) {
          const int64_t pq = (int64_t)pidx[k] * H + h;
          const float mk = pst[2 * pq];
          if (mk == -INFINITY) continue;
          const float ck = pst[2 * pq + 1] * expf(mk - M) / tot;
          const Frag<4> v = load_frag<4>(pout + (int64_t)pidx[k] * ldp + f);
#pragma unroll
          for (int j = 0; j < 4; ++j) o.v[j] = o.v[j] + ck * v.v[j];
        }
        if (agg2) {
          Frag<4> a = load_frag<4>(agg2 + r * F + f);
#pragma unroll
          for (int j = 0; j < 4; ++j) a.v[j] = a.v[j] * c_loc;
          store_frag<4>(agg2 + r * F + f, a);
        }
      }
      if (bias) {
        const Frag<4> b = load_frag<4>(bias + f);
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = o.v[j] + b.v[j];
      }
      store_frag<4>(out + r * ldo + f, o);
    }
    if (k1 <= k0) continue;
    // sweep 2: each head's first lane writes the merged (M, tot) and scales s2
    // (the loads of sweep 1 completed before its stores above; a head's stats
    // are read and written here by that one lane only)
    for (int64_t f0 = 0; f0 < F; f0 += 256) {
      const int64_t f = f0 + 4 * lane;
      if (f >= F || f % C != 0) continue;
      const int h = (int)(f / C);
      const int64_t q = r * H + h;
      float M, tot, c_loc;
      if (merge_head(st[2 * q], st[2 * q + 1], k0, k1, pidx, pst, H, h, M, tot, c_loc)) {
        st[2 * q] = M;
        st[2 * q + 1] = tot;
        if (s2) s2[q] = s2[q] * c_loc;
      }
    }
  }
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_gat_merge_partials_f32(int64_t n_rows, int32_t H, int32_t C, const int32_t* pptr, const int32_t* pidx,
                              int64_t n_parts, const float* part_out, size_t part_out_bytes, int64_t ldp,
                              const float* part_stats, size_t part_stats_bytes, const float* bias, float* out,
                              int64_t ldo, float* row_stats, float* agg2, float* row_s2, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n_rows >= 0 && n_parts >= 0 && H > 0 && C > 0 && C % 4 == 0,
               "mp_gat_merge_partials_f32: needs n_rows, n_parts >= 0 and C %% 4 == 0");
  if (n_rows == 0) return MP_OK;
  const int64_t F = (int64_t)H * C;
  MP_CHECK_ARG(pptr && out && row_stats && (n_parts == 0 || (pidx && part_out && part_stats)),
               "mp_gat_merge_partials_f32: null pointer");
  MP_CHECK_ARG(ldo >= F && ldo % 4 == 0 && (n_parts == 0 || (ldp >= F && ldp % 4 == 0)),
               "mp_gat_merge_partials_f32: leading dimension < H*C or not a multiple of 4");
  if (n_parts > 0) {
    MP_CHECK_EXTENT("mp_gat_merge_partials_f32", "part_out", part_out_bytes, ((n_parts - 1) * ldp + F) * 4);
    MP_CHECK_EXTENT("mp_gat_merge_partials_f32", "part_stats", part_stats_bytes, n_parts * H * 2 * 4);
  }
  MP_CHECK_ARG((uintptr_t)out % 16 == 0 && (uintptr_t)part_out % 16 == 0 && (uintptr_t)bias % 16 == 0 &&
                   (uintptr_t)agg2 % 16 == 0,
               "mp_gat_merge_partials_f32: out, part_out, bias, agg2 must be 16-byte aligned");
  int64_t blocks = ceil_div(n_rows, 4);
  if (blocks > 65536) blocks = 65536;
  k_gat_merge_partials<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(n_rows, H, C, pptr, pidx, part_out, ldp,
                                                                       part_stats, bias, out, ldo, row_stats, agg2,
                                                                       row_s2);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
