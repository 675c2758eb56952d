// GATConv backward pieces on the destination-sorted CSR (gfx950):
//   slot -> row map, alpha / pre-activation score in CSR slot order, and the
//   sampled dense-dense product d alpha[k,h] = <grad_out[row_k,h,:], xw[col_k,h,:]>.
// The alpha-weighted transposed aggregation is mp_aggregate_heads_f32 (the
// main kernel template with a per-head weight).  Reference: GATConv.message
// + utils.softmax autograd (PyG 1.4.3 [U3,U6]).
#include "mp_common.h"

namespace mp {

__global__ void k_slot_rows(const int32_t* __restrict__ rowptr, int64_t n_rows, int64_t n_edges,
                            int32_t* __restrict__ slot_row) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_edges) return;
  int64_t lo = 0, hi = n_rows;  // last r with rowptr[r] <= k
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if ((int64_t)rowptr[mid] <= k) lo = mid;
    else hi = mid - 1;
  }
  slot_row[k] = (int32_t)lo;
}

__global__ void k_gat_alpha_csr(const int32_t* __restrict__ col, const int32_t* __restrict__ slot_row,
                                int64_t n_edges, int32_t H, const float* __restrict__ a_src,
                                const float* __restrict__ a_dst, float slope, const float* __restrict__ stats,
                                float* __restrict__ alpha, float* __restrict__ score) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_edges * (int64_t)H) return;
  const int64_t k = i / H;
  const int h = (int)(i % H);
  const int64_t r = slot_row[k], j = col[k];
  const float sc = a_src[j * H + h] + a_dst[r * H + h];
  const float a = sc > 0.f ? sc : sc * slope;
  alpha[i] = expf(a - stats[(r * H + h) * 2]) / stats[(r * H + h) * 2 + 1];
  if (score) score[i] = sc;
}

// One wave per 256 consecutive slots; lane l owns VEC features f of a
// 64*VEC-feature tile; a head spans G = C/VEC lanes (power of two <= 64) and
// its dot product is reduced with shuffle-xor inside the group.
template <int VEC>
__global__ __launch_bounds__(256) void k_gat_sddmm(const int32_t* __restrict__ col,
                                                    const int32_t* __restrict__ slot_row, int64_t n_edges,
                                                    const float* __restrict__ grow, int64_t ldg,
                                                    const float* __restrict__ x, int64_t ldx, int32_t H,
                                                    int32_t C, int32_t G, float* __restrict__ out) {
  constexpr int U = 8;
  const int lane = lane_id();
  const int64_t k0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 256;
  if (k0 >= n_edges) return;
  const int64_t k1 = k0 + 256 < n_edges ? k0 + 256 : n_edges;
  const int F = H * C;
  const int f = (int)blockIdx.y * 64 * VEC + lane * VEC;
  const bool act = f < F;
  const int fs = act ? f : 0;
  const int h = fs / C;
  for (int64_t kb = k0; kb < k1; kb += 64) {
    const int64_t kk = kb + lane;
    const int rwin = kk < k1 ? slot_row[kk] : 0;
    const int cwin = kk < k1 ? col[kk] : 0;
    const int nb = (int)((k1 - kb) < 64 ? (k1 - kb) : 64);
    for (int b = 0; b < nb; b += U) {
      float d[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int uu = b + u < nb ? b + u : nb - 1;
        const int r = readlane(rwin, uu);
        const int j = readlane(cwin, uu);
        Frag<VEC> gv = load_frag<VEC>(grow + (int64_t)r * ldg + fs);
        Frag<VEC> xv = load_frag<VEC>(x + (int64_t)j * ldx + fs);
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < VEC; ++q) t += gv.v[q] * xv.v[q];
        d[u] = act ? t : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        for (int o = G >> 1; o > 0; o >>= 1) d[u] += __shfl_xor(d[u], o);
        if (b + u < nb && act && (lane & (G - 1)) == 0) out[(kb + b + u) * H + h] = d[u];
      }
    }
  }
}

// general C: one thread per (slot, head)
__global__ void k_gat_sddmm_scalar(const int32_t* __restrict__ col, const int32_t* __restrict__ slot_row,
                                   int64_t n_edges, const float* __restrict__ grow, int64_t ldg,
                                   const float* __restrict__ x, int64_t ldx, int32_t H, int32_t C,
                                   float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_edges * (int64_t)H) return;
  const int64_t k = i / H;
  const int h = (int)(i % H);
  const float* gr = grow + (int64_t)slot_row[k] * ldg + (int64_t)h * C;
  const float* xr = x + (int64_t)col[k] * ldx + (int64_t)h * C;
  float t = 0.f;
  for (int c = 0; c < C; ++c) t += gr[c] * xr[c];
  out[i] = t;
}

// Deterministic block partial: the 4 waves' per-lane sums of one 256-feature
// tile (lane l holds features 4l..4l+3) are added in wave order through LDS
// and stored as one row of the [gridDim.x, F] partial array.
__device__ __forceinline__ void block_partial_store(const float (&v)[4], float* __restrict__ dst, int64_t F) {
  __shared__ float red[3][256];
  const int lane = lane_id();
  const int wid = (int)(threadIdx.x >> 6);
  if (wid > 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wid - 1][lane * 4 + k] = v[k];
  }
  __syncthreads();
  if (wid == 0) {
    float t[4] = {v[0], v[1], v[2], v[3]};
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int k = 0; k < 4; ++k) t[k] += red[q][lane * 4 + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lane * 4 + k < F) dst[lane * 4 + k] = t[k];
  }
}

// Column sums of x [n, F] (F <= 256, F % 4 == 0, 16-B rows) as per-block
// partials [gridDim.x, F]: the bias gradient of a layer whose output adds a
// bias row, sum_i g[i, :].  One wave per row, four rows in flight; the
// partials are added in a fixed order (deterministic).
__global__ __launch_bounds__(256) void k_col_sums(const float* __restrict__ x, int64_t ldx, int64_t n, int32_t F,
                                                  float* __restrict__ part) {
  const int lane = lane_id();
  const int wid = (int)(threadIdx.x >> 6);
  const int64_t f = (int64_t)lane * 4;
  const int64_t fs = f < F ? f : 0;
  const int64_t step = (int64_t)gridDim.x * 4;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t r = (int64_t)blockIdx.x * 4 + wid;
  for (; r + 3 * step < n; r += 4 * step) {
    Frag<4> v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = load_frag<4>(x + (r + u * step) * ldx + fs);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) cs[k] += v[u].v[k];
  }
  for (; r < n; r += step) {
    Frag<4> v = load_frag<4>(x + r * ldx + fs);
#pragma unroll
    for (int k = 0; k < 4; ++k) cs[k] += v.v[k];
  }
  if (f >= F) cs[0] = cs[1] = cs[2] = cs[3] = 0.f;
  block_partial_store(cs, part + (int64_t)blockIdx.x * F, F);
}

// Backward epilogue, one wave per node n (H*C <= 256, C % 4 == 0):
//   gx[n, h*C+c] += ga_dst[n,h] * att[h, c]                (the x_i use of xw in the score)
//   att_part[blk, 0, :] += ga_dst[n,h] * xw[n, :]          (d att_dst, per-block partial)
//   att_part[blk, 1, :] += ga_src[n,h] * xw[n, :]          (d att_src)
__global__ __launch_bounds__(256) void k_gat_bwd_finish(float* __restrict__ gx, const float* __restrict__ xw,
                                                        const float* __restrict__ ga_dst,
                                                        const float* __restrict__ ga_src,
                                                        const float* __restrict__ att, int64_t n, int32_t H,
                                                        int32_t C, float* __restrict__ att_part) {
  const int lane = lane_id();
  const int HC = H * C;
  const int f = lane * 4;
  const bool act = f < HC;
  const int fs = act ? f : 0;
  const int h = fs / C;
  const int c = fs - h * C;
  f32x4 ad = *reinterpret_cast<const f32x4*>(att + (int64_t)h * 2 * C + c);
  float pd[4] = {0.f, 0.f, 0.f, 0.f}, ps[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += nw) {
    const float gd = ga_dst[r * H + h];
    const float gs = ga_src[r * H + h];
    Frag<4> x = load_frag<4>(xw + r * HC + fs);
    if (act) {
      if (gx) {  // (NULL: the transposed pass already added it, mp_gat_backward_train_f32)
        float* d = gx + r * HC + f;
        Frag<4> o = load_frag<4>(d);
        o.v[0] = __builtin_fmaf(gd, ad.x, o.v[0]);
        o.v[1] = __builtin_fmaf(gd, ad.y, o.v[1]);
        o.v[2] = __builtin_fmaf(gd, ad.z, o.v[2]);
        o.v[3] = __builtin_fmaf(gd, ad.w, o.v[3]);
        store_frag<4>(d, o);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        pd[k] = __builtin_fmaf(gd, x.v[k], pd[k]);
        ps[k] = __builtin_fmaf(gs, x.v[k], ps[k]);
      }
    }
  }
  block_partial_store(pd, att_part + (int64_t)blockIdx.x * 2 * HC, HC);
  __syncthreads();
  block_partial_store(ps, att_part + (int64_t)blockIdx.x * 2 * HC + HC, HC);
}

// Backward prologue of the fused GAT pass, per (node n, head h):
//   pack[n,h] = (a_dst[n,h], m[n,h], 1/den[n,h], rs[n,h]),  rs = <g[n,h,:], agg[n,h,:]>
// (rs = sum_j alpha_nj <g_n, xw_j>_h since agg_n = sum_j alpha_nj xw_j).  With
// bias != nullptr, `agg` is the layer output agg + bias and the prologue takes
// agg = out - bias (one rounding per feature): the training forward then writes
// no separate pre-bias copy.
// One wave per node, lane l owns 4 features, a head spans G = C/4 lanes.
__device__ __forceinline__ void write_pack(float* pack, const float* a_dst, const float* stats, int64_t q, float rs) {
  f32x4 v = {a_dst[q], stats[2 * q], 1.f / stats[2 * q + 1], rs};
  *reinterpret_cast<f32x4*>(pack + 4 * q) = v;
}

__global__ __launch_bounds__(256) void k_gat_bwd_prep_wave(const float* __restrict__ g, int64_t ldg,
                                                           const float* __restrict__ agg, int64_t lda,
                                                           const float* __restrict__ a_dst,
                                                           const float* __restrict__ stats, int64_t n, int32_t H,
                                                           int32_t C, int32_t G, float* __restrict__ pack,
                                                           float* __restrict__ gsum_part,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ agg2 = nullptr,
                                                           const float* __restrict__ s2 = nullptr,
                                                           float* __restrict__ ga_dst = nullptr) {
  const int lane = lane_id();
  const int wid = (int)(threadIdx.x >> 6);
  const int64_t HC = (int64_t)H * C;
  const int64_t nw = (int64_t)gridDim.x * 4;
  // bias-gradient partial (column sums of g) for rows of one 256-feature tile
  // (HC <= 256 when gsum_part != nullptr)
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  // per row: rs (and d a_dst from the second accumulator) of the 4 features at fs,
  // the pack / ga_dst stores, the bias-gradient column sums -- rows are folded
  // into cs in the wave's row order, whatever the number in flight
  auto debias = [&](Frag<4>& y, int64_t fs) {
    if (bias) {
      const Frag<4> b = load_frag<4>(bias + fs);
#pragma unroll
      for (int k = 0; k < 4; ++k) y.v[k] = __fsub_rn(y.v[k], b.v[k]);
    }
  };
  auto row = [&](int64_t r, int64_t fs, bool act, const Frag<4>& x, const Frag<4>& y, const Frag<4>& z) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) t = __fadd_rn(t, __fmul_rn(x.v[k], y.v[k]));
    for (int o = 1; o < G; o <<= 1) t = __fadd_rn(t, __shfl_xor(t, o));
    if (act && (lane & (G - 1)) == 0) write_pack(pack, a_dst, stats, r * H + fs / C, t);
    if (agg2) {  // d a_dst = <g, agg2>_h - rs s2  (training forward's second accumulator)
      float t2 = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) t2 = __builtin_fmaf(x.v[k], z.v[k], t2);
      for (int o = 1; o < G; o <<= 1) t2 += __shfl_xor(t2, o);
      const int64_t q = r * H + fs / C;
      // a one-hot softmax row (den == 1) has d a_dst = 0 (GatBwdRed::consume_gatb)
      if (act && (lane & (G - 1)) == 0) ga_dst[q] = stats[2 * q + 1] == 1.f ? 0.f : __builtin_fmaf(-t, s2[q], t2);
    }
    if (gsum_part && act) {
#pragma unroll
      for (int k = 0; k < 4; ++k) cs[k] += x.v[k];
    }
  };
  int64_t r = (int64_t)blockIdx.x * 4 + wid;
  if (HC <= 256) {
    // one 256-feature pass per row: two rows in flight, every load of both issued
    // before the first reduction (the prologue streams 3 rows per node)
    const int64_t f = lane * 4;
    const bool act = f < HC;
    const int64_t fs = act ? f : 0;
    Frag<4> z0 = {}, z1 = {};
    for (; r + nw < n; r += 2 * nw) {
      const int64_t r1 = r + nw;
      Frag<4> x0 = load_frag<4>(g + r * ldg + fs), x1 = load_frag<4>(g + r1 * ldg + fs);
      Frag<4> y0 = load_frag<4>(agg + r * lda + fs), y1 = load_frag<4>(agg + r1 * lda + fs);
      if (agg2) {
        z0 = load_frag<4>(agg2 + r * HC + fs);
        z1 = load_frag<4>(agg2 + r1 * HC + fs);
      }
      debias(y0, fs);
      debias(y1, fs);
      row(r, fs, act, x0, y0, z0);
      row(r1, fs, act, x1, y1, z1);
    }
    if (r < n) {
      Frag<4> x0 = load_frag<4>(g + r * ldg + fs);
      Frag<4> y0 = load_frag<4>(agg + r * lda + fs);
      if (agg2) z0 = load_frag<4>(agg2 + r * HC + fs);
      debias(y0, fs);
      row(r, fs, act, x0, y0, z0);
    }
  } else {
    for (; r < n; r += nw) {
      for (int64_t base = 0; base < HC; base += 256) {
        const int64_t f = base + lane * 4;
        const bool act = f < HC;
        const int64_t fs = act ? f : 0;
        Frag<4> x = load_frag<4>(g + r * ldg + fs);
        Frag<4> y = load_frag<4>(agg + r * lda + fs);
        Frag<4> z = {};
        if (agg2) z = load_frag<4>(agg2 + r * HC + fs);
        debias(y, fs);
        row(r, fs, act, x, y, z);
      }
    }
  }
  if (gsum_part) block_partial_store(cs, gsum_part + (int64_t)blockIdx.x * HC, HC);
}

__global__ void k_gat_bwd_prep_scalar(const float* __restrict__ g, int64_t ldg, const float* __restrict__ agg,
                                      int64_t lda, const float* __restrict__ bias, const float* __restrict__ a_dst,
                                      const float* __restrict__ stats, int64_t n, int32_t H, int32_t C,
                                      float* __restrict__ pack) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * (int64_t)H) return;
  const int64_t r = i / H;
  const int h = (int)(i % H);
  const float* x = g + r * ldg + (int64_t)h * C;
  const float* y = agg + r * lda + (int64_t)h * C;
  const float* b = bias ? bias + (int64_t)h * C : nullptr;
  float t = 0.f;
  for (int c = 0; c < C; ++c) t = __fadd_rn(t, __fmul_rn(x[c], b ? __fsub_rn(y[c], b[c]) : y[c]));
  write_pack(pack, a_dst, stats, i, t);
}

// y[n, h*C + c] += s[n, h] * att[h*att_ld + c]; VEC consecutive features per thread
template <int VEC>
__global__ void k_heads_outer_add(float* __restrict__ y, int64_t ldy, const float* __restrict__ s, int64_t n,
                                  int32_t H, int32_t C, const float* __restrict__ att, int64_t att_ld) {
  const int F = H * C;
  const int per_row = F / VEC;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * per_row) return;
  const int64_t r = i / per_row;
  const int f = (int)(i - r * per_row) * VEC;
  const int h = f / C;
  const float sv = s[r * H + h];
  const float* a = att + (int64_t)h * att_ld + (f - h * C);
  float* d = y + r * ldy + f;
  Frag<VEC> v = load_frag<VEC>(d);
#pragma unroll
  for (int k = 0; k < VEC; ++k) v.v[k] = __fadd_rn(v.v[k], __fmul_rn(sv, a[k]));
  store_frag<VEC>(d, v);
}

}  // namespace mp

using namespace mp;

extern "C" {

int mp_csr_slot_rows(const mp_csr* g, int32_t* slot_row, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(g && g->rowptr && slot_row, "mp_csr_slot_rows: null pointer");
  if (g->n_edges == 0) return MP_OK;
  k_slot_rows<<<(unsigned)ceil_div(g->n_edges, 256), 256, 0, as_stream(stream)>>>(g->rowptr, g->n_rows,
                                                                                  g->n_edges, slot_row);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_alpha_csr_f32(const mp_csr* g, const int32_t* slot_row, const float* a_src, const float* a_dst,
                         int32_t H, float slope, const float* row_stats, float* alpha_csr, float* score,
                         void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(g && H > 0, "mp_gat_alpha_csr_f32: bad argument");
  if (g->n_edges == 0) return MP_OK;
  MP_CHECK_ARG(g->col && slot_row && a_src && a_dst && row_stats && alpha_csr,
               "mp_gat_alpha_csr_f32: null pointer");
  int64_t total = g->n_edges * (int64_t)H;
  k_gat_alpha_csr<<<(unsigned)ceil_div(total, 256), 256, 0, as_stream(stream)>>>(
      g->col, slot_row, g->n_edges, H, a_src, a_dst, slope, row_stats, alpha_csr, score);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_sddmm_f32(const mp_csr* g, const int32_t* slot_row, const float* grow, int64_t ldg, const float* x,
                     int64_t ldx, int32_t H, int32_t C, float* out, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(g && H > 0 && C > 0, "mp_gat_sddmm_f32: bad argument");
  if (g->n_edges == 0) return MP_OK;
  MP_CHECK_ARG(g->col && slot_row && grow && x && out, "mp_gat_sddmm_f32: null pointer");
  const int64_t F = (int64_t)H * C;
  MP_CHECK_ARG(ldg >= F && ldx >= F, "mp_gat_sddmm_f32: leading dimension < H*C");
  hipStream_t s = as_stream(stream);
  auto aligned4 = [](const void* p, int64_t ld) { return (uintptr_t)p % 16 == 0 && ld % 4 == 0; };
  const bool v4 = C % 4 == 0 && aligned4(grow, ldg) && aligned4(x, ldx);
  const int vec = v4 ? 4 : 1;
  const int G = C / vec;
  if (G >= 1 && G <= 64 && (G & (G - 1)) == 0) {
    dim3 grid((unsigned)ceil_div(ceil_div(g->n_edges, 256), 4), (unsigned)ceil_div(F, 64 * vec));
    if (v4) k_gat_sddmm<4><<<grid, 256, 0, s>>>(g->col, slot_row, g->n_edges, grow, ldg, x, ldx, H, C, G, out);
    else k_gat_sddmm<1><<<grid, 256, 0, s>>>(g->col, slot_row, g->n_edges, grow, ldg, x, ldx, H, C, G, out);
  } else {
    int64_t total = g->n_edges * (int64_t)H;
    k_gat_sddmm_scalar<<<(unsigned)ceil_div(total, 256), 256, 0, s>>>(g->col, slot_row, g->n_edges, grow, ldg,
                                                                      x, ldx, H, C, out);
  }
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_backward_prep_train_f32(const float* grad_out, int64_t ldg, const float* agg, int64_t lda,
                                   const float* bias, const float* agg2, const float* row_s2, const float* a_dst,
                                   const float* row_stats, int64_t n, int32_t H, int32_t C, float* pack,
                                   size_t pack_bytes, float* gsum_part, size_t gsum_part_bytes, float* grad_a_dst,
                                   void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(H > 0 && C > 0 && n >= 0, "mp_gat_backward_prep_train_f32: bad sizes");
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(grad_out && agg && agg2 && row_s2 && a_dst && row_stats && pack && grad_a_dst,
               "mp_gat_backward_prep_train_f32: null pointer");
  const int64_t F = (int64_t)H * C;
  MP_CHECK_EXTENT("mp_gat_backward_prep_train_f32", "pack", pack_bytes, (size_t)n * H * 16);
  if (gsum_part)
    MP_CHECK_EXTENT("mp_gat_backward_prep_train_f32", "gsum_part", gsum_part_bytes,
                    (size_t)mp_gat_bwd_blocks(n) * F * 4);
  const int G = C / 4;
  MP_CHECK_ARG(C % 4 == 0 && G <= 64 && (G & (G - 1)) == 0, "mp_gat_backward_prep_train_f32: needs C/4 a power of two");
  MP_CHECK_ARG((uintptr_t)pack % 16 == 0 && (uintptr_t)grad_out % 16 == 0 && (uintptr_t)agg % 16 == 0 &&
                   (uintptr_t)agg2 % 16 == 0 && ldg % 4 == 0 && lda % 4 == 0,
               "mp_gat_backward_prep_train_f32: 16-byte alignment required");
  MP_CHECK_ARG((uintptr_t)bias % 16 == 0, "mp_gat_backward_prep_train_f32: bias must be 16-byte aligned");
  MP_CHECK_ARG(ldg >= F && lda >= F, "mp_gat_backward_prep_train_f32: leading dimension < H*C");
  MP_CHECK_ARG(!gsum_part || F <= 256, "mp_gat_backward_prep_train_f32: gsum_part needs H*C <= 256");
  k_gat_bwd_prep_wave<<<(unsigned)mp_gat_bwd_blocks(n), 256, 0, as_stream(stream)>>>(
      grad_out, ldg, agg, lda, a_dst, row_stats, n, H, C, G, pack, gsum_part, bias, agg2, row_s2, grad_a_dst);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_col_sums_f32(const float* x, int64_t ldx, int64_t n, int32_t F, float* part, size_t part_bytes,
                    void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(n >= 0 && F > 0 && F <= 256 && F % 4 == 0, "mp_col_sums_f32: needs 0 < F <= 256, F %% 4 == 0");
  MP_CHECK_ARG(part && (n == 0 || (x && ldx >= F && ldx % 4 == 0 && (uintptr_t)x % 16 == 0)),
               "mp_col_sums_f32: bad argument (16-byte aligned rows required)");
  const int nb = mp_gat_bwd_blocks(n);
  MP_CHECK_EXTENT("mp_col_sums_f32", "part", part_bytes, (size_t)nb * F * 4);
  if (n == 0) {
    MP_CHECK_HIP(hipMemsetAsync(part, 0, (size_t)nb * F * sizeof(float), as_stream(stream)));
    return MP_OK;
  }
  k_col_sums<<<(unsigned)nb, 256, 0, as_stream(stream)>>>(x, ldx, n, F, part);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_bwd_blocks(int64_t n) {
  int64_t b = ceil_div(n, 4);
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

int mp_gat_backward_prep_f32(const float* grad_out, int64_t ldg, const float* agg, int64_t lda, const float* bias,
                             const float* a_dst,
                             const float* row_stats, int64_t n, int32_t H, int32_t C, float* pack,
                             size_t pack_bytes, float* gsum_part, size_t gsum_part_bytes, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(H > 0 && C > 0 && n >= 0, "mp_gat_backward_prep_f32: bad sizes");
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(grad_out && agg && a_dst && row_stats && pack, "mp_gat_backward_prep_f32: null pointer");
  MP_CHECK_ARG((uintptr_t)pack % 16 == 0, "mp_gat_backward_prep_f32: pack must be 16-byte aligned");
  const int64_t F = (int64_t)H * C;
  MP_CHECK_EXTENT("mp_gat_backward_prep_f32", "pack", pack_bytes, (size_t)n * H * 16);
  if (gsum_part)
    MP_CHECK_EXTENT("mp_gat_backward_prep_f32", "gsum_part", gsum_part_bytes, (size_t)mp_gat_bwd_blocks(n) * F * 4);
  MP_CHECK_ARG(ldg >= F && lda >= F, "mp_gat_backward_prep_f32: leading dimension < H*C");
  hipStream_t s = as_stream(stream);
  const int G = C / 4;
  const bool v4 = C % 4 == 0 && G <= 64 && (G & (G - 1)) == 0 && (uintptr_t)grad_out % 16 == 0 &&
                  (uintptr_t)agg % 16 == 0 && ldg % 4 == 0 && lda % 4 == 0 && (uintptr_t)bias % 16 == 0;
  MP_CHECK_ARG(!gsum_part || (v4 && F <= 256), "mp_gat_backward_prep_f32: gsum_part needs C%%4==0 and H*C<=256");
  if (v4) {
    k_gat_bwd_prep_wave<<<(unsigned)mp_gat_bwd_blocks(n), 256, 0, s>>>(grad_out, ldg, agg, lda, a_dst, row_stats, n,
                                                                      H, C, G, pack, gsum_part, bias);
  } else {
    k_gat_bwd_prep_scalar<<<(unsigned)ceil_div(n * H, 256), 256, 0, s>>>(grad_out, ldg, agg, lda, bias, a_dst,
                                                                         row_stats, n, H, C, pack);
  }
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_gat_backward_finish_f32(float* grad_xw, const float* xw, const float* ga_dst, const float* ga_src,
                                const float* att, int64_t n, int32_t H, int32_t C, float* att_part,
                                size_t att_part_bytes, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(H > 0 && C > 0 && n >= 0, "mp_gat_backward_finish_f32: bad sizes");
  MP_CHECK_ARG(C % 4 == 0 && H * C <= 256, "mp_gat_backward_finish_f32: needs C %% 4 == 0 and H*C <= 256");
  MP_CHECK_ARG(xw && ga_dst && ga_src && att && att_part, "mp_gat_backward_finish_f32: null pointer");
  MP_CHECK_EXTENT("mp_gat_backward_finish_f32", "att_part", att_part_bytes,
                  (size_t)mp_gat_bwd_blocks(n) * 2 * H * C * 4);
  MP_CHECK_ARG((uintptr_t)grad_xw % 16 == 0 && (uintptr_t)xw % 16 == 0 && (uintptr_t)att % 16 == 0,
               "mp_gat_backward_finish_f32: 16-byte alignment required");
  k_gat_bwd_finish<<<(unsigned)mp_gat_bwd_blocks(n), 256, 0, as_stream(stream)>>>(grad_xw, xw, ga_dst, ga_src, att, n,
                                                                                 H, C, att_part);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

int mp_heads_outer_add_f32(float* y, int64_t ldy, const float* s, int64_t n, int32_t H, int32_t C, const float* att,
                           int64_t att_ld, void* stream) {
  MP_DEVICE_GUARD(stream);
  MP_CHECK_ARG(H > 0 && C > 0 && n >= 0, "mp_heads_outer_add_f32: bad sizes");
  if (n == 0) return MP_OK;
  MP_CHECK_ARG(y && s && att && ldy >= (int64_t)H * C && att_ld >= C, "mp_heads_outer_add_f32: bad argument");
  hipStream_t st = as_stream(stream);
  const bool v4 = C % 4 == 0 && (uintptr_t)y % 16 == 0 && ldy % 4 == 0 && (uintptr_t)att % 16 == 0 && att_ld % 4 == 0;
  if (v4) {
    const int64_t total = n * H * C / 4;
    k_heads_outer_add<4><<<(unsigned)ceil_div(total, 256), 256, 0, st>>>(y, ldy, s, n, H, C, att, att_ld);
  } else {
    const int64_t total = n * H * C;
    k_heads_outer_add<1><<<(unsigned)ceil_div(total, 256), 256, 0, st>>>(y, ldy, s, n, H, C, att, att_ld);
  }
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
