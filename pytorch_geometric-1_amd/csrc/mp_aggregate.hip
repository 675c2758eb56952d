// Fused gather -> message -> segment-reduce for gfx950 (MI355X).
//
// Replaces, for one MessagePassing.propagate() [U1]:
//   x_j = x.index_select(0, edge_index[j])             (ATen index_select, [E',F] in HBM)
//   msg = norm.view(-1,1) * x_j   (GCNConv.message)    (elementwise, [E',F] in HBM)
//   out = torch_scatter.scatter_{sum,mean,max,min}(msg, edge_index[i], 0, dim_size=N)
//   out = out + bias              (GCNConv.update)
// with one pass that reads each x_j row once and writes each output row once.
//
// Mapping to CDNA4:
//   * one wave (64 lanes) = one merge-path task: `chunk` work units where a unit
//     is either "gather one CSR slot" or "finish one row" (mp_csr.hip).  Every
//     wave therefore does the same amount of work whatever the in-degree
//     distribution (RMAT hubs have ~1e4-1e5 in-edges, most rows < 10).
//   * a lane owns VEC consecutive features (VEC=4: one dwordx4, a 256-feature
//     row is one 1 KiB coalesced wave load); gridDim.y tiles wider rows.
//   * the wave walks its slots in CSR order; col/weight/eid for 64 slots are
//     loaded once per 64 slots (one coalesced dword per lane, next window
//     prefetched) and broadcast with v_readlane -> the x-row address is a
//     scalar base + lane offset.  U x-row loads are in flight per wave.
//   * accumulation stays in VGPRs; a row is stored once (no atomics).  A row
//     whose slots cross a task boundary leaves partials in a slab; a small
//     fix-up kernel combines them in task order (deterministic).
//   * sum uses separately-rounded mul and add (no FMA contraction) in original
//     edge order, i.e. exactly the arithmetic of the reference's materialised
//     `norm*x_j` followed by CPU scatter_add_: rows that fit in one task are
//     bit-identical to the oracle.
#include <atomic>
#include <cmath>
#include <cxxabi.h>
#include <stdlib.h>
#include <type_traits>
#include <float.h>

#include "mp_common.h"

// Kernel-shape constants.  Every value below was chosen by an in-process A/B
// with bitwise-equal outputs; dispatch-level choices that
// tests and A/B runs switch at run time go through mp_tune (one table, below).
namespace mp {
constexpr int kU_Vec4 = 8;      // x-row loads in flight per task (VEC=4, 64-lane tasks: GAT)
constexpr int kU_Vec2 = 16;     // x-row loads in flight per task (VEC=2: the flat kernel, 128-feature tiles)
constexpr int kU_Vec1 = 16;     // x-row loads in flight per task (VEC=1)
#ifndef MP_U_VEC1_FAR
#define MP_U_VEC1_FAR 8
#endif
constexpr int kU_Vec1Far = MP_U_VEC1_FAR;  // ... scalar-batch sum/mean over an x larger than the Infinity Cache
#ifndef MP_U_GAT_TRAIN
#define MP_U_GAT_TRAIN 4
#endif
constexpr int kU_GatTrain = MP_U_GAT_TRAIN;  // ... the GAT training forward (A/B U=4/6/8: 8.36/8.57/8.52 ms)
constexpr int kU_Narrow = 12;   // x-row loads in flight per task (VEC=4, tasks of < 64 lanes)
constexpr int kWideLanes = 32;  // lanes per task of k_agg_main for rows of >= 256 features (32 beats 64 by ~9%)
constexpr int kGatLanes = 64;   // lanes per GAT task for H*C >= 256
constexpr bool kNtOut = true;   // non-temporal output-row stores (A/B: -0.4%)
constexpr bool kNtIdx = true;   // non-temporal col/weight/eid stream loads (A/B: -0.3%)
constexpr bool kXcdTiles = true;  // feature tile = (block % 8) % tiles when tiles divide 8: each XCD's L2
                                  // holds one tile (A/B: -1.5%)
constexpr int kLaneMaxF = 8;    // rows of 2..this many features: one task per lane (A/B: wins at F=4,8)
constexpr int64_t kSeqTilesMin = 384ll << 20;  // mp_aggregate_tiles_f32: sequential feature tiles above this x
constexpr int kULane = 8;       // slots in flight per lane task
}  // namespace mp

namespace mp {

template <int VEC>
__device__ __forceinline__ void store_out(float* p, const Frag<VEC>& f) {
  if constexpr (kNtOut) store_frag_nt<VEC>(p, f);
  else store_frag<VEC>(p, f);
}

template <class T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (kNtIdx) return __builtin_nontemporal_load(p);
  else return *p;
}

constexpr int kWavesPerBlock = 4;
constexpr int kBlock = 64 * kWavesPerBlock;

struct AggArgs {
  // graph + schedule
  const int32_t* rowptr;
  const int32_t* col;
  const int32_t* eid;
  const int32_t* wave_row;
  const int32_t* wave_slot;
  const int32_t* split_waves;
  int64_t n_rows;
  int64_t n_edges;
  int64_t n_ids;     // edge-id space (empty max/min rows report this arg)
  int32_t chunk;
  int32_t n_waves;
  int32_t n_split;
  int32_t F;
  int32_t n_cols;
  uint32_t x_bytes;  // extent of x for the scalar-batch buffer path (0: not used)
  int32_t flat;      // sum/mean/max/min: run k_agg_flat instead of k_agg_main
  int32_t fix4;      // VEC=2 main kernel: run the fix-up at VEC=4 (slabs are indexed by feature)
  int32_t smem;      // flat sum/mean kernel: slot columns/weights through scalar loads (k_agg_flat SM)
  int32_t seq_tiles; // flat kernel: feature tiles one after another on all XCDs (no XCD-affine map)
  int32_t far;       // flat SM kernel: x larger than the Infinity Cache (batches of kU_Vec1Far)
  int32_t force_flat;  // mp_aggregate_tiles_f32: the scalar-batch flat kernel whatever the layout
  int32_t xr;          // ... and its XR instance (tile-major operands, skipped rows, per-row bias)
  // features
  const float* w;
  const float* x;
  int64_t ldx;
  int32_t flags;
  const float* bias;
  float* out;
  int64_t ldo;
  int64_t* arg_out;
  // partial slabs: slot index s = 2*task + kind (kind 0 = continuation, 1 = head)
  float* slab_v;
  int32_t* slab_a;
  int64_t slab_ld;
  // GAT
  const float* a_src;
  const float* a_dst;
  float* a_src_out;   // GAT forward with in-kernel node scores (GatRed ND): written per owned row
  float* a_dst_out;
  int32_t H;
  int32_t C;
  float slope;
  float* row_stats;
  float* slab_s;
  const int32_t* slot_row;  // two-pass GAT: row owning each CSR slot
  // GAT backward (transposed CSR: rows = source nodes j, col = destination i)
  const float* y;     // xw, the row's own features (d alpha = <g_i, xw_j>)
  int64_t ldy;
  const f32x4* pack;  // [n_cols, H]  (a_dst, m, 1/den, rs) of the destination, rs = <g_i, agg_i>_h
  float* de;          // [n_edges, H] d score per slot (this CSR's slot order)
  float* ga;          // [n_rows, H]  d a_src = row sums of d score
  const float* ga_dst_in;  // [n_rows, H] d a_dst of each row (node-wise, training forward): the
                           // row's d xw also takes d a_dst (x) att_dst at its finish
  const float* att;   // [H, 2C]      (att_dst | att_src)
  // GAT training forward (GatRed<.., TR>): out2[r, f] = sum_k alpha leaky' xw (ld F),
  // row_s2[r, h] = sum_k alpha leaky', and their partial slabs
  float* out2;
  float* row_s2;
  float* agg_nb;  // pre-bias output (ld F), when the output carries the bias
  float* slab_v2;
  float* slab_s2;
  // GAT attention dropout (training: F.dropout on alpha, see drop_bits)
  uint64_t drop_seed;
  uint32_t drop_thr;
  float drop_scale;
  const int32_t* drop_ids;  // (ABI 7) the key of each slot of this CSR (an edge id), or NULL: the dst slot
  // tile-major operands (mp_aggregate_tiles_f32; 0 = row-major): feature f of
  // row r at x[(f / x_tw) * x_ts + r * x_tw + f % x_tw], likewise out with o_tw
  // / o_ts.  Widths are multiples of 64, so a flat-kernel block's 64-feature
  // tile lies inside one operand tile.
  int32_t x_tw;
  int32_t o_tw;
  int64_t x_ts;
  int64_t o_ts;
  // per-row bias flags (mp_aggregate_tiles_f32; NULL = every row): the bias is
  // added to row r only where bias_rows[r] != 0
  const int32_t* bias_rows;
};

// This block's view of tile-major operands: x_tile / ldx_tile / fx0 address
// feature f of row r at x_tile[r * ldx_tile + f - fx0]; out is rebased in place
// so that out + r * ldo + f addresses it (fb: the block's first feature).
__device__ __forceinline__ void tile_view(AggArgs& p, int fb, const float*& x_tile, int64_t& ldx_tile, int& fx0) {
  x_tile = p.x;
  ldx_tile = p.ldx;
  fx0 = 0;
  if (p.x_tw) {
    const int t = fb / p.x_tw;
    x_tile = p.x + (int64_t)t * p.x_ts;
    ldx_tile = p.x_tw;
    fx0 = t * p.x_tw;
  }
  if (p.o_tw) {
    const int t = fb / p.o_tw;
    p.out += (int64_t)t * (p.o_ts - p.o_tw);
    p.ldo = p.o_tw;
  }
}

// ---------------------------------------------------------------------------
// GAT attention dropout (GATConv training: `F.dropout(alpha, p)` after the
// softmax [U6]).  The keep bit of (k, h) -- k the edge's key, h the head -- is
// a counter-based hash of (seed, k * H + h) compared with p * 2^32, so the
// forward and the transposed backward evaluate the same mask without storing
// it; a kept alpha is scaled by 1 / (1 - p).  The key (ABI 7) comes from a
// per-slot array of each pass's CSR (drop_ids): the layer's edge id on one
// GPU, the GLOBAL edge id on a shard -- so a sharded layer draws the
// single-GPU mask; without the array it is the edge's destination-CSR slot.
// oracle/pyg_ref.py restates the hash.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t drop_mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint64_t idx) {
  const uint32_t a = drop_mix32((uint32_t)idx ^ (uint32_t)seed);
  return drop_mix32(a + 0x9E3779B9u * ((uint32_t)(idx >> 32) ^ (uint32_t)(seed >> 32)) + 0x632BE5ABu);
}
// keep bits of slot s, bit h for head h (H <= 32)
__device__ __forceinline__ uint32_t drop_bits(const AggArgs& p, int64_t s) {
  const uint64_t base = (uint64_t)s * (uint64_t)p.H;
  uint32_t b = 0;
  for (int h = 0; h < p.H; ++h) b |= (uint32_t)(drop_hash(p.drop_seed, base + (uint64_t)h) >= p.drop_thr) << h;
  return b;
}
__device__ __forceinline__ float drop_factor(const AggArgs& p, uint32_t bits, int h) {
  return ((bits >> h) & 1u) ? p.drop_scale : 0.f;
}

// ---------------------------------------------------------------------------
// Reducers: per-lane state for VEC features of one (partial) row.
//
// A partial (the state of a row cut at a task boundary) lives in a slab slot
// in HBM between the main kernel and the fix-up, and in LDS between the
// waves of one fix-up block.  PRef points at one lane's share of a partial:
//   v  : VEC values,  a : VEC arg ids (max/min),  st : (m, s) pair (GAT).
// Red::Part is the same state in registers, so a chain of partials can be
// loaded U at a time (U loads in flight) and merged in order.
// ---------------------------------------------------------------------------

struct PRef {
  float* v;
  int32_t* a;
  float* st;
  float* v2;  // GAT training forward: second accumulator, and its per-head sum
  float* s2;
};

template <int VEC, bool HAS_W, bool MEAN>
struct SumRed {
  static constexpr bool kW = HAS_W;
  static constexpr bool kEid = false;
  static constexpr bool kGat = false;
  static constexpr bool kHW = false;
  static constexpr bool kGatB = false;
  static constexpr bool kStat = false;
  struct Part {
    float v[VEC];
  };
  float acc[VEC];
  // the bias features of this lane, read once per task (preload_bias) by the
  // short-row passes of mp_aggregate_tiles_f32 (k_agg_flat XM != 0)
  float bv[VEC];
  bool pre = false;
  int h = 0;  // unused (GAT only)

  __device__ SumRed() {}
  __device__ SumRed(const AggArgs&, int, bool) {}

  // A bias load per row is waited for at the row's end, and the wait (vmcnt
  // retires in order) also drains every gather issued before it -- the next
  // rows' prefetched batch.  On the sharded step's short rows (4.4 edges a row)
  // that cost the interior pass 19 % (tools/exp_interior.py: 0.287 -> 0.245
  // ms); on the one-GPU kernel's long rows the per-row load measured faster
  // (1-3 %), so only the tile launches take it once per task.
  __device__ __forceinline__ void preload_bias(const AggArgs& p, int f, bool act) {
    if (p.bias && act) {
      Frag<VEC> b = load_frag<VEC>(p.bias + f);
#pragma unroll
      for (int k = 0; k < VEC; ++k) bv[k] = b.v[k];
    }
    pre = true;
  }
  __device__ __forceinline__ Frag<VEC> bias_of(const AggArgs& p, int f) const {
    if (pre) {
      Frag<VEC> b;
#pragma unroll
      for (int k = 0; k < VEC; ++k) b.v[k] = bv[k];
      return b;
    }
    return load_frag<VEC>(p.bias + f);
  }

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool owned, int f, bool act) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    if (owned && (p.flags & MP_FLAG_INIT_FROM_OUT) && act) {
      Frag<VEC> o = load_frag<VEC>(p.out + row * p.ldo + f);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = o.v[k];
    }
  }
  __device__ __forceinline__ void consume(const Frag<VEC>& v, float wt, int, float) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __fadd_rn(acc[k], HAS_W ? __fmul_rn(wt, v.v[k]) : v.v[k]);
  }
  __device__ __forceinline__ void save(PRef r, bool) const {
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
    store_frag<VEC>(r.v, o);
  }
  static __device__ __forceinline__ Part load(PRef r) {
    Frag<VEC> o = load_frag<VEC>(r.v);
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = o.v[k];
    return q;
  }
  __device__ __forceinline__ void set(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = q.v[k];
  }
  __device__ __forceinline__ void merge(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __fadd_rn(acc[k], q.v[k]);
  }
  __device__ __forceinline__ Part part() const {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = acc[k];
    return q;
  }
  // sum with the bias scaled by a per-row 0 / 1 flag (k_agg_flat XM 1): o + b * 1
  // is o + b bit for bit; o + b * 0 is o (a -0 row reads +0: equal values)
  __device__ __forceinline__ void finish_scaled_bias(const AggArgs& p, int64_t row, int64_t cnt, int f, bool act,
                                                     float bs) {
    if (!act) return;
    Frag<VEC> o;
    float c = (float)(cnt > 0 ? cnt : 1);
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = MEAN ? __fdiv_rn(acc[k], c) : acc[k];
    if (p.bias) {
      Frag<VEC> b = bias_of(p, f);
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = __fadd_rn(o.v[k], __fmul_rn(b.v[k], bs));
    }
    store_out<VEC>(p.out + row * p.ldo + f, o);
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t cnt, int f, bool act, bool with_bias = true) {
    if (!act) return;
    Frag<VEC> o;
    float c = (float)(cnt > 0 ? cnt : 1);
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = MEAN ? __fdiv_rn(acc[k], c) : acc[k];
    if (p.bias && with_bias) {
      Frag<VEC> b = bias_of(p, f);
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = __fadd_rn(o.v[k], b.v[k]);
    }
    store_out<VEC>(p.out + row * p.ldo + f, o);
  }
};

// torch_scatter CPU scatter_max/min [U9]: out starts at lowest()/max(),
// arg at src.size(0); strict compare so the FIRST edge (in original order)
// wins ties; afterwards out==init -> 0 (only when out was not passed in).
// Partials are merged in task order with the same strict compare: a later
// task only holds later edges of the row, so the first maximum survives.
template <int VEC, bool HAS_W, bool IS_MAX>
struct ArgRed {
  static constexpr bool kW = HAS_W;
  static constexpr bool kEid = true;
  static constexpr bool kGat = false;
  static constexpr bool kHW = false;
  static constexpr bool kGatB = false;
  static constexpr bool kStat = false;
  struct Part {
    float v[VEC];
    int a[VEC];
  };
  float m[VEC];
  int a[VEC];
  int h = 0;
  int sentinel;

  __device__ ArgRed() {}
  __device__ ArgRed(const AggArgs& p, int, bool) : sentinel((int)p.n_ids) {}

  static __device__ __forceinline__ float init_val() { return IS_MAX ? -FLT_MAX : FLT_MAX; }
  static __device__ __forceinline__ bool better(float v, float cur) { return IS_MAX ? (v > cur) : (v < cur); }

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool owned, int f, bool act) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      m[k] = init_val();
      a[k] = sentinel;
    }
    if (owned && (p.flags & MP_FLAG_INIT_FROM_OUT) && act) {
      Frag<VEC> o = load_frag<VEC>(p.out + row * p.ldo + f);
#pragma unroll
      for (int k = 0; k < VEC; ++k) m[k] = o.v[k];
    }
  }
  __device__ __forceinline__ void consume(const Frag<VEC>& v, float wt, int e, float) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      float val = HAS_W ? __fmul_rn(wt, v.v[k]) : v.v[k];
      if (better(val, m[k])) {
        m[k] = val;
        a[k] = e;
      }
    }
  }
  __device__ __forceinline__ void save(PRef r, bool) const {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      r.v[k] = m[k];
      r.a[k] = a[k];
    }
  }
  static __device__ __forceinline__ Part load(PRef r) {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      q.v[k] = r.v[k];
      q.a[k] = r.a[k];
    }
    return q;
  }
  __device__ __forceinline__ void set(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      m[k] = q.v[k];
      a[k] = q.a[k];
    }
  }
  __device__ __forceinline__ void merge(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      if (better(q.v[k], m[k])) {
        m[k] = q.v[k];
        a[k] = q.a[k];
      }
    }
  }
  __device__ __forceinline__ Part part() const {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      q.v[k] = m[k];
      q.a[k] = a[k];
    }
    return q;
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t, int f, bool act, bool with_bias = true) {
    if (!act) return;
    Frag<VEC> o;
    const bool from_out = (p.flags & MP_FLAG_INIT_FROM_OUT) != 0;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      float v = m[k];
      if (!from_out && v == init_val()) v = 0.f;
      if (p.flags & MP_FLAG_PYG_MASK) {
        if (IS_MAX ? (v < -10000.f) : (v > 10000.f)) v = 0.f;
      }
      if (p.bias) v = __fadd_rn(v, p.bias[f + k]);
      o.v[k] = v;
    }
    store_out<VEC>(p.out + row * p.ldo + f, o);
    int64_t* ao = p.arg_out + row * (int64_t)p.F + f;
#pragma unroll
    for (int k = 0; k < VEC; ++k) ao[k] = (int64_t)a[k];
  }
};

// GATConv [U6] + utils.softmax [U3], online: per (row, head) running max m,
// denominator s and accumulator acc, rescaled when the max grows.  Every lane
// of a head carries the same m/s (no cross-lane traffic).
//
// OWN: a_src[j, h] is recomputed from the gathered row itself,
//   a_src[j,h] = <xw[j,h,:], att[h,C:2C]>  (lane partial of its VEC features,
// then group_sum over the head's lanes -- the same arithmetic, in the same
// order, as k_gat_node_scores_wave, so bitwise the value that kernel stores).
// It saves the per-slot a_src gather (one 256-B L1-queue segment per slot on
// top of the row's four).
//
// TR (training forward): also accumulates, with the same online rescaling,
//   acc2 = sum_k alpha_k leaky'_k x_k  and  s2 = sum_k alpha_k leaky'_k
// (leaky' = 1 or slope at the pre-activation a_src + a_dst), written to
// out2 / row_s2.  They make the backward's d a_dst node-wise:
//   d a_dst[i,h] = sum_j de_ij = <g_i, acc2_i>_h - rs_i s2_i
// (de_ij = alpha_ij (<g_i, xw_j> - rs_i) leaky'_ij), so the backward writes no
// per-edge d score and needs no segmented pass over it.
//
// ND (node scores, needs OWN): a_dst[i, h] and a_src[i, h] of each destination
// row come from the row's own xw, loaded at begin() and reduced at the first
// slot (its load completes before the first gathered row's, so the wait is
// hidden) with the node-score kernel's arithmetic -- bitwise its values; the
// row's owner task writes both to a_src_out / a_dst_out, so no separate
// node-score pass over xw is needed.
// DR (attention dropout, training): slot weight pe * keep / (1 - p) on the
// aggregates (acc, acc2), the softmax sums (s, s2) unchanged.
template <int VEC, bool OWN = false, bool TR = false, bool ND = false, bool DR = false>
struct GatRed {
  static_assert(!ND || OWN, "in-kernel node scores reuse the own-a_src reduction");
  static constexpr bool kDrop = DR;
  static constexpr bool kW = false;
  static constexpr bool kEid = false;
  static constexpr bool kGat = true;
  static constexpr bool kOwnAs = OWN;
  static constexpr bool kNodeScores = ND;
  static constexpr bool kHW = false;
  static constexpr bool kGatB = false;
  static constexpr bool kStat = true;
  struct Part {
    float v[VEC];
    float m, s;
    float v2[TR ? VEC : 1];
    float s2;
  };
  float acc[VEC];
  float m, s, ad;
  [[maybe_unused]] float acc2[TR ? VEC : 1];
  [[maybe_unused]] float s2 = 0.f;
  int h;
  [[maybe_unused]] float y[OWN ? VEC : 1];
  [[maybe_unused]] int hl = 1;
  [[maybe_unused]] Frag<ND ? VEC : 1> rowv;  // the destination row's own xw (ND)
  [[maybe_unused]] bool need_ad = false, own_row = false, lead = false;
  [[maybe_unused]] int c_ = 0;               // this lane's first feature within its head (ND)
  [[maybe_unused]] int64_t row_ = 0;

  __device__ GatRed(const AggArgs& p, int f, bool act) : h(act ? f / p.C : 0) {
    if constexpr (OWN) {
      hl = p.C / VEC;
      const int c = act ? f % p.C : 0;
      Frag<VEC> o = load_frag<VEC>(p.att + (int64_t)h * 2 * p.C + p.C + c);
#pragma unroll
      for (int k = 0; k < VEC; ++k) y[k] = act ? o.v[k] : 0.f;
      if constexpr (ND) {
        c_ = c;
        lead = act && c == 0;
      }
    }
  }
  // the row's scores from rowv; the owner writes them (every lane of the
  // wave runs this together: the group sums are cross-lane)
  __device__ __forceinline__ void node_scores(const AggArgs& p) {
    if constexpr (ND) {
      // att_dst slice: an L1-resident 16-B load per row rather than 4 VGPRs held
      // through the slot loop (keeps the kernel at the OWN path's occupancy)
      const Frag<VEC> yd = load_frag<VEC>(p.att + (int64_t)h * 2 * p.C + c_);
      float t = rowv.v[0] * yd.v[0];
#pragma unroll
      for (int k = 1; k < VEC; ++k) t = t + rowv.v[k] * yd.v[k];
      ad = group_sum(t, hl);
      const float as_own = own_as(rowv);
      need_ad = false;
      if (own_row && lead) {
        p.a_dst_out[row_ * p.H + h] = ad;
        p.a_src_out[row_ * p.H + h] = as_own;
      }
    }
  }
  // before a partial of an owned row is saved (its task may have seen none of
  // its slots): make sure the row's scores were written
  __device__ __forceinline__ void flush_scores(const AggArgs& p) {
    if constexpr (ND) {
      if (need_ad) node_scores(p);
    }
  }
  // <row, att_src> over the head's lanes: v.x*y.x + v.y*y.y + ... separately
  // rounded left to right (-ffp-contract=off), then group_sum
  __device__ __forceinline__ float own_as(const Frag<VEC>& v) const {
    float t = v.v[0] * y[0];
#pragma unroll
    for (int k = 1; k < VEC; ++k) t = t + v.v[k] * y[k];
    return group_sum(t, hl);
  }

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool owned, int f, bool act) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    if constexpr (TR) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc2[k] = 0.f;
      s2 = 0.f;
    }
    m = -INFINITY;
    s = 0.f;
    if constexpr (ND) {
      rowv = load_frag<VEC>(p.x + row * p.ldx + (act ? f : 0));
      need_ad = true;
      own_row = owned;
      row_ = row;
    } else {
      ad = p.a_dst[row * p.H + h];
    }
  }
  __device__ __forceinline__ void consume_gat(const AggArgs& p, const Frag<VEC>& v, float as,
                                              [[maybe_unused]] uint32_t dbits = 0) {
    float a = as + ad;
    [[maybe_unused]] const bool pos = a > 0.f;  // leaky' = 1 : slope (the backward's test)
    a = a > 0.f ? a : a * p.slope;  // F.leaky_relu
    // mn = fmaxf(m, a); sc = expf(m - mn); pe = expf(a - mn) with one exp:
    // one of the two arguments is x - x, i.e. 0 (exp 1) or NaN for an
    // infinite x, so (x - x) + 1 reproduces it bit for bit, NaNs included
    // (config 3: 7.81 -> 7.74 ms)
    const bool up = a > m;
    const float e = expf(up ? m - a : a - m);
    const float sc = up ? e : (m - m) + 1.f;
    const float pe = up ? (a - a) + 1.f : e;
    s = s * sc + pe;
    [[maybe_unused]] float dsc = 1.f;
    if constexpr (DR) {
      dsc = drop_factor(p, dbits, h);
      const float pd = pe * dsc;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = acc[k] * sc + pd * v.v[k];
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = acc[k] * sc + pe * v.v[k];
    }
    if constexpr (TR) {
      const float pl = pos ? pe : pe * p.slope;
      s2 = s2 * sc + pl;
      const float pld = DR ? pl * dsc : pl;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc2[k] = acc2[k] * sc + pld * v.v[k];
    }
    m = up ? a : m;
  }
  __device__ __forceinline__ void consume(const Frag<VEC>&, float, int, float) {}
  __device__ __forceinline__ void save(PRef r, bool stat_writer) const {
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
    store_frag<VEC>(r.v, o);
    if (stat_writer) {
      r.st[0] = m;
      r.st[1] = s;
    }
    if constexpr (TR) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = acc2[k];
      store_frag<VEC>(r.v2, o);
      if (stat_writer) *r.s2 = s2;
    }
  }
  static __device__ __forceinline__ Part load(PRef r) {
    Frag<VEC> o = load_frag<VEC>(r.v);
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = o.v[k];
    q.m = r.st[0];
    q.s = r.st[1];
    if constexpr (TR) {
      Frag<VEC> o2 = load_frag<VEC>(r.v2);
#pragma unroll
      for (int k = 0; k < VEC; ++k) q.v2[k] = o2.v[k];
      q.s2 = *r.s2;
    }
    return q;
  }
  __device__ __forceinline__ void set(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = q.v[k];
    m = q.m;
    s = q.s;
    if constexpr (TR) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc2[k] = q.v2[k];
      s2 = q.s2;
    }
  }
  __device__ __forceinline__ void merge(const Part& q) {
    float mn = fmaxf(m, q.m);
    float c0 = expf(m - mn), c1 = expf(q.m - mn);
    s = s * c0 + q.s * c1;
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = acc[k] * c0 + q.v[k] * c1;
    if constexpr (TR) {
      s2 = s2 * c0 + q.s2 * c1;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc2[k] = acc2[k] * c0 + q.v2[k] * c1;
    }
    m = mn;
  }
  __device__ __forceinline__ Part part() const {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = acc[k];
    q.m = m;
    q.s = s;
    if constexpr (TR) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) q.v2[k] = acc2[k];
      q.s2 = s2;
    }
    return q;
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t, int f, bool act, bool with_bias = true) {
    if constexpr (ND) {
      if (need_ad) node_scores(p);  // a row without slots (the fix-up never begins a row: need_ad false)
    }
    if (!act) return;
    Frag<VEC> o;
    float den = s + 1e-16f;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k] / den;
    if constexpr (TR) {  // the pre-bias aggregate the backward's rs needs
      if (p.agg_nb) store_out<VEC>(p.agg_nb + row * (int64_t)p.F + f, o);
    }
    if (p.bias) {
      Frag<VEC> b = load_frag<VEC>(p.bias + f);
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = o.v[k] + b.v[k];
    }
    store_out<VEC>(p.out + row * p.ldo + f, o);
    if (p.row_stats && (f % p.C == 0)) {
      p.row_stats[(row * p.H + h) * 2] = m;
      p.row_stats[(row * p.H + h) * 2 + 1] = den;
    }
    if constexpr (TR) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = acc2[k] / den;
      store_out<VEC>(p.out2 + row * (int64_t)p.F + f, o);
      if (f % p.C == 0) p.row_s2[row * p.H + h] = s2 / den;
    }
  }
};

// Two-pass GAT (mp_gat_softmax_aggregate_f32): utils.softmax's row statistics
// [U3] as their own merge-path passes over x = a_src [N, H] (F = H, one lane
// task per row holding every head, k_agg_lane), then the aggregation as a
// weighted sum whose weights are the reference's alpha.
//   pass 1 (GatMaxRed): m[r,h]   = max_k leaky(a_src[col_k,h] + a_dst[r,h])
//   pass 2 (GatDenRed): den[r,h] = sum_k exp(leaky(.) - m[r,h]) + 1e-16, in
//                       CSR (= original edge) order, separately rounded
// Both write row_stats[r, h, 0|1] (the layout mp_gat_aggregate_f32 leaves).
__device__ __forceinline__ float gat_leaky(float a, float slope) { return a > 0.f ? a : __fmul_rn(a, slope); }

template <int VEC>
struct GatMaxRed {
  static constexpr bool kW = false;
  static constexpr bool kEid = false;
  static constexpr bool kGat = false;
  static constexpr bool kHW = false;
  static constexpr bool kGatB = false;
  static constexpr bool kStat = false;
  struct Part {
    float v[VEC];
  };
  float acc[VEC];
  float ad[VEC];
  float slope = 0.f;
  int h = 0;  // slab_ref: no softmax-stat slab

  __device__ GatMaxRed() {}
  __device__ GatMaxRed(const AggArgs& p, int, bool) : slope(p.slope) {}

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool, int f, bool act) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      acc[k] = -INFINITY;
      ad[k] = (act && f + k < p.F) ? p.a_dst[row * p.H + f + k] : 0.f;
    }
  }
  __device__ __forceinline__ void consume(const Frag<VEC>& v, float, int, float) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = fmaxf(acc[k], gat_leaky(__fadd_rn(v.v[k], ad[k]), slope));
  }
  __device__ __forceinline__ void save(PRef r, bool) const {
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
    store_frag<VEC>(r.v, o);
  }
  static __device__ __forceinline__ Part load(PRef r) {
    Frag<VEC> o = load_frag<VEC>(r.v);
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = o.v[k];
    return q;
  }
  __device__ __forceinline__ void set(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = q.v[k];
  }
  __device__ __forceinline__ void merge(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = fmaxf(acc[k], q.v[k]);
  }
  __device__ __forceinline__ Part part() const {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = acc[k];
    return q;
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t, int f, bool act, bool with_bias = true) {
    if (!act) return;
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      if (f + k < p.F) p.row_stats[(row * p.H + f + k) * 2] = acc[k];
  }
};

template <int VEC>
struct GatDenRed : GatMaxRed<VEC> {
  using Base = GatMaxRed<VEC>;
  using typename Base::Part;
  using Base::acc;
  using Base::ad;
  using Base::slope;
  float m[VEC];

  __device__ GatDenRed() {}
  __device__ GatDenRed(const AggArgs& p, int f, bool act) : Base(p, f, act) {}

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool, int f, bool act) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const bool ok = act && f + k < p.F;
      acc[k] = 0.f;
      ad[k] = ok ? p.a_dst[row * p.H + f + k] : 0.f;
      m[k] = ok ? p.row_stats[(row * p.H + f + k) * 2] : 0.f;
    }
  }
  __device__ __forceinline__ void consume(const Frag<VEC>& v, float, int, float) {
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      acc[k] = __fadd_rn(acc[k], expf(__fsub_rn(gat_leaky(__fadd_rn(v.v[k], ad[k]), slope), m[k])));
  }
  __device__ __forceinline__ void merge(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __fadd_rn(acc[k], q.v[k]);
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t, int f, bool act, bool with_bias = true) {
    if (!act) return;
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      if (f + k < p.F) p.row_stats[(row * p.H + f + k) * 2 + 1] = __fadd_rn(acc[k], 1e-16f);
  }
};

// Per-head weighted sum (GAT backward: d out / d x_j = alpha[e,h]): the weight
// of slot k for this lane's head h = f / C is w[k*H + h].
template <int VEC>
struct HeadSumRed : SumRed<VEC, true, false> {
  static constexpr bool kW = false;
  static constexpr bool kHW = true;
  int h;
  __device__ HeadSumRed(const AggArgs& p, int f, bool act) : SumRed<VEC, true, false>(p, f, act),
                                                              h(act ? f / p.C : 0) {}
};

// GATConv backward in one pass over the TRANSPOSED CSR (row j = source node,
// slots = its out-edges j->i in original edge order).  Per slot the gathered
// row is g_i = d out_i, and with alpha_ij rebuilt from the forward's row
// statistics (m_i, 1/(s_i + 1e-16)):
//   d xw_j    += alpha_ij g_i                               (message part)
//   dalpha_ij  = <g_i, xw_j>_h                              (the row's own xw)
//   de_ij      = alpha_ij (dalpha_ij - rs_i) leaky'(score)  (softmax + leaky_relu backward)
//   d a_src_j += de_ij,  and at the row end d xw_j += d a_src_j (x) att_src.
// rs_i = <g_i, agg_i>_h replaces the per-edge sum_j alpha_ij dalpha_ij, so no
// [E, H*C] product is ever formed.  The destination's (a_dst, m, 1/den, rs)
// come packed in one float4 per (node, head): one 16-byte gather per slot.
// A head spans HL = C/VEC lanes (power of two); its dot product is reduced
// with DPP adds inside the head group.  Gradients are checked to a
// tolerance, so this pass uses FMA and the hardware exp.
template <int VEC, bool DR = false>
struct GatBwdRed {
  static constexpr bool kDrop = DR;
  static constexpr bool kW = false;
  static constexpr bool kEid = true;
  static constexpr bool kGat = false;
  static constexpr bool kHW = false;
  static constexpr bool kGatB = true;
  static constexpr bool kStat = true;
  struct Part {
    float v[VEC];
    float d;
  };
  float acc[VEC];
  float y[VEC];
  float dacc, as;
  float gd = 0.f;  // d a_dst of the row (ga_dst_in)
  int h, hl;
  bool leader;

  __device__ GatBwdRed(const AggArgs& p, int f, bool act)
      : h(act ? f / p.C : 0), hl(p.C / VEC), leader(act && ((f / VEC) & (p.C / VEC - 1)) == 0) {}

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool, int f, bool act) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    dacc = 0.f;
    Frag<VEC> o = load_frag<VEC>(p.y + row * p.ldy + (act ? f : 0));
#pragma unroll
    for (int k = 0; k < VEC; ++k) y[k] = act ? o.v[k] : 0.f;
    as = p.a_src[row * p.H + h];
    row_terms(p, row);
  }
  // the row's node-wise terms needed at finish (the fix-up, which finishes a
  // split row without a begin, calls this itself)
  __device__ __forceinline__ void row_terms(const AggArgs& p, int64_t row) {
    if (p.ga_dst_in) gd = p.ga_dst_in[row * p.H + h];
  }
  // head-group dot product <v, y> (all lanes of the head get the sum)
  __device__ __forceinline__ float dot(const Frag<VEC>& v) const {
    float t = v.v[0] * y[0];
#pragma unroll
    for (int k = 1; k < VEC; ++k) t = __builtin_fmaf(v.v[k], y[k], t);
    return group_sum(t, hl);
  }
  // DR: the message used alpha * keep / (1 - p), so d xw_j takes that weight and
  // d alpha = keep / (1 - p) <g_i, xw_j>
  __device__ __forceinline__ void consume_gatb(const AggArgs& p, const Frag<VEC>& v, float dal, f32x4 q,
                                               int64_t slot, [[maybe_unused]] uint32_t dbits = 0) {
    const float sc = as + q.x;
    const float lk = sc > 0.f ? 1.f : p.slope;
    const float alpha = __expf(sc * lk - q.y) * q.z;
    float aw = alpha;
    if constexpr (DR) {
      const float dsc = drop_factor(p, dbits, h);
      aw = alpha * dsc;
      dal = dal * dsc;
    }
    // a one-hot softmax row (1/den == 1 and this edge's alpha == 1: a single edge, or the others
    // below 2^-24 of it) has d score = alpha (d alpha - rs) = 0 up to those others' weight; the
    // reference's autograd cancels the identical value there, rs = <g_i, agg_i> would leave the
    // rounding of two different evaluations -- so the term is 0, as the reference's
    const float de = (q.z == 1.f && alpha == 1.f) ? 0.f : alpha * (dal - q.w) * lk;
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __builtin_fmaf(aw, v.v[k], acc[k]);
    dacc += de;
    if (leader && p.de) p.de[slot * p.H + h] = de;  // no de: the training forward made d a_dst node-wise
  }
  __device__ __forceinline__ void consume(const Frag<VEC>&, float, int, float) {}
  __device__ __forceinline__ void save(PRef r, bool stat_writer) const {
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
    store_frag<VEC>(r.v, o);
    if (stat_writer) r.st[0] = dacc;
  }
  static __device__ __forceinline__ Part load(PRef r) {
    Frag<VEC> o = load_frag<VEC>(r.v);
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = o.v[k];
    q.d = r.st[0];
    return q;
  }
  __device__ __forceinline__ void set(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = q.v[k];
    dacc = q.d;
  }
  __device__ __forceinline__ void merge(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] += q.v[k];
    dacc += q.d;
  }
  __device__ __forceinline__ Part part() const {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) q.v[k] = acc[k];
    q.d = dacc;
    return q;
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t, int f, bool act, bool with_bias = true) {
    if (!act) return;
    const float* at = p.att + (int64_t)h * 2 * p.C + p.C + (f % p.C);
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = __builtin_fmaf(dacc, at[k], acc[k]);
    if (p.ga_dst_in) {  // the x_i use of xw in the score: + d a_dst (x) att_dst
      const float* ad = p.att + (int64_t)h * 2 * p.C + (f % p.C);
#pragma unroll
      for (int k = 0; k < VEC; ++k) o.v[k] = __builtin_fmaf(gd, ad[k], o.v[k]);
    }
    store_out<VEC>(p.out + row * p.ldo + f, o);
    if (leader) p.ga[row * p.H + h] = dacc;
  }
};

// GATConv backward for heads of any width (C % 4 == 0; a head may span several
// feature tiles, so no per-slot dot product is possible): over the TRANSPOSED
// CSR (row j = source), with alpha_ij rebuilt from the destination's pack
// (a_dst, m, 1/den, rs) and the row's own a_src[j,h], lk = leaky'(score):
//   acc_j  += alpha d g_i              (message part of d xw_j; d = dropout factor)
//   acc2_j += lk alpha d g_i
//   sc_j   += lk alpha rs_i            (per head)
// The per-edge d score never forms: d a_src_j = sum_i lk alpha (d <g_i, xw_j> - rs_i)
// = <acc2_j, xw_j>_h - sc_j, a node-wise dot product taken after this pass
// (mp_gat_backward_epilogue_wide_f32).  Rows write acc to out, acc2 to out2 and
// sc to ga; every lane of a head holds the same sc.  Elementwise per slot:
// FMA and the hardware exp (gradients are tolerance-checked).
template <int VEC, bool DR = false>
struct GatBwdWideRed {
  static constexpr bool kDrop = DR;
  static constexpr bool kW = false;
  static constexpr bool kEid = DR;  // the dropout key: each edge's dst-CSR slot
  static constexpr bool kGat = false;
  static constexpr bool kHW = false;
  static constexpr bool kGatB = false;
  static constexpr bool kStat = true;
  struct Part {
    float v[VEC];
    float v2[VEC];
    float s;
  };
  float acc[VEC], acc2[VEC];
  float sc, as;
  int h;

  __device__ GatBwdWideRed(const AggArgs& p, int f, bool act) : h(act ? f / p.C : 0) {}

  __device__ __forceinline__ void begin(const AggArgs& p, int64_t row, bool, int, bool) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = acc2[k] = 0.f;
    sc = 0.f;
    as = p.a_src[row * p.H + h];
  }
  __device__ __forceinline__ void consume_gatw(const AggArgs& p, const Frag<VEC>& v, f32x4 q,
                                               [[maybe_unused]] uint32_t dbits) {
    const float score = as + q.x;
    const float lk = score > 0.f ? 1.f : p.slope;
    const float alpha = __expf(score * lk - q.y) * q.z;
    // one-hot softmax row (see GatBwdRed::consume_gatb): its d score is 0, so the edge adds
    // nothing to d a_src's two node-wise sums (acc2, sc)
    const bool one_hot = q.z == 1.f && alpha == 1.f;
    sc = one_hot ? sc : __builtin_fmaf(lk * alpha, q.w, sc);
    float aw = alpha;
    if constexpr (DR) aw = alpha * drop_factor(p, dbits, h);
    const float law = one_hot ? 0.f : lk * aw;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      acc[k] = __builtin_fmaf(aw, v.v[k], acc[k]);
      acc2[k] = __builtin_fmaf(law, v.v[k], acc2[k]);
    }
  }
  __device__ __forceinline__ void consume(const Frag<VEC>&, float, int, float) {}
  __device__ __forceinline__ void save(PRef r, bool stat_writer) const {
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
    store_frag<VEC>(r.v, o);
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc2[k];
    store_frag<VEC>(r.v2, o);
    if (stat_writer) r.st[0] = sc;
  }
  static __device__ __forceinline__ Part load(PRef r) {
    Frag<VEC> o = load_frag<VEC>(r.v);
    Frag<VEC> o2 = load_frag<VEC>(r.v2);
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      q.v[k] = o.v[k];
      q.v2[k] = o2.v[k];
    }
    q.s = r.st[0];
    return q;
  }
  __device__ __forceinline__ void set(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      acc[k] = q.v[k];
      acc2[k] = q.v2[k];
    }
    sc = q.s;
  }
  __device__ __forceinline__ void merge(const Part& q) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      acc[k] += q.v[k];
      acc2[k] += q.v2[k];
    }
    sc += q.s;
  }
  __device__ __forceinline__ Part part() const {
    Part q;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      q.v[k] = acc[k];
      q.v2[k] = acc2[k];
    }
    q.s = sc;
    return q;
  }
  __device__ __forceinline__ void finish(const AggArgs& p, int64_t row, int64_t, int f, bool act, bool with_bias = true) {
    if (!act) return;
    Frag<VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
    store_out<VEC>(p.out + row * p.ldo + f, o);
#pragma unroll
    for (int k = 0; k < VEC; ++k) o.v[k] = acc2[k];
    store_out<VEC>(p.out2 + row * (int64_t)p.F + f, o);
    if (f % p.C == 0) p.ga[row * p.H + h] = sc;
  }
};

// this lane's share of slab slot s (2*task + kind)
template <class Red>
__device__ __forceinline__ PRef slab_ref(const AggArgs& p, int64_t s, int f, const Red& red) {
  PRef r;
  r.v = p.slab_v + s * p.slab_ld + f;
  r.a = p.slab_a ? p.slab_a + s * p.slab_ld + f : nullptr;
  r.st = p.slab_s ? p.slab_s + (s * p.H + red.h) * 2 : nullptr;
  r.v2 = p.slab_v2 ? p.slab_v2 + s * p.slab_ld + f : nullptr;
  r.s2 = p.slab_s2 ? p.slab_s2 + s * p.H + red.h : nullptr;
  return r;
}

// ---------------------------------------------------------------------------
// Lane groups.  A wave runs G = 64/L independent merge-path tasks, one per
// group of L lanes (L = 64: one task per wave, every per-task value is
// wave-uniform and lives in SGPRs).  A group covers L*VEC features of a row;
// gridDim.y walks the feature tiles, which the dispatcher runs roughly one
// after another, so the gathered working set of a pass is L*VEC*4 bytes per
// row -- narrow tiles keep more hub rows resident in L2.
// ---------------------------------------------------------------------------
template <int L>
struct Grp {
  static constexpr int G = 64 / L;
  static __device__ __forceinline__ int bc(int v, int idx) {
    if constexpr (L == 64) return readlane(v, idx);
    else return __shfl(v, idx, L);
  }
  static __device__ __forceinline__ float bc(float v, int idx) {
    if constexpr (L == 64) return readlane(v, idx);
    else return __shfl(v, idx, L);
  }
  static __device__ __forceinline__ int un(int v) {
    if constexpr (L == 64) return uni(v);
    else return v;
  }
};

// ---------------------------------------------------------------------------
// Per-group slot window: col / weight / eid of L consecutive CSR slots held one
// per lane, the next L prefetched.  DR: the lane's slot's dropout keep bits,
// computed when its window becomes current (key: the eid channel when EID --
// the transposed backward's dst slot -- else the slot itself).
// ---------------------------------------------------------------------------
template <bool W, bool EID, int L, bool GW = false, bool DR = false>
struct SlotWin {
  int64_t base, limit;
  int col, col_n, eid, eid_n;
  int did = 0, did_n = 0;  // DR with drop_ids: the dropout key of each slot of the window
  float w, w_n;
  uint32_t dr = 0;
  // GAT (GW, 64-lane tasks, H a power of two <= 8): a_src rows of the current
  // window staged in the wave's LDS (one load per lane per window instead of
  // one gather per slot); the column window runs two windows ahead so the
  // next window's a_src loads are issued a window before they are needed.
  int col_nn;
  float asn[8];
  float* lds;
  bool gw;

  __device__ __forceinline__ void fetch(const AggArgs& p, int64_t b, int gl, int& c, float& wt, int& e) {
    int64_t k = b + gl;
    bool ok = k < limit;
    c = ok ? (p.col ? ld_stream(p.col + k) : (int)k) : 0;  // col == nullptr: identity (rows in slot order)
    if (W) wt = ok ? ld_stream(p.w + k) : 0.f;
    if (EID) e = ok ? ld_stream(p.eid + k) : 0;
  }
  // the dropout keys of a window's slots (drop_ids; loaded a window ahead, with its columns)
  __device__ __forceinline__ void fetch_did(const AggArgs& p, int64_t b, int gl, int& d) {
    if constexpr (DR) {
      const int64_t k = b + gl;
      d = (p.drop_ids && k < limit) ? ld_stream(p.drop_ids + k) : 0;
    }
  }
  __device__ __forceinline__ int64_t drop_key(const AggArgs& p, int gl) const {
    return p.drop_ids ? (int64_t)did : (EID ? (int64_t)eid : base + gl);
  }
  __device__ __forceinline__ void load_as(const AggArgs& p, int c) {
    const float* r = p.a_src + (int64_t)c * p.H;
    if (p.H == 8) {
      f32x4 a = *reinterpret_cast<const f32x4*>(r);
      f32x4 b = *reinterpret_cast<const f32x4*>(r + 4);
      asn[0] = a.x; asn[1] = a.y; asn[2] = a.z; asn[3] = a.w;
      asn[4] = b.x; asn[5] = b.y; asn[6] = b.z; asn[7] = b.w;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) asn[k] = k < p.H ? r[k] : 0.f;
    }
  }
  __device__ __forceinline__ void store_as(const AggArgs& p, int gl) {
    __builtin_amdgcn_wave_barrier();  // earlier reads of the previous window come first
    if (p.H == 8) {
      f32x4 a = {asn[0], asn[1], asn[2], asn[3]};
      f32x4 b = {asn[4], asn[5], asn[6], asn[7]};
      *reinterpret_cast<f32x4*>(lds + gl * 8) = a;
      *reinterpret_cast<f32x4*>(lds + gl * 8 + 4) = b;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < p.H) lds[gl * p.H + k] = asn[k];
    }
    __builtin_amdgcn_wave_barrier();  // LDS ops of one wave run in order: later reads see the stores
  }
  __device__ __forceinline__ void init(const AggArgs& p, int64_t b, int64_t lim, int gl, float* wave_lds = nullptr) {
    base = b;
    limit = lim;
    fetch(p, base, gl, col, w, eid);
    fetch(p, base + L, gl, col_n, w_n, eid_n);
    fetch_did(p, base, gl, did);
    fetch_did(p, base + L, gl, did_n);
    if constexpr (DR) dr = drop_bits(p, drop_key(p, gl));
    if constexpr (GW) {
      lds = wave_lds;
      gw = p.H <= 8 && (p.H & (p.H - 1)) == 0;
      if (gw) {
        float dw;
        int de;
        fetch(p, base + 2 * L, gl, col_nn, dw, de);
        load_as(p, col);
        store_as(p, gl);
        load_as(p, col_n);
      }
    }
  }
  __device__ __forceinline__ void ensure(const AggArgs& p, int64_t e, int gl) {
    if (e >= base + L) {  // slots are consumed in order, never skipping a window
      base += L;
      col = col_n;
      w = w_n;
      eid = eid_n;
      did = did_n;
      if constexpr (DR) dr = drop_bits(p, drop_key(p, gl));  // eid_n / did_n were loaded a window ago
      fetch_did(p, base + L, gl, did_n);
      if constexpr (GW) {
        if (gw) {
          col_n = col_nn;
          float dw;
          int de;
          fetch(p, base + 2 * L, gl, col_nn, dw, de);
          store_as(p, gl);      // asn holds the a_src rows of the new current window
          load_as(p, col_n);
          return;
        }
      }
      fetch(p, base + L, gl, col_n, w_n, eid_n);
    }
  }
  __device__ __forceinline__ float a_src_of(const AggArgs& p, int slot_in_win, int c, int h) const {
    if constexpr (GW) {
      if (gw) return lds[slot_in_win * p.H + h];
    }
    return p.a_src[(int64_t)c * p.H + h];
  }
};

// Two-pass GAT aggregation window (k_agg_flat, 64-lane tasks, 64-feature
// tiles): lane k computes the reference's alpha for slot base+k and each of the
// hpt heads of this tile once per window,
//   alpha = exp(leaky(a_src[col,h] + a_dst[r,h]) - m[r,h]) / den[r,h],  r = slot_row,
// into the wave's LDS; a slot then costs one LDS read per lane (lane's head =
// its feature / C).  Columns and slot rows run two windows ahead and the
// per-slot gathers (a_src, a_dst, row stats) one window ahead.
struct GatAlphaWin {
  int64_t base, limit;
  int col, col_n, col_nn, row_n, row_nn;
  float g_as[4], g_ad[4], g_m[4], g_d[4];
  float* lds;
  int h0, hpt, j;

  __device__ __forceinline__ void fetch(const AggArgs& p, int64_t b, int lane, int& c, int& r) {
    const int64_t k = b + lane;
    const bool ok = k < limit;
    c = ok ? ld_stream(p.col + k) : 0;
    r = ok ? ld_stream(p.slot_row + k) : 0;
  }
  __device__ __forceinline__ void gather(const AggArgs& p, int c, int r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < hpt) {
        const int64_t hr = (int64_t)r * p.H + h0 + q;
        g_as[q] = p.a_src[(int64_t)c * p.H + h0 + q];
        g_ad[q] = p.a_dst[hr];
        const f32x2 st = *reinterpret_cast<const f32x2*>(p.row_stats + hr * 2);
        g_m[q] = st.x;
        g_d[q] = st.y;
      }
    }
  }
  __device__ __forceinline__ void publish(const AggArgs& p, int lane) {
    float al[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      al[q] = q < hpt ? __fdiv_rn(expf(__fsub_rn(gat_leaky(__fadd_rn(g_as[q], g_ad[q]), p.slope), g_m[q])), g_d[q])
                      : 0.f;
    __builtin_amdgcn_wave_barrier();  // earlier reads of the previous window come first
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < hpt) lds[lane * hpt + q] = al[q];
    __builtin_amdgcn_wave_barrier();  // LDS ops of one wave run in order: later reads see the stores
  }
  __device__ __forceinline__ void init(const AggArgs& p, int64_t b, int64_t lim, int lane, float* wave_lds,
                                       int tile) {
    base = b;
    limit = lim;
    lds = wave_lds;
    // tile t holds features [64t, 64t+64): heads h0 .. h0+hpt-1, lane's head h0 + lane/C
    h0 = tile * 64 / p.C;
    hpt = p.C >= 64 ? 1 : min(64 / p.C, p.H - h0);  // a last partial tile holds fewer heads
    j = p.C >= 64 ? 0 : lane / p.C;                  // lanes past F read some slot's alpha, unused
    int r;
    fetch(p, base, lane, col, r);
    fetch(p, base + 64, lane, col_n, row_n);
    fetch(p, base + 128, lane, col_nn, row_nn);
    gather(p, col, r);
    publish(p, lane);
    gather(p, col_n, row_n);
  }
  __device__ __forceinline__ void ensure(const AggArgs& p, int64_t e, int lane) {
    if (e >= base + 64) {  // slots are consumed in order, never skipping a window
      base += 64;
      col = col_n;
      publish(p, lane);  // the gathers issued a window ago
      col_n = col_nn;
      row_n = row_nn;
      fetch(p, base + 128, lane, col_nn, row_nn);
      gather(p, col_n, row_n);
    }
  }
  __device__ __forceinline__ float alpha(int slot_in_win) const { return lds[slot_in_win * hpt + j]; }
};

// Process CSR slots [s, t) of the current (partial) row.
// All U row loads are issued unconditionally (indices past the segment are
// clamped to its last slot, inactive lanes read feature 0) so no load sits
// under an exec mask; only the group-uniform consume loop is bounded by n.
// For L = 64 the row address is a uniform base (SGPR pair) + one shared
// 32-bit lane offset, so U rows cost U*VEC data VGPRs only.
// GAT forward: a_src of each 64-slot window staged in LDS (see SlotWin; 8.85 -> 8.66 ms, bitwise the same)
template <class Red>
constexpr bool own_as_v = false;
template <int VEC, bool TR, bool ND, bool DR>
constexpr bool own_as_v<GatRed<VEC, true, TR, ND, DR>> = true;
template <class Red, int L>
constexpr bool kGatWin = Red::kGat && !own_as_v<Red> && L == 64;
template <class Red>
constexpr bool kGatTrain = false;
template <int VEC, bool OWN, bool ND, bool DR>
constexpr bool kGatTrain<GatRed<VEC, OWN, true, ND, DR>> = true;
template <class Red>
constexpr bool kNodeScoresV = false;
template <int VEC, bool OWN, bool TR, bool ND, bool DR>
constexpr bool kNodeScoresV<GatRed<VEC, OWN, TR, ND, DR>> = ND;
template <class Red>
constexpr bool kDropV = false;
template <int VEC, bool OWN, bool TR, bool ND, bool DR>
constexpr bool kDropV<GatRed<VEC, OWN, TR, ND, DR>> = DR;
template <int VEC, bool DR>
constexpr bool kDropV<GatBwdRed<VEC, DR>> = DR;
template <int VEC, bool DR>
constexpr bool kDropV<GatBwdWideRed<VEC, DR>> = DR;
template <class Red>
constexpr bool kGatWideV = false;
template <int VEC, bool DR>
constexpr bool kGatWideV<GatBwdWideRed<VEC, DR>> = true;

template <class Red, int VEC, int U, int L>
__device__ __forceinline__ void run_slots(Red& red, const AggArgs& p,
                                          SlotWin<Red::kW, Red::kEid, L, kGatWin<Red, L>, kDropV<Red>>& win,
                                          int64_t s, int64_t t, uint32_t foff, int gl) {
  using GR = Grp<L>;
  const char* xb = reinterpret_cast<const char*>(p.x);
  const int64_t ldxb = p.ldx * 4;
  int64_t e = s;
  while (e < t) {
    win.ensure(p, e, gl);
    const int off = (int)(e - win.base);
    int64_t rem = t - e;
    int n = L - off;
    if (rem < n) n = (int)rem;
    if (n > U) n = U;
    n = GR::un(n);
    Frag<VEC> v[U];
    float as[U];
    [[maybe_unused]] float hw[U];
    [[maybe_unused]] f32x4 pk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int uu = u < n ? u : n - 1;
      if constexpr (Red::kHW) hw[u] = p.w[(e + uu) * p.H + red.h];
      const int c = GR::bc(win.col, off + uu);
      v[u] = load_frag<VEC>(reinterpret_cast<const float*>(xb + (int64_t)c * ldxb + foff));
      if constexpr (Red::kGat && !own_as_v<Red>) as[u] = win.a_src_of(p, off + uu, c, red.h);
      if constexpr (Red::kGatB || kGatWideV<Red>) pk[u] = p.pack[(int64_t)c * p.H + red.h];
    }
    if constexpr (Red::kGatB) {
#pragma unroll
      for (int u = 0; u < U; ++u) as[u] = red.dot(v[u]);
    }
    if constexpr (kNodeScoresV<Red>) {
      // the row's own scores, once, after this batch's loads are in flight
      if (red.need_ad) red.node_scores(p);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < n) {
        [[maybe_unused]] uint32_t db = 0;
        if constexpr (kDropV<Red>) db = (uint32_t)GR::bc((int)win.dr, off + u);
        if constexpr (Red::kGat) {
          // own_as next to its consume: slot u waits only for its own row
          if constexpr (own_as_v<Red>) red.consume_gat(p, v[u], red.own_as(v[u]), db);
          else red.consume_gat(p, v[u], as[u], db);
        } else if constexpr (kGatWideV<Red>) {
          red.consume_gatw(p, v[u], pk[u], db);
        } else if constexpr (Red::kGatB) {
          red.consume_gatb(p, v[u], as[u], pk[u], GR::bc(win.eid, off + u), db);
        } else {
          const float wt = Red::kHW ? hw[u] : (Red::kW ? GR::bc(win.w, off + u) : 1.f);
          const int ei = Red::kEid ? GR::bc(win.eid, off + u) : 0;
          red.consume(v[u], wt, ei, 0.f);
        }
      }
    }
    e += n;
  }
}

template <class Red, int VEC, int U, int L>
__global__ __launch_bounds__(kBlock) void k_agg_main(AggArgs p) {
  using GR = Grp<L>;
  const int lane = lane_id();
  const int gl = lane & (L - 1);
  int bx = (int)blockIdx.x, tile = (int)blockIdx.y;
  if constexpr (kXcdTiles) {
    // blocks b and b+8 share an XCD (dispatch is round-robin over the 8 XCDs;
    // speed only): give every XCD one feature tile so its L2 holds only that
    // tile of the hot rows.  tiles = gridDim.y divides 8 (checked on the host).
    const int T = (int)gridDim.y;
    if (8 % T == 0) {  // the host pads the grid to a multiple of 8/T blocks per tile
      const int b = (int)(blockIdx.y * gridDim.x + blockIdx.x);
      const int xcd = b & 7;
      tile = xcd % T;
      bx = (b >> 3) * (8 / T) + xcd / T;
    }
  }
  const int wave = bx * kWavesPerBlock + (int)(threadIdx.x >> 6);
  const int w = GR::un(wave * GR::G + lane / L);  // this group's task
  if (w >= p.n_waves) return;
  const int f = tile * L * VEC + gl * VEC;
  const bool act = f < p.F;
  const uint32_t foff = (uint32_t)(act ? f : 0) * 4u;

  const int r_first = GR::un(p.wave_row[w]);
  const int r_last = GR::un(p.wave_row[w + 1]);
  const int64_t e_begin = GR::un(p.wave_slot[w]);
  const int64_t e_end = GR::un(p.wave_slot[w + 1]);

  Red red(p, f, act);
  SlotWin<Red::kW, Red::kEid, L, kGatWin<Red, L>, kDropV<Red>> win;
  [[maybe_unused]] float* wave_lds = nullptr;
  if constexpr (kGatWin<Red, L>) {
    __shared__ float gat_as[kWavesPerBlock][64 * 8];
    wave_lds = gat_as[threadIdx.x >> 6];
  }
  win.init(p, e_begin, e_end, gl, wave_lds);

  // rowptr window: rp = rowptr[rbase + gl]
  int rbase = r_first;
  int rp = (rbase + gl <= p.n_rows) ? p.rowptr[rbase + gl] : 0;

  // continuation of the row owned by an earlier task
  {
    const int64_t ce = GR::bc(rp, 0);  // rowptr[r_first] (== n_edges when r_first == n_rows)
    if (e_begin < ce) {
      red.begin(p, r_first - 1, false, f, act);
      run_slots<Red, VEC, U, L>(red, p, win, e_begin, ce < e_end ? ce : e_end, foff, gl);
      if (act) red.save(slab_ref(p, 2 * (int64_t)w, f, red), Red::kStat && (f % p.C == 0));
    }
  }
  // rows owned by this task
  for (int r = r_first; r < r_last; ++r) {
    if (r + 1 - rbase > L - 1) {
      rbase = r;
      rp = (rbase + gl <= p.n_rows) ? p.rowptr[rbase + gl] : 0;
    }
    const int64_t rs = GR::bc(rp, r - rbase);
    const int64_t re = GR::bc(rp, r - rbase + 1);
    red.begin(p, r, true, f, act);
    if (re <= e_end) {
      run_slots<Red, VEC, U, L>(red, p, win, rs, re, foff, gl);
      red.finish(p, r, re - rs, f, act);
    } else {
      run_slots<Red, VEC, U, L>(red, p, win, rs, e_end, foff, gl);
      if constexpr (kNodeScoresV<Red>) red.flush_scores(p);
      if (act) red.save(slab_ref(p, 2 * (int64_t)w + 1, f, red), Red::kStat && (f % p.C == 0));
    }
  }
}

// ---------------------------------------------------------------------------
// Narrow rows (F <= 16): one merge-path task per LANE.  A lane holds the whole
// row (NV fragments of VEC features, one reducer each) and walks its task's
// slots in CSR order with U slots' loads in flight, so a wave keeps 64*U row
// gathers outstanding instead of 64/L*L.  Same schedule, slab layout and
// fix-up as k_agg_main; rows stay sequential, so results are identical.
// ---------------------------------------------------------------------------
template <class Red, int VEC, int NV, int U>
__device__ __forceinline__ void lane_slots(Red (&red)[NV], const AggArgs& p, int64_t s, int64_t t) {
  for (int64_t e = s; e < t; e += U) {
    const int64_t n = t - e < U ? t - e : U;
    int c[U];
    [[maybe_unused]] float wt[U];
    [[maybe_unused]] int ei[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = e + (u < n ? u : n - 1);
      c[u] = p.col ? p.col[k] : (int)k;
      if constexpr (Red::kW) wt[u] = p.w[k];
      if constexpr (Red::kEid) ei[u] = p.eid[k];
    }
    Frag<VEC> v[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* row = p.x + (int64_t)c[u] * p.ldx;
#pragma unroll
      for (int q = 0; q < NV; ++q) v[u][q] = load_frag<VEC>(row + (q * VEC < p.F ? q * VEC : 0));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < n) {
#pragma unroll
        for (int q = 0; q < NV; ++q)
          red[q].consume(v[u][q], Red::kW ? wt[u] : 1.f, Red::kEid ? ei[u] : 0, 0.f);
      }
    }
  }
}

template <class Red, int VEC, int NV, int U>
__global__ __launch_bounds__(kBlock) void k_agg_lane(AggArgs p) {
  const int w = (int)(blockIdx.x * kBlock + threadIdx.x);
  if (w >= p.n_waves) return;
  const int r_first = p.wave_row[w];
  const int r_last = p.wave_row[w + 1];
  const int64_t e_begin = p.wave_slot[w];
  const int64_t e_end = p.wave_slot[w + 1];
  Red red[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) red[q] = Red(p, q * VEC, q * VEC < p.F);
  const int64_t ce = p.rowptr[r_first];
  if (e_begin < ce) {
#pragma unroll
    for (int q = 0; q < NV; ++q) red[q].begin(p, r_first - 1, false, q * VEC, q * VEC < p.F);
    lane_slots<Red, VEC, NV, U>(red, p, e_begin, ce < e_end ? ce : e_end);
#pragma unroll
    for (int q = 0; q < NV; ++q)
      if (q * VEC < p.F) red[q].save(slab_ref(p, 2 * (int64_t)w, q * VEC, red[q]), false);
  }
  int64_t rs = ce;
  for (int r = r_first; r < r_last; ++r) {
    const int64_t re = p.rowptr[r + 1];
#pragma unroll
    for (int q = 0; q < NV; ++q) red[q].begin(p, r, true, q * VEC, q * VEC < p.F);
    if (re <= e_end) {
      lane_slots<Red, VEC, NV, U>(red, p, rs, re);
#pragma unroll
      for (int q = 0; q < NV; ++q) red[q].finish(p, r, re - rs, q * VEC, q * VEC < p.F);
    } else {
      lane_slots<Red, VEC, NV, U>(red, p, rs, e_end);
#pragma unroll
      for (int q = 0; q < NV; ++q)
        if (q * VEC < p.F) red[q].save(slab_ref(p, 2 * (int64_t)w + 1, q * VEC, red[q]), false);
    }
    rs = re;
  }
}

// ---------------------------------------------------------------------------
// Flat variant of k_agg_main (sum/mean/max/min): a task streams its slots in
// fixed batches of U across row boundaries and closes rows as it crosses
// their ends (row ends come from the rowptr window already in registers).
// k_agg_main starts a new batch at every row, so a short row costs a whole
// batch of U (clamped) loads and a trip of loop overhead; here every batch
// but the task's last carries U useful slots, and the next row's loads are
// in flight while the previous row is finished.  Each row's slots are still
// consumed in CSR order by one task: results are identical.
// ---------------------------------------------------------------------------
// GA: two-pass GAT aggregation (Red = SumRed<1, true, false>, L = 64): the slot
// weights are the reference's alpha from GatAlphaWin instead of w.
// SM (L = 64, no edge ids, col != nullptr, x below 4 GiB): the column and
// weight of every slot of a batch come straight into SGPRs through scalar
// loads (s_load_dwordx16 via the scalar cache) -- the next batch's columns
// issued with the current batch, the current batch's weights consumed only
// after its gathers are in flight -- and each gather is a buffer load with the
// row offset in soffset: per slot one SALU multiply and one VMEM instruction,
// no v_readlane from a one-slot-per-lane window.
template <int U, class T>
__device__ __forceinline__ void scalar_batch(const T* a, int64_t n, int64_t e, T (&v)[U]) {
  typedef T tv __attribute__((ext_vector_type(U), aligned(4)));
  typedef __attribute__((address_space(4))) const tv ctv;
  typedef __attribute__((address_space(4))) const T ct;
  // slots [e, e + U); slots past the end of the array are clamped to the last
  // one (never consumed: the caller stops at the task's end)
  if (e + U <= n) {
    const tv t = *(ctv*)(a + e);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = t[u];
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ((ct*)a)[e + u < n ? e + u : n - 1];
  }
}

// MP_FLAG_SKIP_EMPTY (mp_aggregate_tiles_f32 only): an owned row with no slot
// is left untouched -- no load, no store, no bias.  The sharded step's boundary
// pass (INIT_FROM_OUT) skips its rows without boundary edges this way: their
// read-modify-write of out cost the pass as much as its gathers (measured,
// tools/exp_boundary.py), and the interior pass adds their bias instead
// (AggArgs::bias_rows).  (An out prefetch issued with each batch's gathers was
// also measured there: slower, not kept -- DESIGN Appendix A.)
// XM (mp_aggregate_tiles_f32's launches only): 1 = per-row bias flags (the
// sharded interior pass), 2 = MP_FLAG_SKIP_EMPTY (the boundary pass); TM:
// tile-major operands.  Compile-time, one feature per instance, so every other
// launch runs the kernel without their per-block and per-row work (measured:
// both features as run-time branches of one instance cost short-row passes 13 %).
template <class Red, int VEC, int U, int L, bool GA = false, bool SM = false, int XM = 0, bool TM = false>
__global__ __launch_bounds__(kBlock) void k_agg_flat(AggArgs p) {
  static_assert(!Red::kGat && !Red::kGatB && !Red::kHW, "flat loop: sum/mean/max/min reducers");
  static_assert(!GA || (L == 64 && VEC == 1 && Red::kW), "two-pass GAT: 64-lane tasks, 64-feature tiles");
  static_assert(!SM || (L == 64 && !GA && !Red::kEid), "scalar batches: 64-lane sum/mean tasks");
  static_assert(!(XM || TM) || (SM && VEC == 1), "tile-major / skipped rows: the scalar-batch kernel, 64-feature tiles");
  constexpr bool kSkip = XM == 2, kFlags = XM == 1;
  using GR = Grp<L>;
  const int lane = lane_id();
  const int gl = lane & (L - 1);
  int bx = (int)blockIdx.x, tile = (int)blockIdx.y;
  if constexpr (kXcdTiles) {  // see k_agg_main: one feature tile per XCD
    const int T = (int)gridDim.y;
    if (8 % T == 0 && !p.seq_tiles) {  // the host pads the grid to a multiple of 8/T blocks per tile
      const int b = (int)(blockIdx.y * gridDim.x + blockIdx.x);
      const int xcd = b & 7;
      tile = xcd % T;
      bx = (b >> 3) * (8 / T) + xcd / T;
    }
  }
  const int wave = bx * kWavesPerBlock + (int)(threadIdx.x >> 6);
  const int w = GR::un(wave * GR::G + lane / L);
  if (w >= p.n_waves) return;
  const int f = tile * L * VEC + gl * VEC;
  const bool act = f < p.F;
  const float* x_tile = p.x;
  int64_t ldx_tile = p.ldx;
  int fx0 = 0;
  if constexpr (TM) tile_view(p, tile * L * VEC, x_tile, ldx_tile, fx0);
  const uint32_t foff = (uint32_t)(act ? f - fx0 : 0) * 4u;
  const char* xb = reinterpret_cast<const char*>(x_tile);
  const int64_t ldxb = ldx_tile * 4;
  [[maybe_unused]] __amdgpu_buffer_rsrc_t xr;


  const int r_first = GR::un(p.wave_row[w]);
  const int r_last = GR::un(p.wave_row[w + 1]);
  const int64_t e_begin = GR::un(p.wave_slot[w]);
  const int64_t e_end = GR::un(p.wave_slot[w + 1]);

  Red red(p, f, act);
  if constexpr (XM != 0) red.preload_bias(p, f, act);  // the tile launches: sum / mean only
  // an owned row opens (rs_ / re_: its slot range); an empty one is skipped
  // (no load of out) under MP_FLAG_SKIP_EMPTY
  auto open_row = [&](int rr, int64_t rs_, int64_t re_) {
    red.begin(p, rr, !(kSkip && re_ == rs_), f, act);
  };

  std::conditional_t<GA, GatAlphaWin, SlotWin<Red::kW, Red::kEid, L>> win;
  if constexpr (GA) {
    __shared__ float ga_lds[kWavesPerBlock][64 * 4];
    win.init(p, e_begin, e_end, gl, ga_lds[threadIdx.x >> 6], tile);
  } else if constexpr (!SM) {
    win.init(p, e_begin, e_end, gl);
  }
  [[maybe_unused]] int c_nxt[U];
  if constexpr (SM) {
    xr = __builtin_amdgcn_make_buffer_rsrc((void*)x_tile, (short)0, (int)p.x_bytes, 0x00020000);
    if (e_begin < e_end) scalar_batch<U>(p.col, p.n_edges, e_begin, c_nxt);
  }
  // row window: rowptr (and, kFlags, the per-row bias flags) of rows [rbase,
  // rbase + L) across the lanes.  A kFlags refill for row pointer r starts at
  // r - 1, so the row that r closes -- the one open -- stays in the window
  // until it finishes (its bias flag is read then).
  int rbase = r_first;
  int rp = (rbase + gl <= p.n_rows) ? p.rowptr[rbase + gl] : 0;
  [[maybe_unused]] int bw = 1;
  if constexpr (kFlags) bw = (rbase + gl < p.n_rows) ? p.bias_rows[rbase + gl] : 1;
  auto row_ptr = [&](int r) -> int64_t {
    if (r - rbase > L - 1) {
      rbase = kFlags ? r - 1 : r;
      rp = (rbase + gl <= p.n_rows) ? p.rowptr[rbase + gl] : 0;
      if constexpr (kFlags) bw = (rbase + gl < p.n_rows) ? p.bias_rows[rbase + gl] : 1;
    }
    return GR::bc(rp, r - rbase);
  };
  auto finish_row = [&](int rr, int64_t cnt) {
    if constexpr (kSkip) {
      if (cnt == 0) return;
    }
    if constexpr (kFlags) {
      red.finish_scaled_bias(p, rr, cnt, f, act, GR::bc(bw, rr - rbase) != 0 ? 1.f : 0.f);
    } else {
      red.finish(p, rr, cnt, f, act);
    }
  };

  // current row: the continuation of an earlier task's row, or an owned row
  const int64_t ce = GR::bc(rp, 0);  // rowptr[r_first]
  bool cont = e_begin < ce;
  int r = r_first;
  int64_t rs = ce, re = ce;
  if (cont) {
    red.begin(p, r_first - 1, false, f, act);
  } else if (r < r_last) {
    re = row_ptr(r + 1);
    open_row(r, rs, re);
  }
  // close the current row at slot k (k >= its end) and open the next one(s)
  auto advance = [&](int64_t k) {
    while (k >= re) {
      if (cont) {
        if (act) red.save(slab_ref(p, 2 * (int64_t)w, f, red), false);
        cont = false;
      } else {
        finish_row(r, re - rs);
        ++r;
      }
      if (r >= r_last) {  // cannot happen for a valid schedule: never open a row past the task
        re = INT64_MAX;
        break;
      }
      rs = re;
      re = row_ptr(r + 1);
      open_row(r, rs, re);
    }
  };

  for (int64_t e = e_begin; e < e_end;) {
    if constexpr (SM) {
      // batches start at e_begin + k*U: every batch but the task's last is full
      const int64_t rem = e_end - e;
      const int n = rem < U ? (int)rem : U;
      [[maybe_unused]] float wb[U];
      if constexpr (Red::kW) scalar_batch<U>(p.w, p.n_edges, e, wb);
      Frag<VEC> v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = load_frag_buf<VEC>(xr, foff, (uint32_t)c_nxt[u] * (uint32_t)ldxb);
      // the columns are dead once the gathers are issued: the next batch's
      // land in the same SGPRs while this batch's rows are in flight
      if (e + U < e_end) scalar_batch<U>(p.col, p.n_edges, e + U, c_nxt);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < n) {
          advance(e + u);
          float wt = 1.f;
          if constexpr (Red::kW) wt = wb[u];
          red.consume(v[u], wt, 0, 0.f);
        }
      }
      e += n;
      continue;
    }
    win.ensure(p, e, gl);
    const int off = (int)(e - win.base);
    int64_t rem = e_end - e;
    int n = L - off;
    if (rem < n) n = (int)rem;
    if (n > U) n = U;
    n = GR::un(n);
    Frag<VEC> v[U];
    [[maybe_unused]] float al[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int uu = u < n ? u : n - 1;
      const int c = GR::bc(win.col, off + uu);
      v[u] = load_frag<VEC>(reinterpret_cast<const float*>(xb + (int64_t)c * ldxb + foff));
      if constexpr (GA) al[u] = win.alpha(off + uu);  // LDS reads of the batch issued with its loads
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < n) {
        advance(e + u);
        float wt = 1.f;
        if constexpr (GA) wt = al[u];
        else if constexpr (Red::kW) wt = GR::bc(win.w, off + u);
        int ei = 0;
        if constexpr (!GA && Red::kEid) ei = GR::bc(win.eid, off + u);
        red.consume(v[u], wt, ei, 0.f);
      }
    }
    e += n;
  }
  // tail: the current row, then any rows whose slots all lie in later tasks
  if (cont) {
    if (act) red.save(slab_ref(p, 2 * (int64_t)w, f, red), false);
    cont = false;
    if (r < r_last) {
      rs = ce;
      re = row_ptr(r + 1);
      open_row(r, rs, re);
    }
  }
  while (r < r_last) {
    if (re <= e_end) {
      finish_row(r, re - rs);
    } else {
      if (act) red.save(slab_ref(p, 2 * (int64_t)w + 1, f, red), false);
    }
    ++r;
    if (r < r_last) {
      rs = re;
      re = row_ptr(r + 1);
      open_row(r, rs, re);
    }
  }
}

// One 4-wave block per split row.  The row's partials form a chain in task
// order: item 0 = head slab of the owning task, item k = continuation slab of
// task owner+k.  Wave q reduces items [q*c, (q+1)*c) in order (U loads in
// flight), waves 1..3 hand their result to wave 0 through LDS, wave 0 merges
// them in wave order and finishes the row: a fixed order, so deterministic.
template <class Red, int VEC>
__global__ __launch_bounds__(kBlock) void k_agg_fixup(AggArgs p) {
  constexpr int U = 4;
  __shared__ typename Red::Part lds[kWavesPerBlock - 1][64];
  __shared__ int has[kWavesPerBlock];
  const int lane = lane_id();
  const int wid = uni((int)(threadIdx.x >> 6));
  const int i = (int)blockIdx.x;
  const int f = (int)blockIdx.y * 64 * VEC + lane * VEC;
  const bool act = f < p.F;
  const int fs = act ? f : 0;
  if (p.o_tw) {  // tile-major out (the host runs this fix-up 64 features wide then)
    const float* xt;
    int64_t ldt;
    int fx0;
    tile_view(p, (int)blockIdx.y * 64 * VEC, xt, ldt, fx0);
  }
  const int last = uni(p.split_waves[i]);
  const int r = uni(p.wave_row[last]) - 1;
  const int64_t rs = uni(p.rowptr[r]);
  const int64_t re = uni(p.rowptr[r + 1]);
  // owner = last task whose first owned row is <= r
  int lo = 0, hi = p.n_waves;  // wave_row[n_waves] = n_rows > r
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (p.wave_row[mid] <= r) lo = mid;
    else hi = mid - 1;
  }
  const int owner = uni(lo);
  const int L = last - owner + 1;
  const int c = (L + kWavesPerBlock - 1) / kWavesPerBlock;
  const int b0 = wid * c;
  const int b1 = min(L, b0 + c);
  Red red(p, f, act);
  auto item = [&](int k) {
    int64_t slot = k == 0 ? 2 * (int64_t)owner + 1 : 2 * (int64_t)(owner + k);
    return slab_ref(p, slot, fs, red);
  };
  const bool mine = b0 < b1;
  if (mine) {
    red.set(Red::load(item(b0)));
    for (int k = b0 + 1; k < b1; k += U) {
      typename Red::Part q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) q[u] = Red::load(item(min(k + u, b1 - 1)));
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k + u < b1) red.merge(q[u]);
    }
  }
  if (lane == 0) has[wid] = mine ? 1 : 0;
  if (wid > 0 && mine) lds[wid - 1][lane] = red.part();
  __syncthreads();
  if (wid != 0) return;
  for (int q = 1; q < kWavesPerBlock; ++q)
    if (has[q]) red.merge(lds[q - 1][lane]);
  if constexpr (Red::kGatB) red.row_terms(p, r);
  red.finish(p, r, re - rs, f, act, p.bias_rows == nullptr || p.bias_rows[r] != 0);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

struct Shape {
  int vec, lanes;
};

static int next_pow2(int v) {
  int r = 1;
  while (r < v) r <<= 1;
  return r;
}

// VEC = widest aligned per-lane vector; L = lanes per task: enough to cover
// the row (small F packs several tasks per wave), at most 64.
static Shape pick_shape(int F, int64_t ldx, const void* x, int64_t ldo, const void* out) {
  auto aligned = [](const void* ptr, int64_t ld, int v) {
    return ((uintptr_t)ptr % (4 * v) == 0) && (ld % v == 0);
  };
  int vec = 1;
  if (F % 4 == 0 && aligned(x, ldx, 4) && aligned(out, ldo, 4)) vec = 4;
  else if (F % 2 == 0 && F > 64 && aligned(x, ldx, 2) && aligned(out, ldo, 2)) vec = 2;
  int lanes = 64;
  if (vec == 4) {
    int need = next_pow2((F + 3) / 4);
    lanes = need < 4 ? 4 : (need > 64 ? 64 : need);
    if (F >= 256) lanes = kWideLanes;
  }
  return {vec, lanes};
}

// the same reducer at another lane width (fix-up of a VEC=2 main kernel at VEC=4)
template <class Red, int V>
struct Rebind {
  using type = Red;
};
template <int VEC, bool W, bool M, int V>
struct Rebind<SumRed<VEC, W, M>, V> {
  using type = SumRed<V, W, M>;
};
template <int VEC, bool W, bool M, int V>
struct Rebind<ArgRed<VEC, W, M>, V> {
  using type = ArgRed<V, W, M>;
};

// Kernel query (mp_aggregate_kernel_name): while set, the main-stage launch
// records the kernel the dispatcher chose instead of launching it.
static thread_local bool g_query = false;
static thread_local const void* g_query_kernel = nullptr;

static int launch_main(void (*k)(AggArgs), dim3 grid, hipStream_t s, const AggArgs& a) {
  if (g_query) {
    g_query_kernel = reinterpret_cast<const void*>(k);
    return MP_OK;
  }
  hipLaunchKernelGGL(k, grid, dim3(kBlock), 0, s, a);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

// the mp_aggregate_tiles_f32 instances: XM from the call (per-row bias flags /
// skipped rows / neither), TM when an operand is tile-major
template <class Red, int U, int XM>
static int launch_xm(const AggArgs& a, dim3 grid, hipStream_t s, bool far) {
  const bool tm = a.x_tw || a.o_tw;
  if (tm)
    return far ? launch_main(k_agg_flat<Red, 1, kU_Vec1Far, 64, false, true, XM, true>, grid, s, a)
               : launch_main(k_agg_flat<Red, 1, U, 64, false, true, XM, true>, grid, s, a);
  return far ? launch_main(k_agg_flat<Red, 1, kU_Vec1Far, 64, false, true, XM>, grid, s, a)
             : launch_main(k_agg_flat<Red, 1, U, 64, false, true, XM>, grid, s, a);
}
template <class Red, int U>
static int launch_xr(const AggArgs& a, dim3 grid, hipStream_t s, bool far) {
  if (a.bias_rows) return launch_xm<Red, U, 1>(a, grid, s, far);
  if (a.flags & MP_FLAG_SKIP_EMPTY) return launch_xm<Red, U, 2>(a, grid, s, far);
  return launch_xm<Red, U, 0>(a, grid, s, far);
}

template <class Red, int VEC, int L>
static int launch_l(const AggArgs& a, int stages, hipStream_t s) {
  // the GAT backward holds a 16-B destination pack per slot in flight: U = 8 at every width
  constexpr int U = (Red::kGatB && L == 64) ? kU_Vec4
                    : VEC == 4 ? (L == 64 ? (kGatTrain<Red> ? kU_GatTrain : kU_Vec4) : kU_Narrow)
                               : (VEC == 2 ? kU_Vec2 : (L < kU_Vec1 ? L : kU_Vec1));  // VEC=1 groups < 16 lanes: GAT stats
  const int ftiles = (int)ceil_div(a.F, L * VEC);
  if (stages & MP_STAGE_MAIN) {
    int64_t nb = ceil_div(a.n_waves, kWavesPerBlock * (64 / L));
    if (kXcdTiles && 8 % ftiles == 0) nb = ceil_div(nb, 8 / ftiles) * (8 / ftiles);
    dim3 grid((unsigned)nb, (unsigned)ftiles);
    int rc = MP_OK;
    if (a.flat) {
      if constexpr (!Red::kGat && !Red::kGatB && !Red::kHW && !kGatWideV<Red>) {
        if constexpr (L == 64 && !Red::kEid) {
          bool far = false;
          if constexpr (VEC == 1) {
            far = a.smem && a.far;
            if (far && !a.xr) rc = launch_main(k_agg_flat<Red, 1, kU_Vec1Far, 64, false, true>, grid, s, a);
          }
          if constexpr (VEC == 1) {
            // mp_aggregate_tiles_f32 (scalar batches, 64-feature tiles by construction)
            if (a.xr) rc = launch_xr<Red, U>(a, grid, s, far);
          }
          if (far || a.xr) {
          } else if (a.smem) rc = launch_main(k_agg_flat<Red, VEC, U, 64, false, true>, grid, s, a);
          else rc = launch_main(k_agg_flat<Red, VEC, U, L>, grid, s, a);
        } else {
          rc = launch_main(k_agg_flat<Red, VEC, U, L>, grid, s, a);
        }
      }
    } else {
      rc = launch_main(k_agg_main<Red, VEC, U, L>, grid, s, a);
    }
    if (rc) return rc;
  }
  if ((stages & MP_STAGE_FIXUP) && a.n_split > 0) {
    if constexpr (VEC != 4 && !Red::kGat && !Red::kGatB && !Red::kHW && !kGatWideV<Red>) {
      if (a.fix4) {
        dim3 grid4((unsigned)a.n_split, (unsigned)ceil_div(a.F, 64 * 4));
        hipLaunchKernelGGL((k_agg_fixup<typename Rebind<Red, 4>::type, 4>), grid4, dim3(kBlock), 0, s, a);
        MP_CHECK_LAUNCH();
        return MP_OK;
      }
    }
    dim3 grid((unsigned)a.n_split, (unsigned)ceil_div(a.F, 64 * VEC));
    hipLaunchKernelGGL((k_agg_fixup<Red, VEC>), grid, dim3(kBlock), 0, s, a);
    MP_CHECK_LAUNCH();
  }
  return MP_OK;
}

template <class Red, int VEC, int NV>
static int launch_lane(const AggArgs& a, int stages, hipStream_t s) {
  if (stages & MP_STAGE_MAIN) {
    dim3 grid((unsigned)ceil_div(a.n_waves, kBlock));
    constexpr int U = VEC * NV >= 16 ? (kULane + 1) / 2 : kULane;  // 16-float rows: keep VGPRs < 128
    int rc = launch_main(k_agg_lane<Red, VEC, NV, U>, grid, s, a);
    if (rc) return rc;
  }
  if ((stages & MP_STAGE_FIXUP) && a.n_split > 0) {
    dim3 grid((unsigned)a.n_split, (unsigned)ceil_div(a.F, 64 * VEC));
    hipLaunchKernelGGL((k_agg_fixup<Red, VEC>), grid, dim3(kBlock), 0, s, a);
    MP_CHECK_LAUNCH();
  }
  return MP_OK;
}

// lane-task shape for F <= kLaneMaxF: VEC=4 with NV in {1,2,4} or VEC=1
// with NV in {4,8,16}; -1 when the row is too wide
template <class Red, int VEC>
static int try_lane(const AggArgs& a, int stages, hipStream_t s) {
  if (a.F > kLaneMaxF || a.F < 2) return -1;
  if constexpr (VEC == 4) {
    if (a.F <= 4) return launch_lane<Red, 4, 1>(a, stages, s);
    return launch_lane<Red, 4, 2>(a, stages, s);
  } else if constexpr (VEC == 1) {
    if (a.F <= 4) return launch_lane<Red, 1, 4>(a, stages, s);
    return launch_lane<Red, 1, 8>(a, stages, s);
  }
  return -1;
}

template <class Red, int VEC>
static int launch(const AggArgs& a, int stages, hipStream_t s, int lanes = 64) {
  if constexpr (VEC == 4) {
    switch (lanes) {
      case 4: return launch_l<Red, 4, 4>(a, stages, s);
      case 8: return launch_l<Red, 4, 8>(a, stages, s);
      case 16: return launch_l<Red, 4, 16>(a, stages, s);
      case 32: return launch_l<Red, 4, 32>(a, stages, s);
      default: break;
    }
  }
  return launch_l<Red, VEC, 64>(a, stages, s);
}

template <class Red, int VEC>
static int launch_any(const AggArgs& a, int stages, hipStream_t s, int L) {
  if constexpr (VEC != 2) {
    int rc = try_lane<Red, VEC>(a, stages, s);
    if (rc >= 0) return rc;
  }
  return launch<Red, VEC>(a, stages, s, L);
}

template <int VEC>
static int dispatch_reduce(const AggArgs& a, int reduce, int stages, hipStream_t s, int L) {
  const bool hw = a.w != nullptr;
  switch (reduce) {
    case MP_REDUCE_SUM:
      return hw ? launch_any<SumRed<VEC, true, false>, VEC>(a, stages, s, L)
                : launch_any<SumRed<VEC, false, false>, VEC>(a, stages, s, L);
    case MP_REDUCE_MEAN:
      return hw ? launch_any<SumRed<VEC, true, true>, VEC>(a, stages, s, L)
                : launch_any<SumRed<VEC, false, true>, VEC>(a, stages, s, L);
    case MP_REDUCE_MAX:
      return hw ? launch_any<ArgRed<VEC, true, true>, VEC>(a, stages, s, L)
                : launch_any<ArgRed<VEC, false, true>, VEC>(a, stages, s, L);
    case MP_REDUCE_MIN:
      return hw ? launch_any<ArgRed<VEC, true, false>, VEC>(a, stages, s, L)
                : launch_any<ArgRed<VEC, false, false>, VEC>(a, stages, s, L);
  }
  set_error("mp_aggregate_f32: unknown reduce %d", reduce);
  return MP_ERR_ARG;
}

static int64_t slab_ld_for(int F) { return ceil_div(F, 256) * 256; }

// ---------------------------------------------------------------------------
// mp_tune: the one table of run-time dispatch choices (include/mi355_mp.h).
// Defaults are the A/B winners; every alternative gives
// bitwise-identical results.
// ---------------------------------------------------------------------------
struct Tune {
  std::atomic<int64_t> flat_vec1_min_bytes{0};  // sum/mean: 64-feature tiles at every x size (scalar batches)
  std::atomic<int64_t> flat_smem{1};
  std::atomic<int64_t> flat_min_f{64};
  std::atomic<int64_t> flat_min_f_arg{64};
  std::atomic<int64_t> flat_narrow_vec1{64};  // F=64: one full 64-feature tile, -26% vs a half-used 128 tile
  std::atomic<int64_t> flat_vec{2};
  std::atomic<int64_t> flat_vec_arg{2};
  std::atomic<int64_t> flat_seq_tiles{0};
  std::atomic<int64_t> flat_far_min_bytes{256ll << 20};  // the Infinity Cache
  std::atomic<int64_t> gat_bwd_vec{4};  // features per lane of the GAT backward's transposed pass
};
static Tune g_tune;

static std::atomic<int64_t>* tune_slot(int32_t key) {
  switch (key) {
    case MP_TUNE_FLAT_VEC1_MIN_BYTES: return &g_tune.flat_vec1_min_bytes;
    case MP_TUNE_FLAT_SMEM: return &g_tune.flat_smem;
    case MP_TUNE_FLAT_MIN_F: return &g_tune.flat_min_f;
    case MP_TUNE_FLAT_MIN_F_ARG: return &g_tune.flat_min_f_arg;
    case MP_TUNE_FLAT_NARROW_VEC1: return &g_tune.flat_narrow_vec1;
    case MP_TUNE_FLAT_VEC: return &g_tune.flat_vec;
    case MP_TUNE_FLAT_VEC_ARG: return &g_tune.flat_vec_arg;
    case MP_TUNE_FLAT_SEQ_TILES: return &g_tune.flat_seq_tiles;
    case MP_TUNE_FLAT_FAR_MIN_BYTES: return &g_tune.flat_far_min_bytes;
    case MP_TUNE_GAT_BWD_VEC: return &g_tune.gat_bwd_vec;
  }
  return nullptr;
}

static inline int64_t tuned(std::atomic<int64_t>& v) { return v.load(std::memory_order_relaxed); }

static int check_graph(const mp_csr* g, const char* who) {
  MP_CHECK_ARG(g != nullptr, "%s: null graph", who);
  MP_CHECK_ARG(g->rowptr && g->wave_row && g->wave_slot && (g->n_split == 0 || g->split_waves),
               "%s: graph has null arrays", who);
  MP_CHECK_ARG(g->n_edges == 0 || g->eid, "%s: graph has null eid", who);
  MP_CHECK_ARG(g->n_ids == 0 || (g->n_ids >= g->n_edges && g->n_ids <= INT32_MAX),
               "%s: n_ids must be 0 or in [n_edges, 2^31)", who);
  MP_CHECK_ARG(g->chunk >= 16 && g->chunk % 8 == 0 && g->n_waves >= 1, "%s: bad schedule", who);
  MP_CHECK_ARG(g->col == nullptr || g->n_edges == 0 || g->n_cols > 0,
               "%s: n_cols must be the row count of the gathered x (got %d with a column array)", who,
               (int)g->n_cols);
  return MP_OK;
}

static void fill_graph(AggArgs& a, const mp_csr* g) {
  a.rowptr = g->rowptr;
  a.col = g->col;
  a.eid = g->eid;
  a.wave_row = g->wave_row;
  a.wave_slot = g->wave_slot;
  a.split_waves = g->split_waves;
  a.n_rows = g->n_rows;
  a.n_edges = g->n_edges;
  a.n_ids = g->n_ids > 0 ? g->n_ids : g->n_edges;
  a.chunk = g->chunk;
  a.n_waves = g->n_waves;
  a.n_split = g->n_split;
  a.n_cols = g->n_cols;
}

// Shape selection and launch of one mp_aggregate_f32 call (args checked).
static int aggregate_dispatch(AggArgs& a, const mp_csr* g, int reduce, int stages, hipStream_t s) {
  const int F = a.F;
  const bool is_arg = reduce == MP_REDUCE_MAX || reduce == MP_REDUCE_MIN;
  if (a.x_tw || a.o_tw || a.force_flat) {
    // tile-major operands (mp_aggregate_tiles_f32, arguments checked there): the
    // scalar-batch flat kernel with 64-feature tiles, its fix-up 64 wide
    const int64_t xbytes = (int64_t)g->n_cols * (a.x_tw ? a.x_tw : a.ldx) * 4;
    a.flat = 1;
    a.smem = 1;
    a.x_bytes = (uint32_t)xbytes;
    a.far = xbytes > tuned(g_tune.flat_far_min_bytes) ? 1 : 0;
    // feature tiles one after another when x outgrows the Infinity Cache by up to 4x: then
    // each 64-feature tile of it (a quarter) fits, and the tiles take turns in it (the
    // sharded step's P = 4 passes: interior 0.68 -> 0.65 ms, send 1.26 -> 1.22 ms; at P = 8,
    // x fits whole and XCD-affine tiles stay ahead by 1-2 %; tools/exp_boundary.py)
    const int64_t x_all = (int64_t)g->n_cols * F * 4;
    a.seq_tiles = (tuned(g_tune.flat_seq_tiles) || (x_all > kSeqTilesMin && x_all <= 4 * tuned(g_tune.flat_far_min_bytes)))
                      ? 1 : 0;
    a.fix4 = 0;
    a.xr = 1;
    return dispatch_reduce<1>(a, reduce, stages, s, 64);
  }
  Shape sh = pick_shape(F, a.ldx, a.x, a.ldo, a.out);
  // flat kernel lane width: 64-feature tiles (VEC=1) for sum/mean, where an
  // XCD's L2 holding one narrow tile of the hot rows pays (Reddit-scale x of
  // 238 MB: 8.28 -> 7.25 ms; RMAT21 x of 2 GB 6.98 -> 6.73 ms); 128-feature
  // tiles (VEC=2) for max/min, whose compare-and-select per element is bound
  // by the texture-address unit rather than by L2 misses (VEC=1: +15..29%)
  const int64_t xbytes = (int64_t)g->n_cols * a.ldx * 4;
  int fvec = (int)(is_arg ? tuned(g_tune.flat_vec_arg) : tuned(g_tune.flat_vec));
  // The L1 miss queue holds 256-B segments: a 64-feature
  // tile of a row that does not start on a 256-B boundary straddles two of
  // them.  Such rows take the widest per-lane vector the layout allows, which
  // touches the fewest segments per row (F=200: 8.43 -> 6.93 ms sum, 8.34 ->
  // 7.16 ms max; F=130 sum 6.78 -> 6.44 ms on RMAT21).
  const bool seg_aligned = (a.ldx * 4) % 256 == 0 && (uintptr_t)a.x % 256 == 0;
  if (!seg_aligned) {
    fvec = sh.vec;
  } else {
    if (!is_arg && xbytes >= tuned(g_tune.flat_vec1_min_bytes)) fvec = 1;
    if (F <= tuned(g_tune.flat_narrow_vec1)) fvec = 1;
  }
  // sum/mean: slot columns and weights through scalar loads (k_agg_flat SM),
  // 32-bit buffer offsets (soffset + lane offset) while x spans < 4 GiB.
  // (Max/min through the same batches, edge ids included: bitwise equal and
  // no faster -- Reddit-scale 8.67 vs 8.67 ms, RMAT21 7.77 vs 7.76 ms,
  // profiles/r02_ab_smem_arg.log -- so they keep the slot window.)
  a.smem = tuned(g_tune.flat_smem) && !is_arg && a.col != nullptr && g->n_cols > 0 && xbytes <= 0xFFFFFFF0LL;
  if (a.smem) a.x_bytes = (uint32_t)xbytes;
  // In-flight depth of the scalar-batch kernel: 16 row loads per wave while x
  // fits the Infinity Cache (Reddit-scale, 238 MB: 7.25 ms vs 7.64 at 8); 8
  // beyond it (RMAT21 6.71 -> 6.58 ms, ogbn-products-scale 15.0 -> 14.6 ms;
  // profiles/r02_ab_batch_u.log)
  a.far = xbytes > tuned(g_tune.flat_far_min_bytes) ? 1 : 0;
  a.seq_tiles = (int32_t)tuned(g_tune.flat_seq_tiles);
  const int64_t min_f = is_arg ? tuned(g_tune.flat_min_f_arg) : tuned(g_tune.flat_min_f);
  if (F >= min_f && F % fvec == 0 && sh.vec >= fvec) {
    sh.vec = fvec;  // narrow feature tiles, slot batches across rows
    sh.lanes = 64;
    a.flat = 1;
    // the fix-up reads slabs by feature: run it 4 wide when out (and bias) allow
    a.fix4 = F % 4 == 0 && (uintptr_t)a.out % 16 == 0 && a.ldo % 4 == 0 && (uintptr_t)a.bias % 16 == 0;
  }
  switch (sh.vec) {
    case 4: return dispatch_reduce<4>(a, reduce, stages, s, sh.lanes);
    case 2: return dispatch_reduce<2>(a, reduce, stages, s, 64);
    default: return dispatch_reduce<1>(a, reduce, stages, s, 64);
  }
}

// the dropout keep bits of slots [0, n) (mp_gat_dropout_keep: tests, host-side masks)
__global__ void k_gat_dropout_keep(AggArgs p, int64_t n, uint32_t* bits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) bits[i] = drop_bits(p, p.drop_ids ? (int64_t)p.drop_ids[i] : i);
}

}  // namespace mp

using namespace mp;

extern "C" {

int64_t mp_tune(int32_t key, int64_t value) {
  std::atomic<int64_t>* v = tune_slot(key);
  if (!v) return -1;
  if (value < 0) return v->load();
  if (key == MP_TUNE_FLAT_SMEM || key == MP_TUNE_FLAT_SEQ_TILES) value = value ? 1 : 0;
  if ((key == MP_TUNE_FLAT_VEC || key == MP_TUNE_FLAT_VEC_ARG || key == MP_TUNE_GAT_BWD_VEC) && value != 1 &&
      value != 2 && value != 4)
    return -1;
  return v->exchange(value);
}

size_t mp_aggregate_slab_bytes(const mp_csr* g, int32_t F, int32_t reduce) {
  if (!g || F <= 0) return 256;
  size_t slots = 2 * (size_t)g->n_waves;
  size_t per = (size_t)slab_ld_for(F) * 4;
  size_t v = align_up(slots * per, 256);
  bool arg = reduce == MP_REDUCE_MAX || reduce == MP_REDUCE_MIN;
  return v + (arg ? v : 0) + 256;
}

int mp_aggregate_f32(const mp_csr* g, const float* w, const float* x, int64_t ldx, int32_t F,
                     int32_t reduce, int32_t flags, const float* bias, float* out, int64_t ldo,
                     int64_t* arg_out, void* slab, size_t slab_bytes, int32_t stages, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_aggregate_f32");
  if (rc) return rc;
  MP_CHECK_ARG(F > 0, "mp_aggregate_f32: F must be positive");
  MP_CHECK_ARG(out != nullptr && (g->n_edges == 0 || x != nullptr), "mp_aggregate_f32: null x/out");
  MP_CHECK_ARG(ldx >= F && ldo >= F, "mp_aggregate_f32: leading dimension < F");
  const bool is_arg = reduce == MP_REDUCE_MAX || reduce == MP_REDUCE_MIN;
  MP_CHECK_ARG(!is_arg || arg_out != nullptr, "mp_aggregate_f32: max/min need arg_out");
  MP_CHECK_ARG(slab != nullptr && slab_bytes >= mp_aggregate_slab_bytes(g, F, reduce),
               "mp_aggregate_f32: slab workspace too small (%zu < %zu)", slab_bytes,
               mp_aggregate_slab_bytes(g, F, reduce));
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.w = w;
  a.x = x;
  a.ldx = ldx;
  a.flags = flags;
  a.bias = bias;
  a.out = out;
  a.ldo = ldo;
  a.arg_out = arg_out;
  a.slab_ld = slab_ld_for(F);
  size_t v = align_up(2 * (size_t)g->n_waves * (size_t)a.slab_ld * 4, 256);
  a.slab_v = (float*)slab;
  a.slab_a = is_arg ? (int32_t*)((char*)slab + v) : nullptr;
  return aggregate_dispatch(a, g, reduce, stages, as_stream(stream));
}

int mp_aggregate_tiles_f32(const mp_csr* g, const float* w, const float* x, int64_t ldx, int32_t x_tile_w,
                           int64_t x_tile_stride, int32_t F, int32_t reduce, int32_t flags, const float* bias,
                           const int32_t* bias_rows, float* out, int64_t ldo, int32_t out_tile_w,
                           int64_t out_tile_stride, void* slab, size_t slab_bytes, int32_t stages, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_aggregate_tiles_f32");
  if (rc) return rc;
  MP_CHECK_ARG(reduce == MP_REDUCE_SUM || reduce == MP_REDUCE_MEAN, "mp_aggregate_tiles_f32: sum or mean only");
  MP_CHECK_ARG(F > 0 && F % 64 == 0, "mp_aggregate_tiles_f32: F must be a positive multiple of 64");
  MP_CHECK_ARG((flags & ~(MP_FLAG_INIT_FROM_OUT | MP_FLAG_SKIP_EMPTY)) == 0,
               "mp_aggregate_tiles_f32: flags may only hold INIT_FROM_OUT and SKIP_EMPTY");
  MP_CHECK_ARG(!(bias_rows && bias && (flags & MP_FLAG_SKIP_EMPTY)),
               "mp_aggregate_tiles_f32: per-row bias flags and SKIP_EMPTY are separate calls (one kernel each)");
  MP_CHECK_ARG(out != nullptr && (g->n_edges == 0 || (x != nullptr && g->col != nullptr && g->n_cols > 0)),
               "mp_aggregate_tiles_f32: null x/out or a graph without columns");
  MP_CHECK_ARG(x_tile_w >= 0 && out_tile_w >= 0, "mp_aggregate_tiles_f32: negative tile width");
  const int64_t ncols = g->n_cols > 0 ? g->n_cols : 0;
  if (x_tile_w) {
    MP_CHECK_ARG(x_tile_w % 64 == 0 && F % x_tile_w == 0 && x_tile_stride >= ncols * x_tile_w,
                 "mp_aggregate_tiles_f32: x tiles must be 64k features wide, divide F, and not overlap "
                 "(stride %lld < %lld rows x %d)", (long long)x_tile_stride, (long long)ncols, (int)x_tile_w);
  } else {
    MP_CHECK_ARG(ldx >= F, "mp_aggregate_tiles_f32: ldx < F");
  }
  MP_CHECK_ARG(ncols * (x_tile_w ? x_tile_w : ldx) * 4 <= 0xFFFFFFF0LL,
               "mp_aggregate_tiles_f32: one x tile must span < 4 GiB");
  if (out_tile_w) {
    MP_CHECK_ARG(out_tile_w % 64 == 0 && F % out_tile_w == 0 && out_tile_stride >= g->n_rows * out_tile_w,
                 "mp_aggregate_tiles_f32: out tiles must be 64k features wide, divide F, and not overlap "
                 "(stride %lld < %lld rows x %d)", (long long)out_tile_stride, (long long)g->n_rows,
                 (int)out_tile_w);
  } else {
    MP_CHECK_ARG(ldo >= F, "mp_aggregate_tiles_f32: ldo < F");
  }
  MP_CHECK_ARG(slab != nullptr && slab_bytes >= mp_aggregate_slab_bytes(g, F, reduce),
               "mp_aggregate_tiles_f32: slab workspace too small (%zu < %zu)", slab_bytes,
               mp_aggregate_slab_bytes(g, F, reduce));
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.w = w;
  a.x = x;
  a.ldx = x_tile_w ? x_tile_w : ldx;
  a.x_tw = x_tile_w;
  a.x_ts = x_tile_stride;
  a.flags = flags;
  a.bias = bias;
  a.bias_rows = bias ? bias_rows : nullptr;  // the flags matter only with a bias
  a.out = out;
  a.ldo = out_tile_w ? out_tile_w : ldo;
  a.o_tw = out_tile_w;
  a.o_ts = out_tile_stride;
  a.slab_ld = slab_ld_for(F);
  a.slab_v = (float*)slab;
  // every call takes the scalar-batch flat kernel with 64-feature tiles (its
  // instance chosen by the operands' layout and the call's options), row-major
  // operands included: the same kernel mp_aggregate_f32 picks for such rows,
  // with the feature-tile order chosen for the pass's x (see aggregate_dispatch)
  a.force_flat = 1;
  return aggregate_dispatch(a, g, reduce, stages, as_stream(stream));
}

int mp_aggregate_kernel_name(const mp_csr* g, const float* w, const float* x, int64_t ldx, int32_t F,
                             int32_t reduce, const float* bias, const float* out, int64_t ldo, char* buf,
                             size_t buf_len, void* stream) {
  int rc = check_graph(g, "mp_aggregate_kernel_name");
  if (rc) return rc;
  MP_CHECK_ARG(F > 0 && ldx >= F && ldo >= F && buf != nullptr && buf_len > 0,
               "mp_aggregate_kernel_name: bad arguments");
  MP_CHECK_ARG(reduce >= MP_REDUCE_SUM && reduce <= MP_REDUCE_MIN, "mp_aggregate_kernel_name: unknown reduce %d",
               reduce);
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.w = w;
  a.x = x;
  a.ldx = ldx;
  a.bias = bias;
  a.out = const_cast<float*>(out);
  a.ldo = ldo;
  g_query = true;
  g_query_kernel = nullptr;
  rc = aggregate_dispatch(a, g, reduce, MP_STAGE_MAIN, as_stream(stream));
  g_query = false;
  if (rc) return rc;
  MP_CHECK_ARG(g_query_kernel != nullptr, "mp_aggregate_kernel_name: no main kernel selected");
  const char* mangled = hipKernelNameRefByPtr(g_query_kernel, as_stream(stream));
  MP_CHECK_ARG(mangled != nullptr, "mp_aggregate_kernel_name: HIP has no name for the kernel (no device?)");
  int st = 0;
  char* dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
  const char* name = (st == 0 && dem) ? dem : mangled;
  snprintf(buf, buf_len, "%s", name);
  free(dem);
  return MP_OK;
}

int mp_aggregate_heads_f32(const mp_csr* g, const float* w, int32_t H, const float* x, int64_t ldx, int32_t F,
                           float* out, int64_t ldo, void* slab, size_t slab_bytes, int32_t stages, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_aggregate_heads_f32");
  if (rc) return rc;
  MP_CHECK_ARG(F > 0 && H > 0 && F % H == 0, "mp_aggregate_heads_f32: F must be a positive multiple of H");
  MP_CHECK_ARG(out && (g->n_edges == 0 || (x && w)), "mp_aggregate_heads_f32: null pointer");
  MP_CHECK_ARG(ldx >= F && ldo >= F, "mp_aggregate_heads_f32: leading dimension < F");
  MP_CHECK_ARG(slab && slab_bytes >= mp_aggregate_slab_bytes(g, F, MP_REDUCE_SUM),
               "mp_aggregate_heads_f32: slab workspace too small");
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.w = w;
  a.x = x;
  a.ldx = ldx;
  a.out = out;
  a.ldo = ldo;
  a.H = H;
  a.C = F / H;
  a.slab_ld = slab_ld_for(F);
  a.slab_v = (float*)slab;
  hipStream_t s = as_stream(stream);
  Shape sh = pick_shape(F, ldx, x, ldo, out);
  int vec = sh.vec;
  while (vec > 1 && a.C % vec != 0) vec >>= 1;  // a lane's features must share a head
  if (vec == 4) return launch<HeadSumRed<4>, 4>(a, stages, s, sh.lanes);
  if (vec == 2) return launch<HeadSumRed<2>, 2>(a, stages, s, 64);
  return launch<HeadSumRed<1>, 1>(a, stages, s, 64);
}

size_t mp_gat_slab_bytes(const mp_csr* g, int32_t H, int32_t C) {
  if (!g || H <= 0 || C <= 0) return 256;
  size_t slots = 2 * (size_t)g->n_waves;
  size_t v = align_up(slots * (size_t)slab_ld_for(H * C) * 4, 256);
  size_t st = align_up(slots * (size_t)H * 2 * 4, 256);
  return v + st + 256;
}

size_t mp_gat_train_slab_bytes(const mp_csr* g, int32_t H, int32_t C) {
  if (!g || H <= 0 || C <= 0) return 256;
  size_t slots = 2 * (size_t)g->n_waves;
  size_t v = align_up(slots * (size_t)slab_ld_for(H * C) * 4, 256);
  size_t s2 = align_up(slots * (size_t)H * 4, 256);
  return mp_gat_slab_bytes(g, H, C) + v + s2;
}

int mp_gat_train_ok(int32_t H, int32_t C) {
  const int hl4 = C / 4;
  return H > 0 && C > 0 && C % 4 == 0 && hl4 <= 64 && (hl4 & (hl4 - 1)) == 0 ? 1 : 0;
}

int mp_gat_aggregate_f32(const mp_csr* g, const float* xw, const float* a_src, const float* a_dst,
                         int32_t H, int32_t C, float slope, const float* bias, float* out,
                         int64_t ldo, float* row_stats, void* slab, size_t slab_bytes,
                         int32_t stages, void* stream) {
  return mp_gat_aggregate_att_f32(g, xw, a_src, a_dst, nullptr, H, C, slope, bias, out, ldo, row_stats, slab,
                                  slab_bytes, stages, stream);
}

int mp_gat_aggregate_att_f32(const mp_csr* g, const float* xw, const float* a_src, const float* a_dst,
                             const float* att, int32_t H, int32_t C, float slope, const float* bias, float* out,
                             int64_t ldo, float* row_stats, void* slab, size_t slab_bytes, int32_t stages,
                             void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_gat_aggregate_f32");
  if (rc) return rc;
  MP_CHECK_ARG(H > 0 && C > 0, "mp_gat_aggregate_f32: H, C must be positive");
  MP_CHECK_ARG(xw && a_src && a_dst && out, "mp_gat_aggregate_f32: null input");
  const int F = H * C;
  MP_CHECK_ARG(ldo >= F, "mp_gat_aggregate_f32: ldo < H*C");
  MP_CHECK_ARG(slab != nullptr && slab_bytes >= mp_gat_slab_bytes(g, H, C),
               "mp_gat_aggregate_f32: slab workspace too small");
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.x = xw;
  a.ldx = F;
  a.out = out;
  a.ldo = ldo;
  a.bias = bias;
  a.a_src = a_src;
  a.a_dst = a_dst;
  a.H = H;
  a.C = C;
  a.slope = slope;
  a.row_stats = row_stats;
  a.slab_ld = slab_ld_for(F);
  size_t v = align_up(2 * (size_t)g->n_waves * (size_t)a.slab_ld * 4, 256);
  a.slab_v = (float*)slab;
  a.slab_s = (float*)((char*)slab + v);
  hipStream_t s = as_stream(stream);
  int vec = pick_shape(F, F, xw, ldo, out).vec;
  if (vec == 2 && F <= 64) vec = 1;
  while (vec > 1 && C % vec != 0) vec >>= 1;  // a lane's features must share a head
  // a_src from the gathered rows: the node-score kernel's 4-feature lane
  // partials and head groups of C/4 lanes (a power of two <= 64)
  const int hl4 = C / 4;
  if (att && vec == 4 && C % 4 == 0 && hl4 <= 64 && (hl4 & (hl4 - 1)) == 0 && (uintptr_t)att % 16 == 0) {
    a.att = att;
    return launch<GatRed<4, true>, 4>(a, stages, s, F >= 256 ? kGatLanes : 64);
  }
  switch (vec) {
    case 4: return launch<GatRed<4>, 4>(a, stages, s, F >= 256 ? kGatLanes : 64);
    case 2: return launch<GatRed<2>, 2>(a, stages, s);
    default: return launch<GatRed<1>, 1>(a, stages, s);
  }
}

int mp_gat_forward_f32(const mp_csr* g, const float* xw, const float* att, int32_t H, int32_t C, float slope,
                       const float* bias, float* out, int64_t ldo, float* a_src, float* a_dst, float* row_stats,
                       void* slab, size_t slab_bytes, int32_t stages, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_gat_forward_f32");
  if (rc) return rc;
  MP_CHECK_ARG(mp_gat_train_ok(H, C), "mp_gat_forward_f32: needs C %% 4 == 0 and C/4 a power of two <= 64");
  MP_CHECK_ARG(xw && att && out && a_src && a_dst, "mp_gat_forward_f32: null pointer");
  MP_CHECK_ARG(g->n_cols == g->n_rows, "mp_gat_forward_f32: the graph must be square (row i's own xw is row i)");
  const int F = H * C;
  MP_CHECK_ARG(ldo >= F && ldo % 4 == 0, "mp_gat_forward_f32: ldo < H*C or not a multiple of 4");
  MP_CHECK_ARG((uintptr_t)xw % 16 == 0 && (uintptr_t)att % 16 == 0 && (uintptr_t)out % 16 == 0 &&
                   (uintptr_t)bias % 16 == 0,
               "mp_gat_forward_f32: xw, att, bias, out must be 16-byte aligned");
  MP_CHECK_ARG(slab != nullptr && slab_bytes >= mp_gat_slab_bytes(g, H, C),
               "mp_gat_forward_f32: slab workspace too small");
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.x = xw;
  a.ldx = F;
  a.out = out;
  a.ldo = ldo;
  a.bias = bias;
  a.a_src_out = a_src;
  a.a_dst_out = a_dst;
  a.att = att;
  a.H = H;
  a.C = C;
  a.slope = slope;
  a.row_stats = row_stats;
  a.slab_ld = slab_ld_for(F);
  size_t v = align_up(2 * (size_t)g->n_waves * (size_t)a.slab_ld * 4, 256);
  a.slab_v = (float*)slab;
  a.slab_s = (float*)((char*)slab + v);
  return launch<GatRed<4, true, false, true>, 4>(a, stages, as_stream(stream), F >= 256 ? kGatLanes : 64);
}

// keep threshold p * 2^32 and scale 1 / (1 - p) (in double, then rounded: F.dropout's scale)
static void set_drop(AggArgs& a, uint64_t seed, float p_drop, const int32_t* drop_ids = nullptr) {
  const double t = std::floor((double)p_drop * 4294967296.0);
  a.drop_seed = seed;
  a.drop_ids = drop_ids;
  a.drop_thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  a.drop_scale = (float)(1.0 / (1.0 - (double)p_drop));
}

static int drop_check(float p_drop, int32_t H, const char* who) {
  MP_CHECK_ARG(p_drop > 0.f && p_drop < 1.f, "%s: dropout p must be in (0, 1) (got %g)", who, (double)p_drop);
  MP_CHECK_ARG(H >= 1 && H <= 32, "%s: attention dropout needs H <= 32 (got %d)", who, H);
  return MP_OK;
}

static int gat_train(const mp_csr* g, const float* xw, const float* a_src, const float* a_dst, const float* att,
                     int32_t H, int32_t C, float slope, const float* bias, float* out, int64_t ldo, float* agg,
                     float* row_stats, float* out2, float* row_s2, void* slab, size_t slab_bytes, int32_t stages,
                     void* stream, float* as_out, float* ad_out, uint64_t drop_seed = 0, float p_drop = 0.f,
                     const int32_t* drop_ids = nullptr) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_gat_aggregate_train_f32");
  if (rc) return rc;
  // a_src from each gathered row (OWN) when a head fits one lane group (C/4 a
  // power of two <= 64); any other C % 4 == 0 reads the node-score arrays
  const bool own = mp_gat_train_ok(H, C) && att != nullptr;
  MP_CHECK_ARG(H > 0 && C > 0 && C % 4 == 0, "mp_gat_aggregate_train_f32: needs C %% 4 == 0");
  MP_CHECK_ARG(own || (!as_out && a_src && a_dst),
               "mp_gat_aggregate_train_f32: heads with C/4 not a power of two <= 64 need a_src / a_dst inputs");
  MP_CHECK_ARG(xw && out && row_stats && out2 && row_s2, "mp_gat_aggregate_train_f32: null input");
  const int F = H * C;
  MP_CHECK_ARG(ldo >= F, "mp_gat_aggregate_train_f32: ldo < H*C");
  MP_CHECK_ARG((uintptr_t)xw % 16 == 0 && (uintptr_t)att % 16 == 0 && (uintptr_t)out % 16 == 0 && ldo % 4 == 0 &&
                   (uintptr_t)out2 % 16 == 0 && (uintptr_t)agg % 16 == 0 && (uintptr_t)bias % 16 == 0,
               "mp_gat_aggregate_train_f32: xw, att, bias, out, agg, out2 must be 16-byte aligned (ldo %% 4 == 0)");
  MP_CHECK_ARG(slab != nullptr && slab_bytes >= mp_gat_train_slab_bytes(g, H, C),
               "mp_gat_aggregate_train_f32: slab workspace too small");
  AggArgs a{};
  fill_graph(a, g);
  a.F = F;
  a.x = xw;
  a.ldx = F;
  a.out = out;
  a.ldo = ldo;
  a.a_src = a_src;
  a.a_dst = a_dst;
  a.att = att;
  a.H = H;
  a.C = C;
  a.slope = slope;
  a.row_stats = row_stats;
  a.out2 = out2;
  a.row_s2 = row_s2;
  a.bias = bias;
  a.agg_nb = agg;
  a.a_src_out = as_out;  // mp_gat_forward_train_f32: node scores in-kernel
  a.a_dst_out = ad_out;
  a.slab_ld = slab_ld_for(F);
  const size_t slots = 2 * (size_t)g->n_waves;
  char* b = (char*)slab;
  const size_t v = align_up(slots * (size_t)a.slab_ld * 4, 256);
  a.slab_v = (float*)b;
  a.slab_s = (float*)(b + v);
  b += mp_gat_slab_bytes(g, H, C);
  a.slab_v2 = (float*)b;
  a.slab_s2 = (float*)(b + v);
  const int lanes = F >= 256 ? kGatLanes : 64;
  if (!own) {
    a.att = nullptr;
    if (p_drop > 0.f) {
      set_drop(a, drop_seed, p_drop, drop_ids);
      return launch<GatRed<4, false, true, false, true>, 4>(a, stages, as_stream(stream), lanes);
    }
    return launch<GatRed<4, false, true>, 4>(a, stages, as_stream(stream), lanes);
  }
  if (p_drop > 0.f) {
    set_drop(a, drop_seed, p_drop, drop_ids);
    return launch<GatRed<4, true, true, false, true>, 4>(a, stages, as_stream(stream), lanes);
  }
  if (a.a_src_out) return launch<GatRed<4, true, true, true>, 4>(a, stages, as_stream(stream), lanes);
  return launch<GatRed<4, true, true>, 4>(a, stages, as_stream(stream), F >= 256 ? kGatLanes : 64);
}

int mp_gat_aggregate_train_f32(const mp_csr* g, const float* xw, const float* a_src, const float* a_dst,
                               const float* att, int32_t H, int32_t C, float slope, const float* bias, float* out,
                               int64_t ldo, float* agg, float* row_stats, float* out2, float* row_s2, void* slab,
                               size_t slab_bytes, int32_t stages, void* stream) {
  MP_CHECK_ARG(a_src && a_dst, "mp_gat_aggregate_train_f32: null input");
  return gat_train(g, xw, a_src, a_dst, att, H, C, slope, bias, out, ldo, agg, row_stats, out2, row_s2, slab,
                   slab_bytes, stages, stream, nullptr, nullptr);
}

int mp_gat_forward_train_f32(const mp_csr* g, const float* xw, const float* att, int32_t H, int32_t C, float slope,
                             const float* bias, float* out, int64_t ldo, float* agg, float* row_stats, float* out2,
                             float* row_s2, float* a_src, float* a_dst, void* slab, size_t slab_bytes,
                             int32_t stages, void* stream) {
  MP_CHECK_ARG(a_src && a_dst, "mp_gat_forward_train_f32: null a_src / a_dst");
  MP_CHECK_ARG(!g || g->n_cols == g->n_rows, "mp_gat_forward_train_f32: the graph must be square");
  return gat_train(g, xw, a_src, a_dst, att, H, C, slope, bias, out, ldo, agg, row_stats, out2, row_s2, slab,
                   slab_bytes, stages, stream, a_src, a_dst);
}

int mp_gat_two_pass_ok(int32_t H, int32_t C) {
  return H >= 1 && H <= 16 && (C == 16 || C == 32 || (C >= 64 && C % 64 == 0)) ? 1 : 0;
}

// Two-pass GAT: row statistics (two lane-task passes over a_src), then the
// reference-order weighted aggregation (k_agg_flat<.., GA>, 64-feature tiles).
int mp_gat_softmax_aggregate_f32(const mp_csr* g, const int32_t* slot_row, const float* xw, const float* a_src,
                                 const float* a_dst, int32_t H, int32_t C, float slope, const float* bias,
                                 float* out, int64_t ldo, float* row_stats, void* slab, size_t slab_bytes,
                                 int32_t stages, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(g, "mp_gat_softmax_aggregate_f32");
  if (rc) return rc;
  MP_CHECK_ARG(mp_gat_two_pass_ok(H, C),
               "mp_gat_softmax_aggregate_f32: needs H <= 16 and C in {16, 32} or a multiple of 64");
  MP_CHECK_ARG(g->n_edges == 0 || g->col != nullptr, "mp_gat_softmax_aggregate_f32: graph needs a column array");
  MP_CHECK_ARG(xw && a_src && a_dst && out && row_stats && (g->n_edges == 0 || slot_row),
               "mp_gat_softmax_aggregate_f32: null input");
  MP_CHECK_ARG((uintptr_t)row_stats % 8 == 0, "mp_gat_softmax_aggregate_f32: row_stats must be 8-byte aligned");
  const int F = H * C;
  MP_CHECK_ARG(ldo >= F, "mp_gat_softmax_aggregate_f32: ldo < H*C");
  MP_CHECK_ARG(slab != nullptr && slab_bytes >= mp_gat_slab_bytes(g, H, C),
               "mp_gat_softmax_aggregate_f32: slab workspace too small");
  hipStream_t s = as_stream(stream);
  AggArgs a{};
  fill_graph(a, g);
  a.a_src = a_src;
  a.a_dst = a_dst;
  a.H = H;
  a.C = C;
  a.slope = slope;
  a.row_stats = row_stats;
  a.slot_row = slot_row;
  a.slab_v = (float*)slab;
  if (stages & MP_STAGE_STATS) {
    // passes 1 and 2: x = a_src [N, H], F = H
    AggArgs t = a;
    t.F = H;
    t.x = a_src;
    t.ldx = H;
    t.slab_ld = slab_ld_for(H);
    for (int pass = 0; pass < 2; ++pass) {
      // k_agg_main lane groups, one lane per head: H <= 4 -> 4 lanes, <= 8 -> 8, else 16
      if (H <= 4) rc = pass ? launch_l<GatDenRed<1>, 1, 4>(t, MP_STAGE_ALL, s) : launch_l<GatMaxRed<1>, 1, 4>(t, MP_STAGE_ALL, s);
      else if (H <= 8) rc = pass ? launch_l<GatDenRed<1>, 1, 8>(t, MP_STAGE_ALL, s) : launch_l<GatMaxRed<1>, 1, 8>(t, MP_STAGE_ALL, s);
      else rc = pass ? launch_l<GatDenRed<1>, 1, 16>(t, MP_STAGE_ALL, s) : launch_l<GatMaxRed<1>, 1, 16>(t, MP_STAGE_ALL, s);
      if (rc) return rc;
    }
  }
  a.F = F;
  a.w = a_src;  // any non-null pointer: the HAS_W reducer multiplies by the window's alpha
  a.x = xw;
  a.ldx = F;
  a.bias = bias;
  a.out = out;
  a.ldo = ldo;
  a.slab_ld = slab_ld_for(F);
  a.flat = 1;
  using Red = SumRed<1, true, false>;
  const int ftiles = (int)ceil_div(F, 64);
  if ((stages & MP_STAGE_MAIN) && a.n_waves > 0) {
    int64_t nb = ceil_div(a.n_waves, kWavesPerBlock);
    if (kXcdTiles && 8 % ftiles == 0) nb = ceil_div(nb, 8 / ftiles) * (8 / ftiles);
    hipLaunchKernelGGL((k_agg_flat<Red, 1, kU_Vec1, 64, true>), dim3((unsigned)nb, (unsigned)ftiles),
                       dim3(kBlock), 0, s, a);
    MP_CHECK_LAUNCH();
  }
  if ((stages & MP_STAGE_FIXUP) && a.n_split > 0) {
    if (F % 4 == 0 && (uintptr_t)out % 16 == 0 && ldo % 4 == 0 && (uintptr_t)bias % 16 == 0) {
      hipLaunchKernelGGL((k_agg_fixup<SumRed<4, true, false>, 4>), dim3((unsigned)a.n_split, (unsigned)ceil_div(F, 256)),
                         dim3(kBlock), 0, s, a);
    } else {
      hipLaunchKernelGGL((k_agg_fixup<Red, 1>), dim3((unsigned)a.n_split, (unsigned)ceil_div(F, 64)), dim3(kBlock), 0,
                         s, a);
    }
    MP_CHECK_LAUNCH();
  }
  return MP_OK;
}

static int gat_backward(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* xw, const float* a_src,
                        const float* pack, const float* att, int32_t H, int32_t C, float slope, float* grad_xw,
                        float* grad_a_src, float* de, const float* ga_dst_in, void* slab, size_t slab_bytes,
                        int32_t stages, void* stream, uint64_t drop_seed = 0, float p_drop = 0.f,
                        const int32_t* drop_ids = nullptr) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(gt, "mp_gat_backward_f32");
  if (rc) return rc;
  MP_CHECK_ARG(H > 0 && C > 0, "mp_gat_backward_f32: H, C must be positive");
  MP_CHECK_ARG(grad_out && xw && a_src && pack && att && grad_xw && grad_a_src,
               "mp_gat_backward_f32: null pointer");
  MP_CHECK_ARG((uintptr_t)pack % 16 == 0, "mp_gat_backward_f32: pack must be 16-byte aligned");
  const int F = H * C;
  MP_CHECK_ARG(ldg >= F, "mp_gat_backward_f32: ldg < H*C");
  MP_CHECK_ARG(slab && slab_bytes >= mp_gat_slab_bytes(gt, H, C), "mp_gat_backward_f32: slab workspace too small");
  AggArgs a{};
  fill_graph(a, gt);
  a.F = F;
  a.x = grad_out;
  a.ldx = ldg;
  a.out = grad_xw;
  a.ldo = F;
  a.y = xw;
  a.ldy = F;
  a.a_src = a_src;
  a.pack = reinterpret_cast<const f32x4*>(pack);
  a.att = att;
  a.de = de;
  a.ga = grad_a_src;
  a.ga_dst_in = ga_dst_in;
  a.H = H;
  a.C = C;
  a.slope = slope;
  a.slab_ld = slab_ld_for(F);
  size_t v = align_up(2 * (size_t)gt->n_waves * (size_t)a.slab_ld * 4, 256);
  a.slab_v = (float*)slab;
  a.slab_s = (float*)((char*)slab + v);
  hipStream_t s = as_stream(stream);
  auto pow2 = [](int q) { return q >= 1 && q <= 64 && (q & (q - 1)) == 0; };
  const bool v4 = C % 4 == 0 && pow2(C / 4) && (uintptr_t)grad_out % 16 == 0 && ldg % 4 == 0 &&
                  (uintptr_t)xw % 16 == 0 && (uintptr_t)grad_xw % 16 == 0;
  // narrower feature tiles for the transposed pass (MP_TUNE_GAT_BWD_VEC 2 / 1: 128- / 64-feature
  // tiles, XCD-affine like the flat kernel's; a head stays inside one tile)
  const int bv = (int)tuned(g_tune.gat_bwd_vec);
  if (v4 && bv < 4 && F >= 64 * bv * 2 && pow2(C / bv) && (64 * bv) % C == 0) {
    if (bv == 2) {
      if (p_drop > 0.f) {
        set_drop(a, drop_seed, p_drop, drop_ids);
        return launch<GatBwdRed<2, true>, 2>(a, stages, s);
      }
      return launch<GatBwdRed<2>, 2>(a, stages, s);
    }
    if (p_drop > 0.f) {
      set_drop(a, drop_seed, p_drop, drop_ids);
      return launch<GatBwdRed<1, true>, 1>(a, stages, s);
    }
    return launch<GatBwdRed<1>, 1>(a, stages, s);
  }
  if (v4) {
    int lanes = F >= 256 ? kGatLanes : pick_shape(F, ldg, grad_out, F, grad_xw).lanes;
    if (lanes < C / 4) lanes = C / 4;
    if (p_drop > 0.f) {
      set_drop(a, drop_seed, p_drop, drop_ids);
      return launch<GatBwdRed<4, true>, 4>(a, stages, s, lanes);
    }
    return launch<GatBwdRed<4>, 4>(a, stages, s, lanes);
  }
  MP_CHECK_ARG(p_drop <= 0.f, "mp_gat_backward_train_drop_f32: needs C/4 a power of two <= 64, 16-byte aligned rows");
  MP_CHECK_ARG(pow2(C), "mp_gat_backward_f32: C=%d needs C/4 or C to be a power of two <= 64", C);
  return launch<GatBwdRed<1>, 1>(a, stages, s);
}

int mp_gat_backward_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* xw, const float* a_src,
                        const float* pack, const float* att, int32_t H, int32_t C, float slope, float* grad_xw,
                        float* grad_a_src, float* de, size_t de_bytes, void* slab, size_t slab_bytes, int32_t stages,
                        void* stream) {
  // without the training forward's node-wise d a_dst the per-edge d score is the
  // only way d a_dst comes out: it is required (mp_gat_backward_train_f32 otherwise)
  MP_CHECK_ARG(de != nullptr || !gt || gt->n_edges == 0,
               "mp_gat_backward_f32: de is required (use mp_gat_backward_train_f32 after the training forward)");
  if (gt && H > 0) MP_CHECK_EXTENT("mp_gat_backward_f32", "de", de_bytes, (size_t)gt->n_edges * H * 4);
  return gat_backward(gt, grad_out, ldg, xw, a_src, pack, att, H, C, slope, grad_xw, grad_a_src, de, nullptr, slab,
                      slab_bytes, stages, stream);
}

int mp_gat_backward_train_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* xw,
                              const float* a_src, const float* pack, const float* att, int32_t H, int32_t C,
                              float slope, const float* grad_a_dst, float* grad_xw, float* grad_a_src, void* slab,
                              size_t slab_bytes, int32_t stages, void* stream) {
  MP_CHECK_ARG(grad_a_dst != nullptr, "mp_gat_backward_train_f32: null grad_a_dst");
  return gat_backward(gt, grad_out, ldg, xw, a_src, pack, att, H, C, slope, grad_xw, grad_a_src, nullptr,
                      grad_a_dst, slab, slab_bytes, stages, stream);
}

int mp_gat_aggregate_train_drop_f32(const mp_csr* g, const float* xw, const float* a_src, const float* a_dst,
                                    const float* att, int32_t H, int32_t C, float slope, const float* bias,
                                    float* out, int64_t ldo, float* agg, float* row_stats, float* out2,
                                    float* row_s2, uint64_t seed, float p_drop, const int32_t* drop_ids, void* slab,
                                    size_t slab_bytes, int32_t stages, void* stream) {
  int rc = drop_check(p_drop, H, "mp_gat_aggregate_train_drop_f32");
  if (rc) return rc;
  MP_CHECK_ARG(a_src && a_dst, "mp_gat_aggregate_train_drop_f32: null input");
  return gat_train(g, xw, a_src, a_dst, att, H, C, slope, bias, out, ldo, agg, row_stats, out2, row_s2, slab,
                   slab_bytes, stages, stream, nullptr, nullptr, seed, p_drop, drop_ids);
}

int mp_gat_backward_train_drop_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* xw,
                                   const float* a_src, const float* pack, const float* att, int32_t H, int32_t C,
                                   float slope, const float* grad_a_dst, uint64_t seed, float p_drop,
                                   const int32_t* drop_ids, float* grad_xw, float* grad_a_src, void* slab,
                                   size_t slab_bytes, int32_t stages, void* stream) {
  int rc = drop_check(p_drop, H, "mp_gat_backward_train_drop_f32");
  if (rc) return rc;
  MP_CHECK_ARG(grad_a_dst != nullptr, "mp_gat_backward_train_drop_f32: null grad_a_dst");
  return gat_backward(gt, grad_out, ldg, xw, a_src, pack, att, H, C, slope, grad_xw, grad_a_src, nullptr,
                      grad_a_dst, slab, slab_bytes, stages, stream, seed, p_drop, drop_ids);
}

int mp_gat_backward_wide_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* a_src,
                             const float* pack, int32_t H, int32_t C, float slope, uint64_t seed, float p_drop,
                             const int32_t* drop_ids, float* grad_xw, float* acc2, size_t acc2_bytes, float* sc, size_t sc_bytes, void* slab,
                             size_t slab_bytes, int32_t stages, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = check_graph(gt, "mp_gat_backward_wide_f32");
  if (rc) return rc;
  MP_CHECK_ARG(H > 0 && C > 0 && C % 4 == 0, "mp_gat_backward_wide_f32: needs C %% 4 == 0");
  if (p_drop > 0.f) {
    rc = drop_check(p_drop, H, "mp_gat_backward_wide_f32");
    if (rc) return rc;
  }
  MP_CHECK_ARG(grad_out && a_src && pack && grad_xw && acc2 && sc, "mp_gat_backward_wide_f32: null pointer");
  const int F = H * C;
  MP_CHECK_ARG(ldg >= F && ldg % 4 == 0, "mp_gat_backward_wide_f32: ldg < H*C or not a multiple of 4");
  MP_CHECK_ARG((uintptr_t)grad_out % 16 == 0 && (uintptr_t)grad_xw % 16 == 0 && (uintptr_t)acc2 % 16 == 0 &&
                   (uintptr_t)pack % 16 == 0,
               "mp_gat_backward_wide_f32: grad_out, grad_xw, acc2, pack must be 16-byte aligned");
  MP_CHECK_ARG(slab && slab_bytes >= mp_gat_train_slab_bytes(gt, H, C),
               "mp_gat_backward_wide_f32: slab workspace too small (mp_gat_train_slab_bytes)");
  MP_CHECK_EXTENT("mp_gat_backward_wide_f32", "acc2", acc2_bytes, (size_t)gt->n_rows * F * 4);
  MP_CHECK_EXTENT("mp_gat_backward_wide_f32", "sc", sc_bytes, (size_t)gt->n_rows * H * 4);
  AggArgs a{};
  fill_graph(a, gt);
  a.F = F;
  a.x = grad_out;
  a.ldx = ldg;
  a.out = grad_xw;
  a.ldo = F;
  a.out2 = acc2;
  a.ga = sc;
  a.a_src = a_src;
  a.pack = reinterpret_cast<const f32x4*>(pack);
  a.H = H;
  a.C = C;
  a.slope = slope;
  a.slab_ld = slab_ld_for(F);
  const size_t slots = 2 * (size_t)gt->n_waves;
  char* b = (char*)slab;
  const size_t v = align_up(slots * (size_t)a.slab_ld * 4, 256);
  a.slab_v = (float*)b;
  a.slab_s = (float*)(b + v);
  b += mp_gat_slab_bytes(gt, H, C);
  a.slab_v2 = (float*)b;
  hipStream_t s = as_stream(stream);
  const int lanes = F >= 256 ? 64 : (F / 4 <= 4 ? 4 : next_pow2(F / 4));
  if (p_drop > 0.f) {
    set_drop(a, seed, p_drop, drop_ids);
    return launch<GatBwdWideRed<4, true>, 4>(a, stages, s, lanes);
  }
  return launch<GatBwdWideRed<4>, 4>(a, stages, s, lanes);
}

int mp_gat_dropout_keep(uint64_t seed, float p_drop, int32_t H, int64_t n_slots, const int32_t* drop_ids,
                        uint32_t* bits, void* stream) {
  MP_DEVICE_GUARD(stream);
  int rc = drop_check(p_drop, H, "mp_gat_dropout_keep");
  if (rc) return rc;
  MP_CHECK_ARG(n_slots >= 0, "mp_gat_dropout_keep: negative n_slots");
  if (n_slots == 0) return MP_OK;
  MP_CHECK_ARG(bits != nullptr, "mp_gat_dropout_keep: null bits");
  AggArgs a{};
  a.H = H;
  set_drop(a, seed, p_drop, drop_ids);
  hipLaunchKernelGGL(k_gat_dropout_keep, dim3((unsigned)ceil_div(n_slots, 256)), dim3(256), 0, as_stream(stream), a,
                     n_slots, bits);
  MP_CHECK_LAUNCH();
  return MP_OK;
}

}  // extern "C"
