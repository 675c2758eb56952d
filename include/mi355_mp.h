/*
 * mi355_mp.h — C-ABI of the MI355X (gfx950) message-passing aggregation engine.
 *
 * This is the drop-in boundary for the hot path of PyG 1.4.3
 * `MessagePassing.propagate()` (gather x_j / x_i -> message -> scatter-reduce)
 * and of the torch_scatter 2.0.4 ops it calls.  Upstream those live in
 * unvendored dependencies pinned at /root/reference/requirement.txt:1-7
 * (torch_sparse 0.6.1, torch-scatter 2.0.4, torch-geometric 1.4.3); the
 * reference tree itself only calls them (examples/gcn.py:18-27,
 * ConvexPruning.py:180-224, examples/ppi.py:22-28, README.md:35-49,
 * gmm_conv.py:131-144).  See SURVEY.md section 8b for the schema list.
 *
 * Conventions
 *   - Plain pointers to DEVICE memory, int64 sizes, a hipStream_t passed as
 *     `void* stream` (NULL = default stream).  No torch types.
 *   - Every entry point only enqueues work on `stream`; none allocates, frees
 *     or synchronises, so every call is hipGraph-capturable.  Work runs on
 *     the stream's device: the calling thread's current device is switched
 *     for the call when it differs, and restored.  The caller owns
 *     all outputs and workspaces (sizes from the *_bytes queries).
 *   - Return value: MP_OK or an MP_ERR_* code; mp_last_error() gives the text
 *     (thread-local).
 *   - Extents (ABI 6): every caller-allocated workspace, partial or per-edge
 *     array whose size is not fixed by the call's own row / edge counts alone
 *     is passed with its size in bytes (`*_bytes`).  A buffer shorter than the
 *     call needs is rejected with MP_ERR_ARG before anything is launched, so a
 *     mis-sized array is an error, never an out-of-bounds device write.
 *   - Graph structure is a destination-sorted CSR (stable: inside a row the
 *     edges keep their original order), described by `mp_csr`.  All kernels
 *     are deterministic: no float atomics on any forward output.
 */
#ifndef MI355_MP_H
#define MI355_MP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MP_ABI_VERSION 7

/* status codes */
#define MP_OK 0
#define MP_ERR_ARG 1   /* bad argument (shape, alignment, null pointer) */
#define MP_ERR_HIP 2   /* a HIP runtime call failed */

/* reductions (torch_scatter names: sum/add, mean, max, min) */
#define MP_REDUCE_SUM 0
#define MP_REDUCE_MEAN 1
#define MP_REDUCE_MAX 2
#define MP_REDUCE_MIN 3

/* aggregate flags */
#define MP_FLAG_INIT_FROM_OUT 1 /* torch_scatter `out=` given: reduce into out's values */
#define MP_FLAG_PYG_MASK 2      /* torch_geometric.utils.scatter_: max -> out<-10000 := 0,
                                   min -> out>10000 := 0 */
#define MP_FLAG_SKIP_EMPTY 4    /* (ABI 7, mp_aggregate_tiles_f32 only) rows with no slot are left
                                   untouched: no store, no bias */

/* aggregate stages (bench times the main kernel on its own) */
#define MP_STAGE_MAIN 1
#define MP_STAGE_FIXUP 2
#define MP_STAGE_STATS 4  /* mp_gat_softmax_aggregate_f32: the softmax row-statistics passes */
#define MP_STAGE_ALL 7

/*
 * Destination-sorted CSR plus its edge-balanced ("merge-path") schedule.
 *   rowptr[n_rows+1]      row r owns CSR slots [rowptr[r], rowptr[r+1])
 *   col[n_edges]          gather row for each slot (source node, or message row);
 *                         NULL = identity (row k of x for slot k: values already
 *                         in CSR slot order)
 *   eid[n_edges]          original edge position of each slot (argmax output)
 * Schedule (merge-path over the N+E work items "row r" and "slot k"; row r
 * sits at merged position rowptr[r]+r, slot k of row r at k+r+1):
 *   wave task w covers merged positions [w*chunk, (w+1)*chunk)
 *   wave_row[n_waves+1]   first row whose marker lies in task w (owned rows)
 *   wave_slot[n_waves+1]  first CSR slot processed by task w
 *   split_waves[n_split]  for each row whose slots span several tasks, the
 *                         last task touching it (fix-up list)
 *   n_cols                number of rows of the gathered tensor (x, or the
 *                         messages when col == eid); required (> 0) with col
 */
typedef struct mp_csr {
  const int32_t* rowptr;
  const int32_t* col;
  const int32_t* eid;
  const int32_t* wave_row;
  const int32_t* wave_slot;
  const int32_t* split_waves;
  int64_t n_rows;
  int64_t n_edges;
  int32_t chunk;
  int32_t n_waves;
  int32_t n_split;
  int32_t n_cols;   /* rows of the gathered x; must be > 0 whenever col != NULL (MP_ERR_ARG
                       otherwise).  It bounds the 32-bit buffer offsets of the gather. */
  int64_t n_ids;    /* size of the edge-id space the eid array indexes: the arg an empty
                       max/min row reports (torch_scatter's src.size(0)).  0 = n_edges.  A CSR
                       whose slots are a subset of the edges (first occurrences of repeated
                       (row, column) pairs) sets it to the full edge count.  (ABI 2) */
} mp_csr;

const char* mp_last_error(void);
int mp_abi_version(void);
/* First 16 hex digits of the sha256 of the native sources this library was
 * compiled from (csrc/Makefile computes it; mi355_mp._lib.source_hash() is the
 * same scheme over the tree).  The Python loader refuses a library whose hash
 * differs from the sources beside it: a stale prebuilt .so never runs.  (ABI 3) */
const char* mp_source_hash(void);

/* Process-wide dispatch table (tests and in-process A/B runs).  Sets `key`
 * to `value` and returns the previous value; value < 0 only queries.
 * Unknown keys return -1.  Every setting gives bitwise-identical results;
 * only the kernel shape changes.  "Flat kernel" = k_agg_flat, the
 * sum/mean/max/min kernel whose tasks stream their slots across row ends.
 *   MP_TUNE_FLAT_VEC1_MIN_BYTES: flat sum/mean over a gathered x of at least
 *     this many bytes use 64-feature tiles (VEC=1); smaller x uses
 *     MP_TUNE_FLAT_VEC.  Default 0 (always 64-feature tiles).
 *   MP_TUNE_FLAT_SMEM: 1 (default) = the flat sum/mean kernel reads slot
 *     columns / weights through scalar-cache batches and gathers with 32-bit
 *     buffer offsets whenever the gathered x spans < 4 GiB; 0 = the per-lane
 *     slot window.
 *   MP_TUNE_FLAT_MIN_F: narrowest sum/mean row (features) that takes the
 *     flat kernel (default 64); narrower rows use lane groups / lane tasks.
 *   MP_TUNE_FLAT_MIN_F_ARG: the same for max/min (default 64).
 *   MP_TUNE_FLAT_NARROW_VEC1: flat rows of at most this many features use
 *     64-feature tiles (VEC=1) whatever the other keys say (default 64: a
 *     64-feature row fills one VEC=1 tile, where VEC=2 would idle half the lanes).
 *   MP_TUNE_FLAT_VEC / MP_TUNE_FLAT_VEC_ARG: features per lane of the flat
 *     kernel for sum/mean (below the VEC1 size threshold) and for max/min:
 *     1, 2 (default) or 4 -- feature tiles of 64, 128 or 256.
 *   MP_TUNE_FLAT_SEQ_TILES: 1 = the flat kernel's feature tiles run one after
 *     another on all eight XCDs; 0 (default) = XCD-affine tiles.
 *   MP_TUNE_FLAT_FAR_MIN_BYTES: the scalar-batch sum/mean kernel keeps 8
 *     instead of 16 row loads in flight per wave over a gathered x larger than
 *     this (default 256 MiB, the Infinity Cache).
 *   MP_TUNE_GAT_BWD_VEC: features per lane of the GAT backward's transposed
 *     pass (mp_gat_backward_*_f32 with C/4 a power of two): 4 (default,
 *     256-feature tiles), 2 or 1 (128- / 64-feature XCD-affine tiles, taken
 *     when a head fits inside one tile).  The exception to the rule above:
 *     the per-slot <g_i, xw_j> sums its features in another order, so the
 *     gradients agree to rounding, not bit for bit. */
#define MP_TUNE_FLAT_VEC1_MIN_BYTES 1
#define MP_TUNE_FLAT_SMEM 2
#define MP_TUNE_FLAT_MIN_F 3
#define MP_TUNE_FLAT_MIN_F_ARG 4
#define MP_TUNE_FLAT_NARROW_VEC1 5
#define MP_TUNE_FLAT_VEC 6
#define MP_TUNE_FLAT_VEC_ARG 7
#define MP_TUNE_FLAT_SEQ_TILES 8
#define MP_TUNE_FLAT_FAR_MIN_BYTES 9
#define MP_TUNE_GAT_BWD_VEC 10
int64_t mp_tune(int32_t key, int64_t value);

/* ---- CSR build (replaces the sort/bucketing torch_scatter never did: upstream
 *      scatter_add_ walks edges in original order) ---------------- */

/* Workspace bytes for mp_csr_build. */
size_t mp_csr_build_workspace(int64_t n_edges, int64_t n_rows);

/* Stable sort of edges by key (edge_index[i], the aggregation index).
 *   key[n_edges], other[n_edges]: int64 (rows of edge_index; any stride-1 view)
 *   other may be NULL: then col[k] = eid[k] (aggregating materialised messages).
 *   rowptr[n_rows+1], col[n_edges], eid[n_edges]: int32 outputs.
 *   bad[1]: device int32, set to the number of key/other entries outside
 *   [0,n_rows) / [0,n_other).  Replaces the index->CSR step of
 *   torch_scatter segment_csr callers; PyG 1.4.3 scatter_ itself sorts nothing. */
int mp_csr_build(const int64_t* key, const int64_t* other, int64_t n_edges,
                 int64_t n_rows, int64_t n_other, int32_t* rowptr, int32_t* col,
                 int32_t* eid, int32_t* bad, void* ws, size_t ws_bytes,
                 void* stream);

/* Number of wave tasks for `chunk` merged positions per task (chunk a multiple of 8, >= 16). */
int32_t mp_schedule_n_waves(int64_t n_rows, int64_t n_edges, int32_t chunk);
size_t mp_schedule_workspace(int32_t n_waves);

/* Builds wave_row[n_waves+1], wave_slot[n_waves+1] and split_waves[<=n_waves];
 * writes the split count to n_split_dev[0] (device int32).  A task boundary
 * that falls inside a row of <= snap slots is moved back to that row's start
 * (0 <= snap < chunk-1), so only longer rows are ever split. */
int mp_schedule_build(const int32_t* rowptr, int64_t n_rows, int64_t n_edges,
                      int32_t chunk, int32_t snap, int32_t* wave_row, int32_t* wave_slot,
                      int32_t* split_waves, int32_t* n_split_dev, void* ws,
                      size_t ws_bytes, void* stream);

/* ---- fused gather -> (weight) -> segment reduce ---------------------------
 * out[r, :] = REDUCE_{k in row r} ( w[k] * x[col[k], :] )     (w optional)
 * Replaces: index_select(x, edge_index[j]) (PyG MessagePassing.__collect__),
 * message() = norm.view(-1,1)*x_j (GCNConv) or x_j, and
 * torch_scatter scatter_sum/scatter_mean/scatter_max/scatter_min [U8/U9],
 * torch_geometric.utils.scatter_ [U2] (MP_FLAG_PYG_MASK), update() += bias.
 *   w:      CSR-ordered per-slot weights or NULL
 *   x:      [*, ldx] fp32 rows, F features used
 *   bias:   [F] or NULL (added after the reduction, as GCNConv.update)
 *   out:    [n_rows, ldo] fp32
 *   arg_out:[n_rows, F] int64 (max/min only, else NULL): original edge
 *           position of the first maximal element, n_edges for empty rows
 *   slab:   workspace of mp_aggregate_slab_bytes() bytes
 */
size_t mp_aggregate_slab_bytes(const mp_csr* g, int32_t F, int32_t reduce);
int mp_aggregate_f32(const mp_csr* g, const float* w, const float* x,
                     int64_t ldx, int32_t F, int32_t reduce, int32_t flags,
                     const float* bias, float* out, int64_t ldo,
                     int64_t* arg_out, void* slab, size_t slab_bytes,
                     int32_t stages, void* stream);

/* mp_aggregate_f32 for sum / mean over TILE-MAJOR operands (ABI 7): the
 * sharded step's feature tiles (mi355_mp.dist.OverlappedAggregation) in ONE
 * launch per pass instead of one launch per tile.  With x_tile_w > 0, feature f
 * of row r of x lives at x[(f / x_tile_w) * x_tile_stride + r * x_tile_w +
 * f % x_tile_w] (ldx ignored), else at x[r * ldx + f]; likewise out with
 * out_tile_w / out_tile_stride (ldo ignored), else out[r * ldo + f].  Tile
 * widths are multiples of 64 dividing F (F a multiple of 64) and tiles do not
 * overlap (stride >= rows x width: g->n_cols rows of x, g->n_rows rows of
 * out); bias is [F] as ever, and bias_rows (NULL, or int32 [g->n_rows])
 * limits it to the rows r with bias_rows[r] != 0.  flags: MP_FLAG_INIT_FROM_OUT
 * and / or MP_FLAG_SKIP_EMPTY (rows without slots keep out as it is).  The graph
 * needs its column array.  Per row and feature the arithmetic is exactly
 * mp_aggregate_f32's on the same values laid out row-major: the results are
 * bitwise equal.  Replaces, for one rank's step, the per-tile
 * scatter_add(norm * x_j) of the reference's propagate (gcn_conv.py [U5]). */
int mp_aggregate_tiles_f32(const mp_csr* g, const float* w, const float* x,
                           int64_t ldx, int32_t x_tile_w, int64_t x_tile_stride,
                           int32_t F, int32_t reduce, int32_t flags,
                           const float* bias, const int32_t* bias_rows,
                           float* out, int64_t ldo,
                           int32_t out_tile_w, int64_t out_tile_stride,
                           void* slab, size_t slab_bytes, int32_t stages,
                           void* stream);

/* Name (demangled) of the main kernel mp_aggregate_f32 would launch for these
 * arguments (same shape selection, nothing launched), written to buf.  Lets a
 * profile summary be matched to the dispatched kernel (bench.py).  Needs a
 * HIP device for the name lookup; MP_ERR_ARG when none is available. */
int mp_aggregate_kernel_name(const mp_csr* g, const float* w, const float* x,
                             int64_t ldx, int32_t F, int32_t reduce,
                             const float* bias, const float* out, int64_t ldo,
                             char* buf, size_t buf_len, void* stream);

/* ---- GATConv fused attention aggregation (call stack 3.2) ---
 * a_dst[n,h] = <xw[n,h,:], att[h,0:C]>,  a_src[n,h] = <xw[n,h,:], att[h,C:2C]>
 * (the split of (cat[x_i,x_j]*att).sum(-1) of GATConv.message [U6]). */
int mp_gat_node_scores_f32(const float* xw, int64_t n_nodes, int32_t H,
                           int32_t C, const float* att, float* a_src,
                           float* a_dst, void* stream);

/* out[i,h,:] = sum_k softmax_k(leaky_relu(a_src[col_k,h]+a_dst[i,h])) x[col_k,h,:]
 * with torch_geometric.utils.softmax's +1e-16 denominator, single pass
 * (online max/sum), optional bias [H*C], optional row_stats[n_rows,H,2] =
 * (max, denominator) for mp_gat_alpha_f32. */
size_t mp_gat_slab_bytes(const mp_csr* g, int32_t H, int32_t C);
int mp_gat_aggregate_f32(const mp_csr* g, const float* xw, const float* a_src,
                         const float* a_dst, int32_t H, int32_t C, float slope,
                         const float* bias, float* out, int64_t ldo,
                         float* row_stats, void* slab, size_t slab_bytes,
                         int32_t stages, void* stream);
/* The same with att [H, 2C] (GATConv.att): where C % 4 == 0 and C/4 is a
 * power of two <= 64, the kernel recomputes a_src[j,h] from each gathered xw
 * row (bitwise the value mp_gat_node_scores_f32 stores) instead of gathering
 * it; other shapes, or att == NULL, read a_src. */
int mp_gat_aggregate_att_f32(const mp_csr* g, const float* xw, const float* a_src,
                             const float* a_dst, const float* att, int32_t H,
                             int32_t C, float slope, const float* bias, float* out,
                             int64_t ldo, float* row_stats, void* slab,
                             size_t slab_bytes, int32_t stages, void* stream);

/* The same forward with the node scores computed in-kernel (C % 4 == 0 and
 * C/4 a power of two <= 64: mp_gat_train_ok; xw, att, bias, out 16-byte
 * aligned; the graph square -- row i's own xw is row i of xw): a_src / a_dst
 * [n_rows, H] are OUTPUTS, each destination row's scores reduced from its own
 * xw row with mp_gat_node_scores_f32's arithmetic (bitwise its values), so no
 * separate node-score pass over xw runs.  a_src is also recomputed from every
 * gathered row (as mp_gat_aggregate_att_f32).  (ABI 3) */
int mp_gat_forward_f32(const mp_csr* g, const float* xw, const float* att, int32_t H,
                       int32_t C, float slope, const float* bias, float* out, int64_t ldo,
                       float* a_src, float* a_dst, float* row_stats, void* slab,
                       size_t slab_bytes, int32_t stages, void* stream);

/* Training forward of the same layer (C % 4 == 0; with att given and C/4 a power
 * of two <= 64 -- mp_gat_train_ok -- a_src comes from each gathered row, else
 * from the a_src array).  out = aggregate + bias (bias may be NULL); agg
 * (optional, NULL allowed) also receives the pre-bias aggregate [n_rows, H*C]
 * (contiguous).  The backward's rs needs no such copy: the prologues take the
 * output and the bias (ABI 6: rs over out - bias).  Besides these and row_stats it
 * leaves, with the same online rescaling,
 *   out2[i,h,:]  = sum_j alpha_ij leaky'_ij xw[j,h,:]    ([n_rows, H*C], contiguous)
 *   row_s2[i,h]  = sum_j alpha_ij leaky'_ij             ([n_rows, H])
 * with leaky' = 1 where a_src[j,h] + a_dst[i,h] > 0, else slope.  They turn the
 * backward's d a_dst into a node-wise quantity (mp_gat_backward_prep_train_f32),
 * so mp_gat_backward_f32 then runs with de = NULL.
 * Slab: mp_gat_train_slab_bytes(g, H, C). */
int mp_gat_train_ok(int32_t H, int32_t C);
size_t mp_gat_train_slab_bytes(const mp_csr* g, int32_t H, int32_t C);
int mp_gat_aggregate_train_f32(const mp_csr* g, const float* xw, const float* a_src,
                               const float* a_dst, const float* att, int32_t H, int32_t C,
                               float slope, const float* bias, float* out, int64_t ldo,
                               float* agg, float* row_stats, float* out2, float* row_s2,
                               void* slab, size_t slab_bytes, int32_t stages, void* stream);
/* mp_gat_aggregate_train_f32 with the node scores computed in-kernel (the
 * outputs a_src / a_dst, as mp_gat_forward_f32). */
int mp_gat_forward_train_f32(const mp_csr* g, const float* xw, const float* att, int32_t H,
                             int32_t C, float slope, const float* bias, float* out, int64_t ldo,
                             float* agg, float* row_stats, float* out2, float* row_s2,
                             float* a_src, float* a_dst, void* slab, size_t slab_bytes,
                             int32_t stages, void* stream);

/* Two-pass form of the same layer, in the reference's own arithmetic
 * (utils.softmax [U3] then message x_j * alpha and scatter_add in edge order,
 * GATConv.update + bias [U6]):
 *   MP_STAGE_STATS: row_stats[r,h,0] = m = max_k leaky(a_src[col_k,h] + a_dst[r,h]),
 *                   row_stats[r,h,1] = sum_k exp(leaky(.) - m) + 1e-16 (CSR order)
 *   MP_STAGE_MAIN/FIXUP: out[r,h,:] = sum_k (exp(leaky(.) - m) / den) * xw[col_k,h,:] + bias
 * slot_row from mp_csr_slot_rows.  Shapes: mp_gat_two_pass_ok(H, C) != 0
 * (H <= 16; C = 16, 32 or a multiple of 64).  Rows not split across tasks
 * follow the reference's operation order exactly. */
int mp_gat_two_pass_ok(int32_t H, int32_t C);
int mp_gat_softmax_aggregate_f32(const mp_csr* g, const int32_t* slot_row, const float* xw,
                                 const float* a_src, const float* a_dst, int32_t H, int32_t C,
                                 float slope, const float* bias, float* out, int64_t ldo,
                                 float* row_stats, void* slab, size_t slab_bytes,
                                 int32_t stages, void* stream);

/* ---- GATConv backward pieces ------------------------------ */

/* slot_row[k] = the row owning CSR slot k (one-time per graph). */
int mp_csr_slot_rows(const mp_csr* g, int32_t* slot_row, void* stream);

/* alpha_csr[k,h] = exp(leaky(a_src[col_k,h]+a_dst[r,h]) - m[r,h]) / den[r,h]
 * and (if score != NULL) score[k,h] = a_src[col_k,h] + a_dst[r,h] (the
 * pre-activation), both in CSR slot order, r = slot_row[k]. */
int mp_gat_alpha_csr_f32(const mp_csr* g, const int32_t* slot_row, const float* a_src,
                         const float* a_dst, int32_t H, float slope, const float* row_stats,
                         float* alpha_csr, float* score, void* stream);

/* Per-head weighted aggregation: with C = F / H,
 * out[r, h*C + c] = sum_k w[k*H + h] * x[col[k], h*C + c]   (w in CSR slot order)
 * (GATConv's d out / d x_j = alpha, applied over the transposed CSR). */
int mp_aggregate_heads_f32(const mp_csr* g, const float* w, int32_t H, const float* x,
                           int64_t ldx, int32_t F, float* out, int64_t ldo, void* slab,
                           size_t slab_bytes, int32_t stages, void* stream);

/* Sampled dense-dense product over CSR slots (GAT d alpha):
 * out[k*H + h] = sum_c grow[r, h*C + c] * x[col[k], h*C + c], r = slot_row[k]. */
int mp_gat_sddmm_f32(const mp_csr* g, const int32_t* slot_row, const float* grow, int64_t ldg,
                     const float* x, int64_t ldx, int32_t H, int32_t C, float* out,
                     void* stream);

/* Fused GATConv backward over the TRANSPOSED CSR `gt` (rows = source nodes j,
 * col = destination i, slots in original edge order).  Replaces the autograd
 * of GATConv.message + utils.softmax + scatter_add (PyG 1.4.3 [U3,U6];
 * /root/reference/ConvexPruning.py:209-214) with one gather of grad_out rows:
 *   grad_xw[j]      = sum_i alpha_ij g_i + grad_a_src[j,h] * att[h, C:]
 *   de[k, h]        = alpha_ij (<g_i, xw_j>_h - rs[i,h]) leaky'(a_src[j,h]+a_dst[i,h])
 *   grad_a_src[j,h] = sum over the row of de
 * alpha_ij = exp(leaky(score) - m_i) / den_i from the forward's row_stats.
 * pack [n_dst, H, 4] = mp_gat_backward_prep_f32 output.  de [gt.n_edges, H]
 * (de_bytes >= gt.n_edges * H * 4; ABI 6): de[gt.eid[k], h]
 * receives slot k's value: pass the destination-CSR slot of each edge in
 * gt.eid to get de in destination-CSR order (then d a_dst is a contiguous
 * segmented sum: mp_aggregate_f32 with col = NULL).  de = NULL skips it (the
 * training forward's out2 / row_s2 give d a_dst directly).  Needs C/4 or C to
 * be a power of two <= 64.
 * Slab: mp_gat_slab_bytes(gt, H, C). */
int mp_gat_backward_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* xw,
                        const float* a_src, const float* pack, const float* att, int32_t H,
                        int32_t C, float slope, float* grad_xw, float* grad_a_src, float* de,
                        size_t de_bytes, void* slab, size_t slab_bytes, int32_t stages,
                        void* stream);

/* The same pass after the training forward: no per-edge d score; grad_a_dst
 * [n_rows, H] (mp_gat_backward_prep_train_f32) is an input, and each row's
 * grad_xw also receives grad_a_dst[j,h] * att[h, 0:C] (the term
 * mp_gat_backward_finish_f32 adds otherwise; call that with grad_xw = NULL for
 * the att-gradient partials only). */
int mp_gat_backward_train_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* xw,
                              const float* a_src, const float* pack, const float* att, int32_t H,
                              int32_t C, float slope, const float* grad_a_dst, float* grad_xw,
                              float* grad_a_src, void* slab, size_t slab_bytes, int32_t stages,
                              void* stream);

/* pack[n,h,:] = (a_dst[n,h], m[n,h], 1/den[n,h], rs[n,h]) with
 * rs[n,h] = sum_c grad_out[n, h*C+c] * agg[n, h*C+c]  (agg = pre-bias GAT output;
 * rs = sum_j alpha_nj <g_n, xw_j>_h, the softmax-backward row term).
 * bias (ABI 6; NULL = none): agg is then the layer OUTPUT agg + bias [H*C] and
 * rs is taken over out - bias (one rounding per feature), so the forward need
 * not keep a pre-bias copy; 16-byte aligned.
 * gsum_part (optional, [mp_gat_bwd_blocks(n), H*C], needs C%4==0, H*C<=256):
 * per-block column sums of grad_out (the bias gradient is their sum over blocks).
 * Extents (ABI 6): pack_bytes >= n*H*16, gsum_part_bytes >= mp_gat_bwd_blocks(n)*H*C*4
 * (ignored when gsum_part is NULL). */
int mp_gat_backward_prep_f32(const float* grad_out, int64_t ldg, const float* agg, int64_t lda,
                             const float* bias, const float* a_dst, const float* row_stats, int64_t n, int32_t H,
                             int32_t C, float* pack, size_t pack_bytes, float* gsum_part,
                             size_t gsum_part_bytes, void* stream);

/* The same prologue after mp_gat_aggregate_train_f32 (C % 4 == 0, C/4 a power
 * of two <= 64, 16-byte aligned rows), which also writes
 *   grad_a_dst[n,h] = sum_j de_nj = <grad_out[n,h,:], agg2[n,h,:]> - rs[n,h] * row_s2[n,h]
 * (agg2 / row_s2 = the training forward's out2 / row_s2). */
int mp_gat_backward_prep_train_f32(const float* grad_out, int64_t ldg, const float* agg, int64_t lda,
                                   const float* bias, const float* agg2, const float* row_s2, const float* a_dst,
                                   const float* row_stats, int64_t n, int32_t H, int32_t C,
                                   float* pack, size_t pack_bytes, float* gsum_part,
                                   size_t gsum_part_bytes, float* grad_a_dst, void* stream);

/* ---- GATConv with heads of any width (C % 4 == 0) --------------------------
 * The reference's own GAT stacks (ConvexPruning.py:209-214) use heads = 1 and
 * out_channels drawn at random (:106-114), so a head is often wider than one
 * 256-feature tile or C/4 is not a power of two.  For those shapes:
 *   forward: mp_gat_node_scores_wide_f32 (one wave per node, per-head dot
 *     products in 256-feature chunks), then mp_gat_aggregate_f32 (inference)
 *     or mp_gat_aggregate_train_f32 / _drop_f32 (training; these now take any
 *     C % 4 == 0: a_src is read from the node-score array when C/4 is not a
 *     power of two <= 64 or att is NULL);
 *   backward: mp_gat_backward_prep_wide_f32 (pack + node-wise d a_dst, as
 *     mp_gat_backward_prep_train_f32), mp_gat_backward_wide_f32 over the
 *     transposed CSR (no per-slot dot product:
 *       grad_xw[j] = sum_i alpha d g_i,  acc2[j] = sum_i lk alpha d g_i,
 *       sc[j,h] = sum_i lk alpha rs_i,   lk = leaky'(score), d = dropout factor
 *     (p_drop = 0: none; else the eid channel must hold each edge's dst-CSR
 *     slot), slab mp_gat_train_slab_bytes(gt, H, C)), then
 *     mp_gat_backward_epilogue_wide_f32: grad_a_src = <acc2, xw>_h - sc (written
 *     over sc) and grad_xw += grad_a_src att[h, C:] + grad_a_dst att[h, :C].
 * Rows contiguous [n, H*C] unless an ld is given; 16-byte aligned.
 * Extents (ABI 6): pack_bytes >= n*H*16; acc2_bytes >= gt->n_rows*H*C*4,
 * sc_bytes >= gt->n_rows*H*4. */
int mp_gat_wide_ok(int32_t H, int32_t C);
int mp_gat_node_scores_wide_f32(const float* xw, int64_t n_nodes, int32_t H, int32_t C, const float* att,
                                float* a_src, float* a_dst, void* stream);
int mp_gat_backward_prep_wide_f32(const float* grad_out, int64_t ldg, const float* agg, int64_t lda,
                                  const float* bias, const float* agg2, const float* row_s2, const float* a_dst,
                                  const float* row_stats, int64_t n, int32_t H, int32_t C, float* pack,
                                  size_t pack_bytes, float* grad_a_dst, void* stream);
int mp_gat_backward_wide_f32(const mp_csr* gt, const float* grad_out, int64_t ldg, const float* a_src,
                             const float* pack, int32_t H, int32_t C, float slope, uint64_t seed, float p_drop,
                             const int32_t* drop_ids, float* grad_xw, float* acc2, size_t acc2_bytes, float* sc, size_t sc_bytes,
                             void* slab, size_t slab_bytes, int32_t stages, void* stream);
int mp_gat_backward_epilogue_wide_f32(float* grad_xw, const float* acc2, const float* xw, const float* att,
                                      const float* grad_a_dst, float* sc_grad_a_src, int64_t n, int32_t H,
                                      int32_t C, void* stream);

/* ---- Batch.from_data_list on the replica's device ------------------------
 * torch_geometric.data.Batch.from_data_list (PyG 1.4.3 [U8]; the replica path
 * of DataParallel, /root/reference/ConvexPruning.py:530) collates a graph list
 * on the host: per graph `item + cumsum[key]` for index keys and
 * `torch.full((n_g,), g)` for the batch vector.  With the raw items
 * concatenated and copied to the device once, these apply the same per-graph
 * terms on the device.  Segments: starts[0..G] (int64, starts[0] = 0,
 * starts[G] = n, non-decreasing; empty graphs allowed), device arrays.
 *   mp_segment_offset_i64: data[r*ld + i] += inc[g(i)], r < rows, i < n
 *   mp_segment_ids_i64:    ids[i] = g(i)
 * g(i) = the graph whose segment holds element i.  Bit-exact (integers). */
int mp_segment_offset_i64(int64_t* data, int64_t ld, int32_t rows, int64_t n, const int64_t* starts,
                          const int64_t* inc, int64_t n_graphs, void* stream);
int mp_segment_ids_i64(int64_t* ids, int64_t n, const int64_t* starts, int64_t n_graphs, void* stream);

/* ---- GATConv attention dropout (training) --------------------------------
 * GATConv.message applies `F.dropout(alpha, p, training)` to the softmax output
 * (PyG 1.4.3 [U6]; the reference's generic path materialises alpha [E, H] and
 * the [E, H*C] messages for it).  Here the mask is a function of the edge's
 * key k and the head h:
 *   keep(k, h) = hash(seed, k*H + h) >= floor(p * 2^32),  kept alpha * 1/(1-p)
 * (hash: two rounds of the murmur3 32-bit finaliser, oracle/pyg_ref.py
 * restates it), so the forward and the transposed backward evaluate the same
 * mask without storing one.  0 < p < 1, H <= 32.  The key (ABI 7): drop_ids[s]
 * for slot s of the CSR the call walks (int32, one per slot: the forward's
 * destination CSR, the backward's transposed CSR), or -- drop_ids NULL -- the
 * edge's destination-CSR slot.  mi355_mp passes edge ids: the layer's on one
 * GPU, the GLOBAL ones on a shard, so a sharded GATConv draws exactly the mask
 * of the single-GPU layer.
 *
 * mp_gat_aggregate_train_drop_f32: mp_gat_aggregate_train_f32 with the dropped
 *   alpha on the messages: out / agg / out2 use alpha * keep / (1-p); the
 *   softmax statistics (row_stats, row_s2) are those of the undropped alpha.
 * mp_gat_backward_train_drop_f32: mp_gat_backward_train_f32 for that forward
 *   (the transposed CSR's eid channel must hold each edge's dst-CSR slot);
 *   needs C/4 a power of two <= 64 and 16-byte aligned rows.
 * mp_gat_dropout_keep: bits[s] = keep bits of slot s (bit h), s < n_slots (key drop_ids[s],
 *   or s when drop_ids is NULL). */
int mp_gat_aggregate_train_drop_f32(const mp_csr* g, const float* xw, const float* a_src,
                                    const float* a_dst, const float* att, int32_t H, int32_t C,
                                    float slope, const float* bias, float* out, int64_t ldo,
                                    float* agg, float* row_stats, float* out2, float* row_s2,
                                    uint64_t seed, float p_drop, const int32_t* drop_ids, void* slab,
                                    size_t slab_bytes, int32_t stages, void* stream);
int mp_gat_backward_train_drop_f32(const mp_csr* gt, const float* grad_out, int64_t ldg,
                                   const float* xw, const float* a_src, const float* pack,
                                   const float* att, int32_t H, int32_t C, float slope,
                                   const float* grad_a_dst, uint64_t seed, float p_drop,
                                   const int32_t* drop_ids, float* grad_xw, float* grad_a_src, void* slab,
                                   size_t slab_bytes, int32_t stages, void* stream);
int mp_gat_dropout_keep(uint64_t seed, float p_drop, int32_t H, int64_t n_slots, const int32_t* drop_ids,
                        uint32_t* bits, void* stream);

/* ---- Row-exact feature transform (ABI 7) ----------------------------------
 * C[i, n] = the k-ordered fmaf chain over k = 0..K-1 from 0 of A[i, k] * B[k, n],
 * B = W ([K, N] row-major) or, trans_w != 0, W^T (W [N, K] row-major): every
 * output row is a function of its input row alone, so a shard's rows of X W are
 * bitwise the single-GPU rows whatever M is (GATConv's x @ W [U6]; a hipBLASLt
 * GEMM picks its kernel -- and its rounding -- by M).  K = N = 256 with 16-byte
 * aligned rows of A (lda % 4 == 0): the f32 MFMA kernel; any other shape (or
 * force_generic): a tiled fmaf kernel with the same arithmetic.  lda >= K,
 * ldc >= N; M = 0 is a no-op. */
int mp_gemm_rows_f32(const float* A, int64_t lda, int64_t M, int32_t K, const float* W, int32_t trans_w,
                     int32_t N, float* C, int64_t ldc, int32_t force_generic, void* stream);

/* Per-block column sums of x [n, F] (0 < F <= 256, F % 4 == 0, 16-byte aligned
 * rows): part [mp_gat_bwd_blocks(n), F] (part_bytes >= that * 4; ABI 6);
 * sum_i x[i, :] is their sum over the blocks (a layer's bias gradient, sum over
 * rows of grad_out). */
int mp_col_sums_f32(const float* x, int64_t ldx, int64_t n, int32_t F, float* part, size_t part_bytes,
                    void* stream);

/* Rows of the per-block partial arrays of the prep/finish kernels for n nodes. */
int mp_gat_bwd_blocks(int64_t n);

/* Backward epilogue (C%4==0, H*C<=256), one pass over the nodes:
 *   grad_xw[n, h*C+c] += ga_dst[n,h] * att[h, c]        (att = [H, 2C]: dst half first)
 *   att_part[b, 0, :]  = sum over block b's nodes of ga_dst[n,h] * xw[n, h*C+c]
 *   att_part[b, 1, :]  = ... ga_src[n,h] * xw[n, h*C+c]
 * att_part is [mp_gat_bwd_blocks(n), 2, H*C]; d att = its sum over blocks.
 * att_part_bytes >= mp_gat_bwd_blocks(n) * 2*H*C * 4 (ABI 6: a partial array
 * sized for fewer rows than n -- e.g. a sharded rank's own rows when the pass
 * runs over own + halo rows -- is MP_ERR_ARG, not a device write past its end).
 * grad_xw = NULL: the att-gradient partials only. */
int mp_gat_backward_finish_f32(float* grad_xw, const float* xw, const float* ga_dst,
                               const float* ga_src, const float* att, int64_t n, int32_t H,
                               int32_t C, float* att_part, size_t att_part_bytes, void* stream);

/* y[n, h*C+c] += s[n,h] * att[h*att_ld + c]  (per-head outer-product update) */
int mp_heads_outer_add_f32(float* y, int64_t ldy, const float* s, int64_t n, int32_t H,
                           int32_t C, const float* att, int64_t att_ld, void* stream);

/* alpha[e,h] for edges in ORIGINAL order (return_attention_weights, backward) */
int mp_gat_alpha_f32(const int64_t* src_idx, const int64_t* dst_idx,
                     int64_t n_edges, int32_t H, const float* a_src,
                     const float* a_dst, float slope, const float* row_stats,
                     float* alpha, void* stream);

/* ---- sharded GATConv over the hybrid halo cover ---------------
 * Merge of online-softmax partials into a destination row's local piece.
 * Row i (i < n_rows) holds the local piece: out[i] = acc/den (normalised, no
 * bias) and row_stats[i, h] = (m, den) from mp_gat_aggregate_att_f32 /
 * mp_gat_aggregate_train_f32 over the rank's own + pulled sources; partial
 * rows k in [pptr[i], pptr[i+1]) of pidx name rows of part_out [n_parts, ldp] /
 * part_stats [n_parts, H, 2] (peers' pieces of the same row, the same kernels
 * on their send graphs).  Per head, local piece first, then the partials in
 * list order:  M = max m, w_k = den_k e^(m_k - M), tot = sum w_k,
 *   out[i] = sum_k (w_k / tot) out_k + bias,   row_stats[i, h] = (M, tot),
 * and (training, optional) agg2[i] / row_s2[i] (the local piece's out2 / row_s2
 * [n_rows, H*C] / [n_rows, H]) scaled by w_loc / tot, the merged rows'.  A row
 * with no partial keeps its local piece + bias bit for bit.  pptr [n_rows + 1]
 * (int32, non-decreasing, pptr[n_rows] <= n_parts) and every pidx entry in
 * [0, n_parts) are the caller's contract (device arrays, not read on the host).
 * C % 4 == 0; out, part_out, bias, agg2 16-byte aligned, leading dimensions
 * multiples of 4.  Extents (ABI 7): part_out_bytes >= ((n_parts - 1) * ldp +
 * H*C) * 4 and part_stats_bytes >= n_parts * H * 8 when n_parts > 0 (the
 * pidx range itself is checked by the host that builds the merge list:
 * mi355_mp.gat_cover.GatHaloCover).  Head of any width: a head may span two of
 * the kernel's 256-feature chunks (the merged stats are written after every
 * chunk of the row has read them). */
int mp_gat_merge_partials_f32(int64_t n_rows, int32_t H, int32_t C, const int32_t* pptr, const int32_t* pidx,
                              int64_t n_parts, const float* part_out, size_t part_out_bytes, int64_t ldp,
                              const float* part_stats, size_t part_stats_bytes, const float* bias, float* out,
                              int64_t ldo, float* row_stats, float* agg2, float* row_s2, void* stream);

/* ---- self-loop rewrites (PyG 1.4.3 utils.loop [U4]) -----
 * Output edge order is upstream's: the kept edges in original order, then the
 * loop edges (n, n) for n = 0..N-1.
 *   MP_LOOPS_REMOVE         remove_self_loops: the non-loop edges
 *   MP_LOOPS_ADD            add_self_loops: every edge, then the N loops
 *   MP_LOOPS_ADD_REMAINING  add_remaining_self_loops: the non-loop edges, then
 *                           the N loops
 * out_pos[k] = position of the input edge whose weight output edge k carries:
 * kept edges their own position; a loop of ADD_REMAINING the position of the
 * node's LAST pre-existing loop (upstream's sequential index_put_ keeps the
 * last one), else -1; a loop of ADD -1.  Weights: mp_gather_fill_f32(w, out_pos,
 * fill).  n_kept = n_edges - mp_self_loop_count(...) for REMOVE and
 * ADD_REMAINING, n_edges for ADD; the outputs hold n_kept (+ N) entries.
 * out_pos is also the compaction buffer (needed unless nothing is removed). */
#define MP_LOOPS_REMOVE 0
#define MP_LOOPS_ADD 1
#define MP_LOOPS_ADD_REMAINING 2
/* count_dev: device int64[2]; [0] = number of self loops, [1] = self loops (r, r)
 * with r outside [0, n_nodes) -- upstream's `loop_weight[row[inv_mask]]` raises
 * an IndexError for those, and the caller must reject them before
 * mp_self_loops (whose loop bookkeeping ignores them).  (ABI 3: n_nodes and the
 * second counter.) */
int mp_self_loop_count(const int64_t* row, const int64_t* col, int64_t n_edges,
                       int64_t n_nodes, int64_t* count_dev, void* stream);
size_t mp_self_loops_workspace(int64_t n_edges, int64_t n_nodes);
int mp_self_loops(const int64_t* row, const int64_t* col, int64_t n_edges, int64_t n_nodes,
                  int32_t mode, int64_t n_kept, int64_t* out_row, int64_t* out_col,
                  int64_t* out_pos, void* ws, size_t ws_bytes, void* stream);
/* out[k] = pos[k] >= 0 ? src[pos[k]] : fill */
int mp_gather_fill_f32(const float* src, const int64_t* pos, int64_t n, float fill,
                       float* out, void* stream);

/* ---- shard plan (destination-range shards, halo maps) ---------- */

/* The plan of rank `rank` owning the key rows [lo, hi) = [cuts[rank],
 * cuts[rank + 1]) of a range partition (replaces the torch-op construction in
 * mi355_mp/dist.py ShardPlan: nonzero / unique / searchsorted):
 *   edge_pos[k]     positions of the edges with lo <= key < hi, in edge order;
 *   local_key[k]    key[edge_pos[k]] - lo;
 *   local_other[k]  other - lo when lo <= other < hi, else n_own + the rank of
 *                   `other` among halo_nodes;
 *   halo_nodes      the sorted unique remote `other` values of those edges;
 *   counts (device, int64 [2 + world]): [0] = selected edges, [1] = halo nodes
 *                   (-1 when a selected edge's `other` lies outside
 *                   [0, n_nodes): the outputs are then invalid), [2 + q] = halo
 *                   nodes owned by rank q.
 * key = destination, other = source for flow source_to_target (the forward
 * plan); swapped for the transposed (backward) plan.  cuts: device int64
 * [world + 1].  Outputs are sized at their upper bounds (n_edges, n_nodes);
 * the caller reads counts and slices.  Workspace: mp_shard_plan_workspace. */
size_t mp_shard_plan_workspace(int64_t n_edges, int64_t n_nodes);
int mp_shard_plan(const int64_t* key, const int64_t* other, int64_t n_edges, int64_t n_nodes,
                  const int64_t* cuts, int32_t world, int32_t rank, int64_t lo, int64_t hi,
                  int64_t* edge_pos, int64_t* local_key, int64_t* local_other,
                  int64_t* halo_nodes, int64_t* counts, void* ws, size_t ws_bytes, void* stream);

/* ---- other dtypes (csrc/mp_dtype.hip) -------------------------------------
 * torch_scatter 2.0.4 reduces any dtype ([U8/U9]); the fp32 hot path is
 * mp_aggregate_f32, these are the breadth path for the rest. */
#define MP_DTYPE_F32 0
#define MP_DTYPE_F64 1
#define MP_DTYPE_F16 2
#define MP_DTYPE_BF16 3
#define MP_DTYPE_I64 4

/* out[r, :] = REDUCE_{k in row r} src[col[k], :] (col NULL: src row k), rows
 * of `dtype` with leading dimensions lds / ldo in elements.  Every row is
 * reduced by one wave per 64-feature tile in slot (= original edge) order,
 * never split: float64 / int64 follow the reference's arithmetic bit for bit
 * (int64 sums wrap); float16 / bfloat16 accumulate in fp32 and round once.
 * max / min: strict compare (first edge wins), start at the type's lowest() /
 * max(); a row that keeps it reports 0 and arg = n_ids (n_edges when 0); arg_out
 * int64 [n_rows, F] (contiguous).  mean: (sum [+ out]) / max(count, 1), integer
 * division truncating toward zero.  flags: MP_FLAG_INIT_FROM_OUT (torch_scatter
 * `out=`), MP_FLAG_PYG_MASK (utils.scatter_'s +-10000 masks). */
int mp_segment_reduce(const mp_csr* g, int32_t dtype, const void* src, int64_t lds,
                      int32_t F, int32_t reduce, int32_t flags, void* out, int64_t ldo,
                      int64_t* arg_out, void* stream);

/* out[k, :] = x[idx[k], :] for elements of elem_bytes (2, 4 or 8) bytes. */
int mp_gather_rows_any(int32_t elem_bytes, const void* x, int64_t ldx, const int64_t* idx,
                       int64_t n, int32_t F, void* out, int64_t ldo, void* stream);

/* grad[arg[r, f], f] = grad_out[r, f] for arg in [0, n_edges) (ScatterMax
 * backward on materialised messages; grad zero-initialised by the caller). */
int mp_scatter_arg_any(int32_t elem_bytes, const void* grad_out, const int64_t* arg,
                       int64_t n_rows, int32_t F, int64_t n_edges, void* grad, int64_t ldg,
                       void* stream);

/* ---- helpers on the path -------------------------------------------------- */

/* out[k,:] = x[idx[k],:]  (index_select of __collect__, scatter-sum backward,
 * halo packing for the multi-GPU exchange) */
int mp_gather_rows_f32(const float* x, int64_t ldx, const int64_t* idx,
                       int64_t n, int32_t F, float* out, int64_t ldo,
                       void* stream);

/* dst[k] = src[perm[k]] (CSR-ordering of per-edge weights) */
int mp_permute_f32(const float* src, const int32_t* perm, int64_t n,
                   float* dst, void* stream);

/* ---- deterministic source-side reductions (csrc/mp_segment.hip) ----------- */

/* out[r] = ((0 + v[id(k0)]) + v[id(k0+1)]) + ... over the slots k of row r in
 * slot order, id(k) = eid[k] (eid NULL: k).  Bit-identical to the serial CPU
 * loop.  Over the transposed CSR (rows = edge_index[0]) with v = the edge
 * weights in original order it is GCNConv.norm's deg = scatter_add(w, row) [U5]
 * in the reference's edge order (replaces the float atomics of mp_gcn_norm_f32
 * for real-valued weights). */
int mp_segment_sum_serial_f32(const int32_t* rowptr, const int32_t* eid, const float* v,
                              int64_t n_rows, float* out, void* stream);

/* GCNConv.norm steps 2-3 from a given degree: deg is overwritten with
 * deg^-1/2 (inf -> 0), norm[e] = dinv[row[e]] * w[e] * dinv[col[e]]. */
int mp_gcn_norm_from_deg_f32(const int64_t* row, const int64_t* col, const float* w,
                             int64_t n_edges, int64_t n_nodes, float* deg, float* norm,
                             void* stream);

/* inv[eid[k]] = k for every slot k of g (the slot of each edge id). */
int mp_csr_inverse_eid(const mp_csr* g, int32_t* inv, void* stream);

/* Deterministic ScatterMax/ScatterMin backward of a fused message w_e * x[src_e]
 * ([U8] ScatterMax.backward, then the message's and index_select's backward:
 * an index_add_ by source in edge order).  Three steps over the TRANSPOSED CSR
 * gt (rows = source nodes, slots = out-edges in original order, col = the
 * destination row, eid = the edge id):
 *   1. mp_arg_winner_mask: mask [gt.n_edges, mp_arg_mask_words(F)] uint32 in gt
 *      slot order, bit f of slot inv[e] set when arg[r, f] = e (inv =
 *      mp_csr_inverse_eid(gt)); ids outside [0, n_edges) (empty rows) set nothing.
 *   2. mp_scatter_arg_backward_csr_f32: grad[j, f] = sum over the slots of row j
 *      in order of w_e * grad_out[dst, f] where the slot won (j, f) -- the
 *      reference's edge-order sum, bit for bit; every row of grad is written.
 *      w: per-edge weights in ORIGINAL edge order, or NULL (= 1).
 *   3. (optional) mp_scatter_arg_grad_w_f32: grad_w[e] = sum over the features
 *      e won of grad_out[dst_map[e], f] * x[src_map[e], f] (fixed reduction tree),
 *      0 for edges that won nothing; every entry written.
 * The mask must be 8-byte aligned; mask_bytes >= n_edges * mp_arg_mask_words(F) * 4
 * in all three calls (ABI 6). */
int32_t mp_arg_mask_words(int32_t F);
int mp_arg_winner_mask(const int64_t* arg, int64_t n_rows, int32_t F, int64_t n_edges,
                       const int32_t* inv, uint32_t* mask, size_t mask_bytes, void* stream);
int mp_scatter_arg_backward_csr_f32(const mp_csr* gt, const uint32_t* mask, size_t mask_bytes,
                                    const float* grad_out, int64_t ldg, int32_t F,
                                    const float* w, float* grad, int64_t ldgx, void* stream);
int mp_scatter_arg_grad_w_f32(const int64_t* src_map, const int64_t* dst_map, int64_t n_edges,
                              const int32_t* inv, const uint32_t* mask, size_t mask_bytes, int32_t F,
                              const float* grad_out, int64_t ldg, const float* x, int64_t ldx,
                              float* grad_w, void* stream);

/* ScatterMax/ScatterMin backward [U8] on materialised message rows (torch_scatter
 * scatter_max / scatter_min of src [n_edges, F]): for every (r,f) with
 * arg[r,f] = e != n_edges, grad[e, f] = grad_out[r,f] -- a plain store (row e
 * belongs to one output row), deterministic.  grad must be zero-initialised by
 * the caller.  The fused message w_e * x[src_e] takes the CSR form above.
 * (ABI 5: the float-atomic src_map / grad_w form of ABI <= 4 is gone.) */
int mp_scatter_arg_backward_f32(const float* grad_out, const int64_t* arg,
                                int64_t n_rows, int32_t F, int64_t n_edges,
                                float* grad, int64_t ldg, void* stream);

/* GCNConv.norm [U5]: deg = scatter_add(w, row); dinv = deg^-1/2 (inf -> 0);
 * norm[e] = dinv[row[e]] * w[e] * dinv[col[e]] (original edge order).
 * w == NULL means all ones.  deg_ws: n_nodes floats of workspace.  The degree
 * is summed with float atomics: exact (hence deterministic) only for
 * integer-valued weights (self-loop fills 1 / 2, unweighted graphs); for real
 * weights use mp_segment_sum_serial_f32 + mp_gcn_norm_from_deg_f32. */
int mp_gcn_norm_f32(const int64_t* row, const int64_t* col, const float* w,
                    int64_t n_edges, int64_t n_nodes, float* deg_ws,
                    float* norm, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MI355_MP_H */
