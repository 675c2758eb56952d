/*
 * abi_reject.c -- argument / extent rejection harness for the C-ABI of
 * include/mi355_mp.h (test infrastructure, SURVEY section 5: "ASAN build of the
 * C-ABI harness").
 *
 * Built against the host-only AddressSanitizer build of the library
 * (`make -C pytorch_geometric-1_amd/csrc asan`) and run on a machine with no
 * GPU by tests/test_host.py::test_abi_rejections_under_asan.  Every case calls
 * one entry point with one bad argument and expects MP_ERR_ARG and an error
 * text naming the problem -- no launch, no device access, no host memory
 * error (ASAN aborts the run on one).  The ABI-6 extent cases also call with
 * the exact extent the call needs and expect the argument checks to pass
 * (the call then fails at its first HIP call, MP_ERR_HIP, as there is no GPU):
 * the boundary is the byte count the header documents, not a looser one.
 *
 * Device pointers are fake, 256-byte aligned addresses that the host never
 * dereferences; mp_csr structs are real host structs.
 * Output: one line per case, then "abi_reject: N cases, M failures".
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "mi355_mp.h"

static int n_cases = 0, n_fail = 0;

#define DEV ((void*)(uintptr_t)0x7f0000000000ull) /* fake device pointer, never dereferenced */
#define DEVF ((float*)DEV)
#define DEVI ((int32_t*)DEV)
#define DEVL ((int64_t*)DEV)
#define DEVU ((uint32_t*)DEV)

static void expect(int line, const char* what, int rc, int want_arg, const char* needle) {
  ++n_cases;
  const char* err = mp_last_error();
  int ok;
  if (want_arg) {
    ok = rc == MP_ERR_ARG && (!needle || (err && strstr(err, needle)));
  } else {
    ok = rc != MP_ERR_ARG; /* the argument checks passed (MP_ERR_HIP without a GPU) */
  }
  printf("%s line %d: %s -> rc %d (%s)\n", ok ? "ok  " : "FAIL", line, what, rc, err ? err : "");
  if (!ok) ++n_fail;
}

/* rejected with MP_ERR_ARG, the error text containing `needle` */
#define REJECT(needle, call) expect(__LINE__, #call, (call), 1, needle)
/* passes every argument check */
#define ACCEPT(call) expect(__LINE__, #call, (call), 0, NULL)

/* a well-formed graph of n_rows rows / n_edges slots over n_cols gathered rows */
static mp_csr graph(int64_t n_rows, int64_t n_edges, int32_t n_cols) {
  mp_csr g;
  memset(&g, 0, sizeof g);
  g.rowptr = DEVI;
  g.col = DEVI;
  g.eid = DEVI;
  g.wave_row = DEVI;
  g.wave_slot = DEVI;
  g.split_waves = DEVI;
  g.n_rows = n_rows;
  g.n_edges = n_edges;
  g.chunk = 256;
  g.n_waves = mp_schedule_n_waves(n_rows, n_edges, 256);
  g.n_split = 0;
  g.n_cols = n_cols;
  g.n_ids = 0;
  return g;
}

static void extents_gat_backward(void) {
  /* the round-4 case: a sharded rank's local graph of n_own own rows and halo
   * rows after them; the finish pass runs over all n = n_own + n_halo rows,
   * so att_part needs mp_gat_bwd_blocks(n) blocks, not mp_gat_bwd_blocks(n_own) */
  const int64_t n_own = 1000, n = 1700;
  const int H = 8, C = 32, F = H * C;
  const size_t need = (size_t)mp_gat_bwd_blocks(n) * 2 * F * 4;
  const size_t own_sized = (size_t)mp_gat_bwd_blocks(n_own) * 2 * F * 4;
  REJECT("att_part", mp_gat_backward_finish_f32(DEVF, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, own_sized, NULL));
  REJECT("att_part", mp_gat_backward_finish_f32(NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, need - 1, NULL));
  REJECT("att_part", mp_gat_backward_finish_f32(NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, 0, NULL));
  ACCEPT(mp_gat_backward_finish_f32(NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, need, NULL));
  REJECT("null", mp_gat_backward_finish_f32(NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, NULL, need, NULL));

  /* prep (inference forward) and prep_train: pack [n, H, 4], gsum_part [blocks(n), F] */
  const size_t pack = (size_t)n * H * 16, gsum = (size_t)mp_gat_bwd_blocks(n) * F * 4;
  REJECT("pack", mp_gat_backward_prep_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, n, H, C, DEVF, pack - 1, DEVF, gsum, NULL));
  REJECT("gsum_part", mp_gat_backward_prep_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, n, H, C, DEVF, pack, DEVF, gsum - 4,
                                               NULL));
  ACCEPT(mp_gat_backward_prep_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, n, H, C, DEVF, pack, DEVF, gsum, NULL));
  ACCEPT(mp_gat_backward_prep_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, n, H, C, DEVF, pack, NULL, 0, NULL));
  REJECT("pack", mp_gat_backward_prep_train_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, pack - 16,
                                                DEVF, gsum, DEVF, NULL));
  REJECT("gsum_part", mp_gat_backward_prep_train_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, pack,
                                                     DEVF, mp_gat_bwd_blocks(n_own) * (size_t)F * 4, DEVF, NULL));
  ACCEPT(mp_gat_backward_prep_train_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, pack, DEVF, gsum,
                                        DEVF, NULL));
  REJECT("null", mp_gat_backward_prep_train_f32(DEVF, F, DEVF, F, NULL, DEVF, DEVF, DEVF, DEVF, n, H, C, DEVF, pack, DEVF,
                                                gsum, NULL, NULL));

  /* column sums: part [blocks(n), F] */
  REJECT("part", mp_col_sums_f32(DEVF, F, n, F, DEVF, gsum - 1, NULL));
  REJECT("part", mp_col_sums_f32(DEVF, F, 0, F, DEVF, 0, NULL)); /* n = 0 still zero-fills one block */
  ACCEPT(mp_col_sums_f32(DEVF, F, n, F, DEVF, gsum, NULL));
  REJECT("F <= 256", mp_col_sums_f32(DEVF, 512, n, 512, DEVF, 1 << 30, NULL));

  /* the transposed pass: de [gt.n_edges, H] */
  mp_csr gt = graph(n, 9000, (int32_t)n_own);
  const size_t slab = mp_gat_slab_bytes(&gt, H, C);
  const size_t de = (size_t)gt.n_edges * H * 4;
  REJECT("de", mp_gat_backward_f32(&gt, DEVF, F, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, DEVF, DEVF, de - 1, DEV,
                                   slab, 7, NULL));
  REJECT("de is required", mp_gat_backward_f32(&gt, DEVF, F, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, DEVF, NULL, 0,
                                               DEV, slab, 7, NULL));
  REJECT("slab", mp_gat_backward_f32(&gt, DEVF, F, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, DEVF, DEVF, de, DEV,
                                     slab - 1, 7, NULL));
  ACCEPT(mp_gat_backward_f32(&gt, DEVF, F, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, DEVF, DEVF, de, DEV, slab, 7,
                             NULL));
  REJECT("grad_a_dst", mp_gat_backward_train_f32(&gt, DEVF, F, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, DEVF,
                                                 DEV, slab, 7, NULL));
  REJECT("dropout p", mp_gat_backward_train_drop_f32(&gt, DEVF, F, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, 1, 1.5f, NULL,
                                                      DEVF, DEVF, DEV, slab, 7, NULL));

  /* heads of any width: pack, acc2 [gt.n_rows, F], sc [gt.n_rows, H] */
  const int Cw = 36, Fw = H * Cw;
  const size_t wslab = mp_gat_train_slab_bytes(&gt, H, Cw);
  const size_t acc2 = (size_t)gt.n_rows * Fw * 4, sc = (size_t)gt.n_rows * H * 4;
  REJECT("pack", mp_gat_backward_prep_wide_f32(DEVF, Fw, DEVF, Fw, NULL, DEVF, DEVF, DEVF, DEVF, n, H, Cw, DEVF,
                                               (size_t)n_own * H * 16, DEVF, NULL));
  ACCEPT(mp_gat_backward_prep_wide_f32(DEVF, Fw, DEVF, Fw, NULL, DEVF, DEVF, DEVF, DEVF, n, H, Cw, DEVF, (size_t)n * H * 16,
                                       DEVF, NULL));
  REJECT("acc2", mp_gat_backward_wide_f32(&gt, DEVF, Fw, DEVF, DEVF, H, Cw, 0.2f, 0, 0.f, NULL, DEVF, DEVF, acc2 - 4, DEVF,
                                          sc, DEV, wslab, 7, NULL));
  REJECT("sc", mp_gat_backward_wide_f32(&gt, DEVF, Fw, DEVF, DEVF, H, Cw, 0.2f, 0, 0.f, NULL, DEVF, DEVF, acc2, DEVF,
                                        (size_t)n_own * H * 4, DEV, wslab, 7, NULL));
  ACCEPT(mp_gat_backward_wide_f32(&gt, DEVF, Fw, DEVF, DEVF, H, Cw, 0.2f, 0, 0.f, NULL, DEVF, DEVF, acc2, DEVF, sc, DEV,
                                  wslab, 7, NULL));
  REJECT("C % 4", mp_gat_backward_wide_f32(&gt, DEVF, Fw, DEVF, DEVF, H, 35, 0.2f, 0, 0.f, NULL, DEVF, DEVF, acc2, DEVF, sc,
                                           DEV, wslab, 7, NULL));
  REJECT("null", mp_gat_backward_epilogue_wide_f32(DEVF, NULL, DEVF, DEVF, DEVF, DEVF, n, H, Cw, NULL));
}

static void extents_arg_backward(void) {
  /* max/min backward: mask [n_edges, mp_arg_mask_words(F)] uint32 */
  const int64_t E = 5000, R = 300;
  const int F = 200;
  const size_t mask = (size_t)E * mp_arg_mask_words(F) * 4;
  REJECT("mask", mp_arg_winner_mask(DEVL, R, F, E, DEVI, DEVU, mask - 4, NULL));
  REJECT("mask", mp_arg_winner_mask(DEVL, R, F, E, DEVI, DEVU, (size_t)E * 2 * 4, NULL)); /* sized for F <= 64 */
  ACCEPT(mp_arg_winner_mask(DEVL, R, F, E, DEVI, DEVU, mask, NULL));
  mp_csr gt = graph(400, E, (int32_t)R);
  REJECT("mask", mp_scatter_arg_backward_csr_f32(&gt, DEVU, mask - 1, DEVF, F, F, NULL, DEVF, F, NULL));
  ACCEPT(mp_scatter_arg_backward_csr_f32(&gt, DEVU, mask, DEVF, F, F, NULL, DEVF, F, NULL));
  REJECT("8-byte", mp_scatter_arg_backward_csr_f32(&gt, (const uint32_t*)((char*)DEV + 4), mask, DEVF, F, F, NULL,
                                                    DEVF, F, NULL));
  REJECT("mask", mp_scatter_arg_grad_w_f32(DEVL, DEVL, E, DEVI, DEVU, mask / 2, F, DEVF, F, DEVF, F, DEVF, NULL));
  ACCEPT(mp_scatter_arg_grad_w_f32(DEVL, DEVL, E, DEVI, DEVU, mask, F, DEVF, F, DEVF, F, DEVF, NULL));
}

static void abi7(void) {
  /* the GAT merge list's part_out [n_parts, ldp] / part_stats [n_parts, H, 2] */
  const int64_t n = 1000, np = 300;
  const int H = 6, C = 124, F = H * C;
  const size_t po = (size_t)((np - 1) * F + F) * 4, ps = (size_t)np * H * 2 * 4;
  REJECT("part_out", mp_gat_merge_partials_f32(n, H, C, DEVI, DEVI, np, DEVF, po - 4, F, DEVF, ps, NULL, DEVF, F, DEVF,
                                               NULL, NULL, NULL));
  REJECT("part_stats", mp_gat_merge_partials_f32(n, H, C, DEVI, DEVI, np, DEVF, po, F, DEVF, ps - 1, NULL, DEVF, F,
                                                 DEVF, NULL, NULL, NULL));
  ACCEPT(mp_gat_merge_partials_f32(n, H, C, DEVI, DEVI, np, DEVF, po, F, DEVF, ps, NULL, DEVF, F, DEVF, NULL, NULL,
                                   NULL));
  /* tile-major sum / mean: tiles of 64k features dividing F, no overlap */
  const int64_t N = 2000, E = 9000;
  mp_csr g = graph(N, E, (int32_t)N);
  const size_t slab = mp_aggregate_slab_bytes(&g, 256, MP_REDUCE_SUM);
  REJECT("sum or mean", mp_aggregate_tiles_f32(&g, DEVF, DEVF, 0, 128, N * 128, 256, MP_REDUCE_MAX, 0, NULL, NULL, DEVF, 256,
                                               0, 0, DEV, slab, 7, NULL));
  REJECT("64k features", mp_aggregate_tiles_f32(&g, DEVF, DEVF, 0, 96, N * 96, 192, MP_REDUCE_SUM, 0, NULL, NULL, DEVF, 192,
                                                0, 0, DEV, slab, 7, NULL));
  REJECT("not overlap", mp_aggregate_tiles_f32(&g, DEVF, DEVF, 0, 128, N * 128 - 1, 256, MP_REDUCE_SUM, 0, NULL, NULL, DEVF,
                                               256, 0, 0, DEV, slab, 7, NULL));
  REJECT("not overlap", mp_aggregate_tiles_f32(&g, DEVF, DEVF, 256, 0, 0, 256, MP_REDUCE_SUM, 0, NULL, NULL, DEVF, 0, 64,
                                               N * 64 - 64, DEV, slab, 7, NULL));
  REJECT("flags", mp_aggregate_tiles_f32(&g, DEVF, DEVF, 256, 0, 0, 256, MP_REDUCE_SUM, MP_FLAG_PYG_MASK, NULL, NULL, DEVF,
                                         256, 128, N * 128, DEV, slab, 7, NULL));
  REJECT("slab", mp_aggregate_tiles_f32(&g, DEVF, DEVF, 0, 128, N * 128, 256, MP_REDUCE_SUM, 0, NULL, NULL, DEVF, 256, 0, 0,
                                        DEV, slab - 1, 7, NULL));
  ACCEPT(mp_aggregate_tiles_f32(&g, DEVF, DEVF, 0, 128, N * 128, 256, MP_REDUCE_SUM, MP_FLAG_INIT_FROM_OUT, NULL, NULL, DEVF,
                                256, 0, 0, DEV, slab, 7, NULL));
  ACCEPT(mp_aggregate_tiles_f32(&g, DEVF, DEVF, 256, 0, 0, 256, MP_REDUCE_MEAN, 0, DEVF, NULL, DEVF, 0, 64, N * 64, DEV, slab,
                                7, NULL));
  /* the row-exact feature transform */
  REJECT("null", mp_gemm_rows_f32(NULL, 256, 10, 256, DEVF, 0, 256, DEVF, 256, 0, NULL));
  REJECT("lda >= K", mp_gemm_rows_f32(DEVF, 100, 10, 256, DEVF, 0, 256, DEVF, 256, 0, NULL));
  REJECT("ldc >= N", mp_gemm_rows_f32(DEVF, 256, 10, 256, DEVF, 0, 256, DEVF, 255, 0, NULL));
  REJECT("K > 0", mp_gemm_rows_f32(DEVF, 256, 10, 0, DEVF, 0, 256, DEVF, 256, 0, NULL));
  ACCEPT(mp_gemm_rows_f32(NULL, 256, 0, 256, NULL, 0, 256, NULL, 256, 0, NULL)); /* M = 0: a no-op */
  ACCEPT(mp_gemm_rows_f32(DEVF, 24, 10, 24, DEVF, 0, 64, DEVF, 64, 0, NULL));
}

static void workspaces(void) {
  /* entry points whose workspace extents predate ABI 6 */
  const int64_t E = 10000, N = 2000;
  const size_t csr_ws = mp_csr_build_workspace(E, N);
  REJECT(NULL, mp_csr_build(DEVL, DEVL, E, N, N, DEVI, DEVI, DEVI, DEVI, DEV, csr_ws - 1, NULL));
  ACCEPT(mp_csr_build(DEVL, DEVL, E, N, N, DEVI, DEVI, DEVI, DEVI, DEV, csr_ws, NULL));
  REJECT(NULL, mp_csr_build(NULL, DEVL, E, N, N, DEVI, DEVI, DEVI, DEVI, DEV, csr_ws, NULL));
  const int32_t nw = mp_schedule_n_waves(N, E, 256);
  const size_t sws = mp_schedule_workspace(nw);
  REJECT("chunk", mp_schedule_build(DEVI, N, E, 100, 10, DEVI, DEVI, DEVI, DEVI, DEV, sws, NULL));
  REJECT(NULL, mp_schedule_build(DEVI, N, E, 256, 10, DEVI, DEVI, DEVI, DEVI, DEV, sws - 1, NULL));
  ACCEPT(mp_schedule_build(DEVI, N, E, 256, 10, DEVI, DEVI, DEVI, DEVI, DEV, sws, NULL));

  mp_csr g = graph(N, E, (int32_t)N);
  const int F = 256;
  const size_t ab = mp_aggregate_slab_bytes(&g, F, MP_REDUCE_SUM);
  const size_t ab_arg = mp_aggregate_slab_bytes(&g, F, MP_REDUCE_MAX);
  REJECT("slab", mp_aggregate_f32(&g, NULL, DEVF, F, F, MP_REDUCE_SUM, 0, NULL, DEVF, F, NULL, DEV, ab - 1, 7, NULL));
  REJECT("slab", mp_aggregate_f32(&g, NULL, DEVF, F, F, MP_REDUCE_MAX, 0, NULL, DEVF, F, DEVL, DEV, ab, 7, NULL));
  ACCEPT(mp_aggregate_f32(&g, NULL, DEVF, F, F, MP_REDUCE_MAX, 0, NULL, DEVF, F, DEVL, DEV, ab_arg, 7, NULL));
  REJECT("arg_out", mp_aggregate_f32(&g, NULL, DEVF, F, F, MP_REDUCE_MIN, 0, NULL, DEVF, F, NULL, DEV, ab_arg, 7,
                                     NULL));
  REJECT("leading dimension", mp_aggregate_f32(&g, NULL, DEVF, F - 1, F, MP_REDUCE_SUM, 0, NULL, DEVF, F, NULL, DEV,
                                               ab, 7, NULL));
  REJECT("null x/out", mp_aggregate_f32(&g, NULL, NULL, F, F, MP_REDUCE_SUM, 0, NULL, DEVF, F, NULL, DEV, ab, 7,
                                        NULL));
  REJECT("null graph", mp_aggregate_f32(NULL, NULL, DEVF, F, F, 0, 0, NULL, DEVF, F, NULL, DEV, ab, 7, NULL));
  mp_csr bad = g;
  bad.n_cols = 0;
  REJECT("n_cols", mp_aggregate_f32(&bad, NULL, DEVF, F, F, 0, 0, NULL, DEVF, F, NULL, DEV, ab, 7, NULL));
  bad = g;
  bad.chunk = 12;
  REJECT("schedule", mp_aggregate_f32(&bad, NULL, DEVF, F, F, 0, 0, NULL, DEVF, F, NULL, DEV, ab, 7, NULL));
  bad = g;
  bad.n_ids = 5;
  REJECT("n_ids", mp_aggregate_f32(&bad, NULL, DEVF, F, F, 0, 0, NULL, DEVF, F, NULL, DEV, ab, 7, NULL));
  bad = g;
  bad.eid = NULL;
  REJECT("eid", mp_aggregate_f32(&bad, NULL, DEVF, F, F, 0, 0, NULL, DEVF, F, NULL, DEV, ab, 7, NULL));
  bad = g;
  bad.n_split = 3;
  bad.split_waves = NULL;
  REJECT("null arrays", mp_aggregate_f32(&bad, NULL, DEVF, F, F, 0, 0, NULL, DEVF, F, NULL, DEV, ab, 7, NULL));
  char name[64];
  REJECT("bad arguments", mp_aggregate_kernel_name(&g, NULL, DEVF, F, F, 0, NULL, DEVF, F, NULL, 0, NULL));
  REJECT("unknown reduce", mp_aggregate_kernel_name(&g, NULL, DEVF, F, F, 9, NULL, DEVF, F, name, sizeof name, NULL));
  REJECT("slab", mp_aggregate_heads_f32(&g, DEVF, 8, DEVF, F, F, DEVF, F, DEV, ab - 1, 7, NULL));
  REJECT("multiple of H", mp_aggregate_heads_f32(&g, DEVF, 7, DEVF, F, F, DEVF, F, DEV, ab, 7, NULL));

  const int H = 8, C = 32;
  const size_t gs = mp_gat_slab_bytes(&g, H, C), ts = mp_gat_train_slab_bytes(&g, H, C);
  REJECT("slab", mp_gat_aggregate_f32(&g, DEVF, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, DEVF, DEV, gs - 1, 7, NULL));
  REJECT("null", mp_gat_aggregate_att_f32(&g, DEVF, NULL, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, DEVF, DEV, gs, 7,
                                          NULL));
  REJECT("slab", mp_gat_forward_f32(&g, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, DEVF, DEVF, DEVF, DEV, gs - 1, 7,
                                    NULL));
  REJECT("power of two", mp_gat_forward_f32(&g, DEVF, DEVF, H, 36, 0.2f, NULL, DEVF, F, DEVF, DEVF, DEVF, DEV, gs, 7,
                                            NULL));
  mp_csr rect = graph(N, E, (int32_t)(N + 10));
  REJECT("square", mp_gat_forward_f32(&rect, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, DEVF, DEVF, DEVF, DEV, gs, 7,
                                      NULL));
  REJECT("slab", mp_gat_aggregate_train_f32(&g, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, NULL, DEVF, DEVF,
                                            DEVF, DEV, gs, 7, NULL));
  /* ABI 6: a bias no longer needs the pre-bias copy (the backward takes out - bias) */
  ACCEPT(mp_gat_aggregate_train_f32(&g, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, DEVF, F, NULL, DEVF, DEVF, DEVF,
                                    DEV, ts, 7, NULL));
  REJECT("16-byte", mp_gat_aggregate_train_f32(&g, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, (float*)((char*)DEV + 4), DEVF,
                                               F, NULL, DEVF, DEVF, DEVF, DEV, ts, 7, NULL));
  REJECT("bias", mp_gat_backward_prep_train_f32(DEVF, F, DEVF, F, (float*)((char*)DEV + 8), DEVF, DEVF, DEVF, DEVF,
                                                N, H, C, DEVF, (size_t)N * H * 16, NULL, 0, DEVF, NULL));
  ACCEPT(mp_gat_aggregate_train_f32(&g, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, DEVF, DEVF, F, DEVF, DEVF, DEVF, DEVF,
                                    DEV, ts, 7, NULL));
  REJECT("null", mp_gat_forward_train_f32(&g, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, NULL, DEVF, DEVF, DEVF, NULL,
                                          DEVF, DEV, ts, 7, NULL));
  REJECT("dropout p", mp_gat_aggregate_train_drop_f32(&g, DEVF, DEVF, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, NULL,
                                                       DEVF, DEVF, DEVF, 1, 0.f, NULL, DEV, ts, 7, NULL));
  REJECT("H <= 32", mp_gat_aggregate_train_drop_f32(&g, DEVF, DEVF, DEVF, DEVF, 64, 4, 0.2f, NULL, DEVF, F, NULL,
                                                     DEVF, DEVF, DEVF, 1, 0.5f, NULL, DEV, ts, 7, NULL));
  REJECT("H <= 16", mp_gat_softmax_aggregate_f32(&g, DEVI, DEVF, DEVF, DEVF, 32, 8, 0.2f, NULL, DEVF, F, DEVF, DEV,
                                                  gs, 7, NULL));
  REJECT("slab", mp_gat_softmax_aggregate_f32(&g, DEVI, DEVF, DEVF, DEVF, H, C, 0.2f, NULL, DEVF, F, DEVF, DEV,
                                               gs - 1, 7, NULL));

  const size_t lws = mp_self_loops_workspace(E, N);
  REJECT(NULL, mp_self_loops(DEVL, DEVL, E, N, MP_LOOPS_ADD_REMAINING, E, DEVL, DEVL, DEVL, DEV, lws - 1, NULL));
  ACCEPT(mp_self_loops(DEVL, DEVL, E, N, MP_LOOPS_ADD_REMAINING, E, DEVL, DEVL, DEVL, DEV, lws, NULL));
  REJECT(NULL, mp_self_loops(DEVL, DEVL, E, N, 7, E, DEVL, DEVL, DEVL, DEV, lws, NULL));
  const size_t pws = mp_shard_plan_workspace(E, N);
  REJECT(NULL, mp_shard_plan(DEVL, DEVL, E, N, DEVL, 4, 1, 100, 200, DEVL, DEVL, DEVL, DEVL, DEVL, DEV, pws - 1,
                             NULL));
  REJECT(NULL, mp_shard_plan(DEVL, DEVL, E, N, DEVL, 4, 4, 100, 200, DEVL, DEVL, DEVL, DEVL, DEVL, DEV, pws, NULL));
  ACCEPT(mp_shard_plan(DEVL, DEVL, E, N, DEVL, 4, 1, 100, 200, DEVL, DEVL, DEVL, DEVL, DEVL, DEV, pws, NULL));
}

static void null_pointers(void) {
  /* every other entry point: one required pointer NULL with work to do */
  const int64_t n = 1000, E = 4000;
  mp_csr g = graph(n, E, (int32_t)n);
  REJECT("null", mp_gat_node_scores_f32(NULL, n, 8, 32, DEVF, DEVF, DEVF, NULL));
  REJECT("null", mp_gat_node_scores_wide_f32(DEVF, n, 8, 36, DEVF, NULL, DEVF, NULL));
  REJECT("null", mp_csr_slot_rows(&g, NULL, NULL));
  REJECT("null", mp_gat_alpha_csr_f32(&g, NULL, DEVF, DEVF, 8, 0.2f, DEVF, DEVF, NULL, NULL));
  REJECT("null", mp_gat_sddmm_f32(&g, DEVI, DEVF, 256, NULL, 256, 8, 32, DEVF, NULL));
  REJECT("leading dimension", mp_gat_sddmm_f32(&g, DEVI, DEVF, 255, DEVF, 256, 8, 32, DEVF, NULL));
  REJECT("null", mp_segment_offset_i64(NULL, n, 2, n, DEVL, DEVL, 3, NULL));
  REJECT("null", mp_segment_ids_i64(NULL, n, DEVL, 3, NULL));
  REJECT("null", mp_gat_dropout_keep(1, 0.5f, 8, E, NULL, NULL, NULL));
  REJECT("dropout p", mp_gat_dropout_keep(1, 1.0f, 8, E, NULL, DEVU, NULL));
  const size_t po = 10 * 256 * 4, ps = 10 * 8 * 2 * 4;  /* part_out / part_stats of 10 pieces */
  REJECT("C % 4", mp_gat_merge_partials_f32(n, 8, 30, DEVI, DEVI, 10, DEVF, po, 256, DEVF, ps, NULL, DEVF, 256, DEVF,
                                            NULL, NULL, NULL));
  REJECT("null", mp_gat_merge_partials_f32(n, 8, 32, DEVI, NULL, 10, DEVF, po, 256, DEVF, ps, NULL, DEVF, 256, DEVF,
                                           NULL, NULL, NULL));
  REJECT("leading dimension", mp_gat_merge_partials_f32(n, 8, 32, DEVI, DEVI, 10, DEVF, po, 255, DEVF, ps, NULL,
                                                        DEVF, 256, DEVF, NULL, NULL, NULL));
  REJECT("16-byte", mp_gat_merge_partials_f32(n, 8, 32, DEVI, DEVI, 10, DEVF, po, 256, DEVF, ps,
                                              (float*)((char*)DEV + 4), DEVF, 256, DEVF, NULL, NULL, NULL));
  ACCEPT(mp_gat_merge_partials_f32(n, 8, 32, DEVI, NULL, 0, NULL, 0, 0, NULL, 0, NULL, DEVF, 256, DEVF, NULL, NULL,
                                   NULL));
  REJECT("bad argument", mp_heads_outer_add_f32(DEVF, 256, NULL, n, 8, 32, DEVF, 64, NULL));
  REJECT("bad argument", mp_gat_alpha_f32(DEVL, NULL, E, 8, DEVF, DEVF, 0.2f, DEVF, DEVF, NULL));
  REJECT("bad arguments", mp_self_loop_count(NULL, DEVL, E, n, DEVL, NULL));
  REJECT("bad arguments", mp_gather_fill_f32(DEVF, NULL, E, 1.f, DEVF, NULL));
  REJECT("bad source", mp_segment_reduce(&g, MP_DTYPE_F64, NULL, 16, 16, MP_REDUCE_SUM, 0, DEV, 16, NULL, NULL));
  REJECT("dtype", mp_segment_reduce(&g, 9, DEV, 16, 16, MP_REDUCE_SUM, 0, DEV, 16, NULL, NULL));
  REJECT("element size", mp_gather_rows_any(3, DEV, 16, DEVL, n, 16, DEV, 16, NULL));
  REJECT("bad argument", mp_scatter_arg_any(8, DEV, NULL, n, 16, E, DEV, 16, NULL));
  REJECT("null", mp_gather_rows_f32(DEVF, 16, NULL, n, 16, DEVF, 16, NULL));
  REJECT("bad argument", mp_permute_f32(DEVF, NULL, E, DEVF, NULL));
  REJECT("null", mp_segment_sum_serial_f32(NULL, DEVI, DEVF, n, DEVF, NULL));
  REJECT("null", mp_gcn_norm_from_deg_f32(DEVL, NULL, DEVF, E, n, DEVF, DEVF, NULL));
  REJECT("null", mp_gcn_norm_f32(DEVL, DEVL, NULL, E, n, NULL, DEVF, NULL));
  REJECT("null", mp_csr_inverse_eid(&g, NULL, NULL));
  REJECT("null", mp_scatter_arg_backward_f32(DEVF, NULL, n, 16, E, DEVF, 16, NULL));
}

int main(void) {
  if (mp_abi_version() != MP_ABI_VERSION) {
    printf("FAIL abi version %d != header %d\n", mp_abi_version(), MP_ABI_VERSION);
    return 2;
  }
  extents_gat_backward();
  extents_arg_backward();
  abi7();
  workspaces();
  null_pointers();
  printf("abi_reject: %d cases, %d failures\n", n_cases, n_fail);
  return n_fail ? 1 : 0;
}
