/*
 * Serial restatement of torch_scatter 2.0.4 csrc/cpu/scatter_cpu.cpp (+ its
 * reducer.h update rule) for the layout the hot path uses: src [E, F]
 * row-major, 1-D index [E] along dim 0, out [N, F].   TEST INFRASTRUCTURE.
 *
 *   out initialised to 0 (sum/mean), lowest() (max) or max() (min) unless
 *   `has_out`; arg initialised to E (= src.size(dim)).
 *   for e in [0,E): for k in [0,F): update(out[index[e],k], src[e,k], arg, e)
 *     sum/mean: out += v ; max: if (v > out) {out = v; arg = e} ; min: v < out
 *   mean: out /= max(count, 1) ; max/min (no `out` given): out == init -> 0
 *
 * oracle_gather_sum_f32 is the materialised GCN message + scatter_add_:
 *   out[index[e],k] += (w[e] * x[other[e],k])   (product rounded first).
 * Compile with -ffp-contract=off (oracle/Makefile) so no FMA is formed.
 */
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { R_SUM = 0, R_MEAN = 1, R_MAX = 2, R_MIN = 3 };

void oracle_scatter_f32(const float* src, const int64_t* index, int64_t E, int64_t F, int64_t N,
                        int reduce, int has_out, float* out, int64_t* arg) {
  if (!has_out) {
    float init = reduce == R_MAX ? -FLT_MAX : (reduce == R_MIN ? FLT_MAX : 0.f);
    for (int64_t i = 0; i < N * F; ++i) out[i] = init;
  }
  if (arg)
    for (int64_t i = 0; i < N * F; ++i) arg[i] = E;
  for (int64_t e = 0; e < E; ++e) {
    const int64_t r = index[e];
    const float* s = src + e * F;
    float* o = out + r * F;
    if (reduce == R_SUM || reduce == R_MEAN) {
      for (int64_t k = 0; k < F; ++k) o[k] = o[k] + s[k];
    } else if (reduce == R_MAX) {
      for (int64_t k = 0; k < F; ++k)
        if (s[k] > o[k]) { o[k] = s[k]; arg[r * F + k] = e; }
    } else {
      for (int64_t k = 0; k < F; ++k)
        if (s[k] < o[k]) { o[k] = s[k]; arg[r * F + k] = e; }
    }
  }
  if (reduce == R_MEAN) {
    float* cnt = (float*)calloc((size_t)(N > 0 ? N : 1), sizeof(float));
    for (int64_t e = 0; e < E; ++e) cnt[index[e]] += 1.f;
    for (int64_t r = 0; r < N; ++r) {
      float c = cnt[r] < 1.f ? 1.f : cnt[r];
      for (int64_t k = 0; k < F; ++k) out[r * F + k] = out[r * F + k] / c;
    }
    free(cnt);
  }
  if ((reduce == R_MAX || reduce == R_MIN) && !has_out) {
    float init = reduce == R_MAX ? -FLT_MAX : FLT_MAX;
    for (int64_t i = 0; i < N * F; ++i)
      if (out[i] == init) out[i] = 0.f;
  }
}

void oracle_gather_sum_f32(const float* x, const int64_t* other, const int64_t* index, const float* w,
                           int64_t E, int64_t F, int64_t N, float* out) {
  memset(out, 0, sizeof(float) * (size_t)(N * F));
  for (int64_t e = 0; e < E; ++e) {
    const float* xs = x + other[e] * F;
    float* o = out + index[e] * F;
    const float we = w ? w[e] : 1.f;
    for (int64_t k = 0; k < F; ++k) {
      float m = w ? we * xs[k] : xs[k];
      o[k] = o[k] + m;
    }
  }
}

/* max over gathered rows (GraphConv/SAGE-style message x_j, no materialisation):
 * value and arg exactly as oracle_scatter_f32(R_MAX) on src = x[other]. */
void oracle_gather_max_f32(const float* x, const int64_t* other, const int64_t* index, int64_t E,
                           int64_t F, int64_t N, float* out, int64_t* arg) {
  for (int64_t i = 0; i < N * F; ++i) { out[i] = -FLT_MAX; arg[i] = E; }
  for (int64_t e = 0; e < E; ++e) {
    const float* xs = x + other[e] * F;
    const int64_t r = index[e];
    float* o = out + r * F;
    for (int64_t k = 0; k < F; ++k)
      if (xs[k] > o[k]) { o[k] = xs[k]; arg[r * F + k] = e; }
  }
  for (int64_t i = 0; i < N * F; ++i)
    if (out[i] == -FLT_MAX) out[i] = 0.f;
}
