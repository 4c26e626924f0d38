/*
 * spmm_ref.c -- TEST ORACLE / CPU BASELINE ONLY (see oracle/__init__.py).
 *
 * Plain-C restatement of the fused applyedge MUL -> gather ADD block of the
 * GTA stream (hardware_info.yaml Inst_fused [applyedge,gather] [MUL,ADD];
 * reference code/interpreter.py:575-636 fuses it, :764-802 removes the
 * scatter FETCH):   y[i, c] = sum_{e in row i} w[e, c / (F/heads)] * x[indices[e], c]
 * over a destination-sorted CSR, fp32 accumulation in edge order, OpenMP over
 * rows.  bench.py times it on the GPU box's host cores as `cpu_baseline`
 * ("kind": "port"); tests use it as a second, independent CPU check.
 * Built by oracle/Makefile (gcc), never linked into libgta.
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void oracle_aggregate_f32(const int64_t* indptr, const int32_t* indices, int64_t row_begin, int64_t row_end,
                          const float* x, int64_t ldx, int64_t F, const float* w, int64_t ldw, int64_t heads,
                          float* y, int64_t ldy, int threads) {
  const int64_t g = (w && heads > 0) ? F / heads : 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
#endif
  for (int64_t r = row_begin; r < row_end; ++r) {
    float* yr = y + (r - row_begin) * ldy;
    memset(yr, 0, (size_t)F * sizeof(float));
    for (int64_t e = indptr[r]; e < indptr[r + 1]; ++e) {
      const float* xr = x + (int64_t)indices[e] * ldx;
      if (w) {
        const float* we = w + e * ldw;
        for (int64_t c = 0; c < F; ++c) yr[c] += we[c / g] * xr[c];
      } else {
        for (int64_t c = 0; c < F; ++c) yr[c] += xr[c];
      }
    }
  }
}

/* head-blocked fast path for F % heads == 0 (the metric's 8 heads x 16) */
void oracle_aggregate_heads_f32(const int64_t* indptr, const int32_t* indices, int64_t row_begin, int64_t row_end,
                                const float* x, int64_t ldx, int64_t F, const float* w, int64_t ldw,
                                int64_t heads, float* y, int64_t ldy, int threads) {
  const int64_t g = F / heads;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
#endif
  for (int64_t r = row_begin; r < row_end; ++r) {
    float* yr = y + (r - row_begin) * ldy;
    memset(yr, 0, (size_t)F * sizeof(float));
    for (int64_t e = indptr[r]; e < indptr[r + 1]; ++e) {
      const float* xr = x + (int64_t)indices[e] * ldx;
      const float* we = w + e * ldw;
      for (int64_t h = 0; h < heads; ++h) {
        const float a = we[h];
        const float* xs = xr + h * g;
        float* ys = yr + h * g;
        for (int64_t c = 0; c < g; ++c) ys[c] += a * xs[c];
      }
    }
  }
}
