/*
 * mas_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * CPU restatement of monotonic alignment search as the reference calls it:
 *   call site   emotional-vits/models.py:498
 *               attn = monotonic_align.maximum_path(neg_cent, attn_mask.squeeze(1))
 *   layout      neg_cent [b, t_t(frames), t_s(tokens)]  (models.py:486-497)
 * The `monotonic-align` PyPI package is external, unpinned (README.md:9) and
 * absent from /root/reference, so this restates its published algorithm, the
 * canonical VITS monotonic_align/core.pyx (maximum_path_each / maximum_path_c)
 * and monotonic_align/__init__.py (lengths = mask.sum(1)[:,0] / mask.sum(2)[:,0],
 * neg_cent cast to float32, path int32 zeros).  No reference test or fixture
 * covers it: parity is pinned by brute-force enumeration of all monotone
 * alignments in tests/test_oracle.py (max score + the strict '<' tie rule),
 * see DESIGN.md "Oracle".
 *
 * Only the test suite, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load this file's library.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static void maximum_path_each(int32_t* path, float* value, int t_y, int t_x, int T_x) {
  const float max_neg_val = -1e9f;
  int index = t_x - 1;
  for (int y = 0; y < t_y; ++y) {
    int lo = t_x + y - t_y;
    if (lo < 0) lo = 0;
    int hi = y + 1 < t_x ? y + 1 : t_x;
    for (int x = lo; x < hi; ++x) {
      float v_cur, v_prev;
      if (x == y)
        v_cur = max_neg_val;
      else
        v_cur = value[(y - 1) * T_x + x];
      if (x == 0) {
        if (y == 0)
          v_prev = 0.f;
        else
          v_prev = max_neg_val;
      } else {
        v_prev = value[(y - 1) * T_x + x - 1];
      }
      /* Cython max(v_prev, v_cur) lowers to (v_cur > v_prev) ? v_cur : v_prev */
      float m = (v_cur > v_prev) ? v_cur : v_prev;
      value[y * T_x + x] = value[y * T_x + x] + m;
    }
  }
  for (int y = t_y - 1; y >= 0; --y) {
    if (index >= 0 && index < T_x) path[y * T_x + index] = 1;
    if (index != 0) {
      int dec = (index == y);
      if (!dec && y >= 1 && index >= 1)
        dec = value[(y - 1) * T_x + index] < value[(y - 1) * T_x + index - 1];
      if (dec) index = index - 1;
    }
  }
}

/* paths [B][T_y][T_x] int32 (zeroed here), values [B][T_y][T_x] float32 (modified
 * in place, callers pass a copy), t_ys/t_xs [B]. */
void mas_oracle_maximum_path(int32_t* paths, float* values, const int32_t* t_ys,
                             const int32_t* t_xs, int B, int T_y, int T_x) {
  memset(paths, 0, sizeof(int32_t) * (size_t)B * T_y * T_x);
  for (int b = 0; b < B; ++b) {
    maximum_path_each(paths + (size_t)b * T_y * T_x, values + (size_t)b * T_y * T_x, t_ys[b],
                      t_xs[b], T_x);
  }
}

/* The same, the batch spread over `threads` OpenMP threads (one utterance's
 * DP per task): the CPU baseline of the GPU MAS kernel in bench.py's
 * kernels leg ("MAS CPU = the C++ restatement with OpenMP
 * over batch").  Bitwise the serial result. */
void mas_oracle_maximum_path_mt(int32_t* paths, float* values, const int32_t* t_ys,
                                const int32_t* t_xs, int B, int T_y, int T_x, int threads) {
  const size_t per = (size_t)T_y * T_x;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
  for (int b = 0; b < B; ++b) {
    memset(paths + (size_t)b * per, 0, sizeof(int32_t) * per);
    maximum_path_each(paths + (size_t)b * per, values + (size_t)b * per, t_ys[b], t_xs[b], T_x);
  }
}
