/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
 * cpu_baseline). Never linked into or called by the product path.
 *
 * Plain-C restatement of the reference's e0 scoring + masked top-k
 * (model/LightGCN/recommend.py:83-114; same code at LightGCNOpti/recommend.py:83-114 and
 * LightGCN/evaluation.py:31-51):
 *     score = e0_u @ e0_i^T ; score[train|val positives] = -(1 << 10) ; topk(score, k)
 * with the score of one (u, i) pair fixed to the fp32 fused-multiply-add chain
 *     acc = 0; for s < d/4: for g < 4: acc = fmaf(u[g*d/4+s], i[g*d/4+s], acc)
 * (the element order the library's MFMA kernel uses, include/lgcnhs.h) so the GPU result
 * can be checked bit for bit, and ties broken by (score desc, item asc). The reference's
 * own fp32 matmul rounds in a BLAS-dependent order; tests compare against it tie-aware.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -mfma: fmaf is the hardware fused
 * multiply-add, one rounding, the same result as libm's). Users are independent: both entry
 * points split the user range over ORACLE_THREADS (default: the online CPUs, at most 16)
 * pthreads; each user's result is computed by exactly one thread in the order above.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

float oracle_chain_score(const float *u, const float *it, int d) {
  const int q = d / 4;
  float acc = 0.0f;
  for (int s = 0; s < q; ++s)
    for (int g = 0; g < 4; ++g) acc = fmaf(u[g * q + s], it[g * q + s], acc);
  return acc;
}

/* run fn(arg, u0, u1) over [0, nu) in contiguous user ranges, one pthread each */
typedef void (*user_range_fn)(void *arg, int64_t u0, int64_t u1);
struct range_job { user_range_fn fn; void *arg; int64_t u0, u1; };
static void *range_main(void *p) {
  struct range_job *j = (struct range_job *)p;
  j->fn(j->arg, j->u0, j->u1);
  return NULL;
}
static void for_user_ranges(int64_t nu, user_range_fn fn, void *arg) {
  long t = sysconf(_SC_NPROCESSORS_ONLN);
  const char *e = getenv("ORACLE_THREADS");
  if (e && atoi(e) > 0) t = atoi(e);
  if (t > 16) t = 16;
  if (t > nu) t = (long)nu;
  if (t <= 1) { fn(arg, 0, nu); return; }
  pthread_t th[16];
  struct range_job jobs[16];
  int started[16] = {0};
  for (long w = 0; w < t; ++w) {
    jobs[w].fn = fn; jobs[w].arg = arg;
    jobs[w].u0 = nu * w / t; jobs[w].u1 = nu * (w + 1) / t;
    started[w] = pthread_create(&th[w], NULL, range_main, &jobs[w]) == 0;
    if (!started[w]) range_main(&jobs[w]);  /* (no thread: run it here) */
  }
  for (long w = 0; w < t; ++w)
    if (started[w]) pthread_join(th[w], NULL);
}

struct matrix_args { const float *eu, *ei; int64_t ni; int d; float *out; };
static void matrix_range(void *p, int64_t u0, int64_t u1) {
  const struct matrix_args *a = (const struct matrix_args *)p;
  for (int64_t u = u0; u < u1; ++u)
    for (int64_t b = 0; b < a->ni; ++b)
      a->out[u * a->ni + b] = oracle_chain_score(a->eu + u * a->d, a->ei + b * a->d, a->d);
}

void oracle_score_matrix(const float *eu, const float *ei, int64_t nu, int64_t ni, int d,
                         float *out) {
  struct matrix_args a = {eu, ei, ni, d, out};
  for_user_ranges(nu, matrix_range, &a);
}

/* (a before b) in output order */
static int better(float va, int64_t ia, float vb, int64_t ib) {
  return va > vb || (va == vb && ia < ib);
}

/* min-heap of the current best k by the "better" order (root = worst kept) */
static void sift_down(float *hv, int64_t *hi, int n, int p) {
  for (;;) {
    int l = 2 * p + 1, r = l + 1, w = p;
    if (l < n && better(hv[w], hi[w], hv[l], hi[l])) w = l;
    if (r < n && better(hv[w], hi[w], hv[r], hi[r])) w = r;
    if (w == p) return;
    float tv = hv[p]; hv[p] = hv[w]; hv[w] = tv;
    int64_t ti = hi[p]; hi[p] = hi[w]; hi[w] = ti;
    p = w;
  }
}

static void heap_push_topk(float *hv, int64_t *hi, int *n, int k, float v, int64_t i) {
  if (*n < k) {
    int c = (*n)++;
    hv[c] = v; hi[c] = i;
    while (c > 0) {
      int p = (c - 1) / 2;
      if (better(hv[p], hi[p], hv[c], hi[c])) {
        float tv = hv[p]; hv[p] = hv[c]; hv[c] = tv;
        int64_t ti = hi[p]; hi[p] = hi[c]; hi[c] = ti;
        c = p;
      } else break;
    }
  } else if (better(v, i, hv[0], hi[0])) {
    hv[0] = v; hi[0] = i;
    sift_down(hv, hi, *n, 0);
  }
}

static void heap_sorted(float *hv, int64_t *hi, int n, float *ov, int64_t *oi, int k) {
  /* pop worst first into the tail */
  int m = n;
  while (m > 0) {
    ov[m - 1] = hv[0]; oi[m - 1] = hi[0];
    hv[0] = hv[m - 1]; hi[0] = hi[m - 1];
    --m;
    sift_down(hv, hi, m, 0);
  }
  for (int e = n; e < k; ++e) { ov[e] = -INFINITY; oi[e] = -1; }
}

/* excluded(u, i): binary search in the sorted exclusion row */
static int is_excluded(const int64_t *rp, const int32_t *col, int64_t u, int64_t i) {
  if (!rp) return 0;
  int64_t lo = rp[u], hi = rp[u + 1];
  while (lo < hi) {
    int64_t mid = lo + (hi - lo) / 2;
    if (col[mid] < i) lo = mid + 1; else hi = mid;
  }
  return lo < rp[u + 1] && col[lo] == i;
}

struct topk_args {
  const float *eu, *ei; int64_t ni; int d;
  const int64_t *ex_rowptr; const int32_t *ex_col; float mask_value; int k;
  float *out_val; int64_t *out_idx; int failed;
};
static void topk_range(void *p, int64_t u0, int64_t u1) {
  struct topk_args *a = (struct topk_args *)p;
  float *hv = (float *)malloc(sizeof(float) * (size_t)a->k);
  int64_t *hi = (int64_t *)malloc(sizeof(int64_t) * (size_t)a->k);
  if (!hv || !hi) { free(hv); free(hi); a->failed = 1; return; }
  for (int64_t u = u0; u < u1; ++u) {
    int n = 0;
    for (int64_t i = 0; i < a->ni; ++i) {
      float v = oracle_chain_score(a->eu + u * a->d, a->ei + i * a->d, a->d);
      if (is_excluded(a->ex_rowptr, a->ex_col, u, i)) v = a->mask_value;
      heap_push_topk(hv, hi, &n, a->k, v, i);
    }
    heap_sorted(hv, hi, n, a->out_val + u * a->k, a->out_idx + u * a->k, a->k);
  }
  free(hv); free(hi);
}

int oracle_score_topk(const float *eu, const float *ei, int64_t nu, int64_t ni, int d,
                      const int64_t *ex_rowptr, const int32_t *ex_col, float mask_value,
                      int k, float *out_val, int64_t *out_idx) {
  struct topk_args a = {eu, ei, ni, d, ex_rowptr, ex_col, mask_value, k, out_val, out_idx, 0};
  for_user_ranges(nu, topk_range, &a);
  return a.failed;
}
