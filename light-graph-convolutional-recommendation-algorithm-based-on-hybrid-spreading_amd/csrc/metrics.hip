// K5: recommendation-list metrics on the device.
//
// Reference (pure Python loops over users, pairs of users and pairs of items):
//   metrics/accurate.py:11-46   calPrecisionAndRecall  hit[u][p] = recs[u][p] in test(u)
//   metrics/accurate.py:58-102  calNDCG                dcg = sum_p hit_p / log2(p + 2)
//   metrics/diversity.py:15-63  calHammingDistance     mean over ordered user pairs u != v of
//                                                      1 - |set(R_u) & set(R_v)| / k
//   metrics/diversity.py:66-115 calInternalSimilarity  sum over users and ordered pairs of
//                                                      distinct items (i, j) of the user's
//                                                      list, both of nonzero degree, of
//                                                      co(i, j) / sqrt(k_i * k_j)
// What runs here:
//   * hit flags: one thread per (evaluated user, position), a binary search of the entry in
//     the user's sorted test row (the reference's `item in items` over a Python list).
//   * Hamming: the O(U^2 k) pair loop collapses exactly: sum_{u != v} |R_u & R_v| =
//     sum_i c_i (c_i - 1) with c_i = number of (de-duplicated) lists holding item i, an
//     integer histogram (integer atomics: order-free, exact) and one integer sum.
//   * internal similarity: one wave per (list, position p): item a's user column
//     (co-occurrence = |users(a) & users(b)| over the binary interaction matrix) is staged
//     in LDS once and every later position q > p intersects against it (lanes take 64
//     entries of the shorter column and binary-search the longer); each unordered pair is
//     computed once (s_ab == s_ba bit for bit) with the reference's per-term arithmetic
//     fl(co / fl(sqrt(k_a * k_b))).
#include "common.h"

namespace lg {

constexpr int kSimStage = 2048;  // users of item a staged in LDS (ints per wave)

__global__ __launch_bounds__(256) void k_rec_hits(const int64_t *__restrict__ recs, int k,
                                                  const int64_t *__restrict__ eval_rows,
                                                  int64_t n_eval,
                                                  const int64_t *__restrict__ pos_rowptr,
                                                  const int32_t *__restrict__ pos_col,
                                                  uint8_t *__restrict__ hit) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_eval * k) return;
  const int64_t q = t / k;
  const int p = (int)(t - q * k);
  const int64_t u = eval_rows[q];
  const int64_t it = recs[u * k + p];
  bool h = false;
  if (it >= 0 && it <= 0x7fffffff) {
    const int64_t lo = pos_rowptr[q], hi = pos_rowptr[q + 1];
    const int64_t at = lower_bound_i32(pos_col, lo, hi, (int32_t)it);
    h = at < hi && pos_col[at] == (int32_t)it;
  }
  hit[t] = h;
}

// c_i += 1 for every distinct item of every list (entries < 0 or >= n_items are skipped).
__global__ __launch_bounds__(256) void k_rec_item_counts(const int64_t *__restrict__ recs,
                                                         int64_t n_rows, int k, int64_t n_items,
                                                         int32_t *__restrict__ counts) {
  const int64_t r = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (r >= n_rows) return;
  const int lane = lane_id();
  const int64_t *row = recs + r * k;
  for (int p = lane; p < k; p += 64) {
    const int64_t it = row[p];
    if (it < 0 || it >= n_items) continue;
    bool first = true;
    for (int q = 0; q < p; ++q) first &= row[q] != it;
    if (first) atomicAdd(&counts[it], 1);
  }
}

__global__ __launch_bounds__(256) void k_pair_overlap(const int32_t *__restrict__ counts,
                                                      int64_t n_items,
                                                      unsigned long long *__restrict__ total) {
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = (unsigned long long)counts[i];
    s += c * (c - (c > 0 ? 1ull : 0ull));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane_id() == 0 && s) atomicAdd(total, s);
}

// true if x is in the sorted LDS list s[0..n)
__device__ __forceinline__ bool lds_contains(const int32_t *s, int n, int32_t x) {
  int a = 0, b = n;
  while (a < b) {
    const int mid = (a + b) >> 1;
    if (s[mid] < x) a = mid + 1;
    else b = mid;
  }
  return a < n && s[a] == x;
}

__global__ __launch_bounds__(256) void k_rec_intra_similarity(
    const int64_t *__restrict__ recs, int64_t n_rows, int k,
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int64_t *__restrict__ item_degree, int64_t n_items, double *__restrict__ part) {
  __shared__ int32_t stage[4][kSimStage];
  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int64_t t = (int64_t)blockIdx.x * 4 + wave;  // (row, position)
  if (t >= n_rows * k) return;
  const int64_t r = t / k;
  const int p = (int)(t - r * k);
  const int64_t *row = recs + r * k;
  const int64_t a = row[p];
  const int64_t ka = (a >= 0 && a < n_items) ? item_degree[a] : 0;
  double s = 0.0;
  if (ka > 0) {
    const int64_t a0 = item_rowptr[a], a1 = item_rowptr[a + 1];
    const int64_t na = a1 - a0;
    const bool staged = na <= kSimStage;
    if (staged) {
      for (int e = lane; e < na; e += 64) stage[wave][e] = item_users[a0 + e];
      wave_sync();
    }
    for (int q = p + 1; q < k; ++q) {
      const int64_t b = row[q];
      if (b == a || b < 0 || b >= n_items) continue;
      const int64_t kb = item_degree[b];
      if (kb <= 0) continue;
      const int64_t b0 = item_rowptr[b], b1 = item_rowptr[b + 1];
      const int64_t nb = b1 - b0;
      int64_t co = 0;
      if (staged && nb <= na) {
        // b's column is the shorter: its entries (coalesced) against a's LDS copy
        for (int64_t e0 = 0; e0 < nb; e0 += 64) {
          const int64_t e = e0 + lane;
          const bool in = e < nb && lds_contains(stage[wave], (int)na, item_users[b0 + e]);
          co += __popcll(__ballot(in));
        }
      } else {
        // the shorter column's entries binary-searched in the longer one in global memory
        const bool a_short = na <= nb;
        const int64_t s0 = a_short ? a0 : b0, s1 = a_short ? a1 : b1;
        const int64_t l0 = a_short ? b0 : a0, l1 = a_short ? b1 : a1;
        for (int64_t e0 = s0; e0 < s1; e0 += 64) {
          const int64_t e = e0 + lane;
          bool in = false;
          if (e < s1) {
            const int32_t x = (staged && a_short) ? stage[wave][e - a0] : item_users[e];
            const int64_t at = lower_bound_i32(item_users, l0, l1, x);
            in = at < l1 && item_users[at] == x;
          }
          co += __popcll(__ballot(in));
        }
      }
      // reference: common / np.sqrt(k_i * k_j), the degree product exact in integers
      s += (double)co / sqrt((double)(ka * kb));
    }
  }
  if (lane == 0) part[t] = s;
}

}  // namespace lg

using namespace lg;

extern "C" int lg_rec_hits(const int64_t *recs, int64_t n_rows, int32_t k,
                           const int64_t *eval_rows, int64_t n_eval, const int64_t *pos_rowptr,
                           const int32_t *pos_col, uint8_t *hit, lg_stream_t stream) {
  LG_REQUIRE(n_rows >= 0 && n_eval >= 0 && k >= 1, "lg_rec_hits: bad sizes (k=%d)", k);
  LG_REQUIRE(n_eval == 0 || (recs && eval_rows && pos_rowptr && hit),
             "lg_rec_hits: NULL argument");
  const int64_t n = n_eval * k;
  if (n == 0) return LG_OK;
  k_rec_hits<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream>>>(
      recs, k, eval_rows, n_eval, pos_rowptr, pos_col, hit);
  return launch_status("lg_rec_hits");
}

extern "C" int lg_rec_pair_overlap(const int64_t *recs, int64_t n_rows, int32_t k,
                                   int64_t n_items, int32_t *counts, uint64_t *total,
                                   lg_stream_t stream) {
  LG_REQUIRE(n_rows >= 0 && n_items >= 0 && k >= 1, "lg_rec_pair_overlap: bad sizes (k=%d)",
             k);
  LG_REQUIRE(total && (n_items == 0 || counts) && (n_rows == 0 || recs),
             "lg_rec_pair_overlap: NULL argument");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(total, 0, sizeof(uint64_t), s) != hipSuccess ||
      (n_items && hipMemsetAsync(counts, 0, (size_t)n_items * sizeof(int32_t), s) != hipSuccess)) {
    set_error("lg_rec_pair_overlap: hipMemsetAsync failed");
    return LG_ERR_HIP;
  }
  if (n_rows == 0 || n_items == 0) return launch_status("lg_rec_pair_overlap");
  k_rec_item_counts<<<dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, s>>>(recs, n_rows, k,
                                                                            n_items, counts);
  const int64_t want = (n_items + 255) / 256;
  const unsigned blocks = (unsigned)(want < 2048 ? want : 2048);
  k_pair_overlap<<<dim3(blocks), dim3(256), 0, s>>>(counts, n_items,
                                                    (unsigned long long *)total);
  return launch_status("lg_rec_pair_overlap");
}

extern "C" int lg_rec_intra_similarity_f64(const int64_t *recs, int64_t n_rows, int32_t k,
                                           const int64_t *item_rowptr,
                                           const int32_t *item_users,
                                           const int64_t *item_degree, int64_t n_items,
                                           double *part, lg_stream_t stream) {
  LG_REQUIRE(n_rows >= 0 && n_items >= 0 && k >= 1,
             "lg_rec_intra_similarity_f64: bad sizes (k=%d)", k);
  LG_REQUIRE(n_rows == 0 || (recs && part && (n_items == 0 || (item_rowptr && item_degree))),
             "lg_rec_intra_similarity_f64: NULL argument");
  const int64_t n = n_rows * k;
  if (n == 0) return LG_OK;
  k_rec_intra_similarity<<<dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream>>>(
      recs, n_rows, k, item_rowptr, item_users, item_degree, n_items, part);
  return launch_status("lg_rec_intra_similarity_f64");
}
