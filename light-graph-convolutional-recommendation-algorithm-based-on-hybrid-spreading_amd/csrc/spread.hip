// K3/K4: hybrid spreading (mass diffusion / heat conduction mix) in fp64, gfx950.
//
// Reference (model/SpreadMethod/model.py), all dense numpy fp64 on the host:
//   getSpreadingGeneralMat :14-27   k_u = A.sum(1) (0 -> 1); general_W = (A.T / k_u) @ A
//   HybridS                :63-85   k_i = A.sum(0); den = k_i^(1-l) (x) k_j^l; den==0 -> 1;
//                                    W = general_W / den
//   getResource            :88-99   F = A @ W
//   recommendForAllUser    model/SpreadMethod/recommend.py:31-50: per user
//                                    argsort(F[u])[::-1], drop train|val items, [:k]
//   G * F                  model/SpreadLightGCN/model.py:151 (fp32 G promoted to fp64)
//
// A is 0/1 and sparse, so the GEMMs are replaced by sparse row sums with a deterministic
// ascending summation order:
//   general_W[i][j] = sum_{v in users(i)} [j in items(v)] * fl(1/k_v)   (one block per i)
//   F[u][j]         = sum_{i in items(u)} W[i][j]                        (one block per u)
// which cost E*avg_deg and E*I instead of 2*U*I^2 each. Top-K over the dense rows is the
// candidate-list selection of common.h, one wave per row, 64 columns per step.
#include "common.h"

namespace lg {

__global__ __launch_bounds__(256) void k_spread_general(
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int64_t *__restrict__ user_rowptr, const int32_t *__restrict__ user_items,
    int64_t n_items, double *__restrict__ gW) {
  const int64_t i = blockIdx.x;
  double *row = gW + i * n_items;
  for (int64_t j = threadIdx.x; j < n_items; j += blockDim.x) row[j] = 0.0;
  __syncthreads();
  const int64_t eb = item_rowptr[i], ee = item_rowptr[i + 1];
  for (int64_t e = eb; e < ee; ++e) {
    const int32_t v = item_users[e];
    const int64_t pb = user_rowptr[v], pe = user_rowptr[v + 1];
    // (A.T / k_u)[i][v] = 1.0 / k_v, correctly rounded; times A[v][j] = 1 is exact.
    const double wv = 1.0 / (double)(pe - pb);
    for (int64_t p = pb + threadIdx.x; p < pe; p += blockDim.x) row[user_items[p]] += wv;
    __syncthreads();  // the next user may hit the same columns from other threads
  }
}

// The two factors of HybridS's denominator per item: alpha = k^(1-l), beta = k^l (the pow()
// calls of k_hybrid_weight).
__global__ __launch_bounds__(256) void k_hybrid_factors(const double *__restrict__ k_item,
                                                        int64_t n, double lambda,
                                                        double *__restrict__ alpha,
                                                        double *__restrict__ beta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  alpha[i] = pow(k_item[i], 1.0 - lambda);
  beta[i] = pow(k_item[i], lambda);
}

// general_W and HybridS in one pass, W = general_W / den without general_W in memory. One
// block per (item row i, range of kSpreadCols columns): the range of the row is summed in an
// LDS accumulator with the same fp64 adds in the same order as k_spread_general (users of i
// ascending, one fl(1/k_v) per item of v in the range), then written as
// fl(acc / fl(alpha_i beta_j)) (den == 0 -> 1), k_hybrid_weight's arithmetic. general_W is
// exactly symmetric, so its transposed form gives the same W. Where each user's items enter
// each range comes from a table built once (k_user_range_starts). Users are taken kSpreadG at
// a time: their row bounds and range starts, then every thread's item of each of them, are
// loaded together (one round trip per kind, not one per user), and the adds follow user by
// user (a barrier between users: two may share a column). Rows of hub items (hundreds of
// users) spread over the ranges' blocks instead of one block's chain. At the C3 shape this
// writes one I x I matrix instead of writing general_W, reading it back and writing W.
constexpr int kSpreadCols = 4096;
constexpr int kSpreadG = 8;

// starts[v][r] = the position (relative to v's row) of v's first item >= r kSpreadCols, for
// r = 0 .. n_ranges (the last: the row's length)
__global__ __launch_bounds__(256) void k_user_range_starts(const int64_t *__restrict__ user_rowptr,
                                                           const int32_t *__restrict__ user_items,
                                                           int64_t n_users, int n_ranges,
                                                           int32_t *__restrict__ starts) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n_users * (n_ranges + 1)) return;
  const int64_t v = x / (n_ranges + 1);
  const int r = (int)(x - v * (n_ranges + 1));
  const int64_t pb = user_rowptr[v], pe = user_rowptr[v + 1];
  const int64_t c = (int64_t)r * kSpreadCols;
  const int64_t p = r == n_ranges ? pe : lower_bound_i32(user_items, pb, pe, (int32_t)(c < 0x7fffffff ? c : 0x7fffffff));
  starts[x] = (int32_t)(p - pb);
}

__global__ __launch_bounds__(256) void k_spread_hybrid(
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int64_t *__restrict__ user_rowptr, const int32_t *__restrict__ user_items,
    const int32_t *__restrict__ starts, int n_ranges, int64_t n_items,
    const double *__restrict__ alpha, const double *__restrict__ beta,
    double *__restrict__ W) {
  __shared__ double acc[kSpreadCols];
  const int64_t i = blockIdx.x / n_ranges;
  const int r = (int)(blockIdx.x - i * n_ranges);
  const int64_t c0 = (int64_t)r * kSpreadCols;
  const int64_t c1 = c0 + kSpreadCols < n_items ? c0 + kSpreadCols : n_items;
  const int tid = threadIdx.x;
  for (int t = tid; t < kSpreadCols; t += blockDim.x) acc[t] = 0.0;
  __syncthreads();
  const int64_t eb = item_rowptr[i], ee = item_rowptr[i + 1];
  for (int64_t g0 = eb; g0 < ee; g0 += kSpreadG) {
    const int ng = ee - g0 < kSpreadG ? (int)(ee - g0) : kSpreadG;
    int64_t pb[kSpreadG];
    int32_t sb[kSpreadG], se[kSpreadG];
    int32_t deg[kSpreadG];
#pragma unroll
    for (int g = 0; g < kSpreadG; ++g) {
      const int32_t v = item_users[g0 + (g < ng ? g : 0)];
      pb[g] = user_rowptr[v];
      deg[g] = (int32_t)(user_rowptr[v + 1] - pb[g]);
      sb[g] = starts[(int64_t)v * (n_ranges + 1) + r];
      se[g] = starts[(int64_t)v * (n_ranges + 1) + r + 1];
    }
    int32_t x[kSpreadG];  // this thread's first item of each user in the range (-1: none)
#pragma unroll
    for (int g = 0; g < kSpreadG; ++g)
      x[g] = g < ng && sb[g] + tid < se[g] ? user_items[pb[g] + sb[g] + tid] : -1;
#pragma unroll
    for (int g = 0; g < kSpreadG; ++g) {
      if (g >= ng) break;
      const double wv = 1.0 / (double)deg[g];  // k_spread_general's fl(1/k_v)
      if (x[g] >= 0) acc[x[g] - c0] += wv;
      for (int32_t q = sb[g] + tid + (int32_t)blockDim.x; q < se[g]; q += blockDim.x)
        acc[user_items[pb[g] + q] - c0] += wv;  // (users with > 256 items in the range)
      __syncthreads();  // the next user may hit the same columns from other threads
    }
  }
  double *row = W + i * n_items;
  const double ai = alpha[i];
  for (int64_t j = c0 + tid; j < c1; j += blockDim.x) {
    double den = ai * beta[j];
    if (den == 0.0) den = 1.0;
    row[j] = acc[j - c0] / den;
  }
}

// 32x32 tiles; the transposed source is staged through LDS for coalesced reads. The
// tile's 32 row factors k_i^(1-l) and 32 column factors k_j^l are computed once per tile
// (np.power(item_degrees, 1 - Lambda) / np.power(item_degrees, Lambda)).
__global__ __launch_bounds__(256) void k_hybrid_weight(const double *__restrict__ gW,
                                                       const double *__restrict__ k_item,
                                                       double lambda, int64_t n, int transpose,
                                                       double *__restrict__ W) {
  __shared__ double tile[32][33];
  __shared__ double alpha[32], beta[32];
  const int64_t bi = blockIdx.y * 32, bj = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  if (threadIdx.x < 32) {
    const int64_t i = bi + threadIdx.x;
    alpha[threadIdx.x] = i < n ? pow(k_item[i], 1.0 - lambda) : 1.0;
  } else if (threadIdx.x < 64) {
    const int64_t j = bj + threadIdx.x - 32;
    beta[threadIdx.x - 32] = j < n ? pow(k_item[j], lambda) : 1.0;
  }
  if (transpose) {
    for (int yy = ty; yy < 32; yy += 8) {
      const int64_t si = bj + yy, sj = bi + tx;  // source row = output column
      tile[yy][tx] = (si < n && sj < n) ? gW[si * n + sj] : 0.0;
    }
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    const int64_t i = bi + yy, j = bj + tx;
    if (i >= n || j >= n) continue;
    const double src = transpose ? tile[tx][yy] : gW[i * n + j];
    double den = alpha[yy] * beta[tx];
    if (den == 0.0) den = 1.0;
    W[i * n + j] = src / den;
  }
}

__global__ __launch_bounds__(256) void k_spread_resource(
    const int64_t *__restrict__ user_rowptr, const int32_t *__restrict__ user_items,
    const double *__restrict__ W, int64_t n_items, double *__restrict__ F, int64_t ldf) {
  const int64_t u = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_items) return;
  const int64_t pb = user_rowptr[u], pe = user_rowptr[u + 1];
  double s = 0.0;
  int64_t p = pb;
  for (; p + 4 <= pe; p += 4) {
    const double w0 = W[(int64_t)user_items[p] * n_items + j];
    const double w1 = W[(int64_t)user_items[p + 1] * n_items + j];
    const double w2 = W[(int64_t)user_items[p + 2] * n_items + j];
    const double w3 = W[(int64_t)user_items[p + 3] * n_items + j];
    s = (((s + w0) + w1) + w2) + w3;
  }
  for (; p < pe; ++p) s += W[(int64_t)user_items[p] * n_items + j];
  F[u * ldf + j] = s;
}

// fp32 score in the chain order of lg_score_topk_f32 (see topk.hip header).
template <int D>
__device__ __forceinline__ float chain_score(const float *__restrict__ us,
                                             const float *__restrict__ it) {
  constexpr int Q = D / 4;
  float r[D];
  const float4 *p4 = reinterpret_cast<const float4 *>(it);
#pragma unroll
  for (int t = 0; t < D / 4; ++t) {
    const float4 q = p4[t];
    r[4 * t] = q.x;
    r[4 * t + 1] = q.y;
    r[4 * t + 2] = q.z;
    r[4 * t + 3] = q.w;
  }
  float acc = 0.f;
#pragma unroll
  for (int s = 0; s < Q; ++s)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc = __builtin_fmaf(us[g * Q + s], r[g * Q + s], acc);
  return acc;
}

// NW waves per row (one row per block), D == 0: no G factor. Wave w scans the row's w-th
// column range (whole 64-column steps) in ascending order into its own candidate list --
// at the C3 Douban shape (600 rows x 20,000 columns) one wave per row left the chip mostly
// idle behind each step's load -> 64-FMA chain latency -- then the waves' top-k lists merge
// pairwise in log2(NW) rounds (each merge: the partner's <= k entries appended, the list
// compacted; the (value desc, column asc) order is total, so the result is the single
// scan's). Columns arrive in ascending order within a wave, so a tie with tau loses.
template <int M, int D, int NW>
__global__ __launch_bounds__(64 * NW) void k_rows_topk(
    const double *__restrict__ F, int64_t ldf, int64_t n_rows, int64_t n_cols,
    const float *__restrict__ eu, const float *__restrict__ ei,
    const int64_t *__restrict__ ex_rowptr, const int32_t *__restrict__ ex_col, int excl_mode,
    int k, double *__restrict__ out_val, int64_t *__restrict__ out_idx) {
  constexpr int CAP = 64 * M;
  constexpr int DU = D > 0 ? D : 1;
  static_assert(CAP >= 128 && (NW & (NW - 1)) == 0, "a merge holds two lists of k <= CAP / 2");
  __shared__ double cs[NW][CAP];
  __shared__ int ci[NW][CAP];
  __shared__ float us[DU];
  __shared__ int s_n[NW];
  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int64_t r = blockIdx.x;  // (< n_rows: one block per row)
  if (D > 0) {
    for (int t = threadIdx.x; t < D; t += 64 * NW) us[t] = eu[r * D + t];
    __syncthreads();
  }
  int64_t lo = 0, hi = 0;
  if (ex_rowptr && excl_mode == LG_EXCL_DROP) {
    lo = ex_rowptr[r];
    hi = ex_rowptr[r + 1];
  }
  const int64_t span = ((n_cols + NW - 1) / NW + 63) / 64 * 64;
  const int64_t c0 = wave * span, c1 = c0 + span < n_cols ? c0 + span : n_cols;
  int cnt = 0;
  double tau = neg_inf<double>();
  int tau_id = kPadId;
  const double *row = F + r * ldf;
  // no G: two 64-column steps per round (both loads in flight; the candidates of the first
  // step are taken before the second's, so columns still reach the list in ascending order):
  // 0.141 -> 0.119 ms at the C3 shape. With G one step: two interleaved score chains measured
  // slower (0.52 -> 0.59 ms: 186 instead of 125 VGPRs, half the waves per SIMD)
  constexpr int STEPS = D > 0 ? 1 : 2;
  for (int64_t j00 = c0; j00 < c1; j00 += 64 * STEPS) {
    double v2[STEPS];
#pragma unroll
    for (int h = 0; h < STEPS; ++h) {
      const int64_t j = j00 + 64 * h + lane;
      v2[h] = j < c1 ? row[j] : neg_inf<double>();
    }
    if constexpr (D > 0) {
      if (j00 + lane < c1) v2[0] = (double)chain_score<DU>(us, ei + (j00 + lane) * D) * v2[0];
    }
#pragma unroll
    for (int h = 0; h < STEPS; ++h) {
      const int64_t j0 = j00 + 64 * h;
      if (j0 >= c1) break;  // (wave-uniform)
      const int64_t j = j0 + lane;
      const bool valid = j < c1;
      const double v = v2[h];
      bool cand = valid && v > tau;
      if (__ballot(cand)) {
        if (cand && lo < hi) {
          const int64_t p = lower_bound_i32(ex_col, lo, hi, (int32_t)j);
          lo = p;
          if (p < hi && ex_col[p] == (int32_t)j) cand = false;
        }
        const uint64_t bal = __ballot(cand);
        const int pos = cnt + __popcll(bal & lanemask_lt());
        if (cand) {
          cs[wave][pos] = v;
          ci[wave][pos] = (int)j;
        }
        cnt += __popcll(bal);
        if (cnt > CAP - 64) {
          wave_sync();
          cnt = wave_compact<double, M>(cs[wave], ci[wave], cnt, k, tau, tau_id);
        }
      }
    }
  }
  wave_sync();
  int nc = wave_compact<double, M>(cs[wave], ci[wave], cnt, k, tau, tau_id);
  if (lane == 0) s_n[wave] = nc;
#pragma unroll
  for (int st = 1; st < NW; st <<= 1) {
    __syncthreads();
    if (wave % (2 * st) == 0) {  // (wave + st < NW: NW is a power of two)
      const int n1 = s_n[wave + st];
      for (int e = lane; e < n1; e += 64) {
        cs[wave][nc + e] = cs[wave + st][e];
        ci[wave][nc + e] = ci[wave + st][e];
      }
      wave_sync();
      nc = wave_compact<double, M>(cs[wave], ci[wave], nc + n1, k, tau, tau_id);
      if (lane == 0) s_n[wave] = nc;
    }
  }
  if (wave == 0) {
    for (int e = lane; e < k; e += 64) {
      out_val[r * k + e] = e < nc ? cs[0][e] : neg_inf<double>();
      out_idx[r * k + e] = e < nc ? ci[0][e] : -1;
    }
  }
}

// rows of at least this many columns get 8 waves each, shorter ones one
constexpr int64_t kRowsSplitCols = 4096;

template <int M, int NW>
static void launch_rows_topk_nw(int dim, const double *F, int64_t ldf, int64_t n_rows,
                                int64_t n_cols, const float *eu, const float *ei,
                                const int64_t *ex_rowptr, const int32_t *ex_col, int excl_mode,
                                int k, double *out_val, int64_t *out_idx, hipStream_t s) {
  dim3 grid((unsigned)n_rows), block(64 * NW);
  switch (eu ? dim : 0) {
    case 0: k_rows_topk<M, 0, NW><<<grid, block, 0, s>>>(F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode, k, out_val, out_idx); break;
    case 32: k_rows_topk<M, 32, NW><<<grid, block, 0, s>>>(F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode, k, out_val, out_idx); break;
    case 64: k_rows_topk<M, 64, NW><<<grid, block, 0, s>>>(F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode, k, out_val, out_idx); break;
    default: k_rows_topk<M, 128, NW><<<grid, block, 0, s>>>(F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode, k, out_val, out_idx); break;
  }
}

template <int M>
static void launch_rows_topk(int dim, const double *F, int64_t ldf, int64_t n_rows,
                             int64_t n_cols, const float *eu, const float *ei,
                             const int64_t *ex_rowptr, const int32_t *ex_col, int excl_mode,
                             int k, double *out_val, int64_t *out_idx, hipStream_t s) {
  if (n_cols >= kRowsSplitCols)
    launch_rows_topk_nw<M, 8>(dim, F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode,
                              k, out_val, out_idx, s);
  else
    launch_rows_topk_nw<M, 1>(dim, F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode,
                              k, out_val, out_idx, s);
}

}  // namespace lg

using namespace lg;

extern "C" int lg_spread_general_f64(const int64_t *item_rowptr, const int32_t *item_users,
                                     const int64_t *user_rowptr, const int32_t *user_items,
                                     int64_t n_users, int64_t n_items, double *gW,
                                     lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && item_users && user_rowptr && user_items && gW && n_users >= 0 &&
                 n_items >= 0,
             "lg_spread_general_f64: bad arguments");
  if (n_items == 0) return LG_OK;
  k_spread_general<<<dim3((unsigned)n_items), dim3(256), 0, (hipStream_t)stream>>>(
      item_rowptr, item_users, user_rowptr, user_items, n_items, gW);
  return launch_status("lg_spread_general_f64");
}

static int spread_ranges(int64_t n_items) { return (int)((n_items + kSpreadCols - 1) / kSpreadCols); }

extern "C" size_t lg_spread_hybrid_ws_bytes(int64_t n_items, int64_t n_users) {
  if (n_items <= 0) return 0;
  return (size_t)n_items * 2 * sizeof(double) +
         (size_t)(n_users > 0 ? n_users : 0) * (spread_ranges(n_items) + 1) * sizeof(int32_t);
}

extern "C" int lg_spread_hybrid_f64(const int64_t *item_rowptr, const int32_t *item_users,
                                    const int64_t *user_rowptr, const int32_t *user_items,
                                    const double *k_item, int64_t n_users, int64_t n_items,
                                    double lambda, double *W, void *ws, size_t ws_bytes,
                                    lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && item_users && user_rowptr && user_items && k_item && W &&
                 n_users >= 0 && n_items >= 0 && n_items < 0x7fffffff,
             "lg_spread_hybrid_f64: bad arguments");
  if (n_items == 0) return LG_OK;
  const size_t need = lg_spread_hybrid_ws_bytes(n_items, n_users);
  if (!ws || ws_bytes < need) {
    set_error("lg_spread_hybrid_f64: workspace %zu < %zu bytes", ws_bytes, need);
    return LG_ERR_WORKSPACE;
  }
  const int nr = spread_ranges(n_items);
  LG_REQUIRE((int64_t)nr * n_items < 0x7fffffff, "lg_spread_hybrid_f64: %lld items: too many",
             (long long)n_items);
  hipStream_t s = (hipStream_t)stream;
  double *alpha = (double *)ws, *beta = alpha + n_items;
  int32_t *starts = (int32_t *)(beta + n_items);
  k_hybrid_factors<<<dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, s>>>(
      k_item, n_items, lambda, alpha, beta);
  const int64_t ns = n_users * (nr + 1);
  if (ns > 0)
    k_user_range_starts<<<dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s>>>(
        user_rowptr, user_items, n_users, nr, starts);
  k_spread_hybrid<<<dim3((unsigned)(nr * n_items)), dim3(256), 0, s>>>(
      item_rowptr, item_users, user_rowptr, user_items, starts, nr, n_items, alpha, beta, W);
  return launch_status("lg_spread_hybrid_f64");
}

extern "C" int lg_hybrid_weight_f64(const double *gW, const double *k_item, int64_t n_items,
                                    double lambda, int32_t transpose_gw, double *W,
                                    lg_stream_t stream) {
  LG_REQUIRE(gW && k_item && W && n_items >= 0, "lg_hybrid_weight_f64: bad arguments");
  LG_REQUIRE(gW != W || !transpose_gw, "lg_hybrid_weight_f64: transposed source cannot alias W");
  if (n_items == 0) return LG_OK;
  const unsigned t = (unsigned)((n_items + 31) / 32);
  k_hybrid_weight<<<dim3(t, t), dim3(256), 0, (hipStream_t)stream>>>(gW, k_item, lambda, n_items,
                                                                    transpose_gw, W);
  return launch_status("lg_hybrid_weight_f64");
}

extern "C" int lg_spread_resource_f64(const int64_t *user_rowptr, const int32_t *user_items,
                                      const double *W, int64_t n_users, int64_t n_items,
                                      double *F, int64_t ldf, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && user_items && W && F && n_users >= 0 && n_items >= 0 &&
                 ldf >= n_items,
             "lg_spread_resource_f64: bad arguments");
  if (n_users == 0 || n_items == 0) return LG_OK;
  hipStream_t s = (hipStream_t)stream;
  // grid.y is limited to 65535: walk users in slabs
  for (int64_t u0 = 0; u0 < n_users; u0 += 65535) {
    const int64_t nu = (n_users - u0) < 65535 ? (n_users - u0) : 65535;
    k_spread_resource<<<dim3((unsigned)((n_items + 255) / 256), (unsigned)nu), dim3(256), 0,
                        s>>>(user_rowptr + u0, user_items, W, n_items, F + u0 * ldf, ldf);
  }
  return launch_status("lg_spread_resource_f64");
}

extern "C" int lg_rows_topk_f64(const double *F, int64_t ldf, int64_t n_rows,
                                int64_t n_cols, const float *eu, const float *ei,
                                int32_t dim, const int64_t *ex_rowptr,
                                const int32_t *ex_col, int32_t excl_mode, int32_t k,
                                double *out_val, int64_t *out_idx, lg_stream_t stream) {
  LG_REQUIRE(F && out_val && out_idx && n_rows >= 0 && n_cols >= 0 && ldf >= n_cols &&
                 n_cols < 0x7fffffff,
             "lg_rows_topk_f64: bad arguments");
  LG_REQUIRE(k >= 1 && k <= 128, "lg_rows_topk_f64: k=%d not in [1,128]", k);
  LG_REQUIRE(!eu == !ei, "lg_rows_topk_f64: eu/ei must both be set or both NULL");
  LG_REQUIRE(!eu || dim == 32 || dim == 64 || dim == 128,
             "lg_rows_topk_f64: dim %d not in {32,64,128}", dim);
  LG_REQUIRE(excl_mode == LG_EXCL_DROP || excl_mode == LG_EXCL_NONE,
             "lg_rows_topk_f64: bad excl_mode %d", excl_mode);
  LG_REQUIRE(!ex_rowptr == !ex_col, "lg_rows_topk_f64: ex_rowptr/ex_col must both be set");
  LG_REQUIRE(!(eu && excl_mode == LG_EXCL_NONE && ex_rowptr),
             "lg_rows_topk_f64: a G factor with exclusions requires LG_EXCL_DROP");
  if (n_rows == 0) return LG_OK;
  hipStream_t s = (hipStream_t)stream;
  if (k <= 64)
    launch_rows_topk<2>(dim, F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode, k,
                        out_val, out_idx, s);
  else
    launch_rows_topk<4>(dim, F, ldf, n_rows, n_cols, eu, ei, ex_rowptr, ex_col, excl_mode, k,
                        out_val, out_idx, s);
  return launch_status("lg_rows_topk_f64");
}
