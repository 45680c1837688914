// K3s: factored hybrid spreading for catalogs whose I x I matrices do not fit (SURVEY.md §8
// a9 "K3s", C5: 1M x 1M, 100M interactions -> general_W and W would be 8 TB each).
//
// Reference (dense numpy fp64, model/SpreadMethod/model.py):
//   general_W = (A.T / k_u) @ A            :14-27
//   W = general_W / (k_i^(1-l) (x) k_j^l)   :63-85   (den == 0 -> 1)
//   F = A @ W                               :88-99
//   F_new = G * F; per user argsort desc, drop train|val, [:k]
//                       model/SpreadLightGCN/model.py:151, recommend.py:18-52
//
// The items are processed in column tiles [j0, j0 + T). Per tile:
//   cursor   end[v] = first position of user v's (ascending) item row with item >= j0 + T;
//            cur[v] (the previous tile's end) marks the first item >= j0, so
//            items(v) inside the tile = user_items[cur[v] .. end[v])
//   bound    bound[i] = sum_{v in users(i)} (end[v] - cur[v]) = the (user, item) pairs
//            behind row i of W in the tile
//   weight   row i of W restricted to the tile (format below: the pairs themselves, 4 bytes
//            each, for ordinary rows; merged fp64 values for hub rows)
//   walk     per user: F[u][j - j0] = sum_{i in items(u), ascending} W[i][j] in an LDS
//            accumulator (one wave per user, lg_spread_resource_f64's order and values), then
//            either written out (F mode) or merged straight into the user's running top-K
//            list (top-K mode: (G *) F, G = the fp32 e0 score chain, candidates screened by
//            per-(user, 64-column chunk) score bounds from lg_score_chunk_bound).
// Work: the weight pass costs sum_i deg(i) lookups + the 2-hop pairs once per tile (not per
// user); the walk reads deg(u) short row segments per user and tile (~1e12 paths at C5:
// 4 bytes per path, F never leaves LDS).
#include <stdlib.h>

#include "common.h"

namespace lg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// A W tile is stored as one row segment per item i, in one of two formats (RowMeta, one
// 16-byte load per row: m = ptr | len << 40 | V << 63, and alpha_i):
//
// P rows (<= kSortMax pairs, the common case): one 4-byte slot per (user v, item j) PAIR
//   behind the row (v in users(i), j in items(v) inside the tile), sorted by (j, v):
//     bits 0-15  j - item_begin
//     bits 16-29 the class of v's degree k_v (fl(1 / k_v) = inv[class], classes < kInvTab
//                cached in LDS)
//     bit 30     the next slot is the same column (a run of users of one (i, j))
//     bit 31     this slot continues the previous slot's column
//   The resource pass forms W[i][j] = (sum of the run's fl(1/k_v), ascending v) /
//   (alpha_i * beta_j) per path: the sum of lg_spread_general_f64 and the division of
//   lg_hybrid_weight_f64, bit for bit, without storing an fp64 per entry (4 bytes per path
//   instead of 12; the path count, ~1e12 at C5, sets the runtime).
// V rows (hub items, > kSortMax pairs, merged while building): one 12-byte triple per
//   distinct column: slot 0 = (kClsV << 16) | (j - item_begin), slots 1-2 = the fp64
//   general_W[i][j] (lo, hi), divided by alpha_i * beta_j in the walk like a P run.
// Neither format depends on lambda (only RowMeta's alpha and the walk's beta table do), so
// a lambda sweep reuses the built tiles.
constexpr uint32_t kClsMask = 0x3FFF;
constexpr uint32_t kClsV = 0x3FFF;         // class field of a V-row triple's first slot
constexpr uint32_t kHasNext = 0x40000000u;
constexpr uint32_t kIsCont = 0x80000000u;
constexpr int kLenShift = 40;
constexpr uint64_t kPtrMask = (1ull << kLenShift) - 1;
constexpr uint64_t kLenMask = (1ull << 23) - 1;
constexpr uint64_t kFmtV = 1ull << 63;
constexpr int kInvTab = 512;  // degree classes whose fl(1/k) is cached in LDS

struct RowMeta {
  uint64_t m;
  double alpha;
};

__global__ __launch_bounds__(256) void k_hybrid_factors(const double *__restrict__ k_item,
                                                        int64_t n, double lambda,
                                                        double *__restrict__ alpha,
                                                        double *__restrict__ beta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // the same pow() calls as k_hybrid_weight (spread.hip)
  alpha[i] = pow(k_item[i], 1.0 - lambda);
  beta[i] = pow(k_item[i], lambda);
}

// out[r] = ||x[r]||_2 in fp64 (the bound of the fused top-K prefilter).
__global__ __launch_bounds__(256) void k_row_norms(const float *__restrict__ x, int64_t n,
                                                   int dim, double *__restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  double s = 0.0;
  for (int d = 0; d < dim; ++d) {
    const double v = x[r * dim + d];
    s += v * v;
  }
  out[r] = sqrt(s);
}

__global__ __launch_bounds__(256) void k_inv_degree(const int64_t *__restrict__ rowptr,
                                                    int64_t n, double *__restrict__ inv) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  inv[v] = 1.0 / (double)(rowptr[v + 1] - rowptr[v]);  // k_spread_general's fl(1/k_v)
}

__global__ __launch_bounds__(256) void k_tile_cursor(const int64_t *__restrict__ user_rowptr,
                                                     const int32_t *__restrict__ user_items,
                                                     int64_t n_users, int32_t item_end,
                                                     const int64_t *__restrict__ cur,
                                                     int64_t *__restrict__ end,
                                                     uint16_t *__restrict__ count) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_users) return;
  const int64_t p0 = cur[v];
  int64_t p = p0;
  const int64_t pe = user_rowptr[v + 1];
  while (p < pe && user_items[p] < item_end) ++p;
  end[v] = p;
  count[v] = (uint16_t)(p - p0);  // <= tile <= 8192
}

// cur[v] = first position of user v's item row with item >= item_begin: the cursor state
// of a tile walk that starts at item_begin instead of 0 (an item-range shard).
__global__ __launch_bounds__(256) void k_tile_seek(const int64_t *__restrict__ user_rowptr,
                                                   const int32_t *__restrict__ user_items,
                                                   int64_t n_users, int32_t item_begin,
                                                   int64_t *__restrict__ cur) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_users) return;
  cur[v] = lower_bound_i32(user_items, user_rowptr[v], user_rowptr[v + 1], item_begin);
}

// one wave per item row
__global__ __launch_bounds__(256) void k_tile_bound(const int64_t *__restrict__ item_rowptr,
                                                    const int32_t *__restrict__ item_users,
                                                    int64_t n_items,
                                                    const uint16_t *__restrict__ count,
                                                    int64_t *__restrict__ bound) {
  const int64_t i = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (i >= n_items) return;
  const int lane = lane_id();
  int64_t s = 0;
  for (int64_t e = item_rowptr[i] + lane; e < item_rowptr[i + 1]; e += 64)
    s += count[item_users[e]];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) bound[i] = s;
}

constexpr int kSortMax = 256;  // pairs per row handled by the in-wave sort (P rows)

// Sort the n (<= 64*M) staged pairs (key = -item, id = staging position, which ascends
// with the user) of this wave by (item, user) and write them as P slots.
template <int M>
__device__ __forceinline__ void sort_write_row(int *skey, int *sid, const uint16_t *scls, int n,
                                               int64_t wbase, int32_t item_begin,
                                               uint32_t *__restrict__ wt_ent) {
  const int lane = lane_id();
  int k[M], id[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int e = j * 64 + lane;
    if (e < n) { k[j] = skey[e]; id[j] = sid[e]; }
    else { k[j] = INT32_MIN; id[j] = kPadId; }
  }
  wave_sync();
  // before(): key desc, id asc  ->  item asc, user asc; padding (INT32_MIN) last
  wave_bitonic_sort<int, M>(k, id);
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int e = j * 64 + lane;
    skey[e] = k[j];
    sid[e] = id[j];
  }
  wave_sync();
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int e = j * 64 + lane;
    if (e < n) {
      const int key = skey[e];
      const bool prv = e > 0 && skey[e - 1] == key;
      const bool nxt = e + 1 < n && skey[e + 1] == key;
      wt_ent[wbase + e] = (prv ? kIsCont : 0u) | (nxt ? kHasNext : 0u) |
                          ((uint32_t)scls[sid[e]] << 16) | (uint32_t)(-key - item_begin);
    }
  }
}

// P rows: one wave per item row with bound[i] <= kSortMax pairs (LDS staging per wave).
__global__ __launch_bounds__(256) void k_tile_weight(
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const uint16_t *__restrict__ user_cls,
    int64_t n_items, const int64_t *__restrict__ cur, const uint16_t *__restrict__ count,
    const double *__restrict__ alpha, int32_t item_begin, const int64_t *__restrict__ bound,
    const int64_t *__restrict__ wt_ptr, uint32_t *__restrict__ wt_ent,
    RowMeta *__restrict__ wt_meta) {
  __shared__ int skey[4][kSortMax];
  __shared__ int sid[4][kSortMax];
  __shared__ uint16_t scls[4][kSortMax];
  const int wave = threadIdx.x / 64;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave;
  if (i >= n_items) return;
  const int lane = lane_id();
  const int64_t nb = bound[i];
  if (nb > kSortMax) return;  // hub row: k_tile_weight_hub
  const int64_t wbase = wt_ptr[i];
  if (lane == 0) wt_meta[i] = RowMeta{(uint64_t)wbase | ((uint64_t)nb << kLenShift), alpha[i]};
  if (nb == 0) return;
  // stage the pairs: users of i in ascending order, each user's items inside the tile
  int n = 0;
  for (int64_t e0 = item_rowptr[i]; e0 < item_rowptr[i + 1]; e0 += 64) {
    const int64_t e = e0 + lane;
    int32_t v = 0;
    int c = 0;
    if (e < item_rowptr[i + 1]) {
      v = item_users[e];
      c = count[v];
    }
    int pre = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(pre, o);
      if (lane >= o) pre += y;
    }
    const int total = __shfl(pre, 63);
    pre -= c;
    if (c) {
      const int64_t s0 = cur[v];
      const uint16_t cl = user_cls[v];
      for (int q = 0; q < c; ++q) {
        const int p = n + pre + q;
        skey[wave][p] = -user_items[s0 + q];
        sid[wave][p] = p;
        scls[wave][p] = cl;
      }
    }
    n += total;
  }
  wave_sync();
  if (n <= 64)
    sort_write_row<1>(skey[wave], sid[wave], scls[wave], n, wbase, item_begin, wt_ent);
  else if (n <= 128)
    sort_write_row<2>(skey[wave], sid[wave], scls[wave], n, wbase, item_begin, wt_ent);
  else
    sort_write_row<4>(skey[wave], sid[wave], scls[wave], n, wbase, item_begin, wt_ent);
}

// V rows (bound > kSortMax pairs, hub items): one 256-thread block per row (grid-stride
// over the hub list), the tile as a dense LDS accumulator, users walked in ascending order
// as in k_spread_general, then the touched columns written as merged triples.
__global__ __launch_bounds__(256) void k_tile_weight_hub(
    const int64_t *__restrict__ hub_rows, const int64_t *__restrict__ n_hub,
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const double *__restrict__ inv_deg,
    const int64_t *__restrict__ cur, const uint16_t *__restrict__ count,
    const double *__restrict__ alpha, const double *__restrict__ beta, int32_t item_begin,
    int32_t tile, const int64_t *__restrict__ wt_ptr, uint32_t *__restrict__ wt_ent,
    RowMeta *__restrict__ wt_meta) {
  extern __shared__ double acc[];  // tile doubles
  __shared__ int wsum[4];
  const int64_t nh = *n_hub;
  for (int64_t h = blockIdx.x; h < nh; h += gridDim.x) {
    const int64_t i = hub_rows[h];
    for (int j = threadIdx.x; j < tile; j += blockDim.x) acc[j] = 0.0;
    __syncthreads();
    for (int64_t e = item_rowptr[i]; e < item_rowptr[i + 1]; ++e) {
      const int32_t v = item_users[e];
      const int c = count[v];
      if (c == 0) continue;  // uniform across the block: no barrier skipped unevenly
      const double wv = inv_deg[v];
      const int64_t s0 = cur[v];
      for (int q = threadIdx.x; q < c; q += blockDim.x) acc[user_items[s0 + q] - item_begin] += wv;
      __syncthreads();  // the next user may hit the same columns from other threads
    }
    // compact the touched columns (every contribution is > 0) in ascending order
    const double a = alpha[i];
    const int64_t wbase = wt_ptr[i];
    int base = 0;
    for (int j0 = 0; j0 < tile; j0 += blockDim.x) {
      const int j = j0 + threadIdx.x;
      const bool nz = j < tile && acc[j] != 0.0;
      const uint64_t b = __ballot(nz);
      const int w = threadIdx.x / 64;
      if (lane_id() == 0) wsum[w] = __popcll(b);
      __syncthreads();
      int before_w = 0, total = 0;
      for (int q = 0; q < 4; ++q) {
        if (q < w) before_w += wsum[q];
        total += wsum[q];
      }
      if (nz) {
        const uint64_t bits = (uint64_t)__double_as_longlong(acc[j]);
        const int64_t p = wbase + 3 * (int64_t)(base + before_w + __popcll(b & lanemask_lt()));
        wt_ent[p] = (kClsV << 16) | (uint32_t)j;
        wt_ent[p + 1] = (uint32_t)bits;
        wt_ent[p + 2] = (uint32_t)(bits >> 32);
      }
      base += total;
      __syncthreads();
    }
    if (threadIdx.x == 0)
      wt_meta[i] = RowMeta{(uint64_t)wbase | ((uint64_t)(3 * base) << kLenShift) | kFmtV, a};
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_hub_list(const int64_t *__restrict__ bound,
                                                  int64_t n_items,
                                                  unsigned long long *__restrict__ n_hub,
                                                  int64_t *__restrict__ hub_rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  if (bound[i] > kSortMax) hub_rows[atomicAdd(n_hub, 1ull)] = i;
}

// ------------------------------------------------------------------ the resource pass
// F[u][j] = sum over items(u) ascending of W[i][j]: one wave per user, the tile's
// accumulator in LDS. A user's rows are taken 128 at a time: their RowMeta is fetched in one
// round trip and indexed in LDS (empty rows dropped, inclusive slot prefix, slot base,
// alpha_i); the rows' slots are then flattened: lane l takes slots e = e0 + q*64 + l of the
// concatenated rows, UF loads in flight per lane, its row found by a short scan from the
// previous register's last row (rows are non-empty, so 64 slots span at most 64 rows). Each
// path's W value is formed in registers and added with ds_add_f64; adds of one instruction
// that hit the same column come from rows in lane order and instructions go in slot order,
// so each column receives its rows' values in ascending row order: the order of
// lg_spread_resource_f64, hence the same bits.
constexpr int kResRows = 128;
struct RowIndex {
  int cincl[kResRows];     // inclusive prefix of the rows' 4-slot chunks
  int cexcl[kResRows];     // exclusive prefix
  int len[kResRows];       // slots | 0x80000000 for V rows
  int pad_[kResRows];
  int64_t base[kResRows];  // the row's first slot
  double alpha[kResRows];
};

// Index of a group of up to 128 rows (RowMeta of rows lane and 64 + lane), empty rows
// dropped; returns the group's chunk count.
__device__ __forceinline__ int write_row_index(RowIndex *ix, RowMeta m0, RowMeta m1) {
  const int lane = lane_id();
  const int l0 = (int)((m0.m >> kLenShift) & kLenMask), l1 = (int)((m1.m >> kLenShift) & kLenMask);
  const int c0 = (l0 + 3) >> 2, c1 = (l1 + 3) >> 2;
  int in0 = c0, in1 = c1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y0 = __shfl_up(in0, o), y1 = __shfl_up(in1, o);
    if (lane >= o) { in0 += y0; in1 += y1; }
  }
  in1 += __shfl(in0, 63);
  const int total = __shfl(in1, 63);
  const uint64_t b0 = __ballot(l0 > 0), b1 = __ballot(l1 > 0);
  const int p0 = __popcll(b0 & lanemask_lt());
  const int p1 = __popcll(b0) + __popcll(b1 & lanemask_lt());
  wave_sync();  // earlier readers of this index are done
  ix->cincl[lane] = 0x7fffffff;  // rows past the group's last (binary search sentinel)
  ix->cincl[64 + lane] = 0x7fffffff;
  wave_sync();
  if (l0 > 0) {
    ix->cincl[p0] = in0;
    ix->cexcl[p0] = in0 - c0;
    ix->len[p0] = l0 | ((int64_t)m0.m < 0 ? (int)0x80000000 : 0);
    ix->base[p0] = (int64_t)(m0.m & kPtrMask);
    ix->alpha[p0] = m0.alpha;
  }
  if (l1 > 0) {
    ix->cincl[p1] = in1;
    ix->cexcl[p1] = in1 - c1;
    ix->len[p1] = l1 | ((int64_t)m1.m < 0 ? (int)0x80000000 : 0);
    ix->base[p1] = (int64_t)(m1.m & kPtrMask);
    ix->alpha[p1] = m1.alpha;
  }
  wave_sync();
  return total;
}

__device__ __forceinline__ double inv_of(uint32_t x, const double *s_inv,
                                         const double *__restrict__ g_inv) {
  const uint32_t c = (x >> 16) & kClsMask;
  return c < kInvTab ? s_inv[c] : g_inv[c];
}

// acc[j - item_begin] += the `total` flattened 4-slot chunks of one indexed row group.
// Lane l loads chunk c0 + 64q + l (16 bytes: rows start on 128-byte lines and hold whole
// chunks of capacity), its row found by UC lockstep binary searches over the group's chunk
// prefix; each 256-slot register is then transposed through LDS into slot order, so
// instruction t of it takes slots 64t .. 64t + 63 in lane order, the order that keeps every
// column's adds in ascending row order. The decode is branch-free except for the rare P runs
// of 3+ users and degree classes outside the LDS table.
template <int UC>
__device__ __forceinline__ void accumulate_group(double *acc, const RowIndex *ix, int total,
                                                 const uint32_t *__restrict__ ent,
                                                 const double *s_beta, const double *s_inv,
                                                 const double *__restrict__ g_inv,
                                                 uint32_t *tr) {
  const int lane = lane_id();
  for (int cb = 0; cb < total; cb += 64 * UC) {
    int rr[UC], cc[UC];
#pragma unroll
    for (int q = 0; q < UC; ++q) {
      const int c = cb + q * 64 + lane;
      cc[q] = c < total ? c : total - 1;
      rr[q] = 0;
    }
#pragma unroll
    for (int st = 64; st > 0; st >>= 1)
#pragma unroll
      for (int q = 0; q < UC; ++q) rr[q] += ix->cincl[rr[q] + st - 1] <= cc[q] ? st : 0;
    uint4 w[UC];
#pragma unroll
    for (int q = 0; q < UC; ++q)
      w[q] = *reinterpret_cast<const uint4 *>(ent + ix->base[rr[q]] +
                                              4 * (cc[q] - ix->cexcl[rr[q]]));
    // the first two slots after the block (a V value or a P run that straddles it)
    const int cn = cb + 64 * UC;
    uint32_t pk0 = 0, pk1 = 0;
    if (cn < total) {  // wave-uniform
      int rp = 0;
#pragma unroll
      for (int st = 64; st > 0; st >>= 1) rp += ix->cincl[rp + st - 1] <= cn ? st : 0;
      const uint32_t *p = ent + ix->base[rp] + 4 * (cn - ix->cexcl[rp]);
      pk0 = p[0];
      pk1 = p[1];
    }
#pragma unroll
    for (int q = 0; q < UC; ++q) {
      wave_sync();  // the previous register's readers of tr are done
      reinterpret_cast<uint4 *>(tr)[lane] = w[q];
      wave_sync();
      const uint32_t nx0 = q + 1 < UC ? __builtin_amdgcn_readlane(w[(q + 1 < UC) ? q + 1 : q].x, 0) : pk0;
      const uint32_t nx1 = q + 1 < UC ? __builtin_amdgcn_readlane(w[(q + 1 < UC) ? q + 1 : q].y, 0) : pk1;
      // the register's 4 slot-ordered instructions t: every LDS read of the 4 is issued
      // before any add (the reads then overlap instead of waiting one by one)
      uint32_t X[4], N1[4], N2[4];
      int R[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int m = 64 * t + lane;  // slot of this 256-slot register, in order
        X[t] = tr[m];
        N1[t] = tr[m + 1 < 256 ? m + 1 : 255];
        N2[t] = tr[m + 2 < 256 ? m + 2 : 255];
        R[t] = __shfl(rr[q], m >> 2);
      }
      N1[3] = lane == 63 ? nx0 : N1[3];
      N2[3] = lane == 63 ? nx1 : (lane == 62 ? nx0 : N2[3]);
      int CX[4], LW[4];
      double AL[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        CX[t] = ix->cexcl[R[t]];
        LW[t] = ix->len[R[t]];
        AL[t] = ix->alpha[R[t]];
      }
      bool HEAD[4], ISV[4];
      int COL[4], SROW[4];
      uint32_t CI[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int m = 64 * t + lane;
        const int cabs = cb + q * 64 + (m >> 2);
        SROW[t] = 4 * (cabs - CX[t]) + (m & 3);  // slot within its row
        ISV[t] = LW[t] < 0;
        const bool valid = cabs < total && SROW[t] < (LW[t] & 0x7fffffff);
        HEAD[t] = valid && (ISV[t] ? (SROW[t] % 3) == 0 : !(X[t] & kIsCont));
        COL[t] = HEAD[t] ? (int)(X[t] & 0xffffu) : 0;
        CI[t] = ISV[t] ? 0u : ((X[t] >> 16) & kClsMask);
      }
      double NUM[4], BE[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        NUM[t] = s_inv[CI[t] < (uint32_t)kInvTab ? CI[t] : 0u];
        BE[t] = s_beta[COL[t]];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool far = HEAD[t] && !ISV[t] && CI[t] >= (uint32_t)kInvTab;
        if (__ballot(far))
          if (far) NUM[t] = g_inv[CI[t]];
        if (ISV[t]) NUM[t] = __hiloint2double((int)N2[t], (int)N1[t]);  // general_W[i][j]
        const bool run = HEAD[t] && !ISV[t] && (X[t] & kHasNext);
        if (__ballot(run)) {  // more users behind this (i, j), ascending v
          if (run) {
            NUM[t] += inv_of(N1[t], s_inv, g_inv);
            if (N1[t] & kHasNext) {
              NUM[t] += inv_of(N2[t], s_inv, g_inv);
              if (N2[t] & kHasNext) {  // runs of 4+ (rare): the rest from memory
                const uint32_t *p = ent + ix->base[R[t]] + SROW[t] + 3;
                uint32_t y;
                do {
                  y = *p++;
                  NUM[t] += inv_of(y, s_inv, g_inv);
                } while (y & kHasNext);
              }
            }
          }
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        double den = AL[t] * BE[t];
        if (den == 0.0) den = 1.0;
        NUM[t] = NUM[t] / den;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (HEAD[t])
          __hip_atomic_fetch_add(&acc[COL[t]], NUM[t], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

template <int Q>
__device__ __forceinline__ void load_frag(const float *__restrict__ p, float (&v)[Q]) {
  const float4 *p4 = reinterpret_cast<const float4 *>(p);
#pragma unroll
  for (int t = 0; t < Q / 4; ++t) {
    const float4 q = p4[t];
    v[4 * t + 0] = q.x;
    v[4 * t + 1] = q.y;
    v[4 * t + 2] = q.z;
    v[4 * t + 3] = q.w;
  }
}

// Merge the tile's columns of (G *) F into running per-user top-K lists (io_val/io_idx,
// sorted, index -1 = empty). D = 0: no G factor. One wave = NG groups of 16 users (rows);
// lane (ul, gq) holds user ul of each group and items 4gq..4gq+3 of each 16-item step.
// S = the per-user list stride in LDS (entries): 40 for k <= 24 after a walk's first span
// (30 KiB blocks: 8 waves per CU, VGPR-limited), else 64*M. (A 3-slot load ring under a
// 3-waves-per-SIMD register budget spilled and ran 40 % slower.)
template <int D, int NG, int M, bool VEC, int S>
__global__ __launch_bounds__(128) void k_tile_topk(
    const double *__restrict__ F, int64_t ldf, int64_t n_rows, int32_t item_begin,
    int32_t n_cols, const float *__restrict__ eu, const float *__restrict__ ei,
    const int64_t *__restrict__ ex_rowptr, const int32_t *__restrict__ ex_col, int drop,
    int k, int first, double *__restrict__ io_val, int64_t *__restrict__ io_idx) {
  static_assert(S >= 32 && S <= 64 * M, "list stride");
  constexpr int Q = D > 0 ? D / 4 : 1;
  __shared__ double cs[2][NG][16][S];
  __shared__ int ci[2][NG][16][S];
  __shared__ int exs[2][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);  // uniform: SGPR bases
  const int lane = lane_id();
  const int ul = lane & 15, gq = lane >> 4;
  const int64_t ubase = ((int64_t)blockIdx.x * 2 + wave) * (16 * NG);
  if (ubase >= n_rows) return;

  float uf[NG][Q];
  bool uvalid[NG];
  int cnt[NG], chk[NG];
  bool dirty[NG];  // the user's list gained an entry in this call (first call: always)
  double thr[NG];
  int64_t ex_pos[NG], ex_hi[NG];
  const int lim_end = item_begin + n_cols;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int64_t r = ubase + g * 16 + ul;
    uvalid[g] = r < n_rows;
    const int64_t rr = uvalid[g] ? r : n_rows - 1;
    if (D > 0) load_frag<Q>(eu + rr * D + gq * Q, uf[g]);
    ex_pos[g] = 0;
    ex_hi[g] = 0;
    if (drop && ex_rowptr && uvalid[g]) {
      ex_pos[g] = ex_rowptr[r];
      ex_hi[g] = ex_rowptr[r + 1];
    }
    cnt[g] = 0;
    chk[g] = 0;
    dirty[g] = first != 0;
    thr[g] = uvalid[g] ? neg_inf<double>() : __builtin_huge_val();
  }
  // exclusion cursors: first excluded item >= item_begin, all groups' searches in lockstep
  // so their loads overlap; ex_next caches the item under the cursor (INT_MAX = none left)
  int32_t ex_next[NG];
  {
    int64_t lo[NG], hi[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      lo[g] = ex_pos[g];
      hi[g] = ex_hi[g];
    }
    for (;;) {
      bool busy = false;
      int32_t x[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) x[g] = lo[g] < hi[g] ? ex_col[(lo[g] + hi[g]) >> 1] : 0;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (lo[g] < hi[g]) {
          const int64_t mid = (lo[g] + hi[g]) >> 1;
          if (x[g] < item_begin) lo[g] = mid + 1;
          else hi[g] = mid;
        }
        busy |= lo[g] < hi[g];
      }
      if (!__ballot(busy)) break;
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      ex_pos[g] = lo[g];
      ex_next[g] = lo[g] < ex_hi[g] ? ex_col[lo[g]] : 0x7fffffff;
    }
  }
  // running lists -> LDS (already sorted and exclusion-checked): the wave's NG*16 lists are
  // contiguous in io_*, so they are read in one pass with 8 loads per lane in flight
  if (!first) {
    const int64_t base = ubase * k;
    const int64_t lim = (n_rows - ubase) * k;
    const int total = NG * 16 * k;
    for (int t0 = 0; t0 < total; t0 += 64 * 8) {
      int64_t id[8];
      double vv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int t = t0 + q * 64 + lane;
        const bool in = t < total && t < lim;
        id[q] = in ? io_idx[base + t] : -1;
        vv[q] = in ? io_val[base + t] : neg_inf<double>();
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int t = t0 + q * 64 + lane;
        if (t < total) {
          const int uu = t / k, e = t - uu * k;
          cs[wave][uu >> 4][uu & 15][e] = vv[q];
          ci[wave][uu >> 4][uu & 15][e] = id[q] >= 0 ? (int)id[q] : -1;
        }
      }
    }
    wave_sync();
    // valid entries form a prefix (lists are sorted, drops written as -1 at the end): the
    // 4 lanes of a user count a quarter each
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int *is = &ci[wave][g][ul][0];
      int nv = 0;
      for (int e = gq; e < k; e += 4) nv += is[e] >= 0;
      nv += __shfl_xor(nv, 16);
      nv += __shfl_xor(nv, 32);
      if (uvalid[g]) {
        cnt[g] = nv;
        chk[g] = nv;
        thr[g] = nv == k ? cs[wave][g][ul][k - 1] : neg_inf<double>();
      }
    }
  }
  const uint64_t same_user = 0x0001000100010001ull << ul;

  auto compact_user = [&](int g, int u, int lim) __attribute__((always_inline)) {
    const int n = __shfl(cnt[g], u);
    const int c0 = __shfl(chk[g], u);
    int64_t pos = __shfl(ex_pos[g], u);
    const int64_t hi = __shfl(ex_hi[g], u);
    int32_t nx = __shfl(ex_next[g], u);
    double *ks = &cs[wave][g][u][0];
    int *is = &ci[wave][g][u][0];
    if (n > c0 && nx < lim) {  // the cached next exclusion decides without a load
      while (pos < hi) {  // excluded items in [previous limit, lim): drop their entries
        const int64_t e = pos + lane;
        const int32_t x = e < hi ? ex_col[e] : 0x7fffffff;
        const int nin = __popcll(__ballot(x < lim));
        if (nin < 64) nx = __shfl(x, nin & 63);
        if (nin == 0) break;
        exs[wave][lane] = x;
        wave_sync();
        for (int j = c0 + lane; j < n; j += 64) {
          const int item = is[j];
          int a = 0, b = nin;
          while (a < b) {
            const int mid = (a + b) >> 1;
            if (exs[wave][mid] < item) a = mid + 1;
            else b = mid;
          }
          if (a < nin && exs[wave][a] == item) ks[j] = neg_inf<double>();
        }
        wave_sync();
        pos += nin;
        if (nin < 64) break;
      }
      if (pos >= hi) nx = 0x7fffffff;
    }
    double t;
    int tid;
    const int nc = wave_compact<double, M>(ks, is, n, k, t, tid);
    if (ul == u) {
      cnt[g] = nc;
      chk[g] = nc;
      ex_pos[g] = pos;
      ex_next[g] = nx;
      thr[g] = !uvalid[g] ? __builtin_huge_val() : t;
    }
  };

  // One 16-column step: the item fragment and the F values (clamped to valid memory, so
  // every step issues the same loads) are loaded one step ahead.
  // VEC: ldf >= n_cols rounded up to 16, so a step's 16 columns are always inside the row:
  // the step start is clamped to the last step and each lane reads its 4 columns as two
  // 16-byte loads (columns past n_cols are never inserted: process() checks c < n_cols).
  const int last_step = ((n_cols - 1) / 16) * 16;
  auto load_step = [&](int it, float(&af)[Q], double(&f)[NG][4]) __attribute__((always_inline)) {
    if constexpr (D > 0) {
      const int jc = it + ul < n_cols ? item_begin + it + ul : item_begin + n_cols - 1;
      load_frag<Q>(ei + (int64_t)jc * D + gq * Q, af);
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int64_t row = ubase + g * 16 + ul;
      const double *fr = F + (row < n_rows ? row : n_rows - 1) * ldf;
      if constexpr (VEC) {
        const int c0 = (it < last_step ? it : last_step) + gq * 4;
        const double2 a = *reinterpret_cast<const double2 *>(fr + c0);
        const double2 b = *reinterpret_cast<const double2 *>(fr + c0 + 2);
        f[g][0] = a.x;
        f[g][1] = a.y;
        f[g][2] = b.x;
        f[g][3] = b.y;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = it + gq * 4 + r;
          f[g][r] = fr[c < n_cols ? c : n_cols - 1];
        }
      }
    }
  };
  auto process = [&](int it, const float(&af)[Q], const double(&f)[NG][4]) __attribute__((always_inline)) {
    double v[NG][4];
    if constexpr (D > 0) {
      f32x4 acc[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < Q; ++s)
#pragma unroll
        for (int g = 0; g < NG; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], uf[g][s], acc[g], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[g][r] = (double)acc[g][r] * f[g][r];
    } else {
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[g][r] = f[g][r];
    }
    // fast filter: one ballot per step; the exact per-column insertion only on a hit
    const int c0 = it + gq * 4;
    bool any = false;
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) any |= v[g][r] > thr[g];
    if (__ballot(any)) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool cand = c0 + r < n_cols && v[g][r] > thr[g];
          const uint64_t bal = __ballot(cand);
          if (bal) {
            const int p = cnt[g] + __popcll(bal & same_user & lanemask_lt());
            if (cand) {
              cs[wave][g][ul][p] = v[g][r];
              ci[wave][g][ul][p] = item_begin + c0 + r;
            }
            cnt[g] += __popcll(bal & same_user);
            dirty[g] |= (bal & same_user) != 0;
          }
        }
      }
    }
    bool over = false;
#pragma unroll
    for (int g = 0; g < NG; ++g) over |= cnt[g] > S - 16;
    if (__ballot(over)) {
      const int lim = item_begin + (it + 16 < n_cols ? it + 16 : n_cols);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        uint64_t need = __ballot(cnt[g] > S - 16) & 0xffffull;
        if (need) {
          wave_sync();
          while (need) {
            const int u = __ffsll((long long)need) - 1;
            need &= need - 1;
            compact_user(g, u, lim);
          }
        }
      }
    }
  };

  // ring of 4 register buffers: the loads of step t+3 are in flight while step t is
  // processed (F comes from HBM and is not shared between waves, so the wave needs its
  // own memory-level parallelism); past the end the loads are clamped and harmless
  float af0[Q], af1[Q], af2[Q], af3[Q];
  double f0[NG][4], f1[NG][4], f2[NG][4], f3[NG][4];
  load_step(0, af0, f0);
  load_step(16, af1, f1);
  load_step(32, af2, f2);
  for (int it = 0;; it += 64) {
    load_step(it + 48, af3, f3);
    process(it, af0, f0);
    if (it + 16 >= n_cols) break;
    load_step(it + 64, af0, f0);
    process(it + 16, af1, f1);
    if (it + 32 >= n_cols) break;
    load_step(it + 80, af1, f1);
    process(it + 32, af2, f2);
    if (it + 48 >= n_cols) break;
    load_step(it + 96, af2, f2);
    process(it + 48, af3, f3);
    if (it + 64 >= n_cols) break;
  }

  wave_sync();
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    for (int u = 0; u < 16; ++u) {
      const int64_t r = ubase + g * 16 + u;
      if (r >= n_rows) break;
      if (!__shfl((int)dirty[g], u)) continue;  // list as loaded: nothing to compact or store
      compact_user(g, u, lim_end);
      const int nc = __shfl(cnt[g], u);
      for (int e = lane; e < k; e += 64) {
        const double v = e < nc ? cs[wave][g][u][e] : neg_inf<double>();
        const bool ok = e < nc && v != neg_inf<double>();  // dropped entries never surface
        io_val[r * k + e] = ok ? v : neg_inf<double>();
        io_idx[r * k + e] = ok ? ci[wave][g][u][e] : -1;
      }
      wave_sync();
    }
  }
}

// fp32 score of one (user, item) pair: the chain of lg_score_topk_f32 / the MFMA tile,
//   acc = 0; for s < D/4: for g < 4: acc = fmaf(u[g*D/4+s], i[g*D/4+s], acc),
// with u in LDS (read as a broadcast) and the item row from global memory.
template <int D>
__device__ __forceinline__ float chain_score(const float *us, const float *__restrict__ it) {
  constexpr int Q = D / 4;
  float a = 0.f;
#pragma unroll 1
  for (int s0 = 0; s0 < Q; s0 += 4) {
    float4 q[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) q[g] = *reinterpret_cast<const float4 *>(it + g * Q + s0);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float x = s == 0 ? q[g].x : (s == 1 ? q[g].y : (s == 2 ? q[g].z : q[g].w));
        a = fmaf(us[g * Q + s0 + s], x, a);
      }
  }
  return a;
}

// ------------------------------------------------------------ the tile walk kernel
// One launch per tile. Persistent waves (NW per workgroup, one workgroup per CU; each wave
// takes users u, u + G, u + 2G, ... with G = all waves): a user's chain is row pointers ->
// item ids -> RowMeta -> slots, so while user u's slots are in flight the wave already has
// the RowMeta of u+G, the item ids of u+2G and the row pointers of u+3G in flight (and, for
// the top-K mode, u's list, score bounds, embedding and exclusion window).
//
// MODE_F:    F[u][j - item_begin] = the accumulator (lg_spread_tile_resource_f64).
// MODE_TOPK: the tile's columns of (G *) F merge into the running per-user top-K lists
//            (lg_spread_tile_resource_topk_f64); F never leaves LDS. With a G factor, a
//            column's score can only beat the list's K-th value tau if gb * F > tau, gb =
//            the (user, 64-column chunk) upper bound of the fp32 score chain from
//            lg_score_chunk_bound (bf16 MFMA + a rigorous rounding margin); only those
//            columns get the exact chain score. Ids grow along the walk, so "beats" is
//            v > tau (a tie loses to the older, smaller id).
constexpr int MODE_F = 0, MODE_TOPK = 1;

struct WalkArgs {
  const int64_t *user_rowptr;
  const int32_t *user_items;
  int64_t n_users;
  const RowMeta *wt_meta;
  const uint32_t *wt_ent;
  int32_t item_begin, tile, width;
  const double *beta;   // all items
  const double *g_inv;  // fl(1/k) per degree class
  // MODE_F
  double *F;
  int64_t ldf;
  // MODE_TOPK
  const float *eu, *ei;       // rows' user embeddings / all item embeddings (or NULL)
  const float *gb;            // [n_users][nch] score bounds (with eu)
  int32_t nch;
  const int64_t *ex_rowptr;   // exclusions (dropped), with a per-row cursor
  const int32_t *ex_col;
  int64_t *ex_cur;
  int k, first;
  double *io_val;
  int64_t *io_idx;
};

template <int MODE, int D, int M>
__host__ __device__ constexpr size_t walk_wave_bytes(int tile) {
  return ((size_t)tile * 8 + sizeof(RowIndex) + 1024 +
          (MODE == MODE_TOPK ? (size_t)64 * M * 12 + (size_t)(D > 0 ? D : 4) * 4 +
                                   (D > 0 ? (size_t)128 * 12 : 0)
                             : 0) + 15) &
         ~(size_t)15;
}
__host__ __device__ constexpr size_t walk_shared_bytes(int tile) {
  return (size_t)tile * 8 + (size_t)kInvTab * 8;
}

template <int MODE, int UF, int D, int M>
__global__ __launch_bounds__(512) void k_tile_walk(WalkArgs a) {
  constexpr int CAP = 64 * M;
  extern __shared__ double lds[];
  const int nw = blockDim.x / 64;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const int lane = lane_id();
  const int tile = a.tile;
  double *s_beta = lds;
  double *s_inv = s_beta + tile;
  char *mine = reinterpret_cast<char *>(s_inv + kInvTab) +
               (size_t)wave * walk_wave_bytes<MODE, D, M>(tile);
  double *acc = reinterpret_cast<double *>(mine);
  RowIndex *ix = reinterpret_cast<RowIndex *>(acc + tile);
  uint32_t *tr = reinterpret_cast<uint32_t *>(ix + 1);  // 256-slot transpose scratch
  double *cs = reinterpret_cast<double *>(tr + 256);
  int *ci = reinterpret_cast<int *>(cs + CAP);
  float *us = reinterpret_cast<float *>(ci + CAP);
  double *pf = reinterpret_cast<double *>(us + (D > 0 ? D : 4));  // candidate queue (D > 0)
  int *pj = reinterpret_cast<int *>(pf + 128);
  (void)cs; (void)ci; (void)us; (void)pf; (void)pj;

  for (int j = threadIdx.x; j < tile; j += blockDim.x)
    s_beta[j] = j < a.width ? a.beta[a.item_begin + j] : 0.0;
  for (int c = threadIdx.x; c < kInvTab; c += blockDim.x) s_inv[c] = a.g_inv[c];
  for (int j = lane; j < tile; j += 64) acc[j] = 0.0;
  __syncthreads();

  const int64_t G = (int64_t)gridDim.x * nw;
  int64_t u = (int64_t)blockIdx.x * nw + wave;
  const int64_t n_users = a.n_users;
  if (u >= n_users) return;

  auto rows = [&](int64_t v, int64_t &b, int64_t &e) __attribute__((always_inline)) {
    b = e = 0;
    if (v < n_users) {
      b = a.user_rowptr[v];
      e = a.user_rowptr[v + 1];
    }
  };
  auto items = [&](int64_t b, int64_t e, int32_t &i0, int32_t &i1) __attribute__((always_inline)) {
    i0 = b + lane < e ? a.user_items[b + lane] : -1;
    i1 = b + 64 + lane < e ? a.user_items[b + 64 + lane] : -1;
  };
  auto meta = [&](int32_t i0, int32_t i1, RowMeta &m0, RowMeta &m1) __attribute__((always_inline)) {
    m0 = i0 >= 0 ? a.wt_meta[i0] : RowMeta{0, 0.0};
    m1 = i1 >= 0 ? a.wt_meta[i1] : RowMeta{0, 0.0};
  };

  int64_t b0, e0, b1, e1, b2, e2;
  rows(u, b0, e0);
  rows(u + G, b1, e1);
  rows(u + 2 * G, b2, e2);
  int32_t ia, ib, ja, jb;
  items(b0, e0, ia, ib);
  items(b1, e1, ja, jb);
  RowMeta ma, mb;
  meta(ia, ib, ma, mb);
  int64_t xc_next = 0;  // exclusion cursor of the next user (MODE_TOPK)
  if constexpr (MODE == MODE_TOPK)
    if (a.ex_rowptr) xc_next = a.ex_cur[u];
  int total = write_row_index(ix, ma, mb);
  for (;;) {
    int32_t ka, kb;
    items(b2, e2, ka, kb);           // u+2G
    RowMeta na, nb;
    meta(ja, jb, na, nb);            // u+G
    int64_t b3, e3;
    rows(u + 3 * G, b3, e3);         // u+3G
    // ---- this user's top-K inputs, in flight beside its slots
    const int k = a.k;
    int64_t lid0 = -1, lid1 = -1;
    double lv0 = 0.0, lv1 = 0.0;
    float gbv = 0.f, uev0 = 0.f, uev1 = 0.f;
    int64_t xpos = 0, xhi = 0, xc_after = 0;
    int32_t xw = 0x7fffffff;
    if constexpr (MODE == MODE_TOPK) {
      if (!a.first) {
        if (lane < k) { lid0 = a.io_idx[u * k + lane]; lv0 = a.io_val[u * k + lane]; }
        if (64 + lane < k) { lid1 = a.io_idx[u * k + 64 + lane]; lv1 = a.io_val[u * k + 64 + lane]; }
      }
      if constexpr (D > 0) {
        if (lane < a.nch) gbv = a.gb[u * a.nch + lane];
        if (lane < D) uev0 = a.eu[u * D + lane];
        if (D > 64 && 64 + lane < D) uev1 = a.eu[u * D + 64 + lane];
      }
      if (a.ex_rowptr) {
        xpos = xc_next;
        xhi = a.ex_rowptr[u + 1];
        if (u + G < n_users) xc_after = a.ex_cur[u + G];
        if (xpos + lane < xhi) xw = a.ex_col[xpos + lane];
      }
    }
    accumulate_group<UF>(acc, ix, total, a.wt_ent, s_beta, s_inv, a.g_inv, tr);
    for (int64_t p0 = b0 + kResRows; p0 < e0; p0 += kResRows) {  // rows beyond 128 items
      int32_t xa, xb;
      items(p0, e0, xa, xb);
      RowMeta ya, yb;
      meta(xa, xb, ya, yb);
      const int t2 = write_row_index(ix, ya, yb);
      accumulate_group<UF>(acc, ix, t2, a.wt_ent, s_beta, s_inv, a.g_inv, tr);
    }
    wave_sync();
    if constexpr (MODE == MODE_F) {
      double *row = a.F + u * a.ldf;
      for (int j = lane; j < tile; j += 64) {
        __builtin_nontemporal_store(acc[j], row + j);
        acc[j] = 0.0;
      }
    } else {
      // running list -> LDS (valid entries form a sorted prefix)
      int cnt = __popcll(__ballot(lid0 >= 0)) + __popcll(__ballot(lid1 >= 0));
      if (lid0 >= 0) { cs[lane] = lv0; ci[lane] = (int)lid0; }
      if (lid1 >= 0) { cs[64 + lane] = lv1; ci[64 + lane] = (int)lid1; }
      if constexpr (D > 0) {
        if (lane < D) us[lane] = uev0;
        if (D > 64 && 64 + lane < D) us[64 + lane] = uev1;
      }
      // excluded items of this tile (the next run of the user's sorted exclusion row): -1
      const int32_t lim = a.item_begin + a.width;
      if (a.ex_rowptr) {
        for (;;) {
          const bool in = xw < lim;
          if (in && xw >= a.item_begin) acc[xw - a.item_begin] = -1.0;
          const int nin = __popcll(__ballot(in));
          xpos += nin;
          if (nin < 64) break;
          xw = xpos + lane < xhi ? a.ex_col[xpos + lane] : 0x7fffffff;  // > 64 in one tile
        }
        if (lane == 0) a.ex_cur[u] = xpos;
      }
      wave_sync();
      double tau = neg_inf<double>();
      int tau_id = kPadId;
      if (cnt == k) { tau = cs[k - 1]; tau_id = ci[k - 1]; }
      bool dirty = a.first != 0;
      // insert the lanes' (v, item) with cand set; compact when the list could overflow
      auto insert = [&](bool cand, double v, int item) __attribute__((always_inline)) {
        const uint64_t bal = __ballot(cand);
        if (!bal) return;
        dirty = true;
        const int p = cnt + __popcll(bal & lanemask_lt());
        if (cand) {
          cs[p] = v;
          ci[p] = item;
        }
        cnt += __popcll(bal);
        if (cnt > CAP - 64) {
          wave_sync();
          cnt = wave_compact<double, M>(cs, ci, cnt, k, tau, tau_id);
        }
      };
      if constexpr (D > 0) {
        // columns whose bound gb * F beats tau are queued (pj/pf, ascending), and scored
        // 64 at a time, one lane each: one round of item-row loads per 64 candidates
        int np = 0;
        auto flush = [&](int m) __attribute__((always_inline)) {
          wave_sync();
          bool cand = lane < m;
          double v = 0.0;
          int item = 0;
          if (cand) {
            item = a.item_begin + pj[lane];
            v = (double)chain_score<D>(us, a.ei + (int64_t)item * D) * pf[lane];
            cand = v > tau;
          }
          wave_sync();
          if (np > 64) {  // keep the queue's tail
            if (lane < np - 64) { pj[lane] = pj[64 + lane]; pf[lane] = pf[64 + lane]; }
          }
          np = np > 64 ? np - 64 : 0;
          insert(cand, v, item);
        };
        for (int c0 = 0; c0 < a.width; c0 += 64) {
          const int j = c0 + lane;
          const double f = j < a.width ? acc[j] : -1.0;
          if (j < tile) acc[j] = 0.0;
          const float gbc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gbv), c0 >> 6));
          const bool cand = f >= 0.0 && (double)gbc * f > tau;
          const uint64_t bal = __ballot(cand);
          if (bal) {
            const int p = np + __popcll(bal & lanemask_lt());
            if (cand) {
              pj[p] = j;
              pf[p] = f;
            }
            np += __popcll(bal);
            if (np >= 64) flush(64);
          }
        }
        while (np > 0) flush(np < 64 ? np : 64);
      } else {
        for (int c0 = 0; c0 < a.width; c0 += 64) {
          const int j = c0 + lane;
          const double f = j < a.width ? acc[j] : -1.0;
          if (j < tile) acc[j] = 0.0;
          insert(f >= 0.0 && f > tau, f, a.item_begin + j);
        }
      }
      if (dirty) {
        wave_sync();
        const int nc = wave_compact<double, M>(cs, ci, cnt, k, tau, tau_id);
        for (int e = lane; e < k; e += 64) {
          a.io_val[u * k + e] = e < nc ? cs[e] : neg_inf<double>();
          a.io_idx[u * k + e] = e < nc ? ci[e] : -1;
        }
      }
      wave_sync();
      xc_next = xc_after;
    }
    const bool more = u + G < n_users;
    if (!more) break;
    total = write_row_index(ix, na, nb);
    u += G;
    b0 = b1; e0 = e1;
    b1 = b2; e1 = e2;
    b2 = b3; e2 = e3;
    ja = ka; jb = kb;
  }
}

template <int D, bool VEC>
static void launch_tile_topk_v(int M, const double *F, int64_t ldf, int64_t n_rows, int32_t j0,
                               int32_t n_cols, const float *eu, const float *ei,
                               const int64_t *ex_rowptr, const int32_t *ex_col, int drop,
                               int k, int first, double *io_val, int64_t *io_idx,
                               hipStream_t s) {
  // LDS per block (2 waves): 2 * NG * 16 * S * 12 B (+ 512 B) = 48 KiB (M=1, NG=2, S=64;
  // 3 blocks = 6 waves per CU), 30 KiB at S=40 (k <= 24: 8 waves per CU, VGPR-limited; the
  // list is compacted once it holds more than S-16 entries, so the first span of a walk,
  // where most columns enter, keeps S=64), 48 KiB (M=2), 96 KiB (M=4). Measured per 4096-
  // column span at 1M users: S=40 8.4-8.6 ms vs S=64 8.8-9.1 ms after the first spans,
  // 26.4 vs 16.7 ms on the first. LGCNHS_TILE_TOPK_S64=1 (A/B knob) keeps S=64 throughout.
  static int s64 = -1;
  if (s64 < 0) {
    const char *e = getenv("LGCNHS_TILE_TOPK_S64");
    s64 = e ? atoi(e) : 0;
  }
  if (M == 1 && k <= 24 && !first && !s64) {
    const unsigned b = (unsigned)((n_rows + 63) / 64);
    k_tile_topk<D, 2, 1, VEC, 40><<<b, 128, 0, s>>>(F, ldf, n_rows, j0, n_cols, eu, ei,
                                                    ex_rowptr, ex_col, drop, k, first, io_val,
                                                    io_idx);
  } else if (M == 1) {
    const unsigned b = (unsigned)((n_rows + 63) / 64);
    k_tile_topk<D, 2, 1, VEC, 64><<<b, 128, 0, s>>>(F, ldf, n_rows, j0, n_cols, eu, ei,
                                                    ex_rowptr, ex_col, drop, k, first, io_val,
                                                    io_idx);
  } else if (M == 2) {
    const unsigned b = (unsigned)((n_rows + 31) / 32);
    k_tile_topk<D, 1, 2, VEC, 128><<<b, 128, 0, s>>>(F, ldf, n_rows, j0, n_cols, eu, ei,
                                                     ex_rowptr, ex_col, drop, k, first, io_val,
                                                     io_idx);
  } else {
    const unsigned b = (unsigned)((n_rows + 31) / 32);
    k_tile_topk<D, 1, 4, VEC, 256><<<b, 128, 0, s>>>(F, ldf, n_rows, j0, n_cols, eu, ei,
                                                     ex_rowptr, ex_col, drop, k, first, io_val,
                                                     io_idx);
  }
}

template <int D>
static void launch_tile_topk(int M, const double *F, int64_t ldf, int64_t n_rows, int32_t j0,
                             int32_t n_cols, const float *eu, const float *ei,
                             const int64_t *ex_rowptr, const int32_t *ex_col, int drop, int k,
                             int first, double *io_val, int64_t *io_idx, hipStream_t s) {
  // 16-byte F reads need rows padded to whole steps. (An inline-asm buffer-load form of the
  // ring with hand-counted waits was measured no faster: 9.2 vs 8.9 ms per 4096-column span.)
  const bool vec = ldf >= ((int64_t)n_cols + 15) / 16 * 16 && (ldf % 2) == 0 &&
                   ((uintptr_t)F % 16) == 0;
  if (vec)
    launch_tile_topk_v<D, true>(M, F, ldf, n_rows, j0, n_cols, eu, ei, ex_rowptr, ex_col, drop, k,
                             first, io_val, io_idx, s);
  else
    launch_tile_topk_v<D, false>(M, F, ldf, n_rows, j0, n_cols, eu, ei, ex_rowptr, ex_col, drop, k,
                             first, io_val, io_idx, s);
}

// Merge n_lists sorted top-K lists per row ([n_lists][n_rows][k], index -1 = empty) into one
// ([n_rows][k]): the item-range shards of a multi-GPU spreading run. One wave per row, the
// candidate list in LDS (CAP = 64*M >= k + 64), compacted by the wave-wide bitonic sort.
template <int M>
__global__ __launch_bounds__(256) void k_lists_merge_f64(const double *__restrict__ in_val,
                                                         const int64_t *__restrict__ in_idx,
                                                         int n_lists, int64_t n_rows, int k,
                                                         double *__restrict__ out_val,
                                                         int64_t *__restrict__ out_idx) {
  constexpr int CAP = 64 * M;
  __shared__ double cs[4][CAP];
  __shared__ int ci[4][CAP];
  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= n_rows) return;
  int cnt = 0;
  double tau = neg_inf<double>();
  int tau_id = kPadId;
  for (int s = 0; s < n_lists; ++s) {
    const int64_t base = ((int64_t)s * n_rows + row) * k;
    for (int e0 = 0; e0 < k; e0 += 64) {
      const int e = e0 + lane;
      double v = neg_inf<double>();
      int id = -1;
      if (e < k) {
        const int64_t x = in_idx[base + e];
        if (x >= 0) {
          v = in_val[base + e];
          id = (int)x;
        }
      }
      const bool cand = id >= 0 && before(v, id, tau, tau_id);
      const uint64_t bal = __ballot(cand);
      const int pos = cnt + __popcll(bal & lanemask_lt());
      if (cand) {
        cs[wave][pos] = v;
        ci[wave][pos] = id;
      }
      cnt += __popcll(bal);
      if (cnt > CAP - 64) {
        wave_sync();
        cnt = wave_compact<double, M>(cs[wave], ci[wave], cnt, k, tau, tau_id);
      }
    }
  }
  wave_sync();
  const int nc = wave_compact<double, M>(cs[wave], ci[wave], cnt, k, tau, tau_id);
  for (int e = lane; e < k; e += 64) {
    out_val[row * k + e] = e < nc ? cs[wave][e] : neg_inf<double>();
    out_idx[row * k + e] = e < nc ? ci[wave][e] : -1;
  }
}

}  // namespace lg

using namespace lg;

extern "C" int lg_spread_tile_seek(const int64_t *user_rowptr, const int32_t *user_items,
                                   int64_t n_users, int32_t item_begin, int64_t *cur,
                                   lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && cur && n_users >= 0 && item_begin >= 0,
             "lg_spread_tile_seek: bad arguments");
  if (n_users == 0) return LG_OK;
  k_tile_seek<<<dim3((unsigned)((n_users + 255) / 256)), dim3(256), 0, (hipStream_t)stream>>>(
      user_rowptr, user_items, n_users, item_begin, cur);
  return launch_status("lg_spread_tile_seek");
}

extern "C" int lg_topk_lists_merge_f64(const double *in_val, const int64_t *in_idx,
                                       int32_t n_lists, int64_t n_rows, int32_t k,
                                       double *out_val, int64_t *out_idx, lg_stream_t stream) {
  LG_REQUIRE(n_lists >= 1 && n_rows >= 0, "lg_topk_lists_merge_f64: bad sizes");
  LG_REQUIRE(k >= 1 && k <= 128, "lg_topk_lists_merge_f64: k=%d not in [1,128]", k);
  LG_REQUIRE(n_rows == 0 || (in_val && in_idx && out_val && out_idx),
             "lg_topk_lists_merge_f64: NULL argument");
  if (n_rows == 0) return LG_OK;
  const dim3 grid((unsigned)((n_rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (k <= 64)
    k_lists_merge_f64<2><<<grid, dim3(256), 0, s>>>(in_val, in_idx, n_lists, n_rows, k, out_val,
                                                    out_idx);
  else
    k_lists_merge_f64<4><<<grid, dim3(256), 0, s>>>(in_val, in_idx, n_lists, n_rows, k, out_val,
                                                    out_idx);
  return launch_status("lg_topk_lists_merge_f64");
}

extern "C" int lg_hybrid_factors_f64(const double *k_item, int64_t n_items, double lambda,
                                     double *alpha, double *beta, lg_stream_t stream) {
  LG_REQUIRE(k_item && alpha && beta && n_items >= 0, "lg_hybrid_factors_f64: bad arguments");
  if (n_items == 0) return LG_OK;
  k_hybrid_factors<<<dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream>>>(k_item, n_items, lambda, alpha, beta);
  return launch_status("lg_hybrid_factors_f64");
}

extern "C" int lg_inv_degree_f64(const int64_t *rowptr, int64_t n_rows, double *inv,
                                 lg_stream_t stream) {
  LG_REQUIRE(rowptr && inv && n_rows >= 0, "lg_inv_degree_f64: bad arguments");
  if (n_rows == 0) return LG_OK;
  k_inv_degree<<<dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, (hipStream_t)stream>>>(
      rowptr, n_rows, inv);
  return launch_status("lg_inv_degree_f64");
}

extern "C" int lg_spread_tile_cursor(const int64_t *user_rowptr, const int32_t *user_items,
                                     int64_t n_users, int32_t item_end, const int64_t *cur,
                                     int64_t *end, uint16_t *count, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && cur && end && count && n_users >= 0 && cur != end,
             "lg_spread_tile_cursor: bad arguments");
  if (n_users == 0) return LG_OK;
  k_tile_cursor<<<dim3((unsigned)((n_users + 255) / 256)), dim3(256), 0,
                  (hipStream_t)stream>>>(user_rowptr, user_items, n_users, item_end, cur, end,
                                         count);
  return launch_status("lg_spread_tile_cursor");
}

extern "C" int lg_spread_tile_bound(const int64_t *item_rowptr, const int32_t *item_users,
                                    int64_t n_items, const uint16_t *count, int64_t *bound,
                                    lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && count && bound && n_items >= 0,
             "lg_spread_tile_bound: bad arguments");
  if (n_items == 0) return LG_OK;
  k_tile_bound<<<dim3((unsigned)((n_items + 3) / 4)), dim3(256), 0, (hipStream_t)stream>>>(
      item_rowptr, item_users, n_items, count, bound);
  return launch_status("lg_spread_tile_bound");
}

extern "C" size_t lg_spread_tile_weight_ws_bytes(int64_t n_items) {
  return (size_t)(n_items + 1) * sizeof(int64_t);  // hub count + hub row list
}

extern "C" int lg_spread_tile_weight_f64(const int64_t *item_rowptr, const int32_t *item_users,
                                         const int32_t *user_items, const uint16_t *user_cls,
                                         const double *inv_deg, int64_t n_items,
                                         const int64_t *cur, const uint16_t *count,
                                         const double *alpha, const double *beta,
                                         int32_t item_begin, int32_t tile, const int64_t *bound,
                                         const int64_t *wt_ptr, void *wt_ent, void *wt_meta,
                                         void *ws, size_t ws_bytes, lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && user_cls && inv_deg && cur && count && alpha && beta && bound &&
                 wt_ptr && wt_ent && wt_meta && n_items >= 0,
             "lg_spread_tile_weight_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && item_begin >= 0,
             "lg_spread_tile_weight_f64: tile %d not in [1, 8192]", tile);
  if (n_items == 0) return LG_OK;
  const size_t need = lg_spread_tile_weight_ws_bytes(n_items);
  if (!ws || ws_bytes < need) {
    set_error("lg_spread_tile_weight_f64: workspace %zu < %zu bytes", ws_bytes, need);
    return LG_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  int64_t *n_hub = (int64_t *)ws;
  int64_t *hub_rows = n_hub + 1;
  if (hipMemsetAsync(n_hub, 0, sizeof(int64_t), s) != hipSuccess) {
    set_error("lg_spread_tile_weight_f64: hipMemsetAsync failed");
    return LG_ERR_HIP;
  }
  const unsigned rb = (unsigned)((n_items + 3) / 4);
  k_tile_weight<<<dim3(rb), dim3(256), 0, s>>>(item_rowptr, item_users, user_items, user_cls,
                                               n_items, cur, count, alpha, item_begin, bound,
                                               wt_ptr, (uint32_t *)wt_ent, (RowMeta *)wt_meta);
  k_hub_list<<<dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, s>>>(
      bound, n_items, (unsigned long long *)n_hub, hub_rows);
  k_tile_weight_hub<<<dim3(1024), dim3(256), (size_t)tile * sizeof(double), s>>>(
      hub_rows, n_hub, item_rowptr, item_users, user_items, inv_deg, cur, count, alpha, beta,
      item_begin, tile, wt_ptr, (uint32_t *)wt_ent, (RowMeta *)wt_meta);
  return launch_status("lg_spread_tile_weight_f64");
}

static int n_cus() {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
      n_cu = 256;
  }
  return n_cu;
}

// waves per workgroup: as many as the LDS holds next to the shared tables (<= 8), one
// workgroup per CU, persistent
template <int MODE, int UF, int D, int M>
static int launch_walk(const WalkArgs &a, hipStream_t s) {
  const size_t per = walk_wave_bytes<MODE, D, M>(a.tile);
  const size_t shared = walk_shared_bytes(a.tile);
  const size_t budget = 160 * 1024;
  int nw = (int)((budget - shared) / per);
  if (nw > 8) nw = 8;
  if (nw < 1) {
    set_error("tile walk: tile %d needs %zu bytes of LDS per wave", a.tile, per + shared);
    return LG_ERR_ARG;
  }
  const int64_t want = (a.n_users + nw - 1) / nw;
  const int64_t cap = n_cus();
  const unsigned blocks = (unsigned)(want < cap ? want : cap);
  const size_t lds = shared + (size_t)nw * per;
  k_tile_walk<MODE, UF, D, M><<<dim3(blocks), dim3(64 * nw), lds, s>>>(a);
  return LG_OK;
}

extern "C" int lg_spread_tile_resource_f64(const int64_t *user_rowptr,
                                           const int32_t *user_items, int64_t n_users,
                                           const void *wt_meta, const void *wt_ent,
                                           const double *beta, const double *inv_cls,
                                           int32_t item_begin, int32_t tile, int32_t width,
                                           double *F, int64_t ldf, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && wt_meta && beta && inv_cls && F && n_users >= 0 && ldf >= tile,
             "lg_spread_tile_resource_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && width >= 1 && width <= tile,
             "lg_spread_tile_resource_f64: tile %d / width %d", tile, width);
  if (n_users == 0) return LG_OK;
  WalkArgs a{};
  a.user_rowptr = user_rowptr;
  a.user_items = user_items;
  a.n_users = n_users;
  a.wt_meta = (const RowMeta *)wt_meta;
  a.wt_ent = (const uint32_t *)wt_ent;
  a.item_begin = item_begin;
  a.tile = tile;
  a.width = width;
  a.beta = beta;
  a.g_inv = inv_cls;
  a.F = F;
  a.ldf = ldf;
  const int st = launch_walk<MODE_F, 4, 0, 1>(a, (hipStream_t)stream);
  if (st != LG_OK) return st;
  return launch_status("lg_spread_tile_resource_f64");
}

extern "C" int lg_tile_topk_f64(const double *F, int64_t ldf, int64_t n_rows,
                                int32_t item_begin, int32_t n_cols, const float *eu,
                                const float *ei, int32_t dim, const int64_t *ex_rowptr,
                                const int32_t *ex_col, int32_t excl_mode, int32_t k,
                                int32_t first, double *io_val, int64_t *io_idx,
                                lg_stream_t stream) {
  LG_REQUIRE(F && io_val && io_idx && n_rows >= 0 && n_cols >= 1 && ldf >= n_cols &&
                 item_begin >= 0 && (int64_t)item_begin + n_cols < 0x7fffffff,
             "lg_tile_topk_f64: bad arguments");
  LG_REQUIRE(k >= 1 && k <= 128, "lg_tile_topk_f64: k=%d not in [1,128]", k);
  LG_REQUIRE(!eu == !ei, "lg_tile_topk_f64: eu/ei must both be set or both NULL");
  LG_REQUIRE(!eu || dim == 32 || dim == 64 || dim == 128,
             "lg_tile_topk_f64: dim %d not in {32,64,128}", dim);
  LG_REQUIRE(excl_mode == LG_EXCL_DROP || excl_mode == LG_EXCL_NONE,
             "lg_tile_topk_f64: bad excl_mode %d", excl_mode);
  LG_REQUIRE(!ex_rowptr == !ex_col, "lg_tile_topk_f64: ex_rowptr/ex_col must both be set");
  LG_REQUIRE(!(eu && excl_mode == LG_EXCL_NONE && ex_rowptr),
             "lg_tile_topk_f64: a G factor with exclusions requires LG_EXCL_DROP");
  if (n_rows == 0) return LG_OK;
  hipStream_t s = (hipStream_t)stream;
  const int M = k <= 32 ? 1 : (k <= 64 ? 2 : 4);
  const int drop = excl_mode == LG_EXCL_DROP;
  switch (eu ? dim : 0) {
    case 0: launch_tile_topk<0>(M, F, ldf, n_rows, item_begin, n_cols, eu, ei, ex_rowptr, ex_col, drop, k, first, io_val, io_idx, s); break;
    case 32: launch_tile_topk<32>(M, F, ldf, n_rows, item_begin, n_cols, eu, ei, ex_rowptr, ex_col, drop, k, first, io_val, io_idx, s); break;
    case 64: launch_tile_topk<64>(M, F, ldf, n_rows, item_begin, n_cols, eu, ei, ex_rowptr, ex_col, drop, k, first, io_val, io_idx, s); break;
    default: launch_tile_topk<128>(M, F, ldf, n_rows, item_begin, n_cols, eu, ei, ex_rowptr, ex_col, drop, k, first, io_val, io_idx, s); break;
  }
  return launch_status("lg_tile_topk_f64");
}

extern "C" size_t lg_spread_tile_resource_topk_lds_bytes(int32_t tile, int32_t k, int32_t dim) {
  // one wave's share plus the workgroup's tables (the launch fits as many waves as it can)
  const int M = k <= 64 ? 2 : 4;
  const size_t per = M == 2 ? (dim > 64 ? walk_wave_bytes<MODE_TOPK, 128, 2>(tile)
                                        : walk_wave_bytes<MODE_TOPK, 64, 2>(tile))
                            : walk_wave_bytes<MODE_TOPK, 128, 4>(tile);
  return per + walk_shared_bytes(tile);
}

template <int D>
static int launch_fused(int M, const WalkArgs &a, hipStream_t s) {
  // LGCNHS_WALK_UC (A/B knob): 4-slot chunk registers per block (2 or 8; default 4)
  static int uc = -1;
  if (uc < 0) {
    const char *e = getenv("LGCNHS_WALK_UC");
    uc = e ? atoi(e) : 4;
  }
  if (M == 2 && uc == 2) return launch_walk<MODE_TOPK, 2, D, 2>(a, s);
  if (M == 2 && uc == 8) return launch_walk<MODE_TOPK, 8, D, 2>(a, s);
  return M == 2 ? launch_walk<MODE_TOPK, 4, D, 2>(a, s) : launch_walk<MODE_TOPK, 4, D, 4>(a, s);
}

extern "C" int lg_spread_tile_resource_topk_f64(
    const int64_t *user_rowptr, const int32_t *user_items, int64_t n_users,
    const void *wt_meta, const void *wt_ent, const double *beta, const double *inv_cls,
    int32_t item_begin, int32_t tile, int32_t width, const float *eu, const float *ei,
    int32_t dim, const float *gb, int32_t n_chunks, const int64_t *ex_rowptr,
    const int32_t *ex_col, int64_t *ex_cur, int32_t k, int32_t first, double *io_val,
    int64_t *io_idx, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && wt_meta && beta && inv_cls && io_val && io_idx && n_users >= 0 &&
                 item_begin >= 0,
             "lg_spread_tile_resource_topk_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && width >= 1 && width <= tile &&
                 (int64_t)item_begin + width < 0x7fffffff,
             "lg_spread_tile_resource_topk_f64: tile %d / width %d", tile, width);
  LG_REQUIRE(k >= 1 && k <= 128, "lg_spread_tile_resource_topk_f64: k=%d not in [1,128]", k);
  LG_REQUIRE(!eu == !ei && !eu == !gb,
             "lg_spread_tile_resource_topk_f64: eu, ei and gb go together");
  LG_REQUIRE(!eu || dim == 32 || dim == 64 || dim == 128,
             "lg_spread_tile_resource_topk_f64: dim %d not in {32,64,128}", dim);
  LG_REQUIRE(!eu || n_chunks == (width + 63) / 64,
             "lg_spread_tile_resource_topk_f64: n_chunks %d != ceil(width / 64)", n_chunks);
  LG_REQUIRE(!ex_rowptr == !ex_col && !ex_rowptr == !ex_cur,
             "lg_spread_tile_resource_topk_f64: ex_rowptr/ex_col/ex_cur go together");
  if (n_users == 0) return LG_OK;
  WalkArgs a{};
  a.user_rowptr = user_rowptr;
  a.user_items = user_items;
  a.n_users = n_users;
  a.wt_meta = (const RowMeta *)wt_meta;
  a.wt_ent = (const uint32_t *)wt_ent;
  a.item_begin = item_begin;
  a.tile = tile;
  a.width = width;
  a.beta = beta;
  a.g_inv = inv_cls;
  a.eu = eu;
  a.ei = ei;
  a.gb = gb;
  a.nch = n_chunks;
  a.ex_rowptr = ex_rowptr;
  a.ex_col = ex_col;
  a.ex_cur = ex_cur;
  a.k = k;
  a.first = first;
  a.io_val = io_val;
  a.io_idx = io_idx;
  hipStream_t s = (hipStream_t)stream;
  const int M = k <= 64 ? 2 : 4;
  int st;
  switch (eu ? dim : 0) {
    case 0: st = launch_fused<0>(M, a, s); break;
    case 32: st = launch_fused<32>(M, a, s); break;
    case 64: st = launch_fused<64>(M, a, s); break;
    default: st = launch_fused<128>(M, a, s); break;
  }
  if (st != LG_OK) return st;
  return launch_status("lg_spread_tile_resource_topk_f64");
}

extern "C" int lg_row_norms_f64(const float *x, int64_t n_rows, int32_t dim, double *out,
                                lg_stream_t stream) {
  LG_REQUIRE(x && out && n_rows >= 0 && dim >= 1, "lg_row_norms_f64: bad arguments");
  if (n_rows == 0) return LG_OK;
  k_row_norms<<<dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, (hipStream_t)stream>>>(
      x, n_rows, dim, out);
  return launch_status("lg_row_norms_f64");
}
