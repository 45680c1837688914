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
//   bound    bound[i] = sum_{v in users(i)} (end[v] - cur[v]) >= entries of W's row i in
//            the tile; the caller's exclusive prefix of it is wt_ptr (row capacities)
//   weight   row i of W restricted to the tile: the (item j, user v) pairs of all
//            v in users(i) sorted by (j, v) in one wave (bitonic, <= 256 pairs), each run
//            of equal j summed in ascending v, divided by alpha[i] * beta[j]. Rows with
//            more than 256 pairs (hub items) go through a block-wide dense LDS tile with
//            the users walked in ascending order. Either way the value is, bit for bit,
//            lg_spread_general_f64's sum (ascending v, fl(1/k_v)) / lg_hybrid_weight_f64's
//            den, so the tiled path equals the dense one exactly.
//   resource F[u][j - j0] = sum_{i in items(u), ascending} W[i][j]: one wave per user, the
//            tile's accumulator in LDS; row i's entries are distinct columns, so rows are
//            added one after another without atomics (lg_spread_resource_f64's order).
//   topk     the tile's columns of (G *) F merged into running per-user top-K lists
//            (G = e0 score by f32 MFMA, the chain of lg_score_topk_f32, promoted to fp64).
// Work: the weight pass costs sum_i deg(i) lookups + the 2-hop pairs once per tile (not per
// user); the resource pass reads deg(u) short row segments per user and tile.
#include <stdlib.h>

#include "common.h"

namespace lg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// One entry of a W tile row: 12 bytes, {item, fp64 value as two dwords} (4-byte aligned, so
// a row of n entries is 12n contiguous bytes: fewer 128-B lines per random row than split
// column / value arrays). meta[i] = (row start) | (row length << 48).
struct WEnt {
  int32_t col;
  uint32_t lo, hi;
};
constexpr int kMetaShift = 48;
constexpr uint64_t kMetaPtrMask = (1ull << kMetaShift) - 1;

__device__ __forceinline__ void put_ent(WEnt *__restrict__ ent, int64_t pos, int32_t col,
                                        double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  ent[pos] = WEnt{col, (uint32_t)b, (uint32_t)(b >> 32)};
}

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

constexpr int kSortMax = 256;  // pairs per row handled by the in-wave sort

// Sort the n (<= 64*M) staged pairs (key = -item, id = staging position, which ascends
// with the user) of this wave, then reduce runs of equal items in ascending user order
// (weights sw[position] = fl(1/k_v)) and write the row.
template <int M>
__device__ __forceinline__ int sort_reduce_row(int *skey, int *sid, const double *sw, int n,
                                               int64_t wbase, double alpha_i,
                                               const double *__restrict__ beta,
                                               WEnt *__restrict__ wt_ent) {
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
  int base = 0;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int e = j * 64 + lane;
    const bool head = e < n && (e == 0 || skey[e] != skey[e - 1]);
    const uint64_t hb = __ballot(head);
    if (head) {
      // run e, e+1, ... of one item, users ascending: 0.0 + w0 + w1 + ... in that order
      const int item = -skey[e];
      double s = 0.0;
      for (int m = e; m < n && skey[m] == skey[e]; ++m) s += sw[sid[m]];
      double den = alpha_i * beta[item];
      if (den == 0.0) den = 1.0;
      const int pos = base + __popcll(hb & lanemask_lt());
      put_ent(wt_ent, wbase + pos, item, s / den);
    }
    base += __popcll(hb);
  }
  return base;
}

// one wave per item row; LDS staging of kSortMax pairs per wave
__global__ __launch_bounds__(256) void k_tile_weight(
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const double *__restrict__ inv_deg,
    int64_t n_items, const int64_t *__restrict__ cur, const uint16_t *__restrict__ count,
    const double *__restrict__ alpha, const double *__restrict__ beta,
    const int64_t *__restrict__ wt_ptr, WEnt *__restrict__ wt_ent,
    uint64_t *__restrict__ wt_meta) {
  __shared__ int skey[4][kSortMax];
  __shared__ int sid[4][kSortMax];
  __shared__ double sw[4][kSortMax];
  const int wave = threadIdx.x / 64;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave;
  if (i >= n_items) return;
  const int lane = lane_id();
  const int64_t wbase = wt_ptr[i];
  const int64_t bound = wt_ptr[i + 1] - wbase;
  if (bound == 0) {
    if (lane == 0) wt_meta[i] = (uint64_t)wbase;
    return;
  }
  if (bound > kSortMax) return;  // hub row: k_tile_weight_hub
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
    // exclusive prefix of c over the lanes
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
      const double w = inv_deg[v];
      for (int q = 0; q < c; ++q) {
        const int p = n + pre + q;
        skey[wave][p] = -user_items[s0 + q];
        sid[wave][p] = p;
        sw[wave][p] = w;
      }
    }
    n += total;
  }
  wave_sync();
  int len;
  if (n <= 64)
    len = sort_reduce_row<1>(skey[wave], sid[wave], sw[wave], n, wbase, alpha[i], beta,
                             wt_ent);
  else if (n <= 128)
    len = sort_reduce_row<2>(skey[wave], sid[wave], sw[wave], n, wbase, alpha[i], beta,
                             wt_ent);
  else
    len = sort_reduce_row<4>(skey[wave], sid[wave], sw[wave], n, wbase, alpha[i], beta,
                             wt_ent);
  if (lane == 0) wt_meta[i] = (uint64_t)wbase | ((uint64_t)len << kMetaShift);
}

// Hub rows (> kSortMax pairs): one 256-thread block per row (grid-stride over the hub list),
// the tile as a dense LDS accumulator, users walked in ascending order as in
// k_spread_general.
__global__ __launch_bounds__(256) void k_tile_weight_hub(
    const int64_t *__restrict__ hub_rows, const int64_t *__restrict__ n_hub,
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const double *__restrict__ inv_deg,
    const int64_t *__restrict__ cur, const uint16_t *__restrict__ count,
    const double *__restrict__ alpha, const double *__restrict__ beta, int32_t item_begin,
    int32_t tile, const int64_t *__restrict__ wt_ptr, WEnt *__restrict__ wt_ent,
    uint64_t *__restrict__ wt_meta) {
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
        const int item = item_begin + j;
        double den = a * beta[item];
        if (den == 0.0) den = 1.0;
        const int pos = base + before_w + __popcll(b & lanemask_lt());
        put_ent(wt_ent, wbase + pos, item, acc[j] / den);
      }
      base += total;
      __syncthreads();
    }
    if (threadIdx.x == 0) wt_meta[i] = (uint64_t)wbase | ((uint64_t)base << kMetaShift);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_hub_list(const int64_t *__restrict__ wt_ptr,
                                                  int64_t n_items,
                                                  unsigned long long *__restrict__ n_hub,
                                                  int64_t *__restrict__ hub_rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  if (wt_ptr[i + 1] - wt_ptr[i] > kSortMax) hub_rows[atomicAdd(n_hub, 1ull)] = i;
}

// Resource pass (F = A W over one tile): rows of 128 items per group, see k_tile_resource.
constexpr int kResRows = 128;
constexpr int kResIdxBytes = kResRows * (4 + 8);

// Prefix of a 128-row group's metadata (rows' entry counts and starts) into the wave's
// row index `idx`; returns the group's total entry count.
__device__ __forceinline__ int write_row_index(char *idx, uint64_t m0, uint64_t m1) {
  const int lane = lane_id();
  int64_t *s_base = reinterpret_cast<int64_t *>(idx);
  int *s_incl = reinterpret_cast<int *>(idx + kResRows * 8);
  const int rl0 = (int)(m0 >> kMetaShift), rl1 = (int)(m1 >> kMetaShift);
  int in0 = rl0, in1 = rl1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y0 = __shfl_up(in0, o), y1 = __shfl_up(in1, o);
    if (lane >= o) { in0 += y0; in1 += y1; }
  }
  in1 += __shfl(in0, 63);
  const int total = __shfl(in1, 63);
  wave_sync();  // earlier readers of this index are done
  s_incl[lane] = in0;
  s_incl[64 + lane] = in1;
  s_base[lane] = (int64_t)(m0 & kMetaPtrMask) - (in0 - rl0);
  s_base[64 + lane] = (int64_t)(m1 & kMetaPtrMask) - (in1 - rl1);
  wave_sync();
  return total;
}

// acc[j - item_begin] += the `total` flattened entries of one indexed row group.
template <int UF>
__device__ __forceinline__ void accumulate_group(double *acc, const char *idx, int total,
                                                 const WEnt *__restrict__ wt_ent,
                                                 int32_t item_begin) {
  const int lane = lane_id();
  const int64_t *s_base = reinterpret_cast<const int64_t *>(idx);
  const int *s_incl = reinterpret_cast<const int *>(idx + kResRows * 8);
  for (int e0 = 0; e0 < total; e0 += 64 * UF) {
    // r[q] = number of rows whose inclusive end is <= e[q] (the row holding entry e[q]):
    // the UF binary searches advance in lockstep (independent LDS reads per step, no
    // branch), then the UF entry loads issue back to back. Lanes past the end re-read
    // the last entry and skip the add.
    int e[UF], r[UF];
#pragma unroll
    for (int q = 0; q < UF; ++q) {
      const int x = e0 + q * 64 + lane;
      e[q] = x < total ? x : total - 1;
      r[q] = 0;
    }
#pragma unroll
    for (int st = 64; st > 0; st >>= 1)
#pragma unroll
      for (int q = 0; q < UF; ++q) r[q] += s_incl[r[q] + st - 1] <= e[q] ? st : 0;
    WEnt w[UF];
#pragma unroll
    for (int q = 0; q < UF; ++q) w[q] = wt_ent[s_base[r[q]] + e[q]];
#pragma unroll
    for (int q = 0; q < UF; ++q)
      if (e0 + q * 64 + lane < total)
        __hip_atomic_fetch_add(&acc[w[q].col - item_begin],
                               __hiloint2double((int)w[q].hi, (int)w[q].lo), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// acc[j - item_begin] += W[i][j] for every item i of user u (ascending), acc = the wave's
// LDS tile accumulator (zeroed by the caller), idx = its kResIdxBytes row index.
template <int UF>
__device__ __forceinline__ void accumulate_user_tile(double *acc, char *idx,
                                                     const int64_t *__restrict__ user_rowptr,
                                                     const int32_t *__restrict__ user_items,
                                                     int64_t u,
                                                     const uint64_t *__restrict__ wt_meta,
                                                     const WEnt *__restrict__ wt_ent,
                                                     int32_t item_begin) {
  const int lane = lane_id();
  const int64_t pb = user_rowptr[u], pe = user_rowptr[u + 1];
  for (int64_t p0 = pb; p0 < pe; p0 += kResRows) {
    uint64_t m0 = 0, m1 = 0;
    {
      const int32_t i0 = p0 + lane < pe ? user_items[p0 + lane] : -1;
      const int32_t i1 = p0 + 64 + lane < pe ? user_items[p0 + 64 + lane] : -1;
      if (i0 >= 0) m0 = wt_meta[i0];
      if (i1 >= 0) m1 = wt_meta[i1];
    }
    const int total = write_row_index(idx, m0, m1);
    accumulate_group<UF>(acc, idx, total, wt_ent, item_begin);
  }
  wave_sync();
}

// F[u][j - j0] = sum over items(u) ascending of W[i][j]; the tile's accumulator in LDS (tile
// doubles per wave) plus two 128-row indexes (LDS, 1.5 KiB each). Rows are taken 128 at a
// time: their metadata is fetched in one round trip (two loads per lane), then their entries
// are flattened: lane l takes entries e = e0 + q*64 + l of the concatenated rows (its row
// found by a binary search over the rows' inclusive length prefix in LDS), so each load
// instruction moves 64 useful 12-byte entries whatever the row lengths, UF of them in flight
// per lane. Entries go in with ds_add_f64; entries of one instruction that hit the same
// column come from rows in lane order, and rows are flattened in ascending order, so each
// column still receives its rows' values in ascending row order (the order of
// lg_spread_resource_f64).
//
// Persistent waves, software-pipelined over the users u, u+G, u+2G, ... of a wave (G = waves
// in the grid): a user's chain is row pointers -> item ids -> row metadata -> entries, four
// dependent memory round trips. While user u's entries are in flight the wave also has in
// flight the metadata of u+G, the item ids of u+2G and the row pointers of u+3G, so each user
// costs about one round trip (the first group of 128 items; longer rows add their groups
// unpipelined).
template <int UF, bool NT>
__global__ __launch_bounds__(128) void k_tile_resource(
    const int64_t *__restrict__ user_rowptr, const int32_t *__restrict__ user_items,
    int64_t n_users, const uint64_t *__restrict__ wt_meta, const WEnt *__restrict__ wt_ent,
    int32_t item_begin, int32_t tile, double *__restrict__ F, int64_t ldf) {
  extern __shared__ double lds[];
  const int wave = threadIdx.x / 64;
  const int wpb = blockDim.x / 64;
  const int lane = lane_id();
  const int64_t G = (int64_t)gridDim.x * wpb;
  int64_t u = (int64_t)blockIdx.x * wpb + wave;
  if (u >= n_users) return;
  double *acc = lds + (int64_t)wave * (tile + 2 * kResIdxBytes / 8);
  char *idx0 = reinterpret_cast<char *>(acc + tile);
  char *idx1 = idx0 + kResIdxBytes;
  for (int j = lane; j < tile; j += 64) acc[j] = 0.0;

  auto rows = [&](int64_t v, int64_t &b, int64_t &e) __attribute__((always_inline)) {
    b = e = 0;
    if (v < n_users) {
      b = user_rowptr[v];
      e = user_rowptr[v + 1];
    }
  };
  auto items = [&](int64_t b, int64_t e, int32_t &i0, int32_t &i1) __attribute__((always_inline)) {
    i0 = b + lane < e ? user_items[b + lane] : -1;
    i1 = b + 64 + lane < e ? user_items[b + 64 + lane] : -1;
  };
  auto meta = [&](int32_t i0, int32_t i1, uint64_t &m0, uint64_t &m1) __attribute__((always_inline)) {
    m0 = i0 >= 0 ? wt_meta[i0] : 0;
    m1 = i1 >= 0 ? wt_meta[i1] : 0;
  };

  // prologue: user u indexed; u+G's item ids and u+2G's row pointers loaded
  int64_t b0, e0, b1, e1, b2, e2;
  rows(u, b0, e0);
  rows(u + G, b1, e1);
  rows(u + 2 * G, b2, e2);
  int32_t ia, ib, ja, jb;
  items(b0, e0, ia, ib);
  items(b1, e1, ja, jb);
  uint64_t ma, mb;
  meta(ia, ib, ma, mb);
  char *cur = idx0, *nxt = idx1;
  int total = write_row_index(cur, ma, mb);
  for (;;) {
    int32_t ka, kb;
    items(b2, e2, ka, kb);           // u+2G
    uint64_t na, nb;
    meta(ja, jb, na, nb);            // u+G
    int64_t b3, e3;
    rows(u + 3 * G, b3, e3);         // u+3G
    accumulate_group<UF>(acc, cur, total, wt_ent, item_begin);
    for (int64_t p0 = b0 + kResRows; p0 < e0; p0 += kResRows) {  // rows beyond 128 items
      int32_t xa, xb;
      items(p0, e0, xa, xb);
      uint64_t ya, yb;
      meta(xa, xb, ya, yb);
      const int t2 = write_row_index(cur, ya, yb);
      accumulate_group<UF>(acc, cur, t2, wt_ent, item_begin);
    }
    wave_sync();
    const bool more = u + G < n_users;
    if (more) total = write_row_index(nxt, na, nb);
    double *row = F + u * ldf;
    for (int j = lane; j < tile; j += 64) {
      if constexpr (NT) __builtin_nontemporal_store(acc[j], row + j);
      else row[j] = acc[j];
      acc[j] = 0.0;
    }
    wave_sync();  // zeroes land before the next user's adds
    if (!more) break;
    u += G;
    char *t = cur;
    cur = nxt;
    nxt = t;
    b0 = b1; e0 = e1;
    b1 = b2; e1 = e2;
    b2 = b3; e2 = e3;
    ja = ka; jb = kb;
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
#pragma unroll
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

// Per-wave LDS of the fused kernel: the tile accumulator, the row index of
// accumulate_user_tile, the candidate list (CAP values + ids) and the user's embedding.
__host__ __device__ constexpr size_t fused_wave_bytes(int tile, int M, int D) {
  return (size_t)tile * 8 + kResIdxBytes + (size_t)64 * M * 12 + (size_t)D * 4;
}

// Fused resource + top-K for one tile (lg_spread_tile_resource_topk_f64): one wave per user.
// The user's F columns [item_begin, item_begin + width) are accumulated in LDS exactly as
// k_tile_resource does, the user's excluded items in the tile are marked (-1: F >= 0
// otherwise), and the columns merge straight into the running list: a column can only enter
// if (G *) F beats the current K-th value tau. With a G factor, |G| <= ||u|| ||i|| (1 + 1e-4)
// bounds the fp32 chain (its rounding is < 64 * 2^-24 relative), so once tau > 0 a column
// with F * bound <= tau is skipped without computing G; the rest get the exact chain score.
// Ids grow along the walk, so "beats" is v > tau (a tie loses to the older, smaller id).
template <int UF, int D, int M>
__global__ __launch_bounds__(128) void k_tile_resource_topk(
    const int64_t *__restrict__ user_rowptr, const int32_t *__restrict__ user_items,
    int64_t n_users, const uint64_t *__restrict__ wt_meta, const WEnt *__restrict__ wt_ent,
    int32_t item_begin, int32_t tile, int32_t width, const float *__restrict__ eu,
    const float *__restrict__ ei, const double *__restrict__ item_norm,
    const int64_t *__restrict__ ex_rowptr, const int32_t *__restrict__ ex_col,
    int64_t *__restrict__ ex_cur, int k, int first, double *__restrict__ io_val,
    int64_t *__restrict__ io_idx) {
  constexpr int CAP = 64 * M;
  extern __shared__ double lds[];
  const int wave = threadIdx.x / 64;
  const int wpb = blockDim.x / 64;
  const int lane = lane_id();
  const int64_t u = (int64_t)blockIdx.x * wpb + wave;
  if (u >= n_users) return;
  char *mine = reinterpret_cast<char *>(lds) + (size_t)wave * fused_wave_bytes(tile, M, D);
  double *acc = reinterpret_cast<double *>(mine);
  char *idx = mine + (size_t)tile * 8;
  double *cs = reinterpret_cast<double *>(idx + kResIdxBytes);
  int *ci = reinterpret_cast<int *>(cs + CAP);
  float *us = reinterpret_cast<float *>(ci + CAP);

  // running list (sorted, valid entries first)
  int cnt = 0;
  double tau = neg_inf<double>();
  int tau_id = kPadId;
  if (!first) {
    for (int e0 = 0; e0 < k; e0 += 64) {
      const int e = e0 + lane;
      const int64_t id = e < k ? io_idx[u * k + e] : -1;
      if (id >= 0) {
        cs[e] = io_val[u * k + e];
        ci[e] = (int)id;
      }
      cnt += __popcll(__ballot(id >= 0));
    }
  }
  double ubound = 0.0;
  if constexpr (D > 0) {
    double ss = 0.0;
    for (int d = lane; d < D; d += 64) {
      const float x = eu[u * D + d];
      us[d] = x;
      ss += (double)x * (double)x;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    ubound = sqrt(ss) * (1.0 + 1e-4);
  }
  for (int j = lane; j < tile; j += 64) acc[j] = 0.0;
  // (accumulate_user_tile's first barrier orders the list / embedding / zero stores)
  accumulate_user_tile<UF>(acc, idx, user_rowptr, user_items, u, wt_meta, wt_ent, item_begin);
  if (cnt == k) {
    tau = cs[k - 1];
    tau_id = ci[k - 1];
  }
  const int lim = item_begin + width;
  if (ex_rowptr) {
    // excluded items of the tile: the next run of the user's sorted exclusion row
    int64_t pos = ex_cur[u];
    const int64_t hi = ex_rowptr[u + 1];
    while (pos < hi) {
      const int64_t e = pos + lane;
      const int32_t x = e < hi ? ex_col[e] : 0x7fffffff;
      const bool in = x < lim;
      if (in && x >= item_begin) acc[x - item_begin] = -1.0;
      const int nin = __popcll(__ballot(in));
      pos += nin;
      if (nin < 64) break;
    }
    if (lane == 0) ex_cur[u] = pos;
    wave_sync();
  }
  for (int c0 = 0; c0 < width; c0 += 64) {
    const int j = c0 + lane;
    const double f = j < width ? acc[j] : -1.0;
    bool cand = f >= 0.0;
    double v = f;
    if constexpr (D > 0) {
      if (cand && tau > 0.0) cand = f * (ubound * item_norm[item_begin + j]) > tau;
      if (__ballot(cand)) {
        if (cand) v = (double)chain_score<D>(us, ei + (int64_t)(item_begin + j) * D) * f;
        cand = cand && v > tau;
      }
    } else {
      cand = cand && v > tau;
    }
    const uint64_t bal = __ballot(cand);
    if (bal) {
      const int p = cnt + __popcll(bal & lanemask_lt());
      if (cand) {
        cs[p] = v;
        ci[p] = item_begin + j;
      }
      cnt += __popcll(bal);
      if (cnt > CAP - 64) {
        wave_sync();
        cnt = wave_compact<double, M>(cs, ci, cnt, k, tau, tau_id);
      }
    }
  }
  wave_sync();
  const int nc = wave_compact<double, M>(cs, ci, cnt, k, tau, tau_id);
  for (int e = lane; e < k; e += 64) {
    io_val[u * k + e] = e < nc ? cs[e] : neg_inf<double>();
    io_idx[u * k + e] = e < nc ? ci[e] : -1;
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
                                         const int32_t *user_items, const double *inv_deg,
                                         int64_t n_items, const int64_t *cur,
                                         const uint16_t *count, const double *alpha,
                                         const double *beta, int32_t item_begin, int32_t tile,
                                         const int64_t *wt_ptr, void *wt_ent, uint64_t *wt_meta,
                                         void *ws, size_t ws_bytes, lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && inv_deg && cur && count && alpha && beta && wt_ptr && wt_meta &&
                 n_items >= 0,
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
  k_tile_weight<<<dim3(rb), dim3(256), 0, s>>>(item_rowptr, item_users, user_items, inv_deg,
                                               n_items, cur, count, alpha, beta, wt_ptr,
                                               (WEnt *)wt_ent, wt_meta);
  k_hub_list<<<dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, s>>>(
      wt_ptr, n_items, (unsigned long long *)n_hub, hub_rows);
  k_tile_weight_hub<<<dim3(1024), dim3(256), (size_t)tile * sizeof(double), s>>>(
      hub_rows, n_hub, item_rowptr, item_users, user_items, inv_deg, cur, count, alpha, beta,
      item_begin, tile, wt_ptr, (WEnt *)wt_ent, wt_meta);
  return launch_status("lg_spread_tile_weight_f64");
}

extern "C" int lg_spread_tile_resource_f64(const int64_t *user_rowptr,
                                           const int32_t *user_items, int64_t n_users,
                                           const uint64_t *wt_meta, const void *wt_ent,
                                           int32_t item_begin, int32_t tile, double *F,
                                           int64_t ldf, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && wt_meta && F && n_users >= 0 && ldf >= tile,
             "lg_spread_tile_resource_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192, "lg_spread_tile_resource_f64: tile %d not in [1, 8192]",
             tile);
  if (n_users == 0) return LG_OK;
  // per wave: tile doubles + two row indexes; 2-wave blocks, as many resident per CU as the
  // LDS holds, and a persistent grid of exactly that many (each wave walks users u + k*G)
  const size_t per_wave = (size_t)tile * sizeof(double) + 2 * kResIdxBytes;
  const size_t lds = 2 * per_wave;
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
      n_cu = 256;
  }
  // LGCNHS_RES_BLOCKS_PER_CU (A/B knob): resident-block multiple of the persistent grid;
  // 0 = one wave per user (no persistence)
  static int mult = -1;
  if (mult < 0) {
    const char *e = getenv("LGCNHS_RES_BLOCKS_PER_CU");
    mult = e ? atoi(e) : 0;
  }
  const int64_t per_cu = (int64_t)(160 * 1024 / lds) > 0 ? (int64_t)(160 * 1024 / lds) : 1;
  const int64_t want = (n_users + 1) / 2;
  const int64_t cap = mult > 0 ? per_cu * n_cu * mult : want;
  const unsigned blocks = (unsigned)(want < cap ? want : cap);
  // F rows are written with non-temporal stores: they are read once, by the next top-K
  // span, and should not displace W tile lines (1M users, 40 tiles: 4.08-4.14 vs 4.26 s of
  // resource passes, top-K unchanged; non-temporal F loads in the top-K measured 4 % slower).
  // LGCNHS_RES_NT=0 (A/B knob) restores plain stores.
  static int nt = -1;
  if (nt < 0) {
    const char *e = getenv("LGCNHS_RES_NT");
    nt = e ? atoi(e) : 1;
  }
  if (nt)
    k_tile_resource<16, true><<<dim3(blocks), dim3(128), lds, (hipStream_t)stream>>>(
        user_rowptr, user_items, n_users, wt_meta, (const WEnt *)wt_ent, item_begin, tile, F, ldf);
  else
    k_tile_resource<16, false><<<dim3(blocks), dim3(128), lds, (hipStream_t)stream>>>(
        user_rowptr, user_items, n_users, wt_meta, (const WEnt *)wt_ent, item_begin, tile, F, ldf);
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
  const int M = k <= 64 ? 2 : 4;
  return 2 * fused_wave_bytes(tile, M, dim);
}

template <int D>
static void launch_fused(int M, const int64_t *user_rowptr, const int32_t *user_items,
                         int64_t n_users, const uint64_t *wt_meta, const WEnt *wt_ent,
                         int32_t item_begin, int32_t tile, int32_t width, const float *eu,
                         const float *ei, const double *item_norm, const int64_t *ex_rowptr,
                         const int32_t *ex_col, int64_t *ex_cur, int k, int first,
                         double *io_val, int64_t *io_idx, hipStream_t s) {
  const unsigned b = (unsigned)((n_users + 1) / 2);
  const size_t lds = 2 * fused_wave_bytes(tile, M, D);
  if (M == 2)
    k_tile_resource_topk<16, D, 2><<<b, 128, lds, s>>>(
        user_rowptr, user_items, n_users, wt_meta, wt_ent, item_begin, tile, width, eu, ei,
        item_norm, ex_rowptr, ex_col, ex_cur, k, first, io_val, io_idx);
  else
    k_tile_resource_topk<16, D, 4><<<b, 128, lds, s>>>(
        user_rowptr, user_items, n_users, wt_meta, wt_ent, item_begin, tile, width, eu, ei,
        item_norm, ex_rowptr, ex_col, ex_cur, k, first, io_val, io_idx);
}

extern "C" int lg_spread_tile_resource_topk_f64(
    const int64_t *user_rowptr, const int32_t *user_items, int64_t n_users,
    const uint64_t *wt_meta, const void *wt_ent, int32_t item_begin, int32_t tile,
    int32_t width, const float *eu, const float *ei, int32_t dim, const double *item_norm,
    const int64_t *ex_rowptr, const int32_t *ex_col, int64_t *ex_cur, int32_t k,
    int32_t first, double *io_val, int64_t *io_idx, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && wt_meta && io_val && io_idx && n_users >= 0 && item_begin >= 0,
             "lg_spread_tile_resource_topk_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && width >= 1 && width <= tile &&
                 (int64_t)item_begin + width < 0x7fffffff,
             "lg_spread_tile_resource_topk_f64: tile %d / width %d", tile, width);
  LG_REQUIRE(k >= 1 && k <= 128, "lg_spread_tile_resource_topk_f64: k=%d not in [1,128]", k);
  LG_REQUIRE(!eu == !ei && (!eu || item_norm),
             "lg_spread_tile_resource_topk_f64: eu, ei and item_norm go together");
  LG_REQUIRE(!eu || dim == 32 || dim == 64 || dim == 128,
             "lg_spread_tile_resource_topk_f64: dim %d not in {32,64,128}", dim);
  LG_REQUIRE(!ex_rowptr == !ex_col && !ex_rowptr == !ex_cur,
             "lg_spread_tile_resource_topk_f64: ex_rowptr/ex_col/ex_cur go together");
  LG_REQUIRE(lg_spread_tile_resource_topk_lds_bytes(tile, k, eu ? dim : 0) <= 160 * 1024,
             "lg_spread_tile_resource_topk_f64: tile %d needs too much LDS", tile);
  if (n_users == 0) return LG_OK;
  hipStream_t s = (hipStream_t)stream;
  const int M = k <= 64 ? 2 : 4;
  const WEnt *w = (const WEnt *)wt_ent;
  switch (eu ? dim : 0) {
    case 0: launch_fused<0>(M, user_rowptr, user_items, n_users, wt_meta, w, item_begin, tile, width, eu, ei, item_norm, ex_rowptr, ex_col, ex_cur, k, first, io_val, io_idx, s); break;
    case 32: launch_fused<32>(M, user_rowptr, user_items, n_users, wt_meta, w, item_begin, tile, width, eu, ei, item_norm, ex_rowptr, ex_col, ex_cur, k, first, io_val, io_idx, s); break;
    case 64: launch_fused<64>(M, user_rowptr, user_items, n_users, wt_meta, w, item_begin, tile, width, eu, ei, item_norm, ex_rowptr, ex_col, ex_cur, k, first, io_val, io_idx, s); break;
    default: launch_fused<128>(M, user_rowptr, user_items, n_users, wt_meta, w, item_begin, tile, width, eu, ei, item_norm, ex_rowptr, ex_col, ex_cur, k, first, io_val, io_idx, s); break;
  }
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
