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
// Factored: W[i][j] = general_W[i][j] * ra_i * rb_j with ra = 1/alpha, rb = 1/beta (alpha_i =
// k_i^(1-l), beta_j = k_j^l; a zero factor -> 1, the reference's den == 0 rule), so
//   F[u][j] = rb_j * sum_{i in items(u)} ra_i * sum_{v in users(i) and users(j)} fl(1/k_v)
//           = rb_j * sum over the 3-hop paths u -> i -> v -> j of fl(1/k_v) * ra_i.
// The items are processed in column tiles [j0, j0 + T). Per tile:
//   cursor   end[v] = first position of user v's (ascending) item row with item >= j0 + T;
//            cur[v] (the previous tile's end) marks the first item >= j0, so
//            items(v) inside the tile = user_items[cur[v] .. end[v])
//   bound    bound[i] = sum_{v in users(i)} (end[v] - cur[v]) = the (user, item) pairs
//            behind row i of W in the tile (its paths)
//   rows     row i of general_W restricted to the tile, in the line format below
//   walk     per user (one wave): the paths of its rows added into an LDS accumulator, then
//            scaled by rb_j and either written out (F mode) or merged straight into the
//            user's running top-K list (top-K mode: (G *) F, G = the fp32 e0 score chain,
//            candidates screened by per-(user, 64-column chunk) score bounds).
// Work: the rows pass costs sum_i deg(i) lookups + the 2-hop pairs once per tile (not per
// user); the walk reads one 128-byte line per (user, item) and tile (~5e10 lines at C5) and
// adds ~1e12 paths (one LDS atomic each); F never leaves LDS.
//
// Rounding: every path contributes fl(fl(1/k_v) * ra_i) (P rows) or fl(general_W[i][j] * ra_i)
// (V rows); the sum order is the walk's (fixed: deterministic, but not the dense path's
// ascending-i order), then one multiply by rb_j. Against the reference's
// general_W / (alpha (x) beta) summed by BLAS this is a few ulp per term (tests: 1e-12
// relative), the reference's own BLAS order being unspecified.
#include <stdio.h>
#include <stdlib.h>

#include "common.h"

// LG_REFERENCE_PATHS (test-reference build, lib/liblgcnhs_ref.so, include/lgcnhs_ref.h): the
// per-tile build passes, the F-writing walk and the two-kernel top-K merge, kept as bitwise
// references for the product's group build and fused walk. The product library
// (lib/liblgcnhs.so) is built without them.
#ifndef LG_REFERENCE_PATHS
#define LG_REFERENCE_PATHS 0
#endif
#if LG_REFERENCE_PATHS
#include "lgcnhs_ref.h"
#endif

namespace lg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// A W tile is one 128-byte LINE per item row i at lines[i * 32 ..] (32 words) plus, for rows
// that do not fit, a run of 16-byte units in an overflow array. Word 0 of the line is the
// header: bit 31 = V format, bit 30 = overflow, bit 29 = slow (a V row, or a P row with a
// degree class >= kInvTab: the walk's general decode), bits 0-28 = the overflow run's first
// unit (ovf[u].x = the number of data units that follow it). No per-row metadata: the walk
// reads the line of every item of its user straight from i * 128. Line I (one past the last
// item) is all zero: the walk's padding rows read it.
//
// P rows (<= the hub threshold's pairs, the common case): one 4-byte slot per (user v,
//   item j) PAIR behind the row (v in users(i), j in items(v) inside the tile), in pair order
//   (users ascending, each user's items ascending):
//     bits 0-15  j - item_begin
//     bits 16-30 the 1-based class of v's degree k_v (fl(1 / k_v) = inv[class]; classes
//                < kInvTab are cached in LDS); bit 31 clear (it marks V entries); a zero
//                word is padding
//   line words 1..31 hold the first 31 slots, the overflow units 4 slots each.
// V rows (hub items, more pairs than the threshold; merged while building): one 16-byte
//   entry per distinct column, ascending: {0x80000000 | (j - item_begin), fp64
//   general_W[i][j] (lo, hi), 0}; line units 1..7 hold the first 7, the overflow units one
//   each.
//   A V row with more than width / 2 + 8 entries (hub items held by a large share of the
//   users: nearly every column) is DENSE instead: its line holds only the header, and its
//   overflow run (header x = kRunDense | n, n = ceil(width / 2) data units) holds the row's
//   general_W of columns 2q and 2q + 1 in unit q as two fp64 (zeros included) -- 8 bytes per
//   column instead of 16 per entry, read with no column index (the walk's hub rows are bound
//   by these reads). The sparse run's allocation (1 + min(pairs, width) - 7 units) covers it.
// Neither format depends on lambda (ra / rb are applied by the walk), so a lambda sweep
// reuses the built tiles.
constexpr uint32_t kHdrV = 0x80000000u;
constexpr uint32_t kHdrOvf = 0x40000000u;
constexpr uint32_t kHdrSlow = 0x20000000u;
constexpr uint32_t kHdrPtr = 0x1FFFFFFFu;
constexpr uint32_t kEntV = 0x80000000u;
constexpr uint32_t kRunDense = 0x80000000u;  // overflow run header: a dense V row
constexpr int kLineSlots = 31;  // P slots in a line (word 0 is the header)
constexpr int kLineEnts = 7;    // V entries in a line (unit 0 holds the header)
constexpr int kInvTab = 512;    // degree classes whose fl(1/k) is cached in LDS

__global__ __launch_bounds__(256) void k_inv_degree(const int64_t *__restrict__ rowptr,
                                                    int64_t n, double *__restrict__ inv) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  inv[v] = 1.0 / (double)(rowptr[v + 1] - rowptr[v]);  // k_spread_general's fl(1/k_v)
}

#if LG_REFERENCE_PATHS
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

#endif  // LG_REFERENCE_PATHS
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

#if LG_REFERENCE_PATHS
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

#endif  // LG_REFERENCE_PATHS
// ra[i] = 1 / k_item[i]^(1 - lambda), rb[i] = 1 / k_item[i]^lambda (the same pow() calls as
// k_hybrid_weight); a zero factor -> 1 (its rows / columns hold no paths).
__global__ __launch_bounds__(256) void k_hybrid_recip(const double *__restrict__ k_item,
                                                      int64_t n, double lambda,
                                                      double *__restrict__ ra,
                                                      double *__restrict__ rb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = pow(k_item[i], 1.0 - lambda), b = pow(k_item[i], lambda);
  ra[i] = a != 0.0 ? 1.0 / a : 1.0;
  rb[i] = b != 0.0 ? 1.0 / b : 1.0;
}

// ------------------------------------------------------------------- the rows pass
// Slot p of a row: line word 1 + p for p < 31, else word (p - 31) of the overflow run's
// data units (the run's unit 0 is its header).
__device__ __forceinline__ void put_slot(uint32_t *__restrict__ line, uint32_t *__restrict__ ovf,
                                         int64_t ou, int64_t p, uint32_t w) {
  if (p < kLineSlots) line[1 + p] = w;
  else ovf[(ou + 1) * 4 + (p - kLineSlots)] = w;
}

// The dense form of a V row from its accumulator acc[0 .. width) (threads t = t0 .. of a
// stride-ts group write): the line's header and zero words, the run header, the data units.
__device__ __forceinline__ bool hub_row_dense(int nz, int width) { return nz > width / 2 + 8; }
__device__ void write_hub_row_dense(const double *acc, int width, uint32_t *line, uint32_t *ov,
                                    int64_t ou, int t0, int ts) {
  const int nd = (width + 1) / 2;
  for (int t = t0; t < 32; t += ts) line[t] = t == 0 ? (kHdrV | kHdrSlow | kHdrOvf | (uint32_t)ou) : 0u;
  for (int t = t0; t < 4; t += ts) ov[ou * 4 + t] = t == 0 ? (kRunDense | (uint32_t)nd) : 0u;
  for (int q = t0; q < nd; q += ts) {
    const uint64_t a = (uint64_t)__double_as_longlong(acc[2 * q]);
    const uint64_t b = 2 * q + 1 < width ? (uint64_t)__double_as_longlong(acc[2 * q + 1]) : 0ull;
    *reinterpret_cast<uint4 *>(ov + 4 * (ou + 1 + q)) =
        uint4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
  }
}

#if LG_REFERENCE_PATHS
// P rows: one wave per item row with bound[i] <= vthr pairs. Every word of the line and of
// the overflow run is written exactly once (header, pairs, zero padding), so no stale data
// of an earlier tile survives and no two stores of the wave hit one word.
__global__ __launch_bounds__(256) void k_tile_rows(
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const uint16_t *__restrict__ user_cls,
    int64_t n_items, const int64_t *__restrict__ cur, const uint16_t *__restrict__ count,
    int32_t item_begin, const int64_t *__restrict__ bound, int64_t vthr,
    const int64_t *__restrict__ ovf_ptr, uint32_t *__restrict__ lines,
    uint32_t *__restrict__ ovf, int32_t *__restrict__ row_len) {
  const int64_t i = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (i >= n_items) return;
  const int lane = lane_id();
  const int64_t nb = bound[i];
  if (nb > vthr) return;  // hub row: k_tile_rows_hub
  uint32_t *line = lines + i * 32;
  const bool has_ovf = nb > kLineSlots;
  const int64_t ou = has_ovf ? ovf_ptr[i] : 0;
  const int64_t n_units = has_ovf ? (nb - kLineSlots + 3) / 4 : 0;
  const int64_t cap = kLineSlots + 4 * n_units;
  if (has_ovf && lane < 4) ovf[ou * 4 + lane] = lane == 0 ? (uint32_t)n_units : 0u;
  for (int64_t p = nb + lane; p < cap; p += 64) put_slot(line, ovf, ou, p, 0u);
  // the pairs: users of i ascending, each user's items in the tile ascending
  int64_t n = 0;
  bool far = false;
  const int64_t e1 = item_rowptr[i + 1];
  for (int64_t e0 = item_rowptr[i]; e0 < e1; e0 += 64) {
    const int64_t e = e0 + lane;
    int32_t v = 0;
    int c = 0;
    if (e < e1) {
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
      const uint32_t cl = (uint32_t)user_cls[v];
      far |= cl >= (uint32_t)kInvTab;
      for (int q = 0; q < c; ++q)
        put_slot(line, ovf, ou, n + pre + q,
                 (cl << 16) | (uint32_t)(user_items[s0 + q] - item_begin));
    }
    n += total;
  }
  const bool slow = __ballot(far) != 0;
  if (lane == 0) {
    line[0] = (has_ovf ? (kHdrOvf | (uint32_t)ou) : 0u) | (slow ? kHdrSlow : 0u);
    if (row_len) row_len[i] = (int32_t)nb;
  }
}

// V rows (bound > vthr pairs, hub items): one 256-thread block per row (grid-stride over the
// hub list), the tile as a dense LDS accumulator of general_W, users walked in ascending
// order as in k_spread_general, then the touched columns written as ascending entries.
__global__ __launch_bounds__(256) void k_tile_rows_hub(
    const int64_t *__restrict__ hub_rows, const int64_t *__restrict__ n_hub,
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const double *__restrict__ inv_deg,
    const int64_t *__restrict__ cur, const uint16_t *__restrict__ count, int32_t item_begin,
    int32_t tile, const int64_t *__restrict__ ovf_ptr, uint32_t *__restrict__ lines,
    uint32_t *__restrict__ ovf, int32_t *__restrict__ row_len) {
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
    uint32_t *line = lines + i * 32;
    const int64_t ou = ovf_ptr[i];
    if (threadIdx.x == 0) wsum[0] = 0;
    __syncthreads();
    {
      int c = 0;
      for (int j = threadIdx.x; j < tile; j += blockDim.x) c += acc[j] != 0.0;
      atomicAdd(&wsum[0], c);
    }
    __syncthreads();
    const int nzr = wsum[0];
    __syncthreads();
    if (hub_row_dense(nzr, tile)) {  // (tile = this tile's width here)
      write_hub_row_dense(acc, tile, line, ovf, ou, threadIdx.x, blockDim.x);
      if (threadIdx.x == 0 && row_len) row_len[i] = nzr;
      __syncthreads();
      continue;
    }
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
        const int64_t e = base + before_w + __popcll(b & lanemask_lt());
        uint32_t *u4 = e < kLineEnts ? line + 4 * (1 + e) : ovf + 4 * (ou + 1 + (e - kLineEnts));
        *reinterpret_cast<uint4 *>(u4) =
            uint4{kEntV | (uint32_t)j, (uint32_t)bits, (uint32_t)(bits >> 32), 0u};
      }
      base += total;
      __syncthreads();
    }
    // header, the unused line units, the overflow run's header
    const bool has_ovf = base > kLineEnts;
    if (threadIdx.x < 32) {
      const int t = threadIdx.x;  // line word t
      const int unit = t / 4;
      if (t == 0) line[0] = kHdrV | kHdrSlow | (has_ovf ? (kHdrOvf | (uint32_t)ou) : 0u);
      else if (unit == 0 || unit > base) line[t] = 0u;
    }
    if (has_ovf && threadIdx.x < 4)
      ovf[ou * 4 + threadIdx.x] = threadIdx.x == 0 ? (uint32_t)(base - kLineEnts) : 0u;
    if (threadIdx.x == 0 && row_len) row_len[i] = base;
    __syncthreads();
  }
}

#endif  // LG_REFERENCE_PATHS

__global__ __launch_bounds__(256) void k_hub_list(const int64_t *__restrict__ bound,
                                                  int64_t n_items, int64_t vthr,
                                                  unsigned long long *__restrict__ n_hub,
                                                  int64_t *__restrict__ hub_rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  if (bound[i] > vthr) hub_rows[atomicAdd(n_hub, 1ull)] = i;
}

// ------------------------------------------------------------ group build (S tiles at once)
// The per-tile passes above visit every (item row, user) pair once per TILE, although at C5
// a user has ~0.2 items in a 2048-column tile: 489 tiles x 1e8 visits of gathered counts.
// The group passes visit each pair once per GROUP of up to kGroupMax consecutive tiles and
// write the group's tiles together (tile t of the group at lines + t (n_items + 1) 32 words,
// its overflow runs at ovf + 4 ovf_base[t] words). Every word equals the per-tile build's
// (same slot order, same headers; the caller places the runs with the same exclusive prefix).
constexpr int kGroupMax = 16;
constexpr int kGroupWide = 8;  // groups of tiles wider than 4096 columns (13-bit item codes)

// counts[v][t] (kGroupMax uint16 per user: two 16-byte halves, tiles 0-7 and 8-15) = the
// items of user v in tile t of the group ([group_begin + t tile, min(group_begin + (t + 1)
// tile, stop))), end[v] = the position after the group's last; cur[v] = the first position
// with item >= group_begin.
// rec[v] (16 bytes, what k_group_rows gathers per (item, user) pair instead of counts, cur,
// the class and the items): x = n (the user's items in the group, saturated at 255) |
// class << 8; for n <= kRecItems the items as 16-bit codes t << cs | (item - tile t's first
// item) in y, z, w (low half first; cs = code_shift(n_tiles): 13 for groups of <= 8 tiles,
// 12 for more, whose tiles are <= 4096 wide); else y = cur[v] (the rows read user_items).
constexpr int kRecItems = 6;
__host__ __device__ constexpr int code_shift(int n_tiles) { return n_tiles <= kGroupWide ? 13 : 12; }
__global__ __launch_bounds__(256) void k_group_cursor(const int64_t *__restrict__ user_rowptr,
                                                      const int32_t *__restrict__ user_items,
                                                      const uint16_t *__restrict__ user_cls,
                                                      int64_t n_users, int32_t group_begin,
                                                      int32_t tile, int32_t n_tiles,
                                                      int32_t stop, const int64_t *__restrict__ cur,
                                                      int64_t *__restrict__ end,
                                                      uint4 *__restrict__ counts,
                                                      uint4 *__restrict__ rec) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n_users) return;
  const int cs = code_shift(n_tiles);
  const int64_t p0 = cur[v];
  int64_t p = p0;
  const int64_t pe = user_rowptr[v + 1];
  // the group's items: [group_begin, glim); an item's tile by one division (a user has few
  // items in a group: ~1.6 at C5)
  const int64_t gl = (int64_t)group_begin + (int64_t)n_tiles * tile;
  const int32_t glim = (int32_t)(gl < stop ? gl : stop);
  uint32_t c8[kGroupMax / 2];  // per-tile counts, two tiles per word (16-bit fields)
#pragma unroll
  for (int h = 0; h < kGroupMax / 2; ++h) c8[h] = 0;
  uint32_t code[kRecItems];
#pragma unroll
  for (int k = 0; k < kRecItems; ++k) code[k] = 0;
  int n = 0;
  for (int32_t it = p < pe ? user_items[p] : 0x7fffffff; it < glim;
       it = p < pe ? user_items[p] : 0x7fffffff) {
    const uint32_t rel = (uint32_t)(it - group_begin);  // (cur: it >= group_begin)
    const uint32_t t = rel / (uint32_t)tile;
    const uint32_t cd = t << cs | (rel - t * (uint32_t)tile);
#pragma unroll
    for (int k = 0; k < kRecItems; ++k)
      if (n == k) code[k] = cd;
    const uint32_t inc = 1u << (16 * (t & 1));
#pragma unroll
    for (int h = 0; h < kGroupMax / 2; ++h) c8[h] += t >> 1 == (uint32_t)h ? inc : 0u;
    ++n;
    ++p;
  }
  end[v] = p;  // (the counts of a tile are <= tile <= 8192: no carry between the fields)
  counts[2 * v] = uint4{c8[0], c8[1], c8[2], c8[3]};
  counts[2 * v + 1] = uint4{c8[4], c8[5], c8[6], c8[7]};
  const uint32_t hx = (uint32_t)(n < 255 ? n : 255) | (uint32_t)user_cls[v] << 8;
  rec[v] = n <= kRecItems
               ? uint4{hx, code[0] | code[1] << 16, code[2] | code[3] << 16, code[4] | code[5] << 16}
               : uint4{hx, (uint32_t)p0, 0u, 0u};
}

// tile t's count in a user's 8-tile half c (t < 8)
__device__ __forceinline__ uint32_t count_of(const uint4 &c, int t) {
  const uint32_t w = t < 2 ? c.x : (t < 4 ? c.y : (t < 6 ? c.z : c.w));
  return (t & 1) ? w >> 16 : w & 0xFFFFu;
}
// tile t's count (t < 16) in a user's two halves
__device__ __forceinline__ uint32_t count_of2(const uint4 &lo, const uint4 &hi, int t) {
  return t < 8 ? count_of(lo, t) : count_of(hi, t - 8);
}

// bound[t][i] = sum over the users v of item i of counts[v][t] (the pairs behind row i in
// tile t). 16 lanes per item row, 4 rows per wave (rows of ~100 users fill a 64-lane wave
// poorly, and a wave's fixed costs -- row pointers, the reduction, the stores -- are then
// shared by 4 rows). Per round each lane gathers the counts of 8 of its row's users (128 per
// row; every load is issued, clamped to a valid index, before any is used: one wait for the
// ids, one for the counts; the second 8-tile half only for groups of more than 8), sums them
// per tile in 32 bits (<= 8 x 8192), then into 64 bits. The 16 lanes' 16 per-tile sums are
// reduced by halving exchanges: over xor 8, 4, 2, 1 each lane keeps half of its tiles and
// adds its partner's sums of those (16 -> 8 -> 4 -> 2 -> 1 tiles): lane t of the row ends
// with tile t's total (15 shuffles instead of 16 x 4). At C5 the kernel is bound by the
// random 16-byte count gathers (one per (row, user) pair and group), not by its arithmetic.
static_assert(kGroupMax == 16, "k_group_bound's halving reduction is written for 16 tiles");
__global__ __launch_bounds__(256) void k_group_bound(const int64_t *__restrict__ item_rowptr,
                                                     const int32_t *__restrict__ item_users,
                                                     int64_t n_items,
                                                     const uint4 *__restrict__ counts,
                                                     int32_t n_tiles, int64_t *__restrict__ bound) {
  constexpr int kU = 8;  // users per lane per round
  const int lane = lane_id(), sub = lane & 15;
  const int64_t i = ((int64_t)blockIdx.x * 4 + threadIdx.x / 64) * 4 + (lane >> 4);
  const bool live = i < n_items;  // (no early exit: the reduction needs every lane)
  const bool wide = n_tiles > 8;  // (uniform)
  const int64_t b = live ? item_rowptr[i] : 0, e1 = live ? item_rowptr[i + 1] : 0;
  uint64_t s[kGroupMax];
#pragma unroll
  for (int t = 0; t < kGroupMax; ++t) s[t] = 0;
  // (a round runs only while some row of the wave has users left: there are interactions,
  // so index 0 of item_users and of counts is valid for the clamped lanes)
  for (int64_t r0 = b; __ballot(r0 < e1) != 0; r0 += 16 * kU) {
    int32_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t e = r0 + sub + 16 * u;
      v[u] = item_users[e < e1 ? e : 0];
    }
    uint4 cl[kU], ch[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      cl[u] = counts[2 * (int64_t)v[u]];
      ch[u] = wide ? counts[2 * (int64_t)v[u] + 1] : uint4{0u, 0u, 0u, 0u};
    }
    uint32_t rs[kGroupMax];
#pragma unroll
    for (int t = 0; t < kGroupMax; ++t) rs[t] = 0;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const bool in = r0 + sub + 16 * u < e1;
      const uint4 zl = in ? cl[u] : uint4{0u, 0u, 0u, 0u};
      const uint4 zh = in ? ch[u] : uint4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int t = 0; t < kGroupMax; ++t) rs[t] += count_of2(zl, zh, t);
    }
#pragma unroll
    for (int t = 0; t < kGroupMax; ++t) s[t] += rs[t];
  }
  // halving exchanges within the row's 16 lanes: after the step over xor m the lane keeps
  // the tiles whose bit (m) equals its own
  uint64_t r8[8], r4[4], r2[2];
  const bool h3 = sub & 8, h2 = sub & 4, h1 = sub & 2, h0 = sub & 1;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    r8[j] = (h3 ? s[j + 8] : s[j]) + __shfl_xor(h3 ? s[j] : s[j + 8], 8);  // tiles 8 h3 + j
#pragma unroll
  for (int j = 0; j < 4; ++j)
    r4[j] = (h2 ? r8[j + 4] : r8[j]) + __shfl_xor(h2 ? r8[j] : r8[j + 4], 4);  // + 4 h2 + j
#pragma unroll
  for (int j = 0; j < 2; ++j)
    r2[j] = (h1 ? r4[j + 2] : r4[j]) + __shfl_xor(h1 ? r4[j] : r4[j + 2], 2);  // + 2 h1 + j
  const uint64_t r1 = (h0 ? r2[1] : r2[0]) + __shfl_xor(h0 ? r2[0] : r2[1], 1);  // + h0
  if (live && sub < n_tiles) bound[(int64_t)sub * n_items + i] = (int64_t)r1;
}

// Overflow units (run header + data) of a row with nb pairs in a tile of width w: P rows
// (nb <= vthr) 1 + ceil((nb - 31) / 4) past the line's 31 slots, V rows (hub items)
// 1 + (min(nb, w) - 7) past the line's 7 entries, else 0 (= ops._run_units).
__device__ __forceinline__ int64_t run_units(int64_t nb, int64_t vthr, int64_t w) {
  if (nb > vthr) {
    const int64_t len = nb < w ? nb : w;
    return len > kLineEnts ? 1 + (len - kLineEnts) : 0;
  }
  return nb > kLineSlots ? 1 + (nb - kLineSlots + 3) / 4 : 0;
}

__device__ __forceinline__ int64_t tile_width(int32_t group_begin, int32_t tile, int t,
                                              int32_t stop) {
  const int64_t b = (int64_t)group_begin + (int64_t)t * tile;
  const int64_t e = b + tile < stop ? b + tile : stop;
  return e - b;
}

// units[t][i] = run_units of row i in tile t (the caller's inclusive scan over the flat
// [n_tiles][n_items] array places the runs: tile by tile, rows ascending)
__global__ __launch_bounds__(256) void k_group_units(const int64_t *__restrict__ bound,
                                                     int64_t n_items, int32_t group_begin,
                                                     int32_t tile, int32_t n_tiles, int32_t stop,
                                                     int64_t vthr, int64_t *__restrict__ units) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n_items * n_tiles) return;
  const int t = (int)(x / n_items);
  units[x] = run_units(bound[x], vthr, tile_width(group_begin, tile, t, stop));
}

// Inclusive prefix sum over the wave's 64 lanes by DPP (no LDS round trips): row_shr 1, 2,
// 4, 8 inside each 16-lane row, then row_bcast 15 / 31 add the earlier rows' totals.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// lane t's 64-bit value as a wave-uniform scalar
__device__ __forceinline__ int64_t readlane64(int64_t x, int t) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, t);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), t);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// P rows of every tile of the group: one wave per item row (tiles whose row is a hub row,
// bound > vthr, are left to k_group_rows_hub). The row's lines (kGroupMax x 128 bytes) are
// assembled in the wave's LDS and written with two coalesced 16-byte-per-lane stores at the
// end (the slots of a line come from ~20 lanes over several chunks: written straight to
// global memory they took ~5 sparse store instructions per (row, tile)); slots past a line's
// 31 go to the overflow run directly. Per chunk of 64 users (lane = user, ascending): the
// user's per-tile item counts (from its record's item codes, or its counts for users with
// more than kRecItems items in the group), two tiles per word as 16-bit fields (a P row's
// prefix never exceeds its bound <= vthr < 2^16; hub tiles' counts are masked to 0), one
// DPP prefix sum per word; then per tile t the lane's first slot position minus its item
// index in the group, D_t (an LDS table, [t][lane]), so each of the lane's items k lands
// at slot D_t + k with one table read -- one pass over the user's items instead of one per
// tile. A chunk's user records are gathered one chunk ahead and its users two ahead
// (unconditional loads, clamped into the row).
__global__ __launch_bounds__(256) void k_group_rows(
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, int64_t n_items, const uint4 *__restrict__ counts,
    const uint4 *__restrict__ rec, int32_t group_begin, int32_t tile, int32_t n_tiles,
    int32_t stop, const int64_t *__restrict__ bound, int64_t vthr,
    const int64_t *__restrict__ units_incl,
    uint32_t *__restrict__ lines, uint32_t *__restrict__ ovf, int32_t *__restrict__ row_len) {
  __shared__ __attribute__((aligned(16))) uint32_t s_line[4][kGroupMax * 32];
  __shared__ uint32_t s_pos[4][kGroupMax][64];
  __shared__ uint32_t s_ovw[4][kGroupMax];  // tile t's run: its first data word in ovf
  const int wv = threadIdx.x / 64;
  const int64_t i = (int64_t)blockIdx.x * 4 + wv;
  if (i >= n_items) return;  // (whole waves: the LDS is per wave, no block barrier)
  const int lane = lane_id();
  // lane t < n_tiles: row i's pairs, run offset (relative to the tile's runs) and the
  // tile's first unit in ovf
  int64_t nbl = 0, oul = 0, obl = 0;
  if (lane < n_tiles) {
    const int64_t x = (int64_t)lane * n_items + i;
    nbl = bound[x];
    obl = lane ? units_incl[(int64_t)lane * n_items - 1] : 0;
    oul = units_incl[x] - run_units(nbl, vthr, tile_width(group_begin, tile, lane, stop)) - obl;
  }
  const int64_t eb = item_rowptr[i], e1 = item_rowptr[i + 1];
  const int cs = code_shift(n_tiles);
  const uint32_t cmask = (1u << cs) - 1u;
  const bool wide = n_tiles > 8;  // (uniform)
  uint32_t *line_s = s_line[wv];
  {  // the lines start all zero (padding); 2 x 16 bytes per lane
    uint4 *l4 = reinterpret_cast<uint4 *>(line_s);
    l4[lane] = uint4{0u, 0u, 0u, 0u};
    l4[64 + lane] = uint4{0u, 0u, 0u, 0u};
  }
  wave_sync();
  const bool has_run_l = lane < n_tiles && nbl <= vthr && nbl > kLineSlots;
  if (lane < n_tiles) s_ovw[wv][lane] = (uint32_t)((obl + oul + 1) * 4);
  uint32_t pmask = 0;  // P tiles of this row (uniform)
#pragma unroll
  for (int t = 0; t < kGroupMax; ++t)
    if (t < n_tiles && readlane64(nbl, t) <= vthr) pmask |= 1u << t;
  // overflow runs of the P tiles: header unit and the padding past the row's pairs
  uint32_t runs = (uint32_t)__ballot(has_run_l);
  while (runs) {
    const int t = __builtin_ctz(runs);
    runs &= runs - 1;
    const int64_t nb = readlane64(nbl, t);
    const int64_t ob = readlane64(obl, t) + readlane64(oul, t);  // the run's header unit
    const int64_t n_units = (nb - kLineSlots + 3) / 4;
    if (lane < 4) ovf[ob * 4 + lane] = lane == 0 ? (uint32_t)n_units : 0u;
    for (int64_t p = nb + lane; p < kLineSlots + 4 * n_units; p += 64)
      ovf[(ob + 1) * 4 + (p - kLineSlots)] = 0u;
  }
  uint32_t m8[kGroupMax / 2];
#pragma unroll
  for (int h = 0; h < kGroupMax / 2; ++h) {
    const uint32_t lo = ((pmask >> (2 * h)) & 1) ? 0xFFFFu : 0u;
    const uint32_t hi = ((pmask >> (2 * h + 1)) & 1) ? 0xFFFF0000u : 0u;
    m8[h] = lo | hi;
  }
  uint32_t n[kGroupMax];  // pairs written so far per tile (uniform)
#pragma unroll
  for (int t = 0; t < kGroupMax; ++t) n[t] = 0;
  uint32_t farbits = 0;
  auto user_at = [&](int64_t e0) __attribute__((always_inline)) {
    const int64_t e = e0 + lane;
    return item_users[e < e1 ? e : e1 - 1];
  };
  int32_t v_c = 0, v_n = 0;
  uint4 r_c{0u, 0u, 0u, 0u};
  if (eb < e1) {
    v_c = user_at(eb);
    v_n = user_at(eb + 64);
    r_c = rec[v_c];
  }
  for (int64_t e0 = eb; e0 < e1; e0 += 64) {
    const int32_t v = v_c;
    const uint4 rc = e0 + lane < e1 ? r_c : uint4{0u, 0u, 0u, 0u};
    const uint32_t nu = rc.x & 0xFFu;  // the user's items in the group (saturated)
    const bool longu = nu > (uint32_t)kRecItems;
    uint32_t c8[kGroupMax / 2];  // the user's per-tile counts, two tiles per word
#pragma unroll
    for (int h = 0; h < kGroupMax / 2; ++h) c8[h] = 0;
    // (the rare users with more items than the record holds load their counts before the
    // prefetch below is issued: waiting for these loads then drains nothing younger)
    if (longu) {
      const uint4 lo = counts[2 * (int64_t)v];
      const uint4 hi = wide ? counts[2 * (int64_t)v + 1] : uint4{0u, 0u, 0u, 0u};
      c8[0] = lo.x, c8[1] = lo.y, c8[2] = lo.z, c8[3] = lo.w;
      c8[4] = hi.x, c8[5] = hi.y, c8[6] = hi.z, c8[7] = hi.w;
    }
    v_c = v_n;
    r_c = rec[v_n];           // the next chunk's records
    v_n = user_at(e0 + 128);  // the users of the one after
    if (!longu) {  // per-tile counts from the item codes
#pragma unroll
      for (int k = 0; k < kRecItems; ++k) {
        const uint32_t wd = k < 2 ? rc.y : (k < 4 ? rc.z : rc.w);
        const uint32_t cd = (k & 1) ? wd >> 16 : wd & 0xFFFFu;
        if ((uint32_t)k < nu) {
          const uint32_t t = cd >> cs;
          const uint32_t inc = 1u << (16 * (t & 1));
#pragma unroll
          for (int h = 0; h < kGroupMax / 2; ++h) c8[h] += t >> 1 == (uint32_t)h ? inc : 0u;
        }
      }
    }
    uint32_t any = 0;
#pragma unroll
    for (int h = 0; h < kGroupMax / 2; ++h) any |= c8[h] & m8[h];
    if (__ballot(any != 0) == 0) continue;  // no pair in any P tile
    // D_t per tile: (pairs before this chunk) + (this chunk's lanes before this one) - (the
    // user's items in tiles < t)
    uint32_t off = 0, ntot = 0;
#pragma unroll
    for (int h = 0; h < kGroupMax / 2; ++h) {
      if (2 * h >= n_tiles) break;
      const uint32_t wm = c8[h] & m8[h];
      uint32_t pre = wm;
      if (__ballot(pre != 0) != 0) pre = wave_incl_sum(pre);
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pre, 63);
      pre -= wm;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int t = 2 * h + b;
        const uint32_t pb = (pre >> (16 * b)) & 0xFFFFu;
        s_pos[wv][t][lane] = n[t] + pb - off;
        n[t] += (total >> (16 * b)) & 0xFFFFu;
        off += (c8[h] >> (16 * b)) & 0xFFFFu;
      }
    }
    ntot = off;  // the user's items in the group's tiles (all of them, n_tiles <= 16)
    wave_sync();
    const int64_t s0 = longu ? (int64_t)rc.y : 0;
    const uint32_t cl = rc.x >> 8;
    uint32_t tl = 0;  // (long users: the tile of the current item, items ascending)
    for (uint32_t k = 0; k < ntot; ++k) {
      uint32_t t, col;
      if (!longu) {
        const uint32_t wd = k < 2 ? rc.y : (k < 4 ? rc.z : rc.w);
        const uint32_t cd = (k & 1) ? wd >> 16 : wd & 0xFFFFu;
        t = cd >> cs;
        col = cd & cmask;
      } else {
        const uint32_t rel = (uint32_t)(user_items[s0 + k] - group_begin);
        while (rel >= (tl + 1) * (uint32_t)tile) ++tl;
        t = tl;
        col = rel - tl * (uint32_t)tile;
      }
      if ((pmask >> t) & 1u) {
        const uint32_t pos = s_pos[wv][t][lane] + k;
        const uint32_t word = (cl << 16) | col;
        if (pos < (uint32_t)kLineSlots) line_s[t * 32 + 1 + pos] = word;
        else ovf[(int64_t)s_ovw[wv][t] + (pos - kLineSlots)] = word;
        if (cl >= (uint32_t)kInvTab) farbits |= 1u << t;
      }
    }
  }
  // headers (lane t: tile t) and row lengths, then the lines
  uint32_t slowm = 0;
#pragma unroll
  for (int t = 0; t < kGroupMax; ++t)
    if ((pmask >> t) & 1u) slowm |= __ballot((farbits >> t) & 1u) != 0 ? 1u << t : 0u;
  if (lane < kGroupMax && ((pmask >> lane) & 1u)) {
    line_s[lane * 32] = (nbl > kLineSlots ? (kHdrOvf | (uint32_t)oul) : 0u) |
                        (((slowm >> lane) & 1u) ? kHdrSlow : 0u);
    if (row_len) row_len[(int64_t)lane * n_items + i] = (int32_t)nbl;
  }
  wave_sync();
  const int64_t tstride = (n_items + 1) * 32;  // words per tile of lines
#pragma unroll
  for (int r = 0; r < kGroupMax / 8; ++r) {
    const int t = 8 * r + (lane >> 3), u = lane & 7;
    if ((pmask >> t) & 1u)
      *reinterpret_cast<uint4 *>(lines + (int64_t)t * tstride + i * 32 + 4 * u) =
          reinterpret_cast<const uint4 *>(line_s)[t * 8 + u];
  }
}

__device__ __forceinline__ void lds_add(double *acc, uint32_t col, double v) {
  __hip_atomic_fetch_add(&acc[col], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Hub rows of the group (flat index t * n_items + i of rows with bound > vthr, listed by
// k_hub_list over the [n_tiles][n_items] bounds): the dense accumulation of k_tile_rows_hub --
// general_W[i][j] = the sum over i's users v, ascending, of fl(1/k_v) for each of v's items j
// in tile t (on tile t's cursor cur[v] + v's items in tiles < t) -- by ONE WAVE per row, on
// its own LDS accumulator. A hub item has up to all the users; the per-user metadata (the
// user id, its 32-byte count record, its cursor and fl(1/k_v)) of 64 users is loaded by the
// wave's lanes at once, and their items (~1-3 per user and tile) up to 256 at a time, each
// lane finding the user of its entries by a binary search over the users' running counts;
// the adds then go out user by user in ascending order, each an LDS atomic over the lanes
// holding that user's entries. A wave's LDS operations are performed in order, so every
// column is summed in ascending user order -- k_tile_rows_hub's sums, bit for bit -- with no
// block barrier per user (that kernel's 256-thread block waited at one per user, and walked
// the users one dependent load chain at a time).
__global__ __launch_bounds__(256) void k_group_rows_hub(
    const int64_t *__restrict__ hub_rows, const int64_t *__restrict__ n_hub,
    const int64_t *__restrict__ item_rowptr, const int32_t *__restrict__ item_users,
    const int32_t *__restrict__ user_items, const double *__restrict__ inv_deg,
    int64_t n_items, const int64_t *__restrict__ cur, const uint4 *__restrict__ counts,
    int32_t group_begin, int32_t tile, int32_t stop, const int64_t *__restrict__ bound,
    int64_t vthr, const int64_t *__restrict__ units_incl, uint32_t *__restrict__ lines,
    uint32_t *__restrict__ ovf, int32_t *__restrict__ row_len) {
  extern __shared__ double lds_acc[];  // tile doubles per wave
  const int nwb = blockDim.x / 64, wave = threadIdx.x / 64, lane = lane_id();
  double *acc = lds_acc + (size_t)wave * tile;
  const int64_t nh = *n_hub;
  for (int64_t h = (int64_t)blockIdx.x * nwb + wave; h < nh; h += (int64_t)gridDim.x * nwb) {
    const int64_t flat = hub_rows[h];
    const int t = (int)(flat / n_items);
    const int64_t i = flat - (int64_t)t * n_items;
    const int32_t item_begin = group_begin + t * tile;
    for (int j = lane; j < tile; j += 64) acc[j] = 0.0;
    wave_sync();
    const int64_t eb = item_rowptr[i], ee = item_rowptr[i + 1];
    for (int64_t e0 = eb; e0 < ee; e0 += 64) {
      const int64_t e = e0 + lane;
      int c = 0;
      int64_t s0 = 0;
      double wv = 0.0;
      if (e < ee) {
        const int32_t v = item_users[e];
        const uint4 lo = counts[2 * (int64_t)v], hi = counts[2 * (int64_t)v + 1];
        c = (int)count_of2(lo, hi, t);
        s0 = cur[v];
        for (int q = 0; q < t; ++q) s0 += count_of2(lo, hi, q);
        wv = inv_deg[v];
      }
      int incl = c;  // inclusive running count of the users' items (lane order = user order)
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      const int total = __shfl(incl, 63);
      const int pos = incl - c;
      uint64_t users = __ballot(c > 0);
      if (total <= 256) {
        // entry p = r * 64 + lane: the (p - pos_l)-th item of the user l with
        // pos_l <= p < incl_l (the first lane whose running count passes p)
        int col[4];
        double wt[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 64 * r + lane;
          col[r] = 0;
          wt[r] = 0.0;
          if (64 * r >= total) continue;  // (uniform)
          int lo = 0, hi = 63;
#pragma unroll
          for (int st = 0; st < 6; ++st) {  // first lane l with incl_l > p
            const int mid = (lo + hi) >> 1;
            if (__shfl(incl, mid) > p) hi = mid;
            else lo = mid + 1;
          }
          const int64_t s0l = __shfl(s0, lo);
          const int pl = __shfl(pos, lo);
          const double wl = __shfl(wv, lo);
          if (p < total) {
            col[r] = user_items[s0l + (p - pl)] - item_begin;
            wt[r] = wl;
          }
        }
        while (users) {
          const int l = __builtin_ctzll(users);
          users &= users - 1;
          const int pl = __builtin_amdgcn_readlane(pos, l);
          const int ql = __builtin_amdgcn_readlane(incl, l);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (64 * r >= ql || 64 * r + 64 <= pl) continue;  // (uniform)
            const int p = 64 * r + lane;
            if (p >= pl && p < ql) lds_add(acc, (uint32_t)col[r], wt[r]);
          }
        }
      } else {  // (a chunk of users with more than 256 items in the tile: user by user)
        while (users) {
          const int l = __builtin_ctzll(users);
          users &= users - 1;
          const int cl = __builtin_amdgcn_readlane(c, l);
          const int64_t s0l = __shfl(s0, l);
          const double wl = __shfl(wv, l);
          for (int q = lane; q < cl; q += 64)
            lds_add(acc, (uint32_t)(user_items[s0l + q] - item_begin), wl);
        }
      }
    }
    wave_sync();
    uint32_t *line = lines + (int64_t)t * (n_items + 1) * 32 + i * 32;
    const int64_t tbase = t ? units_incl[(int64_t)t * n_items - 1] : 0;
    uint32_t *ov = ovf + tbase * 4;
    const int width = (int)tile_width(group_begin, tile, t, stop);
    const int64_t ou = units_incl[flat] - run_units(bound[flat], vthr, width) - tbase;
    int nzr = 0;
    for (int j0 = 0; j0 < tile; j0 += 64)
      nzr += __popcll(__ballot(j0 + lane < tile && acc[j0 + lane] != 0.0));
    if (hub_row_dense(nzr, width)) {
      write_hub_row_dense(acc, width, line, ov, ou, lane, 64);
      if (lane == 0 && row_len) row_len[flat] = nzr;
      wave_sync();
      continue;
    }
    int base = 0;
    for (int j0 = 0; j0 < tile; j0 += 64) {
      const int j = j0 + lane;
      const double x = j < tile ? acc[j] : 0.0;
      const bool nz = x != 0.0;
      const uint64_t b = __ballot(nz);
      if (nz) {
        const uint64_t bits = (uint64_t)__double_as_longlong(x);
        const int64_t en = base + __popcll(b & lanemask_lt());
        uint32_t *u4 = en < kLineEnts ? line + 4 * (1 + en) : ov + 4 * (ou + 1 + (en - kLineEnts));
        *reinterpret_cast<uint4 *>(u4) =
            uint4{kEntV | (uint32_t)j, (uint32_t)bits, (uint32_t)(bits >> 32), 0u};
      }
      base += __popcll(b);
    }
    const bool has_ovf = base > kLineEnts;
    if (lane < 32) {
      const int tw = lane;  // line word
      const int unit = tw / 4;
      if (tw == 0) line[0] = kHdrV | kHdrSlow | (has_ovf ? (kHdrOvf | (uint32_t)ou) : 0u);
      else if (unit == 0 || unit > base) line[tw] = 0u;
    }
    if (has_ovf && lane < 4) ov[ou * 4 + lane] = lane == 0 ? (uint32_t)(base - kLineEnts) : 0u;
    if (lane == 0 && row_len) row_len[flat] = base;
    wave_sync();
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

#if LG_REFERENCE_PATHS
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

#endif  // LG_REFERENCE_PATHS

// ------------------------------------------------------------ the tile walk kernel
// One launch per tile. Persistent waves (NW per workgroup, one workgroup per CU; each wave
// takes users u, u + G, u + 2G, ... with G = all waves). A wave's work is a stream of
// BATCHES of at most 64 of a user's rows (every user has at least one, possibly empty):
// lane (g, h) = (lane / 8, lane % 8) loads unit h of row 8q + g for q < 8, so one load
// instruction moves 8 whole lines. The stream is software-pipelined: while batch t is
// decoded, the lines and ra of batch t+1 and the item ids of batch t+2 are in flight (and
// the row pointers of the user after that). Each path is added with one LDS atomic
// (ds_add_f64); rows whose header says "slow" (V rows, far degree classes) take a general
// decode, overflow runs are collected in LDS and loaded together after the batch.
//
// MODE_F:    F[u][j - item_begin] = rb_j * acc[j] (lg_spread_tile_resource_f64).
// MODE_TOPK: the tile's columns of (G *) F merge into the running per-user top-K lists
//            (lg_spread_tile_resource_topk_f64); F never leaves LDS. A column's score can
//            only beat the list's K-th value tau if acc * rb_max (* gb) > tau, rb_max = the
//            tile's largest rb and gb = the (user, 64-column chunk) upper bound of the fp32
//            score chain from lg_score_chunk_bound (bf16 MFMA + a rigorous rounding margin):
//            only those columns get rb_j and (with G) the exact chain score. Ids grow along
//            the walk, so "beats" is v > tau (a tie loses to the older, smaller id).
constexpr int MODE_F = 0, MODE_TOPK = 1;
constexpr int kWalkQ = 8;       // line loads per lane per batch: 8 rows each, 64 rows
constexpr int kBatchRows = 8 * kWalkQ;
// per-wave scratch list: the batch's overflow rows during the decode, the exact-score queue
// (column, f) during the scan -- a drain round can queue one candidate per lane, so it holds
// at least 64 entries whatever the batch size
constexpr int kOvfList = kBatchRows > 64 ? kBatchRows : 64;
constexpr int kDecodePhase = 4;  // lines whose class reads precede their adds
// q dwords per lane loaded with the user's state (256 columns each: a whole 2048-column
// tile); the columns of wider tiles past them are screened by their chunk bound alone (q =
// 255), so the scan issues no memory loads
constexpr int kQPre = 8;
static_assert(kWalkQ % kDecodePhase == 0, "decode phase must divide the batch's line loads");

struct WalkArgs {
  const int64_t *user_rowptr;
  const int32_t *user_items;
  const double *ra_edge;      // ra of user_items[p], aligned with user_items
  int64_t n_users;
  const uint4 *lines;         // n_items + 1 lines (the last all zero)
  const uint4 *ovf;
  int32_t null_row;           // = n_items
  int32_t item_begin, tile, width;
  const double *rbeta;  // all items: 1 / beta
  const double *g_inv;  // fl(1/k) by class number (index 0 unused)
  // MODE_F
  double *F;
  int64_t ldf;
  // MODE_TOPK
  const float *eu, *ei;       // rows' user embeddings / all item embeddings (or NULL)
  const float *gb;            // [n_users][nch] score bounds (with eu)
  int32_t nch;
  const uint8_t *qb;          // [n_users][qstride] per-column 8-bit bounds (or NULL)
  int32_t qstride;
  const int64_t *ex_rowptr;   // exclusions (dropped), with a per-row cursor
  const int32_t *ex_col;
  int64_t *ex_cur;
  int k, first;
  double *io_val;
  int64_t *io_idx;
};

// accumulator columns per wave: the tile rounded up to whole 512-column scan steps
__host__ __device__ constexpr int acc_cols(int tile) { return (tile + 511) / 512 * 512; }

// per wave: acc[acc_cols(tile)] and the overflow list (decode; the exact-score queue during
// the scan); the running list itself lives in registers
template <int MODE, int D, int M>
__host__ __device__ constexpr size_t walk_wave_bytes(int tile) {
  return ((size_t)acc_cols(tile) * 8 + (size_t)kOvfList * 12 + 15) & ~(size_t)15;
}
__host__ __device__ constexpr size_t walk_shared_bytes(int tile) {
  // class table + the block's rb maxima + rb of the tile's columns + its 64-column chunks'
  // rb maxima
  return (size_t)kInvTab * 8 + 16 * 8 + (size_t)((tile + 1) & ~1) * 8 + 64 * 8;
}


// The fast decode's two LDS addresses of a P slot s (class << 16 | column, column < 8192),
// one VALU op each: fl(1/k) of the class at byte s >> 13 (s_inv at LDS address 0; bits
// 13-15 of the column are 0), and the column's acc entry at acc_base + 8 (s & 0xFFFF).
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ double slot_inv_fast(uint32_t s) {
  return *(const lds_f64 *)(uintptr_t)(s >> 13);
}
// Branch-free form: an empty slot (s == 0, value 0) adds its 0.0 to the lane's own dummy
// word instead (no exec-mask branch per slot; the dummies are lane-distinct: no conflicts).
__device__ __forceinline__ void slot_add_nobranch(uint32_t acc_base, uint32_t dummy, uint32_t s,
                                                  double v) {
  uint32_t addr;
  asm("v_mad_u32_u16 %0, %1, 8, %2" : "=v"(addr) : "v"(s), "v"(acc_base));
  addr = s ? addr : dummy;
  __hip_atomic_fetch_add((lds_f64 *)(uintptr_t)addr, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}

// fl(1/k) of a P slot's degree class (general decode: classes >= kInvTab from memory)
__device__ __forceinline__ double slot_inv(uint32_t s, const double *s_inv,
                                           const double *__restrict__ g_inv) {
  const uint32_t c = s >> 16;
  const bool far = c >= (uint32_t)kInvTab;
  const double inv = s_inv[far ? 0u : c];
  if (__builtin_expect(__ballot(far) != 0, 0)) {  // (a separate load: not a flat select)
    const double g = __builtin_nontemporal_load(g_inv + (far ? c : 0u));
    return far ? g : inv;
  }
  return inv;
}

// General decode of one 16-byte unit: a V entry (x has bit 31) or 4 P slots (zero words:
// padding). head: unit 0 of a line, whose word x is the row header (y, z, w are slots of a
// P row and zero in a V row).
__device__ __forceinline__ void add_unit(double *acc, uint4 w, bool head, double ra,
                                         const double *s_inv, const double *__restrict__ g_inv) {
  const bool isv = !head && (w.x & kEntV);
  const uint32_t sx = head ? 0u : w.x;
  // P slot words only (a V entry's y / z are its value: never decoded as classes)
  const uint32_t py = isv ? 0u : w.y, pz = isv ? 0u : w.z, pw = isv ? 0u : w.w;
  const double i0 = slot_inv(isv ? 0u : sx, s_inv, g_inv);
  const double v0 = (isv ? __hiloint2double((int)w.z, (int)w.y) : i0) * ra;
  const double v1 = slot_inv(py, s_inv, g_inv) * ra;
  const double v2 = slot_inv(pz, s_inv, g_inv) * ra;
  const double v3 = slot_inv(pw, s_inv, g_inv) * ra;
  if (sx) lds_add(acc, sx & 0xFFFFu, v0);
  if (py) lds_add(acc, py & 0xFFFFu, v1);
  if (pz) lds_add(acc, pz & 0xFFFFu, v2);
  if (pw) lds_add(acc, pw & 0xFFFFu, v3);
}

// A unit of a V row's overflow run: one entry (or a zero padding unit), ra * general_W into
// its column (add_unit's V case without its four class reads of P slots)
__device__ __forceinline__ void add_unit_v(double *acc, uint4 w, double ra) {
  if (w.x & kEntV) lds_add(acc, w.x & 0xFFFFu, __hiloint2double((int)w.z, (int)w.y) * ra);
}
// data unit q of a dense V row's run: columns 2q and 2q + 1 (zero values skipped)
__device__ __forceinline__ void add_unit_d(double *acc, uint4 w, int q, double ra) {
  const double a = __hiloint2double((int)w.y, (int)w.x), b = __hiloint2double((int)w.w, (int)w.z);
  if (a != 0.0) lds_add(acc, (uint32_t)(2 * q), a * ra);
  if (b != 0.0) lds_add(acc, (uint32_t)(2 * q + 1), b * ra);
}

// Fast decode (P rows whose classes are all < kInvTab): s_inv sits at LDS address 0.
__device__ __forceinline__ void add_slot_fast(double *acc, uint32_t s, double ra,
                                              const double *s_inv) {
  const double inv = s_inv[s >> 16];
  if (s) lds_add(acc, s & 0xFFFFu, inv * ra);
}

// A batch of the wave's stream: rows [r0, r1) of user u (whose rows end at e); xc / xh =
// the user's exclusion cursor and row end (prefetched with its row pointers). 32-bit fields
// (the host requires users, interactions and exclusions < 2^31): the stream state then fits
// the SGPRs without spilling into VGPR lanes.
struct Batch {
  int32_t u, r0, r1, e;
  bool first;
  int32_t xc, xh;
};

// The top-K state of a batch's user, loaded with the batch's lines (every batch loads it:
// the loads are unconditional, so the compiler's vmcnt bookkeeping never waits for a
// younger load than the one it needs): the running list (lane, 64 + lane), the chunk score
// bound, the per-column 8-bit bounds of the first kQPre * 256 columns and the next 64
// excluded items.
struct UState {
  int lid0, lid1;
  double lv0, lv1;
  float gb;
  uint32_t q[kQPre];
  int32_t xw;
};

// SEED: the first tile's instance (lists start empty): the finish scores the columns with the
// largest bounds first (below); a separate instance so the other tiles' code is untouched
template <int MODE, int D, int M, bool SEED = false>
__global__ __launch_bounds__(512) void k_tile_walk(WalkArgs a) {
  constexpr int Q = kWalkQ;
  extern __shared__ double lds[];
  const int nw = blockDim.x / 64;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  const int lane = lane_id();
  const int gh = lane & 7;     // unit of the line this lane loads
  const int grow = lane >> 3;  // row of the 8-row load group
  const uint32_t hmask = gh == 0 ? 0u : 0xFFFFFFFFu;  // word x of unit 0 is the header
  const int tile = a.tile;
  double *s_inv = lds;  // at LDS address 0 (the fast decode indexes it with class * 8)
  double *s_red = s_inv + kInvTab;
  double *s_rb = s_red + 16;  // rb of the tile's columns (0 past the width)
  // per 64-column chunk: the largest rb (G screen, tile <= 4096); the waves' areas after it
  // (16-byte aligned: the tile's rb padded to an even count)
  double *s_rbc = s_rb + ((tile + 1) & ~1);
  char *mine = reinterpret_cast<char *>(s_rbc + 64) +
               (size_t)wave * walk_wave_bytes<MODE, D, M>(tile);
  double *acc = reinterpret_cast<double *>(mine);
  const uint32_t acc_base = (uint32_t)(uintptr_t)(lds_f64 *)acc;
  // the lane's dummy word for empty slots: its entry of the overflow list (rewritten before
  // every use; adding 0.0 leaves it unchanged meanwhile)
  const uint32_t dummy_addr = acc_base + 8u * (uint32_t)(acc_cols(tile) + lane);
  double *ovl_ra = acc + acc_cols(tile);  // overflow list (decode)
  uint32_t *ovl_ent = reinterpret_cast<uint32_t *>(ovl_ra + kOvfList);

  for (int c = threadIdx.x; c < kInvTab; c += blockDim.x) s_inv[c] = a.g_inv[c];
  double rmax = 0.0;  // the tile's largest rb (top-K prefilter)
  for (int j = threadIdx.x; j < tile; j += blockDim.x) {
    const double rb = j < a.width ? a.rbeta[a.item_begin + j] : 0.0;
    s_rb[j] = rb;
    rmax = fmax(rmax, rb);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) rmax = fmax(rmax, __shfl_xor(rmax, o));
  if (lane == 0) s_red[wave] = rmax;
  for (int j = lane; j < acc_cols(tile); j += 64) acc[j] = 0.0;
  __syncthreads();
  if (MODE == MODE_TOPK && D > 0) {
    for (int c = wave; 64 * c < tile && c < 64; c += nw) {
      double m = s_rb[64 * c + lane < tile ? 64 * c + lane : 0];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
      if (lane == 0) s_rbc[c] = m;
    }
    __syncthreads();
  }
  rmax = 0.0;
  for (int w = 0; w < nw; ++w) rmax = fmax(rmax, s_red[w]);
  // acc * rb_j > tau  implies  acc * rb_max * (1 + 2^-50) > tau (rounding of both products)
  const double rscale = rmax * (1.0 + 0x1p-50);

  const int64_t G = (int64_t)gridDim.x * nw;
  const int64_t n_users = a.n_users;
  const int64_t u_first = (int64_t)blockIdx.x * nw + wave;
  if (u_first >= n_users) return;

  // row pointers (and exclusion cursor) of the next new user of the stream, prefetched one
  // user ahead. Lane-varying loads (lane 0 / 1: the row's start / end, resp. exclusion cursor /
  // row end) keep the values in VGPRs until the user starts: a wave-uniform load is read into
  // SGPRs right away, and hipcc then waits for it where it is issued -- vmcnt(0), draining
  // every batch line in flight at each new user. Reissued unconditionally at every step
  // (clamped past the last user; the same address until a user starts): a load issued only
  // when a user starts leaves a register copy at the join, which hipcc also guards with
  // vmcnt(0).
  const bool has_ex = MODE == MODE_TOPK && a.ex_rowptr != nullptr;
  int32_t uq = (int32_t)u_first;
  int32_t pr = 0, px = 0;  // lanes 0, 1: the prefetched (start, end) / (cursor, end)
  // (positions < 2^31: the low dword of each int64 entry, one 4-byte load -- a whole int64
  // load's unused high half would pin a register whose reuse hipcc guards with a vmcnt wait)
  auto pre_load = [&]() __attribute__((always_inline)) {
    const int64_t uu = uq < n_users ? uq : n_users - 1;
    pr = reinterpret_cast<const int32_t *>(a.user_rowptr)[2 * (uu + (lane & 1))];
    if (has_ex) {  // (uniform)
      const int64_t *p = (lane & 1) ? a.ex_rowptr + uu + 1 : a.ex_cur + uu;
      px = *reinterpret_cast<const int32_t *>(p);
    }
  };
  pre_load();
  auto new_user = [&]() __attribute__((always_inline)) {
    const int32_t bq = __builtin_amdgcn_readlane(pr, 0), eq = __builtin_amdgcn_readlane(pr, 1);
    const int32_t xcq = has_ex ? __builtin_amdgcn_readlane(px, 0) : 0;
    const int32_t xhq = has_ex ? __builtin_amdgcn_readlane(px, 1) : 0;
    Batch y{uq, bq, bq + kBatchRows < eq ? bq + kBatchRows : eq, eq, true, xcq, xhq};
    uq += (int32_t)G;
    return y;
  };
  const Batch kEnd{(int32_t)n_users, 0, 0, 0, false, 0, 0};  // past the end of the stream
  auto next_batch = [&](const Batch &x) __attribute__((always_inline)) {
    if (x.u >= n_users) return kEnd;
    if (x.r1 < x.e) {
      Batch y{x.u, x.r1, x.r1 + kBatchRows < x.e ? x.r1 + kBatchRows : x.e, x.e, false, x.xc,
              x.xh};
      return y;
    }
    if (x.u + G >= n_users) return kEnd;
    return new_user();
  };
  // item ids of a batch's rows (lanes of one 8-lane group: one row)
  // Buffer loads with 32-bit offsets: a batch's item ids and ra through a descriptor based
  // at its first row (lane offsets are per-lane constants + immediates; rows past the batch
  // are out of range and read 0), the lines through one descriptor for the tile.
  const __amdgpu_buffer_rsrc_t r_lines = __builtin_amdgcn_make_buffer_rsrc(
      (void *)a.lines, 0, (int)((uint32_t)(a.null_row + 1) * 128u), 0x00020000);
  auto load_ids = [&](const Batch &x, int32_t (&it)[Q]) __attribute__((always_inline)) {
    {  // (unconditional: an empty batch reads 0 through a 0-byte descriptor)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(a.user_items + x.r0), 0, (int)((x.r1 - x.r0) * 4), 0x00020000);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        it[q] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(grow * 4 + 32 * q),
                                                              0, 0);
    }
  };
  // lines and ra of a batch (rows past r1 read the zero line, and ra 0)
  auto load_rows = [&](const Batch &x, const int32_t (&it)[Q], uint4 (&w)[Q], double (&ra)[Q])
      __attribute__((always_inline)) {
    // (every load group is issued even past a short last batch: skipping them with a
    // uniform branch measured 40 % slower -- the branches cost the loads their overlap)
    const int nr = (int)(x.r1 - x.r0);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.ra_edge + x.r0), 0, nr * 8, 0x00020000);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const bool in = 8 * q + grow < nr;
      const uint32_t row = in ? (uint32_t)it[q] : (uint32_t)a.null_row;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r_lines, row * 128u + 16u * gh, 0, 0);
      w[q] = uint4{v[0], v[1], v[2], v[3]};
      const auto d = __builtin_amdgcn_raw_buffer_load_b64(rr, (uint32_t)(grow * 8 + 64 * q), 0, 0);
      ra[q] = __builtin_bit_cast(double, d);
    }
  };

  // ---- top-K state of a batch's user (MODE_TOPK), loaded with the batch's lines: every load
  // is issued (clamped user, 0-byte descriptors for absent operands), the consumers apply the
  // masks at the finish
  constexpr bool kTwo = M > 2;  // k > 64: the list spans two registers per lane
  const bool has_qb = MODE == MODE_TOPK && D > 0 && a.qb != nullptr;
  auto load_state = [&](const Batch &x, UState &st) __attribute__((always_inline)) {
    if constexpr (MODE == MODE_TOPK) {
      const int k = a.k;
      const int64_t us = x.u < n_users ? x.u : n_users - 1;
      // ids < 2^31 (and -1): the low dword of the int64 entry
      const int *idx32 = reinterpret_cast<const int *>(a.io_idx);
      const int e0 = lane < k ? lane : k - 1;
      st.lid0 = idx32[2 * (us * k + e0)];
      st.lv0 = a.io_val[us * k + e0];
      if constexpr (kTwo) {
        const int e1 = 64 + lane < k ? 64 + lane : k - 1;
        st.lid1 = idx32[2 * (us * k + e1)];
        st.lv1 = a.io_val[us * k + e1];
      }
      if constexpr (D > 0) {
        st.gb = a.gb[us * a.nch + (lane < a.nch ? lane : 0)];
        const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
            has_qb ? (void *)(a.qb + us * a.qstride) : (void *)a.lines, 0,
            has_qb ? a.qstride : 0, 0x00020000);
        // (the whole offset in voffset + the immediate, both range-checked against qstride:
        // a tile narrower than kQPre * 256 columns reads 0 past its row instead of the next
        // user's -- or, for the last user, past the allocation)
#pragma unroll
        for (int kk = 0; kk < kQPre; ++kk)
          st.q[kk] = __builtin_amdgcn_raw_buffer_load_b32(rq, (uint32_t)(4 * lane + 256 * kk), 0, 0);
      }
      const int32_t nx = x.xh - x.xc;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          has_ex ? (void *)(a.ex_col + x.xc) : (void *)a.lines, 0,
          has_ex ? (int)(4 * (nx < 64 ? nx : 64)) : 0, 0x00020000);
      st.xw = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rx, (uint32_t)(4 * lane), 0, 0);
    }
  };

  // ---- decode one batch into acc
  auto decode = [&](const Batch &x, uint4 (&w)[Q], const double (&ra)[Q])
      __attribute__((always_inline)) {
#ifdef LG_WALK_PROBE  // measurement builds only (wrong lists): 2 = no decode (lines loaded only)
    if (LG_WALK_PROBE == 2) {
      uint32_t h = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) h ^= w[q].x ^ w[q].y ^ w[q].z ^ w[q].w ^ (uint32_t)ra[q];
      if (h == 0x12345678u && lane == 64) acc[0] = 1.0;  // (keeps the loads; never true)
      return;
    }
#endif
    uint32_t hdr = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) hdr |= w[q].x & ~hmask;  // the group heads' headers
    const bool slow = __ballot(hdr & kHdrSlow) != 0;
    const bool ovf = __ballot(hdr & kHdrOvf) != 0;
    if (!slow) {
      // The LDS serves a wave's operations in order, so a class-table read issued after an
      // atomic returns only once the atomic is done: the reads of H lines' slots go out
      // first, then their adds (one wait per phase, not one per slot).
      // (line groups wholly past a short batch's rows hold the zero line: their reads and
      // adds are skipped with a wave-uniform branch; their loads were issued regardless)
      constexpr int H = kDecodePhase;
      const int nr = (int)(x.r1 - x.r0);
#pragma unroll
      for (int q0 = 0; q0 < Q; q0 += H) {
        if (8 * q0 >= nr) break;
        double inv[H][4];
#pragma unroll
        for (int q = 0; q < H; ++q) {
          if (8 * (q0 + q) >= nr) break;
          inv[q][0] = slot_inv_fast(w[q0 + q].x & hmask);
          inv[q][1] = slot_inv_fast(w[q0 + q].y);
          inv[q][2] = slot_inv_fast(w[q0 + q].z);
          inv[q][3] = slot_inv_fast(w[q0 + q].w);
        }
#pragma unroll
        for (int q = 0; q < H; ++q) {
          if (8 * (q0 + q) >= nr) break;
          const uint32_t sv[4] = {w[q0 + q].x & hmask, w[q0 + q].y, w[q0 + q].z, w[q0 + q].w};
#pragma unroll
          for (int t = 0; t < 4; ++t)
            slot_add_nobranch(acc_base, dummy_addr, sv[t], inv[q][t] * ra[q0 + q]);
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) add_unit(acc, w[q], gh == 0, ra[q], s_inv, a.g_inv);
    }
    if (ovf) {  // overflow runs: collected, then up to 4 rows' first 64 units in flight
      int nov = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const bool o = gh == 0 && (w[q].x & kHdrOvf);
        const uint64_t bal = __ballot(o);
        if (o) {
          const int p = nov + __popcll(bal & lanemask_lt());
          ovl_ent[p] = w[q].x & (kHdrPtr | kHdrV);  // (the run's first unit; a V row's bit)
          ovl_ra[p] = ra[q];
        }
        nov += __popcll(bal);
      }
      wave_sync();
      for (int t0 = 0; t0 < nov; t0 += 4) {
        uint4 y4[4];
        uint32_t ou4[4];
        double r4[4];
        bool v4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool in = t0 + j < nov;
          const uint32_t e = ovl_ent[in ? t0 + j : t0];
          v4[j] = (e & kHdrV) != 0;
          ou4[j] = e & kHdrPtr;
          r4[j] = ovl_ra[in ? t0 + j : t0];
          y4[j] = a.ovf[(int64_t)ou4[j] + lane];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (t0 + j >= nov) continue;
          const uint32_t n0 = (uint32_t)__shfl((int)y4[j].x, 0);
          const bool dn = (n0 & kRunDense) != 0;  // (a dense V row: unit q -> columns 2q, 2q+1)
          const uint32_t n = n0 & ~kRunDense;
          if (lane == 0 || (uint32_t)lane > n) y4[j] = uint4{0u, 0u, 0u, 0u};
          if (dn) add_unit_d(acc, y4[j], lane - 1, r4[j]);
          else if (v4[j]) add_unit_v(acc, y4[j], r4[j]);
          else add_unit(acc, y4[j], false, r4[j], s_inv, a.g_inv);
          // runs longer than 63 units (hub items' V rows: up to a whole tile of entries): 4
          // chunks of 64 units in flight per round instead of one load -> add at a time
          for (uint32_t c = 64; c <= n; c += 256) {
            uint4 z[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
              const uint32_t cc = c + 64 * p + lane;
              z[p] = cc <= n ? a.ovf[(int64_t)ou4[j] + cc] : uint4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int p = 0; p < 4; ++p) {
              if (c + 64 * p > n) break;  // (uniform)
              if (dn) add_unit_d(acc, z[p], (int)(c + 64 * p) + lane - 1, r4[j]);
              else if (v4[j]) add_unit_v(acc, z[p], r4[j]);
              else add_unit(acc, z[p], false, r4[j], s_inv, a.g_inv);
            }
          }
        }
      }
      wave_sync();
    }
  };

  // ---- the user's tile of F: written out (MODE_F) or merged into its top-K list
  auto finish_user = [&](const Batch &x, UState &st) __attribute__((always_inline)) {
    const int64_t u = x.u;
    wave_sync();
#ifdef LG_WALK_PROBE  // measurement builds only (wrong lists): 1 = no scan (acc zeroed only)
    if (LG_WALK_PROBE == 1) {
      for (int j = 2 * lane; j < acc_cols(tile); j += 128)
        *reinterpret_cast<double2 *>(acc + j) = double2{0.0, 0.0};
      wave_sync();
      return;
    }
#endif
    if constexpr (MODE == MODE_F) {
      double *row = a.F + u * a.ldf;
      for (int j = lane; j < tile; j += 64) {
        __builtin_nontemporal_store(acc[j] * s_rb[j], row + j);
        acc[j] = 0.0;
      }
    } else {
      const int k = a.k;
      // the running list in registers: entry lane (L0, I0) and 64 + lane (L1, I1), sorted by
      // (value desc, id asc); empty entries (-inf, kPadId); a first tile starts empty
      const bool ok0 = !a.first && lane < k && st.lid0 >= 0;
      double L0 = ok0 ? st.lv0 : neg_inf<double>();
      int I0 = ok0 ? st.lid0 : kPadId;
      double L1 = neg_inf<double>();
      int I1 = kPadId;
      if constexpr (kTwo) {
        const bool ok1 = !a.first && 64 + lane < k && st.lid1 >= 0;
        L1 = ok1 ? st.lv1 : neg_inf<double>();
        I1 = ok1 ? st.lid1 : kPadId;
      }
      const float gbv = st.gb;
      uint32_t (&qr)[kQPre] = st.q;
      if (!has_qb) {
#pragma unroll
        for (int kk = 0; kk < kQPre; ++kk) qr[kk] = 0xFFFFFFFFu;
      }
      int64_t xpos = x.xc;
      const int64_t xhi = x.xh;
      int32_t xw = has_ex && xpos + lane < xhi ? st.xw : 0x7fffffff;
      auto kth = [&](double &tv, int &ti) __attribute__((always_inline)) {
        if (!kTwo || k <= 64) {
          tv = __shfl(L0, k - 1);
          ti = __shfl(I0, k - 1);
        } else {
          tv = __shfl(L1, k - 65);
          ti = __shfl(I1, k - 65);
        }
      };
      double tau;
      int tau_id;
      kth(tau, tau_id);
      bool dirty = a.first != 0;
      // insert (v, id) (wave-uniform) if it beats the k-th entry: its rank is the number of
      // entries before it; the entries from that rank on move one place down
      auto insert1 = [&](double v, int id) __attribute__((always_inline)) {
        if (!before(v, id, tau, tau_id)) return;
        dirty = true;
        int pos = __popcll(__ballot(before(L0, I0, v, id)));
        if constexpr (kTwo) pos += __popcll(__ballot(before(L1, I1, v, id)));
        const double up0 = __shfl_up(L0, 1);
        const int iu0 = __shfl_up(I0, 1);
        if constexpr (kTwo) {
          const double up1 = __shfl_up(L1, 1);
          const int iu1 = __shfl_up(I1, 1);
          const double c0 = __shfl(L0, 63);
          const int ic0 = __shfl(I0, 63);
          const int p1 = 64 + lane;
          const double n1 = p1 > pos ? (lane == 0 ? c0 : up1) : (p1 == pos ? v : L1);
          const int m1 = p1 > pos ? (lane == 0 ? ic0 : iu1) : (p1 == pos ? id : I1);
          L1 = p1 < k ? n1 : neg_inf<double>();
          I1 = p1 < k ? m1 : kPadId;
        }
        L0 = lane > pos ? up0 : (lane == pos ? v : L0);
        I0 = lane > pos ? iu0 : (lane == pos ? id : I0);
        if (lane >= k) { L0 = neg_inf<double>(); I0 = kPadId; }
        kth(tau, tau_id);
      };
      // excluded items of this tile (the next run of the user's sorted exclusion row): -1
      const int32_t lim = a.item_begin + a.width;
      if (has_ex) {
        for (;;) {
          const bool in = xw < lim;
          if (in && xw >= a.item_begin) acc[xw - a.item_begin] = neg_inf<double>();
          const int nin = __popcll(__ballot(in));
          xpos += nin;
          if (nin < 64) break;
          xw = xpos + lane < xhi ? a.ex_col[xpos + lane] : 0x7fffffff;  // > 64 in one tile
        }
        if (lane == 0) a.ex_cur[u] = xpos;
      }
      wave_sync();
      // The scan: lane l reads columns c0 + 2l, c0 + 2l + 1 (ds_read_b128), 4 reads in flight
      // (512 columns). A column can enter only if acc > thr, thr = tau / (rb_max (1 + 2^-50)
      // [* max(gb, 0)]) (>= -0.5: excluded columns hold -1; every rounding of
      // fl(gb fl(acc rb_j)) > tau is covered by the 2^-50 margin); those get rb_j and (with G)
      // the exact score. The list order (value desc, id asc) is total, so the order in which
      // candidates are inserted does not matter.
      // Exact scores in batches (D > 0): the columns that pass the bound test are queued in
      // LDS (column, f) and scored 16 at a time by v_mfma_f32_16x16x4_f32 -- candidate m as
      // A row m (its item row), the user row as every B column -- whose per-element sums are
      // the fp32 chain acc = fmaf(u[g*D/4+s], i[g*D/4+s], acc) (s outer, g inner) of
      // lg_score_topk_f32. One load round trip per 16 candidates instead of a dependent
      // per-lane chain of item-row loads; the queue is flushed when it holds 16, when the list
      // is not full yet (tau = -inf: every column passes), and at the end of the scan.
      int ncand = 0;
      double *cq_f = ovl_ra;     // queued f (the decode's overflow list, free during the scan)
      uint32_t *cq_j = ovl_ent;  // queued column
      auto flush = [&]() __attribute__((always_inline)) {
#ifdef LG_WALK_PROBE  // 3 = no exact scores: candidates inserted with their f as the score
        if (LG_WALK_PROBE == 3) {
          wave_sync();
          for (int mm = 0; mm < ncand; ++mm) insert1(cq_f[mm], a.item_begin + (int)cq_j[mm]);
          ncand = 0;
          wave_sync();
          return;
        }
#endif
        if constexpr (D > 0) {
          constexpr int Qd = D / 4;              // MFMA steps
          constexpr int H = Qd < 16 ? Qd : 16;   // steps per load round (<= 16 VGPRs each)
          wave_sync();
          const int m = lane & 15, g = lane >> 4;
          for (int b0 = 0; b0 < ncand; b0 += 16) {
            const int nb = ncand - b0 < 16 ? ncand - b0 : 16;
            const int ci = b0 + (m < nb ? m : 0);
            const float *ir = a.ei + (int64_t)(a.item_begin + (int)cq_j[ci]) * D + g * Qd;
            const float *ur = a.eu + u * D + g * Qd;
            f32x4 sc4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int h0 = 0; h0 < Qd; h0 += H) {
              float av[H], bv[H];
              load_frag<H>(ir + h0, av);
              load_frag<H>(ur + h0, bv);
#pragma unroll
              for (int s = 0; s < H; ++s)
                sc4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], sc4, 0, 0, 0);
            }
            // candidate mm's sum: lane 16 (mm / 4), element mm % 4
            for (int mm = 0; mm < nb; ++mm) {
              const float e = (mm & 3) == 0 ? sc4[0] : (mm & 3) == 1 ? sc4[1]
                            : (mm & 3) == 2 ? sc4[2] : sc4[3];
              const float sc = __shfl(e, 16 * (mm >> 2));
              insert1((double)sc * cq_f[b0 + mm], a.item_begin + (int)cq_j[b0 + mm]);
            }
          }
          ncand = 0;
          wave_sync();
        }
      };
      // The scan, 512 columns per iteration: lane l takes columns c0 + 4l .. + 3 and
      // c0 + 256 + 4l .. + 3 (ds_read_b128 x 4). A column can enter only if
      //   no G:  acc > thr = tau / (rb_max (1 + 2^-50))            (excluded: acc = -inf)
      //   G:     acc * q * (rbmax_c (1 + 2^-50) max(gb, 0) / 255) > tau   (c = the chunk)
      // (gb * q / 255 >= the exact score, q = the column's 8-bit bound, 255 without qb; the
      // 2^-50 margin covers every rounding of fl(G fl(acc rb_j)) > tau). The lanes' passing
      // columns form a bit mask that one loop drains (one candidate per lane per round): rb_j,
      // then (G) the column bound times f and the exact chain score, then the insertion. The
      // list order (value desc, id asc) is total, so the insertion order does not matter.
      double thr_s = tau / rscale;
      double sc_v = 0.0, bq_v = 0.0;  // per 64-column chunk c in lane c (D > 0)
      if constexpr (D > 0) {
        // the pre-screen scale of chunk c: its own largest rb (not the tile's), so a column
        // passes only if acc * q * rbmax_c (1 + 2^-50) gb / 255 > tau
        const double gp = (double)fmaxf(gbv, 0.f);
        sc_v = s_rbc[lane < a.nch ? lane : 0] * (1.0 + 0x1p-50) * gp * (1.0 / 255.0);
        bq_v = gp * (1.0 / 255.0) * (1.0 + 0x1p-50);
      }
      // Seeding (the first tile's instance; G, k <= 64, a list that is not full): with tau = -inf
      // every column would pass and be scored exactly until the list fills and tau climbs from
      // whatever the first columns scored. Instead the columns whose pre-screen bound
      // b = acc q sc is at least t_hi = the k-th largest of the lanes' maximum bounds (so at
      // least k columns) are scored first (pass A), tau starts at the k-th best of them, and
      // the scan below skips exactly those columns (the same b, computed the same way). The
      // candidate set and the list order are unchanged, so the list is the same.
      bool seeded = false;
      double t_hi = 0.0;
      if constexpr (SEED && D > 0 && !kTwo) {  // (kTwo: k > 64, two list registers per lane)
        if (tau == neg_inf<double>()) {
          // step s8's columns c0 = 512 s8 + ...: the 8 accumulator values of the lane (read
          // only; the scan below zeroes them) and their bounds b, computed as the scan does
          auto read8 = [&](int c0, double (&sv)[8]) __attribute__((always_inline)) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
#pragma unroll
              for (int pp = 0; pp < 2; ++pp) {
                const int j = c0 + 256 * hh + 4 * lane + 2 * pp;
                const double2 x = *reinterpret_cast<const double2 *>(acc + j);
                sv[4 * hh + 2 * pp] = x.x;
                sv[4 * hh + 2 * pp + 1] = x.y;
              }
            if (c0 + 512 > a.width) {
#pragma unroll
              for (int t = 0; t < 8; ++t) {
                const int j = c0 + 256 * (t >> 2) + 4 * lane + (t & 3);
                if (j >= a.width) sv[t] = neg_inf<double>();
              }
            }
          };
          auto qsel = [&](int i) __attribute__((always_inline)) {  // qr[i] for a uniform i
            uint32_t v = 0xFFFFFFFFu;  // (columns past 256 kQPre: the chunk bound alone)
#pragma unroll
            for (int x = 0; x < kQPre; ++x) v = i == x ? qr[x] : v;
            return v;
          };
          auto bound = [&](int c0, int t, double svt, uint32_t qa, uint32_t qb2)
              __attribute__((always_inline)) {
            const double sc = __shfl(sc_v, ((c0 + 256 * (t >> 2) + 4 * lane) >> 6) & 63);
            const uint32_t qq = t < 4 ? qa : qb2;
            const double qv = (double)((qq >> (8 * (t & 3))) & 0xFFu);
            return svt * qv * sc;
          };
          double lmax = neg_inf<double>();
#pragma unroll 1
          for (int c0 = 0; c0 < a.width; c0 += 512) {
            double sv[8];
            read8(c0, sv);
            const uint32_t qa = qsel(c0 >> 8), qb2 = qsel((c0 >> 8) + 1);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const double bt = bound(c0, t, sv[t], qa, qb2);
              lmax = bt > lmax ? bt : lmax;  // (NaN: skipped)
            }
          }
          // the k-th largest lane maximum: bitonic sort of the 64 values, descending
          double v = lmax;
#pragma unroll
          for (int sz = 2; sz <= 64; sz <<= 1)
#pragma unroll
            for (int st2 = sz >> 1; st2 > 0; st2 >>= 1) {
              const double o = __shfl_xor(v, st2);
              const bool keep_max = ((lane & sz) == 0) == ((lane & st2) == 0);
              v = keep_max ? (o > v ? o : v) : (o < v ? o : v);
            }
          t_hi = __shfl(v, k - 1);
          seeded = true;
          // pass A: score every column with b >= t_hi (16 at a time), insert
#pragma unroll 1
          for (int c0 = 0; c0 < a.width; c0 += 512) {
            double sv[8];
            read8(c0, sv);
            const uint32_t qa = qsel(c0 >> 8), qb2 = qsel((c0 >> 8) + 1);
            uint32_t mask = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {  // (excluded columns: b = -inf or NaN, never taken)
              const double bt = bound(c0, t, sv[t], qa, qb2);
              mask |= bt >= t_hi && bt > neg_inf<double>() ? 1u << t : 0u;
            }
            while (__ballot(mask != 0)) {
              const bool has = mask != 0;
              const int t = has ? __ffs(mask) - 1 : 0;
              mask &= mask - 1;
              double sx = sv[0];
#pragma unroll
              for (int x = 1; x < 8; ++x) sx = t == x ? sv[x] : sx;
              const int j = c0 + 256 * (t >> 2) + 4 * lane + (t & 3);
              const double f = has ? sx * s_rb[has ? j : 0] : -1.0;
              const uint64_t bal = __ballot(has);
              const int nb = __popcll(bal);
              if (ncand + nb > kOvfList) flush();
              if (has) {
                const int p = ncand + __popcll(bal & lanemask_lt());
                cq_f[p] = f;
                cq_j[p] = (uint32_t)j;
              }
              ncand += nb;
              if (ncand >= 16) flush();
            }
          }
          if (ncand) flush();
        }
      }
      const double2 zero2{0.0, 0.0};
      for (int c0 = 0; c0 < a.width; c0 += 512) {
        const uint32_t qa = qr[0], qb2 = qr[1];
#pragma unroll
        for (int k = 0; k + 2 < kQPre; ++k) qr[k] = qr[k + 2];
        qr[kQPre - 2] = 0xFFFFFFFFu;  // (columns past 256 kQPre: the chunk bound alone)
        qr[kQPre - 1] = 0xFFFFFFFFu;
        double sv[8];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            const int j = c0 + 256 * hh + 4 * lane + 2 * pp;
            // (acc holds whole 512-column steps: no bounds branch, the 4 reads go out together)
            const double2 x = *reinterpret_cast<const double2 *>(acc + j);
            *reinterpret_cast<double2 *>(acc + j) = zero2;
            sv[4 * hh + 2 * pp] = x.x;
            sv[4 * hh + 2 * pp + 1] = x.y;
          }
        if (c0 + 512 > a.width) {  // the last step of a partial tile: columns past the width
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int j = c0 + 256 * (t >> 2) + 4 * lane + (t & 3);
            if (j >= a.width) sv[t] = neg_inf<double>();
          }
        }
        double sc0 = 0.0, sc1 = 0.0;
        if constexpr (D > 0) {
          sc0 = __shfl(sc_v, ((c0 + 4 * lane) >> 6) & 63);
          sc1 = __shfl(sc_v, ((c0 + 256 + 4 * lane) >> 6) & 63);
        }
        uint32_t mask = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          bool pre;
          if constexpr (D > 0) {
            const uint32_t qq = t < 4 ? qa : qb2;
            const double qv = (double)((qq >> (8 * (t & 3))) & 0xFFu);
            const double b = sv[t] * qv * (t < 4 ? sc0 : sc1);
            // (seeded: pass A scored the columns with b >= t_hi, b > -inf)
            pre = b > tau && !(seeded && b >= t_hi && b > neg_inf<double>());
          } else {
            pre = sv[t] > thr_s;
          }
          mask |= pre ? 1u << t : 0u;
        }
        while (__ballot(mask != 0)) {
          const bool has = mask != 0;
          const int t = has ? __ffs(mask) - 1 : 0;
          mask &= mask - 1;
          double s = sv[0];
#pragma unroll
          for (int x = 1; x < 8; ++x) s = t == x ? sv[x] : s;
          const int j = c0 + 256 * (t >> 2) + 4 * lane + (t & 3);
          const double f = has ? s * s_rb[has ? j : 0] : -1.0;
          if constexpr (D > 0) {
            const uint32_t qq = t < 4 ? qa : qb2;
            const double bq = (double)((qq >> (8 * (t & 3))) & 0xFFu) *
                              __shfl(bq_v, (j >> 6) & 63);
            const bool cand = has && bq * f > tau;
            const uint64_t bal = __ballot(cand);
            if (bal) {
              const int nb = __popcll(bal);
              if (ncand + nb > kOvfList) flush();  // (nb <= 64 <= kOvfList)
              if (cand) {
                const int p = ncand + __popcll(bal & lanemask_lt());
                cq_f[p] = f;
                cq_j[p] = (uint32_t)j;
              }
              ncand += nb;
              if (ncand >= 16 || tau == neg_inf<double>()) flush();
            }
          } else {
            uint64_t bal = __ballot(has && before(f, a.item_begin + j, tau, tau_id));
            while (bal) {
              const int l = __ffsll((long long)bal) - 1;
              bal &= bal - 1;
              insert1(__shfl(f, l), a.item_begin + __shfl(j, l));
            }
            thr_s = tau / rscale;
          }
        }
      }
      if (ncand) flush();
      if (dirty) {
        if (lane < k) {
          a.io_val[u * k + lane] = I0 != kPadId ? L0 : neg_inf<double>();
          a.io_idx[u * k + lane] = I0 != kPadId ? I0 : -1;
        }
        if (kTwo && 64 + lane < k) {
          a.io_val[u * k + 64 + lane] = I1 != kPadId ? L1 : neg_inf<double>();
          a.io_idx[u * k + 64 + lane] = I1 != kPadId ? I1 : -1;
        }
      }
      wave_sync();
    }
  };

  // ---- the pipeline: c (decoded now; lines in wc), d (lines in flight in wd), n2 (ids in
  // flight in it2). Two register sets (lines, ra, user state) alternate between c and d. Every
  // step issues the same loads (empty batches read the zero line / 0 bytes), so the wait
  // before a decode counts the two younger batches' loads instead of draining them.
  int32_t it2[Q];
  uint4 w0[Q], w1[Q];
  double ra0[Q], ra1[Q];
  UState s0, s1;
  Batch c = new_user();
  pre_load();
  load_ids(c, it2);
  load_rows(c, it2, w0, ra0);
  load_state(c, s0);
  Batch d = next_batch(c);
  pre_load();
  load_ids(d, it2);
  load_rows(d, it2, w1, ra1);
  load_state(d, s1);
  Batch n2 = next_batch(d);
  pre_load();
  load_ids(n2, it2);
  auto step = [&](uint4 (&wc)[Q], double (&rc)[Q], UState &sc) __attribute__((always_inline)) {
    // c's user state (loaded two steps ago) is taken here, where the wait for it counts the
    // younger batches' loads; at the finish, behind the exclusion loop's load, the compiler
    // would drain every load in flight
    if constexpr (MODE == MODE_TOPK) {
      asm volatile("" : "+v"(sc.lid0), "+v"(sc.lv0), "+v"(sc.xw));
      if constexpr (kTwo) asm volatile("" : "+v"(sc.lid1), "+v"(sc.lv1));
      if constexpr (D > 0) {
        asm volatile("" : "+v"(sc.gb));
#pragma unroll
        for (int kk = 0; kk < kQPre; ++kk) asm volatile("" : "+v"(sc.q[kk]));
      }
    }
    decode(c, wc, rc);
    if (c.r1 >= c.e) finish_user(c, sc);
    // batch t+2 into the freed registers (issued before the scan instead: 1.5 % slower)
    load_rows(n2, it2, wc, rc);
    load_state(n2, sc);
    const Batch n3 = next_batch(n2);
    pre_load();
    load_ids(n3, it2);
    c = d;
    d = n2;
    n2 = n3;
    return c.u < n_users;
  };
  for (;;) {
    if (!step(w0, ra0, s0)) break;
    if (!step(w1, ra1, s1)) break;
  }
}

#if LG_REFERENCE_PATHS
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
  // 26.4 vs 16.7 ms on the first.
  if (M == 1 && k <= 24 && !first) {
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

#endif  // LG_REFERENCE_PATHS

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

extern "C" int lg_hybrid_recip_f64(const double *k_item, int64_t n_items, double lambda,
                                   double *ra, double *rb, lg_stream_t stream) {
  LG_REQUIRE(k_item && ra && rb && n_items >= 0, "lg_hybrid_recip_f64: bad arguments");
  if (n_items == 0) return LG_OK;
  k_hybrid_recip<<<dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0,
                   (hipStream_t)stream>>>(k_item, n_items, lambda, ra, rb);
  return launch_status("lg_hybrid_recip_f64");
}

extern "C" int lg_inv_degree_f64(const int64_t *rowptr, int64_t n_rows, double *inv,
                                 lg_stream_t stream) {
  LG_REQUIRE(rowptr && inv && n_rows >= 0, "lg_inv_degree_f64: bad arguments");
  if (n_rows == 0) return LG_OK;
  k_inv_degree<<<dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, (hipStream_t)stream>>>(
      rowptr, n_rows, inv);
  return launch_status("lg_inv_degree_f64");
}

#if LG_REFERENCE_PATHS
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

extern "C" size_t lg_spread_tile_rows_ws_bytes(int64_t n_items) {
  return (size_t)(n_items + 1) * sizeof(int64_t);  // hub count + hub row list
}

extern "C" int lg_spread_tile_rows_f64(const int64_t *item_rowptr, const int32_t *item_users,
                                       const int32_t *user_items, const uint16_t *user_cls,
                                       const double *inv_deg, int64_t n_items,
                                       const int64_t *cur, const uint16_t *count,
                                       int32_t item_begin, int32_t tile, const int64_t *bound,
                                       int64_t vthr, const int64_t *ovf_ptr, void *lines,
                                       void *ovf, int32_t *row_len, void *ws, size_t ws_bytes,
                                       lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && user_cls && inv_deg && cur && count && bound && ovf_ptr && lines &&
                 ovf && n_items >= 0 && vthr >= kLineSlots,
             "lg_spread_tile_rows_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && item_begin >= 0,
             "lg_spread_tile_rows_f64: tile %d not in [1, 8192]", tile);
  if (n_items == 0) return LG_OK;
  const size_t need = lg_spread_tile_rows_ws_bytes(n_items);
  if (!ws || ws_bytes < need) {
    set_error("lg_spread_tile_rows_f64: workspace %zu < %zu bytes", ws_bytes, need);
    return LG_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  int64_t *n_hub = (int64_t *)ws;
  int64_t *hub_rows = n_hub + 1;
  if (hipMemsetAsync(n_hub, 0, sizeof(int64_t), s) != hipSuccess) {
    set_error("lg_spread_tile_rows_f64: hipMemsetAsync failed");
    return LG_ERR_HIP;
  }
  k_tile_rows<<<dim3((unsigned)((n_items + 3) / 4)), dim3(256), 0, s>>>(
      item_rowptr, item_users, user_items, user_cls, n_items, cur, count, item_begin, bound, vthr,
      ovf_ptr, (uint32_t *)lines, (uint32_t *)ovf, row_len);
  k_hub_list<<<dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, s>>>(
      bound, n_items, vthr, (unsigned long long *)n_hub, hub_rows);
  k_tile_rows_hub<<<dim3(1024), dim3(256), (size_t)tile * sizeof(double), s>>>(
      hub_rows, n_hub, item_rowptr, item_users, user_items, inv_deg, cur, count, item_begin, tile,
      ovf_ptr, (uint32_t *)lines, (uint32_t *)ovf, row_len);
  return launch_status("lg_spread_tile_rows_f64");
}

#endif  // LG_REFERENCE_PATHS

extern "C" int lg_spread_group_cursor(const int64_t *user_rowptr, const int32_t *user_items,
                                      const uint16_t *user_cls, int64_t n_users,
                                      int32_t group_begin, int32_t tile, int32_t n_tiles,
                                      int32_t stop, const int64_t *cur, int64_t *end,
                                      uint16_t *counts, void *rec, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && user_cls && cur && end && counts && rec && n_users >= 0 &&
                 cur != end && group_begin >= 0 && stop > group_begin,
             "lg_spread_group_cursor: bad arguments");
  LG_REQUIRE(((uintptr_t)rec & 15) == 0, "lg_spread_group_cursor: rec not 16-byte aligned");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && n_tiles >= 1 && n_tiles <= kGroupMax &&
                 (n_tiles <= kGroupWide || tile <= 4096),
             "lg_spread_group_cursor: tile %d / n_tiles %d (groups of more than %d tiles need tile <= 4096)",
             tile, n_tiles, kGroupWide);
  LG_REQUIRE(((uintptr_t)counts & 15) == 0, "lg_spread_group_cursor: counts not 16-byte aligned");
  if (n_users == 0) return LG_OK;
  k_group_cursor<<<dim3((unsigned)((n_users + 255) / 256)), dim3(256), 0,
                   (hipStream_t)stream>>>(user_rowptr, user_items, user_cls, n_users,
                                          group_begin, tile, n_tiles, stop, cur, end,
                                          (uint4 *)counts, (uint4 *)rec);
  return launch_status("lg_spread_group_cursor");
}

extern "C" int lg_spread_group_bound(const int64_t *item_rowptr, const int32_t *item_users,
                                     int64_t n_items, const uint16_t *counts, int32_t n_tiles,
                                     int64_t *bound, lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && counts && bound && n_items >= 0 && n_tiles >= 1 &&
                 n_tiles <= kGroupMax && ((uintptr_t)counts & 15) == 0,
             "lg_spread_group_bound: bad arguments");
  if (n_items == 0) return LG_OK;
  k_group_bound<<<dim3((unsigned)((n_items + 15) / 16)), dim3(256), 0, (hipStream_t)stream>>>(
      item_rowptr, item_users, n_items, (const uint4 *)counts, n_tiles, bound);
  return launch_status("lg_spread_group_bound");
}

extern "C" int lg_spread_group_units(const int64_t *bound, int64_t n_items, int32_t group_begin,
                                     int32_t tile, int32_t n_tiles, int32_t stop, int64_t vthr,
                                     int64_t *units, lg_stream_t stream) {
  LG_REQUIRE(bound && units && n_items >= 0 && group_begin >= 0 && stop > group_begin &&
                 vthr >= kLineSlots,
             "lg_spread_group_units: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && n_tiles >= 1 && n_tiles <= kGroupMax &&
                 (n_tiles <= kGroupWide || tile <= 4096),
             "lg_spread_group_units: tile %d / n_tiles %d (groups of more than %d tiles need tile <= 4096)",
             tile, n_tiles, kGroupWide);
  const int64_t n = n_items * n_tiles;
  if (n == 0) return LG_OK;
  k_group_units<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream>>>(
      bound, n_items, group_begin, tile, n_tiles, stop, vthr, units);
  return launch_status("lg_spread_group_units");
}

extern "C" size_t lg_spread_group_rows_ws_bytes(int64_t n_items, int32_t n_tiles) {
  return (size_t)(n_items * (n_tiles > 0 ? n_tiles : 1) + 1) * sizeof(int64_t);
}

extern "C" int lg_spread_group_rows_f64(
    const int64_t *item_rowptr, const int32_t *item_users, const int32_t *user_items,
    const double *inv_deg, int64_t n_items, const int64_t *cur, const uint16_t *counts,
    const void *rec, int32_t group_begin, int32_t tile, int32_t n_tiles, int32_t stop,
    const int64_t *bound, int64_t vthr, const int64_t *units_incl, void *lines, void *ovf,
    int32_t *row_len, void *ws, size_t ws_bytes, lg_stream_t stream) {
  LG_REQUIRE(item_rowptr && rec && inv_deg && cur && counts && bound && units_incl &&
                 lines && ovf && n_items >= 0 && group_begin >= 0 && stop > group_begin,
             "lg_spread_group_rows_f64: bad arguments");
  LG_REQUIRE(vthr >= kLineSlots && vthr < 65536,
             "lg_spread_group_rows_f64: vthr %lld not in [31, 65535]", (long long)vthr);
  LG_REQUIRE(tile >= 1 && tile <= 8192 && n_tiles >= 1 && n_tiles <= kGroupMax &&
                 (n_tiles <= kGroupWide || tile <= 4096),
             "lg_spread_group_rows_f64: tile %d / n_tiles %d (groups of more than %d tiles need tile <= 4096)",
             tile, n_tiles, kGroupWide);
  LG_REQUIRE(((uintptr_t)counts & 15) == 0, "lg_spread_group_rows_f64: counts not 16-byte aligned");
  if (n_items == 0) return LG_OK;
  const size_t need = lg_spread_group_rows_ws_bytes(n_items, n_tiles);
  if (!ws || ws_bytes < need) {
    set_error("lg_spread_group_rows_f64: workspace %zu < %zu bytes", ws_bytes, need);
    return LG_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  int64_t *n_hub = (int64_t *)ws;
  int64_t *hub_rows = n_hub + 1;
  if (hipMemsetAsync(n_hub, 0, sizeof(int64_t), s) != hipSuccess) {
    set_error("lg_spread_group_rows_f64: hipMemsetAsync failed");
    return LG_ERR_HIP;
  }
  const uint4 *c4 = (const uint4 *)counts;
  k_group_rows<<<dim3((unsigned)((n_items + 3) / 4)), dim3(256), 0, s>>>(
      item_rowptr, item_users, user_items, n_items, c4, (const uint4 *)rec, group_begin, tile,
      n_tiles, stop, bound, vthr, units_incl, (uint32_t *)lines, (uint32_t *)ovf, row_len);
  const int64_t nflat = n_items * n_tiles;
  k_hub_list<<<dim3((unsigned)((nflat + 255) / 256)), dim3(256), 0, s>>>(
      bound, nflat, vthr, (unsigned long long *)n_hub, hub_rows);
  const int hub_waves = tile <= 4096 ? 4 : 2;  // (LDS: one tile of doubles per wave)
  k_group_rows_hub<<<dim3(1024), dim3(64 * hub_waves), (size_t)hub_waves * tile * sizeof(double),
                     s>>>(
      hub_rows, n_hub, item_rowptr, item_users, user_items, inv_deg, n_items, cur, c4,
      group_begin, tile, stop, bound, vthr, units_incl, (uint32_t *)lines, (uint32_t *)ovf,
      row_len);
  return launch_status("lg_spread_group_rows_f64");
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
template <int MODE, int D, int M>
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
  bool seeded = false;
  if constexpr (D > 0 && M <= 2) {  // (the seeded finish: k <= 64 with a G factor)
    if (a.first) {
      k_tile_walk<MODE, D, M, true><<<dim3(blocks), dim3(64 * nw), lds, s>>>(a);
      seeded = true;
    }
  }
  if (!seeded) k_tile_walk<MODE, D, M><<<dim3(blocks), dim3(64 * nw), lds, s>>>(a);
  return LG_OK;
}

#if LG_REFERENCE_PATHS
extern "C" int lg_spread_tile_resource_f64(const int64_t *user_rowptr,
                                           const int32_t *user_items, const double *ra_edge,
                                           int64_t n_users, const void *lines, const void *ovf,
                                           int32_t null_row,
                                           const double *rbeta, const double *inv_cls,
                                           int32_t item_begin, int32_t tile, int32_t width,
                                           double *F, int64_t ldf, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && user_items && ra_edge && lines && ovf && rbeta && inv_cls && F &&
                 n_users >= 0 && ldf >= tile,
             "lg_spread_tile_resource_f64: bad arguments");
  LG_REQUIRE(tile >= 1 && tile <= 8192 && width >= 1 && width <= tile,
             "lg_spread_tile_resource_f64: tile %d / width %d", tile, width);
  LG_REQUIRE(null_row >= 0 && null_row < (1 << 25) - 1,
             "tile walk: %d items exceed the 32-bit line offsets", null_row);
  if (n_users == 0) return LG_OK;
  WalkArgs a{};
  a.user_rowptr = user_rowptr;
  a.user_items = user_items;
  a.ra_edge = ra_edge;
  a.n_users = n_users;
  a.lines = (const uint4 *)lines;
  a.ovf = (const uint4 *)ovf;
  a.null_row = null_row;
  a.item_begin = item_begin;
  a.tile = tile;
  a.width = width;
  a.rbeta = rbeta;
  a.g_inv = inv_cls;
  a.F = F;
  a.ldf = ldf;
  const int st = launch_walk<MODE_F, 0, 1>(a, (hipStream_t)stream);
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

#endif  // LG_REFERENCE_PATHS

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
  return M == 2 ? launch_walk<MODE_TOPK, D, 2>(a, s) : launch_walk<MODE_TOPK, D, 4>(a, s);
}

extern "C" int lg_spread_tile_resource_topk_f64(
    const int64_t *user_rowptr, const int32_t *user_items, const double *ra_edge,
    int64_t n_users, const void *lines, const void *ovf, int32_t null_row, const double *rbeta,
    const double *inv_cls, int32_t item_begin, int32_t tile, int32_t width, const float *eu,
    const float *ei, int32_t dim, const float *gb, int32_t n_chunks, const uint8_t *qb,
    int32_t qstride, const int64_t *ex_rowptr,
    const int32_t *ex_col, int64_t *ex_cur, int32_t k, int32_t first, double *io_val,
    int64_t *io_idx, int64_t n_positions, int64_t n_ex_positions, lg_stream_t stream) {
  LG_REQUIRE(user_rowptr && user_items && ra_edge && lines && ovf && rbeta && inv_cls &&
                 io_val && io_idx && n_users >= 0 && n_users < 0x7fffffff && item_begin >= 0,
             "lg_spread_tile_resource_topk_f64: bad arguments");
  // (the walk's stream positions are 32-bit)
  LG_REQUIRE(n_positions >= 0 && n_positions < 0x7fffffff && n_ex_positions >= 0 &&
                 n_ex_positions < 0x7fffffff,
             "lg_spread_tile_resource_topk_f64: %lld interactions / %lld exclusions exceed the "
             "walk's 32-bit positions", (long long)n_positions, (long long)n_ex_positions);
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
  LG_REQUIRE(!qb || (eu && qstride >= (width + 255) / 256 * 256),
             "lg_spread_tile_resource_topk_f64: qb needs eu and qstride >= width rounded to 256");
  LG_REQUIRE(!eu || n_chunks <= 64,
             "lg_spread_tile_resource_topk_f64: a G factor needs width <= 4096 (one chunk "
             "bound per lane), got %d", width);
  LG_REQUIRE(!ex_rowptr == !ex_col && !ex_rowptr == !ex_cur,
             "lg_spread_tile_resource_topk_f64: ex_rowptr/ex_col/ex_cur go together");
  LG_REQUIRE(null_row >= 0 && null_row < (1 << 25) - 1,
             "tile walk: %d items exceed the 32-bit line offsets", null_row);
  if (n_users == 0) return LG_OK;
  WalkArgs a{};
  a.user_rowptr = user_rowptr;
  a.user_items = user_items;
  a.ra_edge = ra_edge;
  a.n_users = n_users;
  a.lines = (const uint4 *)lines;
  a.ovf = (const uint4 *)ovf;
  a.null_row = null_row;
  a.item_begin = item_begin;
  a.tile = tile;
  a.width = width;
  a.rbeta = rbeta;
  a.g_inv = inv_cls;
  a.eu = eu;
  a.ei = ei;
  a.gb = gb;
  a.nch = n_chunks;
  a.qb = qb;
  a.qstride = qstride;
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

