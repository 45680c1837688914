// K1: one LightGCN propagation layer as a CSR row-gather SpMM, gfx950.
//
// Replaces PyG 2.6.1 MessagePassing.propagate at model/LightGCN/model.py:62 (and
// LightGCNOpti/model.py:74):  x_j = x.index_select(0, row)  [nnz, d] materialised;
// msg = norm.view(-1,1) * x_j  (message, :84);  out = zeros.scatter_add_(0, col, msg).
// Here every destination row is owned by one wave, the nnz x d message tensor never
// exists, the edge weight dis[s]*dis[g] (gcn_norm) is streamed per entry or recomputed,
// and the running layer sum of torch.stack(...).mean(1) (:66-69) is fused into the
// epilogue.
//
// Layout / mapping (HBM-bound gather):
//   - embedding rows are fp32 [N, D]; a row is D*4 bytes = LPR lanes x 16 B (float4).
//   - one wave64 per destination row; the wave's 64/LPR lane groups take interleaved
//     edges (group gi takes edges gi, gi+G, gi+2G, ... of the row) so each wave-level
//     load instruction fetches G whole source rows (1 KiB) fully coalesced.
//   - edge ids and weights are fetched 64 at a time (coalesced non-temporal loads of src
//     and of the precomputed gcn_norm weights w, or a gather of dis when w is NULL) and
//     broadcast to the groups with ds_bpermute (__shfl). Streaming w costs 4 B/edge but
//     removes a random 4-byte gather per edge from an 8 MB table that does not fit one
//     XCD's L2 (each miss moves a whole line).
//   - outputs are written with non-temporal stores so they do not evict the gathered
//     table from the Infinity Cache.
//   - UNROLL edge slots per group are in flight before the accumulate.
//   - group partial sums are combined with an xor butterfly; deterministic order.
//
// Power-law rows: a row longer than `long_threshold` would serialise on one wave (a
// 10M-edge hub = 2.4 GB through one wave). The main kernel skips such rows; the caller
// cuts them into segments, k_spmm_segments gives each segment its own wave (partial sums
// in a workspace) and k_spmm_long_reduce adds a row's segments in order and runs the same
// epilogue. Still atomic-free and bitwise reproducible.
//
// Sparse inputs (the backward pass: dL/d(e_final) is non-zero only on the mini-batch's
// rows, and one layer later only on their neighbours): lg_spmm_layer_live_f32 takes a
// per-source-node byte mask and skips the 4*D-byte gather of rows marked dead (their
// contribution w*0 = 0 is added as a register zero, so the sums are the unmasked kernel's).
// The edge ids and weights are still streamed: 8 B/edge instead of 8 + 4*D.
#include "common.h"

namespace lg {

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void nt_store4(float *p, const float4 &v) {
  const f32x4v t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4v *>(p));
}

__device__ __forceinline__ void add4(float4 &a, const float4 &b) {
  a.x = __fadd_rn(a.x, b.x);
  a.y = __fadd_rn(a.y, b.y);
  a.z = __fadd_rn(a.z, b.z);
  a.w = __fadd_rn(a.w, b.w);
}

// sum over entries [beg, end) of w_e * x[src_e] for this lane's float4 slice, combined over
// the wave's lane groups (every group ends with the full sum).
template <int D, int UNROLL, bool LIVE = false>
__device__ __forceinline__ float4 gather_sum(int64_t beg, int64_t end,
                                             const int32_t *__restrict__ src,
                                             const float *__restrict__ w,
                                             const float *__restrict__ dis, float dg,
                                             const float *__restrict__ x,
                                             const uint8_t *__restrict__ live = nullptr) {
  constexpr int LPR = D / 4;
  constexpr int G = 64 / LPR;
  const int lane = lane_id();
  const int gi = lane / LPR;
  const int li = lane % LPR;
  const float4 *__restrict__ x4 = reinterpret_cast<const float4 *>(x);
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  // LIVE: the next 64 edges' ids/weights are loaded while this chunk's mask bytes are in
  // flight (the chain edge id -> mask byte bounds the layer, not bandwidth)
  int nx_s = 0;
  float nx_w = 0.f;
  if constexpr (LIVE) {
    if (beg + lane < end) {
      nx_s = __builtin_nontemporal_load(src + beg + lane);
      nx_w = w ? __builtin_nontemporal_load(w + beg + lane) : __fmul_rn(dis[nx_s], dg);
    }
  }
  for (int64_t cb = beg; cb < end; cb += 64) {
    const int n = (int)((end - cb) < 64 ? (end - cb) : 64);
    int my_s = 0;
    float my_w = 0.f;
    int my_l = 0;  // LIVE: this lane's edge source row is non-zero (one load per 64 edges)
    if constexpr (LIVE) {
      my_s = nx_s;
      my_w = nx_w;
      if (lane < n) my_l = live[my_s];
      nx_s = 0;
      nx_w = 0.f;
      if (cb + 64 + lane < end) {
        nx_s = __builtin_nontemporal_load(src + cb + 64 + lane);
        nx_w = w ? __builtin_nontemporal_load(w + cb + 64 + lane) : __fmul_rn(dis[nx_s], dg);
      }
      // no live source in the chunk: its terms are all +0 and sum is never -0, so
      // skipping them leaves the sum bitwise unchanged
      if (__ballot(my_l) == 0) continue;
    } else if (lane < n) {
      my_s = __builtin_nontemporal_load(src + cb + lane);
      // PyG: deg_inv_sqrt[row] * edge_weight(=1) * deg_inv_sqrt[col]; row = source.
      my_w = w ? __builtin_nontemporal_load(w + cb + lane) : __fmul_rn(dis[my_s], dg);
    }
    for (int j0 = 0; j0 < n; j0 += UNROLL * G) {
      int s[UNROLL];
      float wv[UNROLL];
      float4 xv[UNROLL];
      int lv[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int jj = j0 + u * G + gi;
        s[u] = __shfl(my_s, jj & 63);
        wv[u] = __shfl(my_w, jj & 63);
        if constexpr (LIVE) lv[u] = __shfl(my_l, jj & 63);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int jj = j0 + u * G + gi;
        if constexpr (LIVE) {
          xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (lv[u]) xv[u] = x4[(int64_t)s[u] * LPR + li];  // 0 for lanes >= n
        } else {
          if (jj < n) xv[u] = x4[(int64_t)s[u] * LPR + li];
        }
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int jj = j0 + u * G + gi;
        if (jj < n) {
          // message = norm * x_j, then scatter-add: a rounded product, then a rounded sum.
          sum.x = __fadd_rn(sum.x, __fmul_rn(wv[u], xv[u].x));
          sum.y = __fadd_rn(sum.y, __fmul_rn(wv[u], xv[u].y));
          sum.z = __fadd_rn(sum.z, __fmul_rn(wv[u], xv[u].z));
          sum.w = __fadd_rn(sum.w, __fmul_rn(wv[u], xv[u].w));
        }
      }
    }
  }
#pragma unroll
  for (int off = LPR; off < 64; off <<= 1) {
    sum.x = __fadd_rn(sum.x, __shfl_xor(sum.x, off));
    sum.y = __fadd_rn(sum.y, __shfl_xor(sum.y, off));
    sum.z = __fadd_rn(sum.z, __shfl_xor(sum.z, off));
    sum.w = __fadd_rn(sum.w, __shfl_xor(sum.w, off));
  }
  return sum;
}

// y / layer-mean epilogue for node g, float4 slice li (called by lane group 0 only).
template <int D>
__device__ __forceinline__ void epilogue(int64_t g, int li, const float4 &sum,
                                         float *__restrict__ y, const float *__restrict__ x0,
                                         float *acc, float *out, int mode, float denom) {
  constexpr int LPR = D / 4;
  const int64_t o = g * LPR + li;
  if (y) nt_store4(y + o * 4, sum);
  float4 a;
  switch (mode) {
    case LG_ACC_FIRST:
    case LG_ACC_ONLY: a = reinterpret_cast<const float4 *>(x0)[o]; break;
    case LG_ACC_MID:
    case LG_ACC_LAST: a = reinterpret_cast<const float4 *>(acc)[o]; break;
    default: return;
  }
  add4(a, sum);
  if (mode == LG_ACC_LAST || mode == LG_ACC_ONLY) {
    a.x = __fdiv_rn(a.x, denom);
    a.y = __fdiv_rn(a.y, denom);
    a.z = __fdiv_rn(a.z, denom);
    a.w = __fdiv_rn(a.w, denom);
    nt_store4(out + o * 4, a);
  } else {
    nt_store4(acc + o * 4, a);
  }
}

template <int D, int UNROLL, bool LIVE>
__global__ __launch_bounds__(256) void k_spmm_layer(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ src,
    const float *__restrict__ dis, const float *__restrict__ w, const float *__restrict__ x,
    float *__restrict__ y, const float *__restrict__ x0, float *acc, float *out,
    int64_t n_rows, int64_t row_offset, int mode, float denom, int64_t long_threshold,
    const uint8_t *__restrict__ live) {
  constexpr int LPR = D / 4;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (r >= n_rows) return;  // wave-uniform
  const int64_t beg = rowptr[r];
  const int64_t end = rowptr[r + 1];
  if (end - beg > long_threshold) return;  // done by the segmented path
  const int64_t g = row_offset + r;
  const float4 sum = gather_sum<D, UNROLL, LIVE>(beg, end, src, w, dis, dis[g], x, live);
  const int lane = lane_id();
  if (lane / LPR != 0) return;
  epilogue<D>(g, lane % LPR, sum, y, x0, acc, out, mode, denom);
}

// Output-restricted layer (the BPR training forward: the loss reads the final embedding only
// at the mini-batch's rows, so layer L is needed only there, layer L-1 only there and at their
// neighbours, ...): rows whose byte in row_mask (per node) is 0 are not computed -- their y /
// acc / out rows are left as they are. One wave per 64 consecutive rows: the lanes read the
// rows' mask bytes and bounds, and the wave runs the marked rows one after the other through
// the unmasked kernel's gather_sum and epilogue, so every computed row is bitwise
// k_spmm_layer's.
template <int D, int UNROLL>
__global__ __launch_bounds__(256) void k_spmm_layer_rows(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ src,
    const float *__restrict__ dis, const float *__restrict__ w, const float *__restrict__ x,
    float *__restrict__ y, const float *__restrict__ x0, float *acc, float *out,
    int64_t n_rows, int64_t row_offset, int mode, float denom, int64_t long_threshold,
    const uint8_t *__restrict__ row_mask) {
  constexpr int LPR = D / 4;
  const int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 64;
  if (r0 >= n_rows) return;  // wave-uniform
  const int lane = lane_id();
  const int64_t r = r0 + lane;
  int64_t beg = 0, end = 0;
  bool want = false;
  if (r < n_rows && row_mask[row_offset + r]) {
    beg = rowptr[r];
    end = rowptr[r + 1];
    want = end - beg <= long_threshold;  // (longer rows: the segmented path)
  }
  uint64_t rows = __ballot(want);
  while (rows) {
    const int b = __builtin_ctzll(rows);
    rows &= rows - 1;
    const int64_t rb = __shfl(beg, b), re = __shfl(end, b);
    const int64_t g = row_offset + r0 + b;
    const float4 sum = gather_sum<D, UNROLL, false>(rb, re, src, w, dis, dis[g], x);
    if (lane / LPR == 0) epilogue<D>(g, lane % LPR, sum, y, x0, acc, out, mode, denom);
  }
}

// row_mask (per node): out[r] = 1 for every r with in[r] set and for every source of its
// edges (the rows the next-lower layer must produce for it); one wave per 64 rows, each
// marked row's edges 64 at a time. Byte stores of 1 only: concurrent duplicates are benign.
__global__ __launch_bounds__(256) void k_mark_neighbors(const int64_t *__restrict__ rowptr,
                                                        const int32_t *__restrict__ src,
                                                        int64_t n_rows,
                                                        const uint8_t *__restrict__ in,
                                                        uint8_t *__restrict__ out) {
  const int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 64;
  if (r0 >= n_rows) return;
  const int lane = lane_id();
  const int64_t r = r0 + lane;
  int64_t beg = 0, end = 0;
  const bool want = r < n_rows && in[r];
  if (want) {
    beg = rowptr[r];
    end = rowptr[r + 1];
    out[r] = 1;
  }
  uint64_t rows = __ballot(want);
  while (rows) {
    const int b = __builtin_ctzll(rows);
    rows &= rows - 1;
    const int64_t rb = __shfl(beg, b), re = __shfl(end, b);
    for (int64_t e = rb + lane; e < re; e += 64) out[src[e]] = 1;
  }
}

// one wave per segment: partial[s] = sum over [seg_beg[s], seg_end[s]) of w_e * x[src_e]
// (row_mask, optional: segments of unmarked rows are skipped)
template <int D, int UNROLL>
__global__ __launch_bounds__(256) void k_spmm_segments(
    const int64_t *__restrict__ seg_beg, const int64_t *__restrict__ seg_end,
    const int32_t *__restrict__ seg_node, const int32_t *__restrict__ src,
    const float *__restrict__ dis, const float *__restrict__ w, const float *__restrict__ x,
    float *__restrict__ partial, int64_t n_seg, const uint8_t *__restrict__ row_mask) {
  constexpr int LPR = D / 4;
  const int64_t sgi = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (sgi >= n_seg) return;
  if (row_mask && !row_mask[seg_node[sgi]]) return;
  const float4 sum = gather_sum<D, UNROLL>(seg_beg[sgi], seg_end[sgi], src, w, dis,
                                           dis[seg_node[sgi]], x);
  const int lane = lane_id();
  if (lane / LPR != 0) return;
  reinterpret_cast<float4 *>(partial)[sgi * LPR + lane % LPR] = sum;
}

// one wave per long row j: its segments [seg_ptr[j], seg_ptr[j+1]) summed in order.
template <int D>
__global__ __launch_bounds__(256) void k_spmm_long_reduce(
    const int32_t *__restrict__ long_node, const int64_t *__restrict__ seg_ptr,
    const float *__restrict__ partial, float *__restrict__ y, const float *__restrict__ x0,
    float *acc, float *out, int64_t n_long, int mode, float denom,
    const uint8_t *__restrict__ row_mask) {
  constexpr int LPR = D / 4;
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (j >= n_long) return;
  if (row_mask && !row_mask[long_node[j]]) return;
  const int lane = lane_id();
  if (lane / LPR != 0) return;  // one lane group sums the segments sequentially
  const int li = lane % LPR;
  const float4 *p4 = reinterpret_cast<const float4 *>(partial);
  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t s = seg_ptr[j]; s < seg_ptr[j + 1]; ++s) add4(sum, p4[s * LPR + li]);
  epilogue<D>(long_node[j], li, sum, y, x0, acc, out, mode, denom);
}

template <int D>
static void launch_spmm(const int64_t *rowptr, const int32_t *src, const float *dis,
                        const float *w, const float *x, float *y, const float *x0, float *acc,
                        float *out, int64_t n_rows, int64_t row_offset, int mode, float denom,
                        int64_t long_threshold, const uint8_t *live, hipStream_t stream,
                        const uint8_t *row_mask = nullptr) {
  constexpr int WPB = 4;  // waves (rows) per 256-thread block
  constexpr int UNROLL = (D <= 64) ? 4 : 8;
  const int64_t blocks = (n_rows + WPB - 1) / WPB;
  if (row_mask)  // (64 rows per wave)
    k_spmm_layer_rows<D, UNROLL><<<dim3((unsigned)((n_rows + 64 * WPB - 1) / (64 * WPB))),
                                   dim3(64 * WPB), 0, stream>>>(
        rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, mode, denom,
        long_threshold, row_mask);
  else if (live)
    k_spmm_layer<D, UNROLL, true><<<dim3((unsigned)blocks), dim3(64 * WPB), 0, stream>>>(
        rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, mode, denom,
        long_threshold, live);
  else
    k_spmm_layer<D, UNROLL, false><<<dim3((unsigned)blocks), dim3(64 * WPB), 0, stream>>>(
        rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, mode, denom,
        long_threshold, nullptr);
}

template <int D>
static void launch_long(const int64_t *seg_beg, const int64_t *seg_end,
                        const int32_t *seg_node, int64_t n_seg, const int32_t *long_node,
                        const int64_t *seg_ptr, int64_t n_long, const int32_t *src,
                        const float *dis, const float *w, const float *x, float *y,
                        const float *x0, float *acc, float *out, int mode, float denom,
                        float *partial, hipStream_t stream, const uint8_t *row_mask) {
  constexpr int UNROLL = (D <= 64) ? 4 : 8;
  if (n_seg > 0)
    k_spmm_segments<D, UNROLL><<<dim3((unsigned)((n_seg + 3) / 4)), dim3(256), 0, stream>>>(
        seg_beg, seg_end, seg_node, src, dis, w, x, partial, n_seg, row_mask);
  k_spmm_long_reduce<D><<<dim3((unsigned)((n_long + 3) / 4)), dim3(256), 0, stream>>>(
      long_node, seg_ptr, partial, y, x0, acc, out, n_long, mode, denom, row_mask);
}

static int check_modes(int acc_mode, const float *x0, const float *acc, const float *out,
                       float denom, const float *x, const float *y, const char *fn) {
  LG_REQUIRE(acc_mode >= LG_ACC_NONE && acc_mode <= LG_ACC_ONLY, "%s: bad acc_mode %d", fn,
             acc_mode);
  LG_REQUIRE(!(acc_mode == LG_ACC_FIRST || acc_mode == LG_ACC_ONLY) || x0,
             "%s: acc_mode needs x0", fn);
  LG_REQUIRE(!(acc_mode == LG_ACC_FIRST || acc_mode == LG_ACC_MID || acc_mode == LG_ACC_LAST) ||
                 acc,
             "%s: acc_mode needs acc", fn);
  LG_REQUIRE(!(acc_mode == LG_ACC_LAST || acc_mode == LG_ACC_ONLY) || (out && denom != 0.f),
             "%s: acc_mode needs out and a non-zero denom", fn);
  LG_REQUIRE(y != x || !y, "%s: y must not alias x (ping-pong the layer buffers)", fn);
  return LG_OK;
}

}  // namespace lg

using namespace lg;

static int spmm_layer(const int64_t *rowptr, const int32_t *src, const float *dis,
                      const float *w, const float *x, float *y, const float *x0, float *acc,
                      float *out, int64_t n_rows, int64_t row_offset, int32_t dim,
                      int32_t acc_mode, float denom, int64_t long_threshold,
                      const uint8_t *live, lg_stream_t stream, const char *fn,
                      const uint8_t *row_mask = nullptr) {
  LG_REQUIRE(rowptr && dis && x && n_rows >= 0 && row_offset >= 0,
             "%s: null pointer or negative size", fn);
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128 || dim == 256,
             "%s: dim %d not in {32,64,128,256}", fn, dim);
  const int st = check_modes(acc_mode, x0, acc, out, denom, x, y, fn);
  if (st != LG_OK) return st;
  if (n_rows == 0) return LG_OK;
  if (long_threshold <= 0) long_threshold = INT64_MAX;
  hipStream_t s = (hipStream_t)stream;
  switch (dim) {
    case 32: launch_spmm<32>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, long_threshold, live, s, row_mask); break;
    case 64: launch_spmm<64>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, long_threshold, live, s, row_mask); break;
    case 128: launch_spmm<128>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, long_threshold, live, s, row_mask); break;
    default: launch_spmm<256>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, long_threshold, live, s, row_mask); break;
  }
  return launch_status(fn);
}

extern "C" int lg_spmm_layer_f32(const int64_t *rowptr, const int32_t *src,
                                 const float *dis, const float *w, const float *x, float *y,
                                 const float *x0, float *acc, float *out, int64_t n_rows,
                                 int64_t row_offset, int32_t dim, int32_t acc_mode,
                                 float denom, int64_t long_threshold, lg_stream_t stream) {
  return spmm_layer(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, dim,
                    acc_mode, denom, long_threshold, nullptr, stream, "lg_spmm_layer_f32");
}

extern "C" int lg_spmm_layer_live_f32(const int64_t *rowptr, const int32_t *src,
                                      const float *dis, const float *w, const float *x,
                                      float *y, const float *x0, float *acc, float *out,
                                      int64_t n_rows, int64_t row_offset, int32_t dim,
                                      int32_t acc_mode, float denom, int64_t long_threshold,
                                      const uint8_t *live, lg_stream_t stream) {
  LG_REQUIRE(live, "lg_spmm_layer_live_f32: null live mask");
  return spmm_layer(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, dim,
                    acc_mode, denom, long_threshold, live, stream, "lg_spmm_layer_live_f32");
}

static int long_rows(const int64_t *seg_beg, const int64_t *seg_end, const int32_t *seg_node,
                     int64_t n_seg, const int32_t *long_node, const int64_t *seg_ptr,
                     int64_t n_long, const int32_t *src, const float *dis, const float *w,
                     const float *x, float *y, const float *x0, float *acc, float *out,
                     int32_t dim, int32_t acc_mode, float denom, float *partial,
                     const uint8_t *row_mask, lg_stream_t stream, const char *fn) {
  LG_REQUIRE(n_seg >= 0 && n_long >= 0, "%s: negative size", fn);
  if (n_long == 0) return LG_OK;
  LG_REQUIRE(seg_beg && seg_end && seg_node && long_node && seg_ptr && src && dis && x &&
                 partial,
             "%s: null pointer", fn);
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128 || dim == 256,
             "%s: dim %d not in {32,64,128,256}", fn, dim);
  const int st = check_modes(acc_mode, x0, acc, out, denom, x, y, fn);
  if (st != LG_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  switch (dim) {
    case 32: launch_long<32>(seg_beg, seg_end, seg_node, n_seg, long_node, seg_ptr, n_long, src, dis, w, x, y, x0, acc, out, acc_mode, denom, partial, s, row_mask); break;
    case 64: launch_long<64>(seg_beg, seg_end, seg_node, n_seg, long_node, seg_ptr, n_long, src, dis, w, x, y, x0, acc, out, acc_mode, denom, partial, s, row_mask); break;
    case 128: launch_long<128>(seg_beg, seg_end, seg_node, n_seg, long_node, seg_ptr, n_long, src, dis, w, x, y, x0, acc, out, acc_mode, denom, partial, s, row_mask); break;
    default: launch_long<256>(seg_beg, seg_end, seg_node, n_seg, long_node, seg_ptr, n_long, src, dis, w, x, y, x0, acc, out, acc_mode, denom, partial, s, row_mask); break;
  }
  return launch_status(fn);
}

extern "C" int lg_spmm_long_rows_f32(const int64_t *seg_beg, const int64_t *seg_end,
                                     const int32_t *seg_node, int64_t n_seg,
                                     const int32_t *long_node, const int64_t *seg_ptr,
                                     int64_t n_long, const int32_t *src, const float *dis,
                                     const float *w, const float *x, float *y,
                                     const float *x0, float *acc, float *out, int32_t dim,
                                     int32_t acc_mode, float denom, float *partial,
                                     lg_stream_t stream) {
  return long_rows(seg_beg, seg_end, seg_node, n_seg, long_node, seg_ptr, n_long, src, dis, w,
                   x, y, x0, acc, out, dim, acc_mode, denom, partial, nullptr, stream,
                   "lg_spmm_long_rows_f32");
}

extern "C" int lg_spmm_long_rows_masked_f32(
    const int64_t *seg_beg, const int64_t *seg_end, const int32_t *seg_node, int64_t n_seg,
    const int32_t *long_node, const int64_t *seg_ptr, int64_t n_long, const int32_t *src,
    const float *dis, const float *w, const float *x, float *y, const float *x0, float *acc,
    float *out, int32_t dim, int32_t acc_mode, float denom, float *partial,
    const uint8_t *row_mask, lg_stream_t stream) {
  LG_REQUIRE(row_mask, "lg_spmm_long_rows_masked_f32: null row mask");
  return long_rows(seg_beg, seg_end, seg_node, n_seg, long_node, seg_ptr, n_long, src, dis, w,
                   x, y, x0, acc, out, dim, acc_mode, denom, partial, row_mask, stream,
                   "lg_spmm_long_rows_masked_f32");
}

extern "C" int lg_spmm_layer_rows_f32(const int64_t *rowptr, const int32_t *src,
                                      const float *dis, const float *w, const float *x,
                                      float *y, const float *x0, float *acc, float *out,
                                      int64_t n_rows, int64_t row_offset, int32_t dim,
                                      int32_t acc_mode, float denom, int64_t long_threshold,
                                      const uint8_t *row_mask, lg_stream_t stream) {
  LG_REQUIRE(row_mask, "lg_spmm_layer_rows_f32: null row mask");
  return spmm_layer(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, dim,
                    acc_mode, denom, long_threshold, nullptr, stream, "lg_spmm_layer_rows_f32",
                    row_mask);
}

extern "C" int lg_mark_neighbors_u8(const int64_t *rowptr, const int32_t *src, int64_t n_rows,
                                    const uint8_t *in_mask, uint8_t *out_mask,
                                    lg_stream_t stream) {
  LG_REQUIRE(rowptr && src && in_mask && out_mask && n_rows >= 0 && in_mask != out_mask,
             "lg_mark_neighbors_u8: bad arguments");
  if (n_rows == 0) return LG_OK;
  k_mark_neighbors<<<dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream>>>(rowptr, src, n_rows, in_mask, out_mask);
  return launch_status("lg_mark_neighbors_u8");
}
