// K1: one LightGCN propagation layer as a CSR row-gather SpMM, gfx950.
//
// Replaces PyG 2.6.1 MessagePassing.propagate at model/LightGCN/model.py:62 (and
// LightGCNOpti/model.py:74):  x_j = x.index_select(0, row)  [nnz, d] materialised;
// msg = norm.view(-1,1) * x_j  (message, :84);  out = zeros.scatter_add_(0, col, msg).
// Here every destination row is owned by one wave, the nnz x d message tensor never
// exists, the edge weight dis[s]*dis[g] (gcn_norm) is streamed per entry or recomputed,
// and the running layer sum of torch.stack(...).mean(1) (:66-69) is fused into the epilogue.
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
#include "common.h"

namespace lg {

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void nt_store4(float *p, const float4 &v) {
  const f32x4v t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4v *>(p));
}

template <int D, int UNROLL>
__global__ __launch_bounds__(256) void k_spmm_layer(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ src,
    const float *__restrict__ dis, const float *__restrict__ w, const float *__restrict__ x,
    float *__restrict__ y,
    const float *__restrict__ x0, float *acc, float *out, int64_t n_rows,
    int64_t row_offset, int mode, float denom) {
  constexpr int LPR = D / 4;   // lanes per embedding row (float4 each)
  constexpr int G = 64 / LPR;  // rows gathered per wave-instruction
  const int lane = lane_id();
  const int gi = lane / LPR;
  const int li = lane % LPR;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (r >= n_rows) return;  // wave-uniform
  const int64_t g = row_offset + r;
  const int64_t beg = rowptr[r];
  const int64_t end = rowptr[r + 1];
  const float dg = dis[g];
  const float4 *__restrict__ x4 = reinterpret_cast<const float4 *>(x);

  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t cb = beg; cb < end; cb += 64) {
    const int n = (int)((end - cb) < 64 ? (end - cb) : 64);
    int my_s = 0;
    float my_w = 0.f;
    if (lane < n) {
      my_s = __builtin_nontemporal_load(src + cb + lane);
      // PyG: deg_inv_sqrt[row] * edge_weight(=1) * deg_inv_sqrt[col]; row = source.
      my_w = w ? __builtin_nontemporal_load(w + cb + lane) : __fmul_rn(dis[my_s], dg);
    }
    for (int j0 = 0; j0 < n; j0 += UNROLL * G) {
      int s[UNROLL];
      float wv[UNROLL];
      float4 xv[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int jj = j0 + u * G + gi;
        s[u] = __shfl(my_s, jj & 63);
        wv[u] = __shfl(my_w, jj & 63);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int jj = j0 + u * G + gi;
        if (jj < n) xv[u] = x4[(int64_t)s[u] * LPR + li];
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
  if (gi != 0) return;
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
  a.x = __fadd_rn(a.x, sum.x);
  a.y = __fadd_rn(a.y, sum.y);
  a.z = __fadd_rn(a.z, sum.z);
  a.w = __fadd_rn(a.w, sum.w);
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

template <int D>
static void launch_spmm(const int64_t *rowptr, const int32_t *src, const float *dis,
                        const float *w, const float *x, float *y, const float *x0, float *acc, float *out,
                        int64_t n_rows, int64_t row_offset, int mode, float denom,
                        hipStream_t stream) {
  constexpr int WPB = 4;  // waves (rows) per 256-thread block
  constexpr int UNROLL = (D <= 64) ? 4 : 8;
  const int64_t blocks = (n_rows + WPB - 1) / WPB;
  k_spmm_layer<D, UNROLL><<<dim3((unsigned)blocks), dim3(64 * WPB), 0, stream>>>(
      rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, mode, denom);
}

}  // namespace lg

using namespace lg;

extern "C" int lg_spmm_layer_f32(const int64_t *rowptr, const int32_t *src,
                                 const float *dis, const float *w, const float *x, float *y,
                                 const float *x0, float *acc, float *out, int64_t n_rows,
                                 int64_t row_offset, int32_t dim, int32_t acc_mode,
                                 float denom, lg_stream_t stream) {
  LG_REQUIRE(rowptr && dis && x && n_rows >= 0 && row_offset >= 0,
             "lg_spmm_layer_f32: null pointer or negative size");
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128 || dim == 256,
             "lg_spmm_layer_f32: dim %d not in {32,64,128,256}", dim);
  LG_REQUIRE(acc_mode >= LG_ACC_NONE && acc_mode <= LG_ACC_ONLY,
             "lg_spmm_layer_f32: bad acc_mode %d", acc_mode);
  LG_REQUIRE(!(acc_mode == LG_ACC_FIRST || acc_mode == LG_ACC_ONLY) || x0,
             "lg_spmm_layer_f32: acc_mode needs x0");
  LG_REQUIRE(!(acc_mode == LG_ACC_FIRST || acc_mode == LG_ACC_MID || acc_mode == LG_ACC_LAST) ||
                 acc,
             "lg_spmm_layer_f32: acc_mode needs acc");
  LG_REQUIRE(!(acc_mode == LG_ACC_LAST || acc_mode == LG_ACC_ONLY) || (out && denom != 0.f),
             "lg_spmm_layer_f32: acc_mode needs out and a non-zero denom");
  LG_REQUIRE(y != x, "lg_spmm_layer_f32: y must not alias x (ping-pong the layer buffers)");
  if (n_rows == 0) return LG_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (dim) {
    case 32: launch_spmm<32>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, s); break;
    case 64: launch_spmm<64>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, s); break;
    case 128: launch_spmm<128>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, s); break;
    default: launch_spmm<256>(rowptr, src, dis, w, x, y, x0, acc, out, n_rows, row_offset, acc_mode, denom, s); break;
  }
  return launch_status("lg_spmm_layer_f32");
}
