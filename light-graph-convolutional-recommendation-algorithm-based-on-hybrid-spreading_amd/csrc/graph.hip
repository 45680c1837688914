// Graph format + normalisation kernels (K0).
//
// Replaces, for the propagation input:
//   - utils/graph.py:22-35  convertEdgeIndexToAdjMatrix: a dense (U+I)^2 fp32 matrix turned
//     into a coalesced COO. Here the caller hands over entries sorted by target row and the
//     row pointer is found by binary search, one thread per row (no dense matrix).
//   - PyG 2.6.1 gcn_norm(add_self_loops=False) at model/LightGCN/model.py:53:
//       deg = scatter_add(ones, col); dis = deg^-1/2; dis[inf] = 0; w = dis[row]*dis[col].
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "common.h"

namespace lg {

static thread_local char g_err[512] = {0};

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return LG_ERR_HIP;
  }
  return LG_OK;
}

__global__ void k_rowptr_from_sorted(const int64_t *__restrict__ keys, int64_t nnz,
                                     int64_t n_rows, int64_t *__restrict__ rowptr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n_rows) return;
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (keys[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = lo;
}

__global__ void k_gcn_norm(const int64_t *__restrict__ rowptr, int64_t n,
                           float *__restrict__ dis) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // PyG sums fp32 ones; an integer count is exact up to 2^24 edges per node and equal to
  // the fp32 sum there. pow(-0.5) is computed as 1/sqrt in IEEE fp32 (correctly rounded
  // sqrt and division), inf (deg 0) -> 0.
  const float deg = (float)(rowptr[i + 1] - rowptr[i]);
  dis[i] = deg > 0.f ? __fdiv_rn(1.0f, __fsqrt_rn(deg)) : 0.f;
}

// One wave per row, lanes over the row's entries.
__global__ void k_gcn_edge_weight(const int64_t *__restrict__ rowptr,
                                  const int32_t *__restrict__ src,
                                  const float *__restrict__ dis, int64_t n_rows,
                                  int64_t row_offset, float *__restrict__ w) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (r >= n_rows) return;
  const float dg = dis[row_offset + r];
  for (int64_t e = rowptr[r] + lane_id(); e < rowptr[r + 1]; e += 64)
    w[e] = __fmul_rn(dis[src[e]], dg);
}

}  // namespace lg

using namespace lg;

extern "C" int lg_abi_version(void) { return LG_ABI_VERSION; }

extern "C" const char *lg_last_error(void) { return g_err; }

extern "C" int lg_csr_rowptr_from_sorted(const int64_t *keys, int64_t nnz, int64_t n_rows,
                                         int64_t *rowptr, lg_stream_t stream) {
  LG_REQUIRE(rowptr && n_rows >= 0 && nnz >= 0 && (nnz == 0 || keys),
             "lg_csr_rowptr_from_sorted: bad arguments");
  const int64_t n = n_rows + 1;
  const int bs = 256;
  k_rowptr_from_sorted<<<dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0,
                         (hipStream_t)stream>>>(keys, nnz, n_rows, rowptr);
  return launch_status("lg_csr_rowptr_from_sorted");
}

extern "C" int lg_gcn_norm_f32(const int64_t *rowptr, int64_t n_nodes, float *dis,
                               lg_stream_t stream) {
  LG_REQUIRE(rowptr && dis && n_nodes >= 0, "lg_gcn_norm_f32: bad arguments");
  if (n_nodes == 0) return LG_OK;
  const int bs = 256;
  k_gcn_norm<<<dim3((unsigned)((n_nodes + bs - 1) / bs)), dim3(bs), 0,
               (hipStream_t)stream>>>(rowptr, n_nodes, dis);
  return launch_status("lg_gcn_norm_f32");
}

extern "C" int lg_gcn_edge_weight_f32(const int64_t *rowptr, const int32_t *src,
                                      const float *dis, int64_t n_rows, int64_t row_offset,
                                      float *w, lg_stream_t stream) {
  LG_REQUIRE(rowptr && src && dis && w && n_rows >= 0 && row_offset >= 0,
             "lg_gcn_edge_weight_f32: bad arguments");
  if (n_rows == 0) return LG_OK;
  const int rows_per_block = 4;
  k_gcn_edge_weight<<<dim3((unsigned)((n_rows + rows_per_block - 1) / rows_per_block)),
                      dim3(64 * rows_per_block), 0, (hipStream_t)stream>>>(
      rowptr, src, dis, n_rows, row_offset, w);
  return launch_status("lg_gcn_edge_weight_f32");
}
