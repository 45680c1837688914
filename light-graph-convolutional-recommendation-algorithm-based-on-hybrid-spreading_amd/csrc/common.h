// Shared device/host helpers for the lgcnhs HIP library (gfx950 only).
//
// - error plumbing for the C ABI (thread-local message, status codes)
// - wave64 helpers
// - WaveSort: a register-resident bitonic sort of CAP (key, id) pairs across one wave,
//   CAP/64 pairs per lane, used by every top-K selection kernel to compact its candidate
//   buffer. Order = (key desc, id asc): the canonical tie rule of this library (the
//   reference's torch.topk / np.argsort leave tie order unspecified).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lgcnhs.h"

namespace lg {

void set_error(const char *fmt, ...);
int launch_status(const char *what);

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// rocPRIM-style wave barrier: orders this wave's LDS traffic between lanes.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : ((~0ull) >> (64 - l));
}

template <typename K>
__device__ __forceinline__ K neg_inf();
template <>
__device__ __forceinline__ float neg_inf<float>() { return -__builtin_huge_valf(); }
template <>
__device__ __forceinline__ double neg_inf<double>() { return -__builtin_huge_val(); }

constexpr int kPadId = 0x7fffffff;

// (a before b) in the output order.
template <typename K>
__device__ __forceinline__ bool before(K ka, int ia, K kb, int ib) {
  return ka > kb || (ka == kb && ia < ib);
}

// Bitonic sort of CAP = 64*M elements held as k[j], id[j] (element e = j*64 + lane) into
// ascending "before" order over e: after the call element 0 is the best.
template <typename K, int M>
__device__ __forceinline__ void wave_bitonic_sort(K (&k)[M], int (&id)[M]) {
  constexpr int CAP = 64 * M;
  const int lane = lane_id();
#pragma unroll
  for (int size = 2; size <= CAP; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int js = stride / 64;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          if (j & js) continue;
          const int e = j * 64 + lane;            // lower element of the pair
          const bool desc = (e & size) == 0;      // this block sorts best-first
          const int p = j | js;
          const bool lo_better = before(k[j], id[j], k[p], id[p]);
          if (lo_better != desc) {
            K tk = k[j]; k[j] = k[p]; k[p] = tk;
            int ti = id[j]; id[j] = id[p]; id[p] = ti;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const int e = j * 64 + lane;
          const K ok = __shfl_xor(k[j], stride);
          const int oi = __shfl_xor(id[j], stride);
          const bool lower = (e & stride) == 0;
          const bool desc = (e & size) == 0;
          const bool mine_better = before(k[j], id[j], ok, oi);
          // lower slot of a best-first block keeps the better one, etc.
          const bool keep_mine = (lower == desc) ? mine_better : !mine_better;
          if (!keep_mine) { k[j] = ok; id[j] = oi; }
        }
      }
    }
  }
}

// Compact a wave-owned LDS candidate list (n valid entries, capacity CAP = 64*M) down to
// its best `keep` entries, written back sorted at [0, keep). Returns the new count and sets
// `tau` to the key of the last kept entry when the list is full (count == keep), else -inf
// (every future candidate must still be admitted).
template <typename K, int M>
__device__ __forceinline__ int wave_compact(K *ks, int *ids, int n, int keep, K &tau,
                                            int &tau_id) {
  const int lane = lane_id();
  K k[M];
  int id[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int e = j * 64 + lane;
    if (e < n) { k[j] = ks[e]; id[j] = ids[e]; }
    else { k[j] = neg_inf<K>(); id[j] = kPadId; }
  }
  wave_sync();
  wave_bitonic_sort<K, M>(k, id);
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int e = j * 64 + lane;
    if (e < keep) { ks[e] = k[j]; ids[e] = id[j]; }
  }
  wave_sync();
  const int cnt = n < keep ? n : keep;
  if (cnt == keep && keep > 0) { tau = ks[keep - 1]; tau_id = ids[keep - 1]; }
  else { tau = neg_inf<K>(); tau_id = kPadId; }
  wave_sync();
  return cnt;
}

// First position p in [lo, hi) with col[p] >= x (binary search over a sorted row).
__device__ __forceinline__ int64_t lower_bound_i32(const int32_t *col, int64_t lo, int64_t hi,
                                                   int32_t x) {
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (col[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

}  // namespace lg

#define LG_REQUIRE(cond, ...)        \
  do {                               \
    if (!(cond)) {                   \
      lg::set_error(__VA_ARGS__);    \
      return LG_ERR_ARG;             \
    }                                \
  } while (0)
