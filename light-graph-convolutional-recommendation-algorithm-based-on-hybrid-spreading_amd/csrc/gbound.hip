// Score bounds for the LGCNHS top-K walk (SURVEY.md §8 a9-a12 at C5): for every user u and
// 64-column chunk c of an item tile, gb[u][c] >= the fp32 chain score G(u, j) =
// e0_u . e0_j (model/SpreadLightGCN/model.py:74-77, the chain of lg_score_topk_f32) of
// every column j of the chunk. The walk (lg_spread_tile_resource_topk_f64) computes the
// exact chain only for columns whose gb * F can beat the user's K-th value.
//
// The bound is a bf16 MFMA product plus a rigorous margin. With the operands rounded to
// bf16 (relative error <= 2^-8 each) and an fp32-accumulated dot product of 64..128 terms,
//   |G_bf16 - G_chain| <= sum_k |u_k j_k| (2^-7 + 2^-16 + 2 gamma_D (1 + 2^-7))
//                      <= 0.00785 ||u|| ||j||           (gamma_128 = 128 * 2^-24)
// so gb = max_{j in c} G_bf16 + 0.008 ||u|| max_{j in c} ||j|| (norms rounded up to fp32),
// nudged up by 2^-22 relative for the fp32 operations that formed it, is an upper bound.
// Per column (optional qb): q_j = rne(v_j + 0.5) >= v_j, v_j = 255 (G_bf16_j + the same
// margin) / gb (1 + 2^-20), saturated to [0, 255] by v_cvt_pk_u8_f32 (measured on the box:
// round to nearest even, negative / NaN -> 0, above 255 -> 255, scripts/micro/cvt_pk_u8.hip),
// so gb * q_j / 255 >= G_chain_j as well (q_j = 0 when the bound is negative; gb <= 0 makes
// every column's bound <= 0). Stored row-major, one byte per column, rows of qstride bytes. (Folding the walk's rb_j / rbmax_c into q as well made the walk no
// faster -- 2.68 vs 2.67 s over the 489 C5 tiles -- and the bounds 0.34 s slower: dropped.)
// Then fl(G_chain * F) <= fl(gb * F) for every F >= 0 (rounding is monotone), so a column
// with gb * F <= tau can not beat tau. Cost per tile: 2 * U * T * D flop on bf16 MFMA
// (v_mfma_f32_16x16x32_bf16: 16 items x 16 users x 32 dims per instruction; 64 users per
// wave share every item fragment).
#include <math.h>

#include "common.h"

namespace lg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr float kBoundMargin = 0.008f;
#ifndef LG_BOUND_DEPTH
#define LG_BOUND_DEPTH 1  // item-fragment chunks in flight ahead (2 measured no faster at D = 64)
#endif

// max of three floats without the NaN-quieting canonicalisation fmaxf adds (the operands are
// finite or -inf)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float m;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(a), "v"(b), "v"(c));
  return m;
}

__device__ __forceinline__ float round_up_f32(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, __builtin_huge_valf());
  return f;
}

// xb[r] = bf16(x[r]) (round to nearest even), norm[r] = ||x[r]||_2 rounded up to fp32.
// One wave per row.
__global__ __launch_bounds__(256) void k_bound_prep(const float *__restrict__ x, int64_t n,
                                                    int dim, __bf16 *__restrict__ xb,
                                                    float *__restrict__ norm) {
  const int64_t r = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (r >= n) return;
  const int lane = lane_id();
  double ss = 0.0;
  for (int d = lane; d < dim; d += 64) {
    const float v = x[r * dim + d];
    xb[r * dim + d] = (__bf16)v;
    ss += (double)v * (double)v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  // sqrt of an fp64 sum of squares of fp32 values: relative error ~1e-16, far below the
  // fp32 round-up (the margin constant leaves 2 % slack besides)
  if (lane == 0) norm[r] = round_up_f32(sqrt(ss) * (1.0 + 1e-12));
}

// One wave = 64 users (4 groups of 16 MFMA columns) x every chunk of the tile. W = waves per
// SIMD the registers are sized for: D <= 64 runs 3 (152 VGPRs) and loads each chunk's item
// fragments at its start (the other waves cover the latency; 393 vs 437 ms at C5 against 2
// waves with the next chunk prefetched into 32 more registers), D = 128 runs 2 with the
// prefetch (3 would spill).
template <int D, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, W))) void k_chunk_bound(const __bf16 *__restrict__ ub,
                                                     const float *__restrict__ unorm,
                                                     int64_t n_users,
                                                     const __bf16 *__restrict__ ib,
                                                     const float *__restrict__ inorm,
                                                     int32_t item_begin, int32_t width,
                                                     int32_t nch, float *__restrict__ gb,
                                                     uint8_t *__restrict__ qb, int32_t qstride) {
  constexpr int S = D / 32;  // k-steps
  const int lane = lane_id();
  const int64_t ubase = ((int64_t)blockIdx.x * 4 + threadIdx.x / 64) * 64;
  if (ubase >= n_users) return;
  const int ul = lane & 15, kg = lane >> 4;
  bf16x8 bfr[4][S];
  float un[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    int64_t uu = ubase + 16 * g + ul;
    uu = uu < n_users ? uu : n_users - 1;
#pragma unroll
    for (int s = 0; s < S; ++s)
      bfr[g][s] = *reinterpret_cast<const bf16x8 *>(ub + uu * D + 32 * s + 8 * kg);
    un[g] = unorm[uu];
  }
  // q bytes of two chunks (64 users x 128 columns) staged in LDS, then written as whole
  // 128-byte row segments (8 lanes x 16 bytes per user)
  constexpr int QS = 36;  // dwords per user row: 32 + 4 (no bank conflicts, 16-B aligned)
  __shared__ uint32_t qs_all[4][64 * QS];
  uint32_t *qs = qs_all[threadIdx.x / 64];
  // item fragments of a chunk: [tile t][k-step s]; the next chunk's are loaded while this
  // chunk's MFMAs and bounds run
  auto load_items = [&](int cb, bf16x8 (&fr)[4][S], float &nm) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      int it = cb + 16 * t + ul;  // A row = item
      it = it < width ? it : width - 1;
#pragma unroll
      for (int s = 0; s < S; ++s)
        fr[t][s] = *reinterpret_cast<const bf16x8 *>(ib + (int64_t)(item_begin + it) * D +
                                                     32 * s + 8 * kg);
    }
    nm = cb + lane < width ? inorm[item_begin + cb + lane] : 0.f;
  };
  bf16x8 fa[4][S], fb[4][S];
  float na = 0.f, nb = 0.f;
  constexpr bool kNoPre = W >= 3;  // each chunk's fragments loaded at its start
  if (!kNoPre) load_items(0, fa, na);
  // D <= 64: chunk c + 2's fragments in flight during chunk c (c + 1's already landed);
  // D = 128 keeps one chunk ahead (the registers of a third set would spill)
  constexpr bool kDeep = LG_BOUND_DEPTH > 1 && D <= 64;
  bf16x8 fc[4][S];
  float nc = 0.f;
  if (kDeep && nch > 1) load_items(64, fb, nb);
  for (int c = 0; c < nch; ++c) {
    const int cb = 64 * c;  // chunk start inside the tile
    if constexpr (kNoPre) {
      load_items(cb, fa, na);
    } else if constexpr (kDeep) {
      if (c + 2 < nch) load_items(cb + 128, fc, nc);
    } else {
      if (c + 1 < nch) load_items(cb + 64, fb, nb);
    }
    // the chunk's largest item norm (wave-uniform)
    float inm = na;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) inm = fmaxf(inm, __shfl_xor(inm, o));
    float gmax[4];
    f32x4 accs[4][4];  // [item tile t][user group g]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; ++s)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][s], bfr[g][s], acc, 0, 0, 0);
        accs[t][g] = acc;
      }
    }
    // lane holds rows (items) 4 kg + r of each 16-item tile, column (user) ul; columns past
    // the width (a partial last chunk only) do not count
    if (cb + 64 > width) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (cb + 16 * t + 4 * kg + r >= width)
#pragma unroll
            for (int g = 0; g < 4; ++g) accs[t][g][r] = -__builtin_huge_valf();
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float m = max3f(accs[0][g][0], accs[0][g][1], accs[0][g][2]);
      m = max3f(m, accs[0][g][3], accs[1][g][0]);
      m = max3f(m, accs[1][g][1], accs[1][g][2]);
      m = max3f(m, accs[1][g][3], accs[2][g][0]);
      m = max3f(m, accs[2][g][1], accs[2][g][2]);
      m = max3f(m, accs[2][g][3], accs[3][g][0]);
      m = max3f(m, accs[3][g][1], accs[3][g][2]);
      gmax[g] = fmaxf(m, accs[3][g][3]);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float m = gmax[g];
      m = fmaxf(m, __shfl_xor(m, 16));
      m = fmaxf(m, __shfl_xor(m, 32));
      const float marg = kBoundMargin * un[g] * inm;
      float b = m + marg;
      b += fabsf(b) * 0x1p-22f + 1e-30f;
      const int64_t uu = ubase + 16 * g + ul;
      if (kg == 0 && uu < n_users) gb[uu * nch + c] = b;
      if (qb) {
        // per column: q = rne(v') with v' = fl(acc sc + msc) >= 255 (acc + marg) / b + 0.5 (sc
        // and msc carry (1 + 2^-20) factors over their own roundings and the fma's; msc holds
        // the 0.5 plus 1e-4 for the fma's absolute rounding near 0), so q >= the ratio; the
        // conversion saturates to [0, 255]; 4 consecutive items of one user per lane and
        // tile -> one dword
        const float sc = b > 0.f ? 255.f / b * (1.f + 0x1p-20f) * (1.f + 0x1p-20f) : 0.f;
        const float msc = (marg * sc * (1.f + 0x1p-20f) + 0.5001f) * (1.f + 0x1p-20f);
        const f32x2 sc2 = {sc, sc}, ms2 = {msc, msc};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f32x2 lo = __builtin_elementwise_fma(f32x2{accs[t][g][0], accs[t][g][1]}, sc2, ms2);
          const f32x2 hi = __builtin_elementwise_fma(f32x2{accs[t][g][2], accs[t][g][3]}, sc2, ms2);
          float v[4] = {lo[0], lo[1], hi[0], hi[1]};
          uint32_t w = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) w = __builtin_amdgcn_cvt_pk_u8_f32(v[r], r, w);
          // user 16 g + ul, columns (c & 1) * 64 + 16 t + 4 kg of the pair
          qs[(16 * g + ul) * QS + (c & 1) * 16 + 4 * t + kg] = w;
        }
      }
    }
    if (qb && ((c & 1) || c + 1 == nch)) {  // a chunk pair is complete: write it out
      wave_sync();
      const int cp = 64 * (c & ~1);  // the pair's first column
#pragma unroll
      for (int r8 = 0; r8 < 8; ++r8) {
        const int uloc = 8 * r8 + (lane >> 3);
        const int64_t uu = ubase + uloc;
        const int col = cp + 16 * (lane & 7);
        const uint4 v = *reinterpret_cast<const uint4 *>(qs + uloc * QS + 4 * (lane & 7));
        if (uu < n_users && col + 16 <= qstride)
          *reinterpret_cast<uint4 *>(qb + uu * qstride + col) = v;
      }
      wave_sync();
    }
    if constexpr (!kNoPre) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < S; ++s) fa[t][s] = fb[t][s];
      na = nb;
    }
    if constexpr (kDeep) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < S; ++s) fb[t][s] = fc[t][s];
      nb = nc;
    }
  }
}

}  // namespace lg

using namespace lg;

extern "C" int lg_bound_prep_f32(const float *x, int64_t n_rows, int32_t dim, void *x_bf16,
                                 float *norm_up, lg_stream_t stream) {
  LG_REQUIRE(x && x_bf16 && norm_up && n_rows >= 0 && dim >= 1,
             "lg_bound_prep_f32: bad arguments");
  if (n_rows == 0) return LG_OK;
  k_bound_prep<<<dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream>>>(
      x, n_rows, dim, (__bf16 *)x_bf16, norm_up);
  return launch_status("lg_bound_prep_f32");
}

extern "C" int lg_score_chunk_bound(const void *u_bf16, const float *u_norm, int64_t n_users,
                                    const void *i_bf16, const float *i_norm, int32_t dim,
                                    int32_t item_begin, int32_t width, float *gb, uint8_t *qb,
                                    int32_t qstride, lg_stream_t stream) {
  LG_REQUIRE(u_bf16 && u_norm && i_bf16 && i_norm && gb && n_users >= 0 && item_begin >= 0 &&
                 width >= 1,
             "lg_score_chunk_bound: bad arguments");
  LG_REQUIRE(!qb || (qstride >= (width + 255) / 256 * 256 && qstride % 4 == 0),
             "lg_score_chunk_bound: qstride %d < width %d rounded up to 256", qstride, width);
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128, "lg_score_chunk_bound: dim %d not in "
             "{32,64,128}", dim);
  if (n_users == 0) return LG_OK;
  const int nch = (width + 63) / 64;
  const dim3 grid((unsigned)((n_users + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  const __bf16 *u = (const __bf16 *)u_bf16, *i = (const __bf16 *)i_bf16;
  switch (dim) {
    case 32: k_chunk_bound<32, 3><<<grid, 256, 0, s>>>(u, u_norm, n_users, i, i_norm, item_begin, width, nch, gb, qb, qstride); break;
    case 64: k_chunk_bound<64, 3><<<grid, 256, 0, s>>>(u, u_norm, n_users, i, i_norm, item_begin, width, nch, gb, qb, qstride); break;
    default: k_chunk_bound<128, 2><<<grid, 256, 0, s>>>(u, u_norm, n_users, i, i_norm, item_begin, width, nch, gb, qb, qstride); break;
  }
  return launch_status("lg_score_chunk_bound");
}
