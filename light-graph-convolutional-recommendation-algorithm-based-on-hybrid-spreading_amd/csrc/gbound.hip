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
// widest tile lg_score_chunk_bound takes: 64 chunks of 64 columns (LG_BOUND_MAX_WIDTH)
constexpr int kBoundMaxWidth = LG_BOUND_MAX_WIDTH;

// max of three floats: one v_maximum3_f32 (gfx950), compiler-visible, so hipcc pads the
// MFMA-result wait states itself (no NaN-quieting canonicalisation as fmaxf would add; the
// operands are finite or -inf, and a NaN would propagate into the bound)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  return __builtin_elementwise_maximum(a, __builtin_elementwise_maximum(b, c));
}

// max of a value over the lanes l, l ^ 16, l ^ 32, l ^ 48 (the four 16-lane rows) by the
// gfx950 row swaps (VALU; a __shfl_xor is an LDS-pipe ds_bpermute and a wait per step). Inline
// asm: hipcc's __builtin_amdgcn_permlane{16,32}_swap returns the swapped vdst as both halves of
// its result (the second register is lost -- seen in the ISA of a two-output test kernel). The
// nops cover the VALU-write -> permlane read and permlane -> VALU read hazards.
__device__ __forceinline__ float row_max4(float m) {
  uint32_t x = __builtin_bit_cast(uint32_t, m), y = x;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  m = fmaxf(__builtin_bit_cast(float, x), __builtin_bit_cast(float, y));
  x = __builtin_bit_cast(uint32_t, m);
  y = x;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  return fmaxf(__builtin_bit_cast(float, x), __builtin_bit_cast(float, y));
}

// Half exchanges over the 16-lane rows (gfx950): v_permlane32_swap x, y -- rows 2-3 of x <->
// rows 0-1 of y; v_permlane16_swap x, y -- rows 1, 3 of x <-> rows 0, 2 of y. Inline asm with
// the waits inside: 2 wait states between a VALU write and a swap reading it, and between a
// swap and a VALU reading its result (hipcc's builtins pad the first only: a value read right
// after its swap came out wrong on the box, the last chunk's q bytes in
// test_score_bounds_cover_chain_scores_many_blocks).
__device__ __forceinline__ void swap32x2(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\t"
               "s_nop 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void swap16x2(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\t"
               "s_nop 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void swap16(uint32_t &a, uint32_t &b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
}

// 4 x 4 transpose of (register t, lane row): afterwards row r's register t holds what row t's
// register r held
__device__ __forceinline__ void rows_transpose(uint32_t w[4]) {
  asm volatile("s_nop 1\n\t"
               "v_permlane32_swap_b32 %0, %2\n\tv_permlane32_swap_b32 %1, %3\n\t"
               "s_nop 1\n\t"
               "v_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\t"
               "s_nop 1" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
}

// maximum of two floats given as bits (v_maximum_f32: a NaN propagates)
__device__ __forceinline__ float fmax_bits(uint32_t a, uint32_t b) {
  return __builtin_elementwise_maximum(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b));
}

// u, v hold at lane row kg the value of group P(kg) = {0, 2, 1, 3}[kg] (of the lane's
// column); ou[g], ov[g] = group g's values on every row
__device__ __forceinline__ void rows_broadcast2(float u, float v, float ou[4], float ov[4]) {
  uint32_t x = __builtin_bit_cast(uint32_t, u), y = x;
  uint32_t p = __builtin_bit_cast(uint32_t, v), q = p;
  swap16x2(x, y, p, q);  // x = [u0 u0 u1 u1], y = [u2 u2 u3 u3] (p, q likewise)
  uint32_t x2 = x, y2 = y, p2 = p, q2 = q;
  swap32x2(x, x2, y, y2);
  swap32x2(p, p2, q, q2);
  ou[0] = __builtin_bit_cast(float, x), ou[1] = __builtin_bit_cast(float, x2);
  ou[2] = __builtin_bit_cast(float, y), ou[3] = __builtin_bit_cast(float, y2);
  ov[0] = __builtin_bit_cast(float, p), ov[1] = __builtin_bit_cast(float, p2);
  ov[2] = __builtin_bit_cast(float, q), ov[3] = __builtin_bit_cast(float, q2);
}

__device__ __forceinline__ float round_up_f32(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, __builtin_huge_valf());
  return f;
}

// xb[r] = bf16(x[r]) (round to nearest even), norm[r] = ||x[r]||_2 rounded up to fp32, and
// (err, optional) err[r] = ||x[r] - bf16(x[r])||_2 rounded up: the per-row rounding error the
// screened top-K's tight margin is built from (lgcnhs.ops.screen_margins). x - bf16(x) is
// exact in fp32 (it has at most 16 significant bits). One wave per row.
__global__ __launch_bounds__(256) void k_bound_prep(const float *__restrict__ x, int64_t n,
                                                    int dim, __bf16 *__restrict__ xb,
                                                    float *__restrict__ norm,
                                                    float *__restrict__ err) {
  const int64_t r = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (r >= n) return;
  const int lane = lane_id();
  double ss = 0.0, se = 0.0;
  for (int d = lane; d < dim; d += 64) {
    const float v = x[r * dim + d];
    const __bf16 b = (__bf16)v;
    xb[r * dim + d] = b;
    ss += (double)v * (double)v;
    const double e = (double)v - (double)(float)b;
    se += e * e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ss += __shfl_xor(ss, o);
    se += __shfl_xor(se, o);
  }
  // sqrt of an fp64 sum of squares of fp32 values: relative error ~1e-16, far below the
  // fp32 round-up (the margin constant leaves 2 % slack besides)
  if (lane == 0) {
    norm[r] = round_up_f32(sqrt(ss) * (1.0 + 1e-12));
    if (err) err[r] = round_up_f32(sqrt(se) * (1.0 + 1e-12));
  }
}

// The same for dim = 4 LPR (LPR = 8, 16, 32 lanes per row: dim 32, 64, 128): each lane takes
// 4 consecutive elements (one 16-byte load, one 8-byte store), 64 / LPR rows per wave, the
// row's sums over its LPR lanes in log2(LPR) xor steps -- the one-wave-per-row form above spent
// its time in six fp64 shuffle steps per row (0.28 ms for a 1M x 64 table).
template <int LPR>
__global__ __launch_bounds__(256) void k_bound_prep4(const float *__restrict__ x, int64_t n,
                                                     __bf16 *__restrict__ xb,
                                                     float *__restrict__ norm,
                                                     float *__restrict__ err) {
  constexpr int dim = 4 * LPR, RPW = 64 / LPR;
  const int lane = lane_id();
  const int64_t r = ((int64_t)blockIdx.x * 4 + threadIdx.x / 64) * RPW + lane / LPR;
  const bool in = r < n;
  const int64_t rr = in ? r : n - 1;
  const int c = 4 * (lane % LPR);
  const float4 v = *reinterpret_cast<const float4 *>(x + rr * dim + c);
  const float vv[4] = {v.x, v.y, v.z, v.w};
  double ss = 0.0, se = 0.0;
  __bf16 b[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    b[t] = (__bf16)vv[t];
    ss += (double)vv[t] * (double)vv[t];
    const double e = (double)vv[t] - (double)(float)b[t];
    se += e * e;
  }
  if (in) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<bf16x4 *>(xb + r * dim + c) = bf16x4{b[0], b[1], b[2], b[3]};
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) {
    ss += __shfl_xor(ss, o);
    se += __shfl_xor(se, o);
  }
  if (in && lane % LPR == 0) {
    norm[r] = round_up_f32(sqrt(ss) * (1.0 + 1e-12));
    if (err) err[r] = round_up_f32(sqrt(se) * (1.0 + 1e-12));
  }
}

// s_waitcnt vmcnt(n) for a uniform run-time n <= K (the count is an immediate: a chain of
// scalar compares picks the instruction)
template <int K>
__device__ __forceinline__ void vm_wait_le(int n) {
  if constexpr (K > 0) {
    if (n < K) {
      vm_wait_le<K - 1>(n);
      return;
    }
  }
  static_assert(K <= 63, "vmcnt holds 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(K) : "memory");
}

// chunk buffers of the score-bound kernel's ring (D = 128: 4 x 16 KB, 2 blocks per CU)
#ifndef LG_BOUND_NB
#define LG_BOUND_NB(D) ((D) <= 64 ? 5 : 4)
#endif

// cache-policy bits of the q and gb stores (measurement builds): nt on the q stores measured
// 0.84 -> 0.75 ms per C5 tile alone (scripts/micro_bound.py) but 0.728 -> 0.778 ms inside the
// LGCNHS pipeline (scripts/gpu_r06_qab.sh), so the default is plain stores
#ifndef LG_QSTORE_AUX
#define LG_QSTORE_AUX 0
#endif
#ifndef LG_GB_AUX
#define LG_GB_AUX 0
#endif
// One wave = 64 users (4 groups of 16 MFMA columns) x every chunk of the tile; a block = 4
// waves = 256 users. The chunk's item fragments (64 items x D bf16) are shared by the block's
// waves through LDS: an NB-buffer ring filled by LDS-DMA NB - 1 chunks ahead, one barrier per
// chunk hands a buffer over -- a quarter of the L2 fragment reads, their latency hidden by
// NB - 2 chunks of work. W = waves per SIMD the registers are sized for (D <= 64: 3, D = 128:
// 2). Waves past the last user still load and synchronise (their stores are dropped by the
// descriptors' range checks).
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
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));  // (uniform)
  const int64_t ubase = ((int64_t)blockIdx.x * 4 + wv) * 64;
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
  // the staged chunks: 64 item rows of D bf16 (2 D bytes), written by LDS-DMA
  // (global_load_lds_dwordx4: each wave instruction fills 1 KB contiguously, no VGPRs); the
  // 16-byte pieces of row r sit XOR-swizzled by sw(r) = (r / (128 / D)) & (D / 8 - 1), so the
  // fragment reads of any 16 consecutive lanes (16 rows, one piece) hit distinct banks
  constexpr int PR = D / 8;               // 16-byte pieces per item row
  constexpr int RB = 2 * D;               // bytes per staged row
  constexpr int NL = 64 * PR / 256;       // DMA instructions per thread per chunk (D = 32: 1)
  static_assert(NL >= 1 && 64 * PR % 256 == 0, "chunk pieces must spread over the block");
  // a ring of NB chunk buffers: chunk c + NB - 1's DMA goes out while chunk c is computed, so
  // the wait at a chunk's end (for chunk c + 1) leaves the stores of the last NB - 1 chunks in
  // flight -- vmcnt completes in issue order, and with 2 buffers every chunk waited for the
  // previous chunk's q stores to be acknowledged (the q bytes' write latency then set the
  // pace: 0.74 ms per C5 tile with 3 buffers, 0.24 without q)
  constexpr int NB = LG_BOUND_NB(D);
  __shared__ __attribute__((aligned(16))) char frs[NB][64 * RB];
  auto sw = [](int r) { return (r / (128 / D)) & (PR - 1); };
  // per thread and DMA instruction j: the chunk row of its piece and the piece's byte offset
  // from the chunk's first item row (loop-invariant; the chunk's base address is uniform and
  // goes in the instruction's SGPR pair)
  int drow[NL];
  uint32_t doff[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int p = 256 * j + 64 * wv + lane;
    drow[j] = p / PR;
    doff[j] = (uint32_t)(2 * (drow[j] * D + 8 * ((p % PR) ^ sw(drow[j]))));
  }
  auto dma = [&](int cb, int buf) __attribute__((always_inline)) {
    const __bf16 *base = ib + (int64_t)(item_begin + cb) * D;
    const bool part = cb + 64 > width;  // a partial last chunk: rows past the width re-read
#pragma unroll                          // the tile's last item
    for (int j = 0; j < NL; ++j) {
      uint32_t off = doff[j];
      if (part) {
        const int rr = drow[j] < width - cb ? drow[j] : width - 1 - cb;
        off -= (uint32_t)(2 * D * (drow[j] - rr));
      }
      const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(
          __attribute__((address_space(3))) char *)(frs[buf] + 16 * (256 * j + 64 * wv)));
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(off), "s"(base), "s"(dst) : "memory");
    }
  };
  // the wave's 64 rows of gb through one descriptor (32-bit offsets)
  const int64_t nrow_w = n_users - ubase < 64 ? n_users - ubase : 64;
  const __amdgpu_buffer_rsrc_t rgb = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(gb + (ubase < n_users ? ubase : 0) * nch), 0,
      nrow_w > 0 ? (int)(nrow_w * nch * 4) : 0, 0x00020000);
  // the wave's 64 q rows through one descriptor (rows past n_users are out of range: their
  // stores are dropped), 32-bit offsets
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
      qb ? (void *)(qb + (ubase < n_users ? ubase : 0) * (int64_t)qstride) : nullptr, 0,
      qb && nrow_w > 0 ? (int)(nrow_w * qstride) : 0, 0x00020000);
  // every chunk's largest item norm (the margin's ||j|| factor), once per block: wave w folds
  // chunks w, w + 4, ... (the loads first, then the reductions side by side)
  __shared__ float s_cmax[kBoundMaxWidth / 64];
  {
    constexpr int CPW = kBoundMaxWidth / 64 / 4;  // chunks per wave (nch <= 64, checked at the ABI)
    float v[CPW];
#pragma unroll
    for (int k = 0; k < CPW; ++k) {
      const int j = 64 * (wv + 4 * k) + lane;
      v[k] = j < width ? inorm[item_begin + j] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < CPW; ++k) {
      if (64 * (wv + 4 * k) >= width) break;
      float m = row_max4(v[k]);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      if (lane == 0) s_cmax[wv + 4 * k] = m;
    }
  }
#pragma unroll
  for (int j = 0; j < NB - 1; ++j)
    if (j < nch) dma(64 * j, j);
  // the DMA is inline asm, invisible to hipcc's waits: this wave's copies have landed only
  // after an explicit vmcnt wait, which must precede the barrier that publishes the buffer
  // (the later chunks' copies may stay in flight)
  vm_wait_le<NL * (NB - 2)>(NL * ((nch < NB - 1 ? nch : NB - 1) - 1));
  __syncthreads();
  // every prologue load (the user fragments and norms above) is taken here, before the loop:
  // a load still pending at the loop head gets its wait inside the loop, where it also drains
  // the next chunk's DMA in every iteration
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int s = 0; s < S; ++s) asm volatile("" : "+v"(bfr[g][s]));
    asm volatile("" : "+v"(un[g]));
  }
  // lane row kg reduces and stores the bound of user group P(kg) = {0, 2, 1, 3}[kg] (the row
  // exchanges below leave the groups in that order)
  const float unl = kg == 0 ? un[0] : kg == 1 ? un[2] : kg == 2 ? un[1] : un[3];
  const uint32_t gbo = (uint32_t)(4 * (16 * (kg == 1 ? 2 : kg == 2 ? 1 : kg) + ul) * nch);
  // q: user 16 g + ul's row, lane row kg's 16 columns (all in the VGPR offset, which the
  // descriptor's range check covers: rows past n_users are dropped). The SGPR offset stays 0:
  // with a register there hipcc does not pad the 16-byte store's data hazard (a VALU writing
  // the data registers right after the store), and on the box such an overwrite reached the
  // store (q bytes of lanes 12-15 of every row wrong, the last chunk's second dword)
  uint32_t qo[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) qo[g] = (uint32_t)((16 * g + ul) * qstride + 16 * kg);
  // gb: the lane's user's bounds of 8 consecutive chunks are collected in registers (a shift
  // register, gq[7] the latest) and leave as 32 contiguous bytes -- one dword store per chunk
  // wrote each 32-byte memory sector 8 times over (WRITE_SIZE 1.2 GB per C5 tile for 128 MB
  // of bounds)
  float gq[8];
  // the vector-memory operations each chunk issues after its DMA (the loop issues no loads):
  // with q one 16-byte q store per lane and user group -- the waits at the loop's end leave
  // these in flight (below); the gb stores of every 8th chunk are not counted, so the wait
  // after them is stricter than it needs to be, never looser
  constexpr int kQStores = 4;   // the `g` loop's raw_buffer_store_b128
  for (int c = 0; c < nch; ++c) {
    const int cb = 64 * c;  // chunk start inside the tile
    if (c + NB - 1 < nch)  // into the buffer every wave finished reading at the last barrier
      dma(cb + 64 * (NB - 1), (c + NB - 1) % NB);
    const float inm = s_cmax[c];  // the chunk's largest item norm
    f32x4 accs[4][4];  // [item tile t][user group g]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // item tile t's A fragments from the staged chunk (read per tile: 8 S VGPRs live)
      bf16x8 fa[S];
#pragma unroll
      for (int s = 0; s < S; ++s)
        fa[s] = *reinterpret_cast<const bf16x8 *>(frs[c % NB] + (16 * t + ul) * RB +
                                                  16 * ((4 * s + kg) ^ sw(16 * t + ul)));
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; ++s)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s], bfr[g][s], acc, 0, 0, 0);
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
    // the lane's maximum per group (16 scores), then over the 4 lane rows for all groups at
    // once: row exchanges pair rows 0 <-> 2, 1 <-> 3 of groups 0 and 1 (2 and 3) in one
    // maximum, then rows 0 <-> 1 across the pairs -- row kg ends with group P(kg)'s maximum
    uint32_t gm[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float m0 = max3f(accs[0][g][0], accs[0][g][1], accs[0][g][2]);
      const float m1 = max3f(accs[0][g][3], accs[1][g][0], accs[1][g][1]);
      const float m2 = max3f(accs[1][g][2], accs[1][g][3], accs[2][g][0]);
      const float m3 = max3f(accs[2][g][1], accs[2][g][2], accs[2][g][3]);
      const float m4 = max3f(accs[3][g][0], accs[3][g][1], accs[3][g][2]);
      gm[g] = __builtin_bit_cast(
          uint32_t, __builtin_elementwise_maximum(max3f(m0, m1, m2), max3f(m3, m4, accs[3][g][3])));
    }
    swap32x2(gm[0], gm[1], gm[2], gm[3]);
    uint32_t ma = __builtin_bit_cast(uint32_t, fmax_bits(gm[0], gm[1]));
    uint32_t mb = __builtin_bit_cast(uint32_t, fmax_bits(gm[2], gm[3]));
    swap16(ma, mb);
    const float m = fmax_bits(ma, mb);
    const float marg = kBoundMargin * unl * inm;
    float b = m + marg;
    b += fabsf(b) * 0x1p-22f + 1e-30f;
    b = b == b ? b : __builtin_huge_valf();  // NaN (a non-finite score): no bound, +inf
    // (every lane stores; rows past n_users fall outside the descriptor's range and are
    // dropped; the chunk goes in the VGPR offset, see qo below)
#pragma unroll
    for (int k = 0; k < 7; ++k) gq[k] = gq[k + 1];
    gq[7] = b;
    if ((c & 7) == 7) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, (f32x4){gq[0], gq[1], gq[2], gq[3]}), rgb,
          gbo + 4 * (c - 7), 0, LG_GB_AUX);
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, (f32x4){gq[4], gq[5], gq[6], gq[7]}), rgb,
          gbo + 4 * (c - 3), 0, LG_GB_AUX);
    } else if (c + 1 == nch) {  // the last chunk: the held bounds of chunks c - (c & 7) .. c
#pragma unroll
      for (int k = 0; k < 7; ++k)
        if (k >= 7 - (c & 7))
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, gq[k]), rgb,
                                                gbo + 4 * (c - 7 + k), 0, LG_GB_AUX);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, gq[7]), rgb, gbo + 4 * c,
                                            0, LG_GB_AUX);
    }
    if (qb) {
      // per column: q = rne(v') with v' = fl(acc sc + msc) >= 255 (acc + marg) / b + 0.5 (sc
      // and msc carry (1 + 2^-20) factors over their own roundings and the fma's; msc holds
      // the 0.5 plus 1e-4 for the fma's absolute rounding near 0), so q >= the ratio; the
      // conversion saturates to [0, 255]. sc and msc are the lane row's group's; row
      // exchanges hand every group's pair to all 4 rows
      const float scl = b > 0.f ? 255.f / b * (1.f + 0x1p-20f) * (1.f + 0x1p-20f) : 0.f;
      const float mscl = (marg * scl * (1.f + 0x1p-20f) + 0.5001f) * (1.f + 0x1p-20f);
      float sc[4], msc[4];
      rows_broadcast2(scl, mscl, sc, msc);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // 4 consecutive items of one user per lane and tile -> one dword w[t] (lane row kg:
        // items 16 t + 4 kg .. + 3)
        // (the fma on pairs: v_pk_fma_f32, two columns per instruction, the same roundings)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 s2 = {sc[g], sc[g]}, m2 = {msc[g], msc[g]};
        uint32_t w[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f32x2 lo = __builtin_elementwise_fma(
              (f32x2){accs[t][g][0], accs[t][g][1]}, s2, m2);
          const f32x2 hi = __builtin_elementwise_fma(
              (f32x2){accs[t][g][2], accs[t][g][3]}, s2, m2);
          const float v[4] = {lo[0], lo[1], hi[0], hi[1]};
          w[t] = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) w[t] = __builtin_amdgcn_cvt_pk_u8_f32(v[r], r, w[t]);
        }
        // 4 x 4 transpose of (tile t, lane row kg): lane row kg then holds tile kg's 16
        // consecutive columns, w[0..3] = its 4 dwords in order
        rows_transpose(w);
        // user 16 g + ul, columns cb + 16 kg .. + 15: 16 users x 64 contiguous bytes per
        // store (every lane stores; a partial last chunk's columns past the width land in
        // the row's padding, qstride >= the width rounded up to 256)
        __builtin_amdgcn_raw_buffer_store_b128(
            (__attribute__((ext_vector_type(4))) uint32_t){w[0], w[1], w[2], w[3]}, rq,
            qo[g] + cb, 0, LG_QSTORE_AUX);
      }
    }
    // chunk c + 1's DMA (this wave's share) landed, then the barrier publishes the buffer.
    // vmcnt counts stores as well, and completes in issue order: the wait leaves in flight
    // what was issued after that DMA (it went out in chunk c + 2 - NB, or in the prologue) --
    // the q stores of chunks max(0, c + 2 - NB) .. c and the DMAs of chunks c + 2 ..
    // min(c + NB - 1, nch - 1). kQStores per chunk: the unconditional store statements above
    // (every lane issues every store; a store made conditional or merged would have to change
    // the count); the gb stores are not counted (stricter, never looser). The last chunk
    // waits for nothing: the kernel ends.
    if (c + 1 < nch) {
      const int nst = (qb ? kQStores : 0) * (c + 1 < NB - 1 ? c + 1 : NB - 1);
      const int ndma = NL * (nch - 2 - c < NB - 2 ? nch - 2 - c : NB - 2);
      vm_wait_le<kQStores * (NB - 1) + NL * (NB - 2)>(nst + ndma);
      __syncthreads();
    }
  }
}

}  // namespace lg

using namespace lg;

extern "C" int lg_bound_prep_f32(const float *x, int64_t n_rows, int32_t dim, void *x_bf16,
                                 float *norm_up, float *err_up, lg_stream_t stream) {
  LG_REQUIRE(x && x_bf16 && norm_up && n_rows >= 0 && dim >= 1,
             "lg_bound_prep_f32: bad arguments");
  if (n_rows == 0) return LG_OK;
  hipStream_t s = (hipStream_t)stream;
  __bf16 *xb = (__bf16 *)x_bf16;
  const bool al = ((uintptr_t)x & 15) == 0 && ((uintptr_t)x_bf16 & 7) == 0;
#define LG_PREP4(LPR)                                                                         \
  k_bound_prep4<LPR><<<dim3((unsigned)((n_rows + 4 * (64 / LPR) - 1) / (4 * (64 / LPR)))),     \
                       dim3(256), 0, s>>>(x, n_rows, xb, norm_up, err_up)
  if (al && dim == 32) LG_PREP4(8);
  else if (al && dim == 64) LG_PREP4(16);
  else if (al && dim == 128) LG_PREP4(32);
  else
    k_bound_prep<<<dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, s>>>(
        x, n_rows, dim, xb, norm_up, err_up);
#undef LG_PREP4
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
  // the per-chunk norm maxima live in a 64-entry LDS table (s_cmax, 16 chunks per wave)
  LG_REQUIRE(width <= kBoundMaxWidth, "lg_score_chunk_bound: width %d > %d", width,
             kBoundMaxWidth);
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
