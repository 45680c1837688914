// K2: full-catalog scoring + exclusion mask + streaming top-K, gfx950 f32 MFMA.
//
// Replaces model/LightGCN/recommend.py:83-114 (identical in LightGCNOpti/recommend.py and
// LightGCN/evaluation.py:31-51):
//     score = torch.matmul(users_emb.weight, items_emb.weight.T)       # [U, I] fp32
//     score[train positives] = -(1 << 10); score[val positives] = -(1 << 10)
//     _, recommendations = torch.topk(score, k)
// and the dense masked matrix of getAllocateMat (model/SpreadLightGCN/model.py:74-104).
//
// Score definition (bit-exact, checked against oracle/score_chain.c): v_mfma_f32_16x16x4_f32
// computes a k-ordered fp32 fma chain. Lane l of a wave holds item row (l & 15) as the A
// operand and user column (l & 15) as the B operand, k-slot (l >> 4); step s of the chain
// uses element g*Q + s of k-slot g (Q = D/4), so each lane reads one contiguous 16*Q-byte
// piece of each embedding row, and the fp32 result equals
//     acc = 0; for s < Q: for g < 4: acc = fmaf(u[g*Q+s], i[g*Q+s], acc).
// Top-K: per user a candidate list of CAP entries in LDS; a score enters only if it beats
// the user's current K-th best (tau), so after the first few hundred items almost nothing
// enters and the VALU cost per score is one compare. The exclusion row (sorted) is
// binary-searched only for list entries, in batch when the list is compacted: an excluded
// item takes mask_value (-1024) before the sort, which is exactly the reference's masked
// top-k. Lists are compacted by the wave-wide bitonic sort of common.h. Order: (score
// desc, item asc). The main loop thus issues no global load but the item tiles.
#include <stdlib.h>

#include "common.h"

namespace lg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int Q>
__device__ __forceinline__ void load_piece(const float *__restrict__ p, float (&v)[Q]) {
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

typedef float f32x4v __attribute__((ext_vector_type(4)));

// Item-tile loads: raw buffer loads through a per-tile descriptor whose base is the tile's
// first row and whose record count is the bytes left in the table (0 past its end), so rows
// beyond n_items read as 0 and every tile issues the same LT loads with no branch and no
// per-lane address arithmetic. Compiler-visible (__builtin_amdgcn_raw_buffer_load_b128):
// hipcc counts these loads itself and places each s_waitcnt vmcnt before the first use.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
template <int D>
__device__ __forceinline__ void load_item_tile(const float *ei, int64_t n_items, int64_t it,
                                               int voff, f32x4v (&v)[D / 16]) {
  constexpr int TB = 16 * D * 4;  // bytes of one 16-item tile
  const int rem = (int)(n_items - it);  // items left in the table (n_items < 2^31)
  const int num = rem >= 16 ? TB : (rem > 0 ? rem * (D * 4) : 0);
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void *)(ei + it * D), 0, num, 0x00020000);
#pragma unroll
  for (int t = 0; t < D / 16; ++t)
    v[t] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16 * t, 0, 0));
}

// max of the four scores of an MFMA result: two v_maximum3_f32 (gfx950), compiler-visible, so
// hipcc pads the MFMA-result wait states itself. NaN-propagating: callers test
// !(max4(a) <= thr), which sends a NaN score to the exact per-element test (sc > thr) instead
// of hiding the tile's other scores behind it.
__device__ __forceinline__ float max4(f32x4 a) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a[0], a[1]),
                                       __builtin_elementwise_maximum(a[2], a[3]));
}
__device__ __forceinline__ bool above(float m, float thr) { return !(m <= thr); }

// One wave: NG groups of 16 users; the block's waves work independently.
//
// Software pipeline (per wave, one 16-item tile per step t):
//   wait for tile t+1  ->  MFMAs of tile t+1 into acc[(t+1)%2], interleaved with the
//   one-max-one-compare filter of tile t's scores in acc[t%2]  ->  issue the loads of tile
//   t+3 into the register buffer tile t+1 just left  ->  (rare) insert tile t's candidates
//   ->  compact lists that could overflow.
// The filter's vector instructions fill the MFMA issue gaps (an f32 16x16x4 MFMA holds the
// SIMD's vector issue for 8 of its 32 cycles), and each tile's loads are in flight for two
// steps. All loads are compiler-visible: hipcc places the vmcnt waits.
template <int D, int NG, int M, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_score_topk(
    const float *__restrict__ eu, const float *__restrict__ ei, int64_t n_users,
    int64_t n_items, const int64_t *__restrict__ ex_rowptr,
    const int32_t *__restrict__ ex_col, float mask_value, int k, int n_splits,
    int64_t items_per_split, float *__restrict__ out_val, int64_t *__restrict__ out_idx,
    float *__restrict__ part_val, int32_t *__restrict__ part_idx, int probe) {
  constexpr int Q = D / 4;
  constexpr int LT = Q / 4;  // buffer loads per tile per lane
  constexpr int CAP = 64 * M;
  __shared__ float cs[WAVES][NG][16][CAP];
  __shared__ int ci[WAVES][NG][16][CAP];
  __shared__ int exs[WAVES][64];

  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int ul = lane & 15;
  const int gq = lane >> 4;
  const int64_t tile = blockIdx.x / n_splits;
  const int split = blockIdx.x % n_splits;
  const int64_t ubase = (tile * WAVES + wave) * (16 * NG);
  if (ubase >= n_users) return;  // wave-uniform; no block-level barriers below
  const int64_t i0 = (int64_t)split * items_per_split;
  int64_t i1 = i0 + items_per_split;
  if (i1 > n_items) i1 = n_items;
  const int n_valid = i1 > i0 ? (int)(i1 - i0) : 0;  // items of this split
  const int n_t = (n_valid + 15) / 16;                // tiles of this split

  float uf[NG][Q];
  bool uvalid[NG];
  int64_t ex_pos[NG], ex_hi[NG];
  int cnt[NG], chk[NG];
  float tau[NG], thr[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int64_t u = ubase + g * 16 + ul;
    uvalid[g] = u < n_users;
    const int64_t uu = uvalid[g] ? u : n_users - 1;
    load_piece<Q>(eu + uu * D + gq * Q, uf[g]);
    ex_pos[g] = 0;
    ex_hi[g] = 0;
    if (ex_rowptr && uvalid[g]) {
      ex_pos[g] = ex_rowptr[u];
      ex_hi[g] = ex_rowptr[u + 1];
    }
    cnt[g] = 0;
    chk[g] = 0;
    tau[g] = neg_inf<float>();
    thr[g] = (uvalid[g] && probe != 1) ? neg_inf<float>() : __builtin_huge_valf();
    // probe == 1 (measurement builds only, see topk_probe()): no candidate ever enters
  }
  const uint64_t same_user = 0x0001000100010001ull << ul;

  // Exclusion is applied lazily: a candidate enters on its raw score (or on the mask value
  // when that alone beats tau), and the entries [chk, n) added since the user's last
  // compaction are checked when the list is compacted. Their items all lie in
  // [previous limit, lim), and ex_pos is the user's first excluded item not yet passed
  // (>= the previous limit, or the row start: items below i0 are harmless), so the
  // excluded items to test are one ascending run ex_col[ex_pos ..) read 64 at a time,
  // coalesced, and binary-searched in LDS. Exact: an excluded item would enter with
  // mask_value, and mask_value > tau admits every item.
  auto compact_user = [&](int g, int u, int lim) __attribute__((always_inline)) {
    const int n = __shfl(cnt[g], u);
    const int c0 = __shfl(chk[g], u);
    int64_t pos = __shfl(ex_pos[g], u);
    const int64_t hi = __shfl(ex_hi[g], u);
    float *ks = &cs[wave][g][u][0];
    int *is = &ci[wave][g][u][0];
    if (n > c0) {
      while (pos < hi) {
        const int64_t e = pos + lane;
        const int32_t x = e < hi ? ex_col[e] : 0x7fffffff;
        const int nin = __popcll(__ballot(x < lim));  // ascending: a prefix of the lanes
        if (nin == 0) break;
        exs[wave][lane] = x;
        wave_sync();
        for (int j = c0 + lane; j < n; j += 64) {
          const int item = is[j];
          int a = 0, b = nin;  // first index with exs[] >= item
          while (a < b) {
            const int mid = (a + b) >> 1;
            if (exs[wave][mid] < item) a = mid + 1;
            else b = mid;
          }
          if (a < nin && exs[wave][a] == item) ks[j] = mask_value;
        }
        wave_sync();
        pos += nin;
        if (nin < 64) break;
      }
    }
    float t;
    int tid;
    const int nc = wave_compact<float, M>(ks, is, n, k, t, tid);
    if (ul == u) {
      cnt[g] = nc;
      chk[g] = nc;
      tau[g] = t;
      ex_pos[g] = pos;
      // a masked (excluded) item would enter with mask_value: admit everything then
      thr[g] = !uvalid[g] ? __builtin_huge_valf() : (mask_value > t ? neg_inf<float>() : t);
    }
  };

  // acc[g][r] = score(user ubase + 16g + ul, item i0 + 16t + 4gq + r)
  auto mfma_tile = [&](const f32x4v(&af)[LT], f32x4 (&acc)[NG]) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    // s outer / g inner: NG independent accumulation chains interleave on the MFMA pipe
#pragma unroll
    for (int s = 0; s < Q; ++s)
#pragma unroll
      for (int g = 0; g < NG; ++g)
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s / 4][s % 4], uf[g][s], acc[g], 0,
                                                      0, 0);
  };

  // Fast filter: one max and one compare per group against thr = the entry threshold (tau,
  // or -inf while the mask value itself would enter, +inf for padding users).
  auto any_cand = [&](const f32x4 (&acc)[NG]) __attribute__((always_inline)) {
    bool any = false;
#pragma unroll
    for (int g = 0; g < NG; ++g) any |= above(max4(acc[g]), thr[g]);
    return __ballot(any) != 0;
  };

  // Slow path, taken when some lane of the wave has a candidate in tile t.
  auto insert_tile = [&](int t, const f32x4 (&acc)[NG]) __attribute__((always_inline)) {
    const int rel = t * 16 + gq * 4;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (__ballot(above(max4(acc[g]), thr[g])) == 0) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sc = acc[g][r];
        const bool cand = rel + r < n_valid && sc > thr[g];
        const uint64_t bal = __ballot(cand);
        if (bal) {
          const int pos = cnt[g] + __popcll(bal & same_user & lanemask_lt());
          if (cand) {
            cs[wave][g][ul][pos] = sc;
            ci[wave][g][ul][pos] = (int)i0 + rel + r;
          }
          cnt[g] += __popcll(bal & same_user);
        }
      }
    }
  };

  // compact every user whose list could overflow on the next tile (+16 max per tile)
  auto maybe_compact = [&](int lim) __attribute__((always_inline)) {
    bool over = false;
#pragma unroll
    for (int g = 0; g < NG; ++g) over |= cnt[g] > CAP - 16;
    if (__ballot(over) == 0) return;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      uint64_t need = __ballot(cnt[g] > CAP - 16) & 0xffffull;
      if (need) {
        wave_sync();
        while (need) {
          const int u = __ffsll((long long)need) - 1;
          need &= need - 1;
          compact_user(g, u, lim);
        }
      }
    }
  };

  const int voff = (ul * D + gq * Q) * 4;
  const int lim_end = (int)i1;
  auto step_lim = [&](int t) __attribute__((always_inline)) {
    const int l = (int)i0 + (t + 1) * 16;
    return l < lim_end ? l : lim_end;
  };
  // retire the prologue loads with a wait hipcc sees (vmcnt(0)): otherwise its waitcnt pass
  // merges their pending state into the loop header and waits for them inside the loop
  __builtin_amdgcn_s_waitcnt(0x0F70);
  if (n_t > 0) {
    f32x4v afA[LT], afB[LT];
    f32x4 accA[NG], accB[NG];
    load_item_tile<D>(ei, n_items, i0, voff, afA);
    load_item_tile<D>(ei, n_items, i0 + 16, voff, afB);
    mfma_tile(afA, accA);
    load_item_tile<D>(ei, n_items, i0 + 32, voff, afA);
    // invariant at step t: acc[t%2] = tile t; buffer (t+1)%2 = tile t+1 (landed or in
    // flight); buffer t%2 = tile t+2 in flight
    for (int t = 0;; t += 2) {
      // ---- even step: tile t in accA, tile t+1 in afB
      mfma_tile(afB, accB);
      bool hit = any_cand(accA);
      load_item_tile<D>(ei, n_items, i0 + (int64_t)(t + 3) * 16, voff, afB);
      if (hit) insert_tile(t, accA);
      maybe_compact(step_lim(t));
      if (t + 1 >= n_t) break;
      // ---- odd step: tile t+1 in accB, tile t+2 in afA
      mfma_tile(afA, accA);
      hit = any_cand(accB);
      load_item_tile<D>(ei, n_items, i0 + (int64_t)(t + 4) * 16, voff, afA);
      if (hit) insert_tile(t + 1, accB);
      maybe_compact(step_lim(t + 1));
      if (t + 2 >= n_t) break;
    }
  }

  // final lists
  wave_sync();
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    for (int u = 0; u < 16; ++u) {
      const int64_t user = ubase + g * 16 + u;
      if (user >= n_users) break;
      compact_user(g, u, lim_end);
      const int nc = __shfl(cnt[g], u);
      for (int e = lane; e < k; e += 64) {
        const float v = e < nc ? cs[wave][g][u][e] : neg_inf<float>();
        const int id = e < nc ? ci[wave][g][u][e] : -1;
        if (n_splits == 1) {
          out_val[user * k + e] = v;
          out_idx[user * k + e] = id;
        } else {
          const int64_t o = ((int64_t)split * n_users + user) * k + e;
          part_val[o] = v;
          part_idx[o] = id;
        }
      }
      wave_sync();
    }
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// the largest float below a finite x
__device__ __forceinline__ float next_below(float x) {
  const int32_t b = __builtin_bit_cast(int32_t, x);
  if (x == 0.f) return -__builtin_bit_cast(float, 1);  // (-0 as well)
  return __builtin_bit_cast(float, x > 0.f ? b - 1 : b + 1);
}

// a float at or below t - m (finite t and m: fl(t - m) moved one ulp down; t = +-inf stays; NaN
// m gives NaN)
__device__ __forceinline__ float thr_minus(float t, float m) {
  const float d = t - m;
  if (!(d > -__builtin_huge_valf() && d < __builtin_huge_valf())) return d;
  return next_below(d);
}

// K2r: the screened top-K (every k <= 128), with bound-side lists -- no exact score inside
// the streaming loop. A bf16 MFMA product (v_mfma_f32_16x16x32_bf16, 16x the f32 MFMA's rate)
// plus a rigorous per-user margin m_u (umarg, include/lgcnhs.h: |G_bf16 - G_chain| <= m_u for
// every item) bounds the exact fp32 chain score of k_score_topk from both sides.
//
// Every item i of user u has, from its bf16 product b = G_bf16(u, i), a lower bound
// LB = fl(b - m_u) and an upper bound UB = fl(b + m_u) of its exact chain score (nudged
// outward past the roundings; excluded items and already exact entries have LB = UB = their
// final value). A user's list holds (b, item) entries; at each compaction
// tau = the k-th largest LB of the list. Every list entry whose UB is below tau (or below the
// seed floor, below) can not be in the final top-k -- k items of lower id reach tau, which
// exceeds its exact score -- and is dropped; an item enters only if fl(b + m_u) > tau, for the
// same reason. Nothing else is dropped, so the final list holds every item of the exact
// top-k; at the end of the stream its entries get the exact fp32 chain (k_score_topk's MFMA
// chain, bit for bit), and the best k by (value desc, item asc) are the output -- identical to
// k_score_topk's. If a compaction leaves more entries than a tile could still add room for,
// the entries are made exact right there (the same chain) and the list cut to k.
// The loop thus issues no load but the fragment ring's DMA, and a hit costs an insertion
// instead of a global fp32 load round trip + a chain (round 4's exact-tile kernel kept ~70 %
// of its time in those). The cost: a few more entries per list -- those within 2 m_u of the k-th value --
// which the tight per-user margin keeps small (~k + 9 at C5, d = 64).
//
// The item fragments are shared by the block's waves through LDS, as the fragment ring
// described at the loop; lists live in LDS (CAP entries per user, M per lane).
// Seeded thresholds. In a streaming top-K most insertions happen early: k ln(N / k) of them
// over N items, three quarters within the first 1/16 of the range. So a first, screen-only pass
// (SEEDP) over the first 1/16 of the items keeps, per user, the largest LB of each of C classes
// of items (item index mod C, C = 16 x the tiles per ring chunk, at most 64), no insertions at
// all. If E_u of the user's excluded items lie in that range, the (K + E_u)-th largest class
// maximum s_u is a lower bound of the final K-th value: K + E_u distinct items reach it, at most
// E_u of them excluded (their final value is the mask value), so K scoring items of the
// catalog score >= s_u (no seed when K + E_u > C). The main pass never lets a user's entry
// threshold fall under the float below s_u (unless the mask value is above it: then an
// excluded item could rank, and everything enters). Several splits: each split's seed is
// valid on its own, the largest is kept.

// float <-> uint32 with the same order (NaN excluded by the callers)
__device__ __forceinline__ uint32_t ford(float f) {
  const uint32_t b = __builtin_bit_cast(uint32_t, f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float funord(uint32_t o) {
  return __builtin_bit_cast(float, (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// fl(b - m) nudged down past the subtraction's rounding (<= b - m exactly); fl(b + m) up
__device__ __forceinline__ float lbound(float b, float m) {
  const float d = b - m;
  return d - (fabsf(d) * 0x1p-22f + 1e-30f);
}
__device__ __forceinline__ float ubound(float b, float m) {
  const float e = b + m;
  return e + (fabsf(e) * 0x1p-22f + 1e-30f);
}

// List entries are 6 bytes: a 32-bit key and the item's 16-bit tile index in its split (so a
// split holds at most 2^20 items). The key is a float whose 6 low mantissa bits are replaced:
// bits 0-3 the item's row in its tile, bit 4 kExact (the key is the exact chain score, LB = UB
// up to the truncation), bit 5 kExcl (an excluded item: its final value is the mask value
// exactly). Clearing 6 low bits moves a float by < 64 ulp <= 2^-17 |key| (toward zero), which
// the bounds widen by: lbound_t / ubound_t below.
constexpr uint32_t kRowMask = 15u, kExact = 16u, kExcl = 32u, kLowBits = 63u;
constexpr int kTileBits = 16;  // tile index field: splits of at most 2^20 items
__device__ __forceinline__ float key_value(uint32_t kb) {
  return __builtin_bit_cast(float, kb & ~kLowBits);
}
__device__ __forceinline__ uint32_t key_pack(float v, uint32_t low) {
  return (__builtin_bit_cast(uint32_t, v) & ~kLowBits) | low;
}
// bounds of the true value from a truncated key v = key_value(kb): widened by |v| 2^-16 (> the
// truncation's 2^-17 |v| and the roundings of the sum)
__device__ __forceinline__ float lbound_t(float v, float m) {
  const float d = v - m;
  return d - (fabsf(d) * 0x1p-22f + fabsf(v) * 0x1p-16f + 1e-30f);
}
__device__ __forceinline__ float ubound_t(float v, float m) {
  const float e = v + m;
  return e + (fabsf(e) * 0x1p-22f + fabsf(v) * 0x1p-16f + 1e-30f);
}

#ifdef LG_TOPK_COUNT  // measurement builds only: event counts of k_topk_ring (lg_topk_counts)
__device__ unsigned long long g_topk_counts[16];
#define LG_COUNT(i, v) (cnt_ev[i] += (v))
// cycles of a phase: LG_CLK0(t) before it, LG_CLK1(i, t) after it (slot i)
#define LG_CLK0(t) const unsigned long long t = clock64()
#define LG_CLK1(i, t) (cnt_ev[i] += clock64() - (t))
#else
#define LG_COUNT(i, v) ((void)0)
#define LG_CLK0(t) ((void)0)
#define LG_CLK1(i, t) ((void)0)
#endif

// The ring kernel's shapes per list size (k <= 32 / <= 64 / <= 128): list capacity,
// fragment-ring buffers, chunks a wave issues ahead, chunks between a piece's issue and its
// arrival signal (measurement builds may override them: -DLG_RING_CAP=... etc.). LDS: lists
// users x CAP x 6 B + NBUF x 8 KiB + 2 KiB within 160 KiB.
#ifndef LG_RING_CAP
#define LG_RING_CAP 56
#endif
#ifndef LG_RING_LEAN  // the leaner ring check and chunk test (-DLG_RING_LEAN=0: round 5's)
#define LG_RING_LEAN 1  // (C5 k = 20: 9.05 -> 8.89 ms, k = 100: 16.85 -> 16.72 ms)
#endif
#ifndef LG_RING_NBUF
#define LG_RING_NBUF 9
#endif
#ifndef LG_RING_LA
#define LG_RING_LA 5
#endif
#ifndef LG_RING_LAG
#define LG_RING_LAG 1
#endif
#ifndef LG_RING2_CAP
#define LG_RING2_CAP 112
#endif
#ifndef LG_RING2_NBUF
#define LG_RING2_NBUF 9
#endif
#ifndef LG_RING4_CAP
#define LG_RING4_CAP 160
#endif
#ifndef LG_RING4_NBUF
#define LG_RING4_NBUF 4
#endif
#ifndef LG_RING4_LA
#define LG_RING4_LA 2
#endif
#ifndef LG_RING4_W  // waves (16 users each) per block at k <= 128
#define LG_RING4_W 8
#endif
// user groups per wave at k <= 32 (2: 8 waves, two per SIMD; 4: 4 waves, one per SIMD)
#ifndef LG_RING_NG
#define LG_RING_NG 2
#endif
#ifndef LG_RING_W  // waves per block at k <= 32 (default: 256 users per block)
#define LG_RING_W (16 / LG_RING_NG)
#endif

// the fragment ring's chunk: 8 KiB for 8 waves (64 items at d = 64), 4 or 8 KiB for 4; other
// wave counts (measurement shapes): the smallest multiple of one 16-byte piece per thread of
// >= 4 KiB that holds whole 16-item tiles
constexpr int ring_chunk_bytes(int D, int W) {
  if (W == 8 || W == 4) return D >= 64 || W >= 8 ? 8192 : 4096;
  for (int m = 1; m < 64; ++m) {
    const int cb = 1024 * W * m;
    if (cb >= 4096 && (cb / (2 * D)) % 16 == 0) return cb;
  }
  return 0;
}

template <int D, int NG, int WAVES, int M, int CAP, int NBUF, int LA, int LAG, bool SEEDP,
          bool GL = false>
__global__ __launch_bounds__(64 * WAVES) void k_topk_ring(
    const float *__restrict__ eu, const float *__restrict__ ei, const __bf16 *__restrict__ eub,
    const __bf16 *__restrict__ eib, const float *__restrict__ umarg, int64_t n_users,
    int64_t n_items, const int64_t *__restrict__ ex_rowptr,
    const int32_t *__restrict__ ex_col, float mask_value, int k, int n_splits,
    int64_t items_per_split, float *__restrict__ out_val, int64_t *__restrict__ out_idx,
    float *__restrict__ part_val, int32_t *__restrict__ part_idx,
    const float *__restrict__ seed_val, uint2 *__restrict__ gl_list) {
  // WAVES waves x NG groups of 16 users (the MFMA columns); a list of CAP entries per user, up
  // to M per lane (entry e = 64 j + lane in slab j). The host picks CAP > k + 16 (k <= 32: 256
  // users and CAP 56; k <= 64: 128 users and CAP 112; k <= 128: 128 users and CAP 160).
  // GL (global lists): each user's list is a slab of CAPG = 64 M entries {key, item} in global
  // memory (gl_list + (split n_users + user) CAPG, L2/MALL-resident), and the LDS holds only a
  // staging list of CAP (<= 64) entries per user in front of it: insertions go to the staging
  // list as above; one that could overflow on the next tile is spilled (appended to the slab:
  // one store per entry), and a slab that could not take the next spill is compacted (the same
  // compaction, on the slab). The LDS left over goes to the fragment ring, and the lists --
  // which hold k + the entries inside the margins -- compact every CAPG - k - CAP insertions
  // instead of every CAP - k - 16.
  static_assert(M == 1 || M == 2 || M == 4, "list slabs");
  static_assert(GL ? (CAP <= 64 && CAP > 16) : (CAP <= 64 * M && CAP > 32 * M), "list capacity");
  constexpr int CAPG = 64 * M;  // (GL: the slab's capacity)
  constexpr int Q = D / 4;   // f32 MFMA steps
  constexpr int S = D / 32;  // bf16 MFMA k-blocks
  // the fragment ring: chunks of CI items (CB bytes, PPT 16-byte LDS-DMA pieces per thread)
  constexpr int CB = ring_chunk_bytes(D, WAVES);
  constexpr int CI = CB / (2 * D), TPC = CI / 16, PR = D / 8, RB = 2 * D;
  constexpr int PPT = CB / 16 / (64 * WAVES);
  static_assert(PPT >= 1 && CI * PR == 64 * WAVES * PPT, "whole DMA pieces per thread");
  static_assert(LAG >= 1 && LA > LAG && NBUF > LA, "ring shape");
  // seed classes: 16 x the tiles per ring chunk (at most 4 of them: one class per lane); the
  // seed pass keeps the R largest lower bounds of each class (R = 4 for k > 32)
  constexpr int TPC_S = TPC < 4 ? TPC : 4;
  constexpr int NCLS = 16 * TPC_S;
  // (k <= 32: at least 64 candidates -- d = 128 has 32 classes; 2 per class at d = 64 measured
  // 9.21 vs 9.07 ms, at d = 128 13.96 vs 14.13 ms)
  constexpr int R = M == 1 ? (NCLS >= 64 ? 1 : 2) : 4;
  // the lists: keys and tile indices (6-byte entries, above)
  __shared__ uint32_t lk[WAVES][NG][16][SEEDP ? 1 : CAP];
  __shared__ uint16_t lt[WAVES][NG][16][SEEDP ? 1 : CAP];
  __shared__ int exs[WAVES][64];  // exclusion runs; the exact chain's results
  __shared__ __attribute__((aligned(16))) char frs[NBUF][CI * RB];
  __shared__ uint32_t prog[WAVES];  // the fragment ring's progress words (below)

  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int ul = lane & 15;
  const int gq = lane >> 4;
  const int64_t tile = blockIdx.x / n_splits;
  const int split = blockIdx.x % n_splits;
  const int64_t ubase = (tile * WAVES + wave) * (16 * NG);
  // (waves past the last user still stage their share of every chunk; their users are
  // invalid, so they never hit the screen and write nothing)
  const int64_t i0 = (int64_t)split * items_per_split;
  int64_t i1 = i0 + items_per_split;
  if (i1 > n_items) i1 = n_items;
  const int n_valid = i1 > i0 ? (int)(i1 - i0) : 0;
  const int n_t = (n_valid + 15) / 16;

  bf16x8 ub[NG][S];
  float marg[NG];
  bool uvalid[NG];
  int64_t ex_pos[NG], ex_hi[NG];
  int cnt[NG], chk[NG];
  int gcnt[NG];  // (GL) entries in the user's slab; chk: its count at the last compaction
  float thr[NG];
  // LG_RING_LEAN: the chunk test's threshold on the product itself, at or below thr - marg
  // (a product b with fl(b + m) > thr has b >= thr - m >= thrm; NaN margins give NaN: every
  // chunk hits), kept with thr
  float thrm[NG];
  float sthr[NG];  // the seeded floor of the threshold (-inf without a seed)
  // the entry threshold over a list's k-th lower bound tau and the seed floor st: an
  // excluded item ranks at the mask value, so while that reaches the floor anything enters
  auto entry_thr = [&](float tau, float st) __attribute__((always_inline)) {
    const float tf = fmaxf(tau, st);
    return mask_value > tf ? neg_inf<float>() : tf;
  };
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int64_t u = ubase + g * 16 + ul;
    uvalid[g] = u < n_users;
    const int64_t uu = uvalid[g] ? u : n_users - 1;
    sthr[g] = neg_inf<float>();
    if (seed_val && uvalid[g]) {  // (a non-finite seed -- NaN embeddings -- seeds nothing)
      const float sv = seed_val[u * k + k - 1];
      if (sv > neg_inf<float>() && sv < __builtin_huge_valf()) sthr[g] = next_below(sv);
    }
#pragma unroll
    for (int s = 0; s < S; ++s)
      ub[g][s] = *reinterpret_cast<const bf16x8 *>(eub + uu * D + 32 * s + 8 * gq);
    // A margin that is no bound (NaN, negative) becomes NaN: every bound of that user is NaN
    // and enters (the compares below are !(bound <= thr)), so the user's items all get the
    // exact chain -- k_score_topk's lists for any input. (+inf works as it is: every bound is
    // +inf or NaN.) Padding users take 0: their thr = +inf keeps them out of every list unless
    // a product itself is NaN (then the entry is harmless: exact_entries clamps the user and
    // padding lists are never written out).
    {
      const float mr = umarg[uu];
      marg[g] = !uvalid[g] ? 0.f : (mr >= 0.f ? mr : __builtin_nanf(""));
    }
    ex_pos[g] = 0;
    ex_hi[g] = 0;
    if (ex_rowptr && uvalid[g]) {
      ex_pos[g] = ex_rowptr[u];
      ex_hi[g] = ex_rowptr[u + 1];
    }
    cnt[g] = 0;
    chk[g] = 0;
    gcnt[g] = 0;
    thr[g] = uvalid[g] ? entry_thr(neg_inf<float>(), sthr[g]) : __builtin_huge_valf();
    thrm[g] = thr_minus(thr[g], marg[g]);
  }
  // (GL) the slab of user u of group g (valid users only: padding users never insert)
  auto gslab = [&](int g, int u) __attribute__((always_inline)) {
    return gl_list + ((int64_t)split * n_users + ubase + 16 * g + u) * CAPG;
  };
#ifdef LG_TOPK_COUNT
  // 0 inserted entries, 1 group-tiles with a hit, 2 compactions, 3 escapes (lists made exact
  // mid-stream), 4 exclusion-row loads, 5 entries ranked exactly at the end, 6 users finished;
  // cycles (clock64) in 8 ring waits, 9 screen + tests, 10 insertion, 11 compaction, 12 the
  // final ranking, 13 the whole wave
  unsigned long long cnt_ev[16] = {};
  LG_CLK0(t_all);
#endif
  const uint64_t same_user = 0x0001000100010001ull << ul;
  // retire the prologue loads with a wait hipcc sees (vmcnt(0)): otherwise its waitcnt pass
  // merges their pending state into the loop header, and the screen loop's waits for them
  // also drained the fragment ring's DMA issued at the chunk start
  __builtin_amdgcn_s_waitcnt(0x0F70);

  // The exact chain scores of the list entries of user `user` on the lanes in `want` (lane e:
  // entry e, item `item`): k_score_topk's f32 MFMA chain with 16 entries as the A rows and the
  // user in every B column, so column ul of the result is the chain of (user, entry) bit for
  // bit. One slab of a list per call (lane e: entry 64 j + e); results pass through exs (lane
  // e reads its own).
  auto exact_entries = [&](int64_t user, uint64_t want, int item) __attribute__((always_inline)) {
    float uf[Q];
    user = user < n_users ? user : n_users - 1;  // (callers pass valid users; a clamp is cheap)
    load_piece<Q>(eu + user * D + gq * Q, uf);
    constexpr int CS = !GL && CAP < 64 ? CAP : 64;     // entries of one slab
    constexpr int NB = CS / 16 + (CS % 16 ? 1 : 0);    // 16-entry batches
    constexpr int BL = D <= 64 ? 4 : 2;               // batches whose rows load together
#pragma unroll
    for (int b0 = 0; b0 < NB; b0 += BL) {
      float af[BL][Q];
#pragma unroll
      for (int b = 0; b < BL; ++b) {
        const int e = 16 * (b0 + b) + ul;
        const int it = __shfl(item, e < 64 ? e : 63);
        const bool w = b0 + b < NB && e < 64 && ((want >> e) & 1ull) && it >= 0 &&
                       it < n_items;
        load_piece<Q>(ei + (int64_t)(w ? it : 0) * D + gq * Q, af[b]);
      }
#pragma unroll
      for (int b = 0; b < BL; ++b) {
        if (b0 + b >= NB || ((want >> (16 * (b0 + b))) & 0xffffull) == 0) continue;  // (uniform)
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < Q; ++s)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[b][s], uf[s], acc, 0, 0, 0);
        // rows 4 gq + r of column ul: every column holds the same user
        if (ul == 0)
          *reinterpret_cast<f32x4 *>(&exs[wave][16 * (b0 + b) + 4 * gq]) = acc;
      }
    }
    wave_sync();
    const float raw = __builtin_bit_cast(float, exs[wave][lane]);
    wave_sync();
    return raw;
  };

  // Compaction of user u of group g (the whole wave; lane e holds entry e). (1) The lazy
  // exclusion of k_score_topk: the entries [chk, n) added since the last compaction lie in
  // [previous limit, lim) and the user's excluded items there are the next run of its sorted
  // exclusion row; an excluded entry takes the mask value as its final value. (2) tau = the
  // k-th largest LB (radix select over ballots); entries with UB below max(tau, seed floor)
  // go. (3) With `fin` (the end of the stream), or when more entries remain than leave room
  // for a tile, the rest get their exact chain scores: entries whose score is NaN or -inf go
  // (k_score_topk never inserts them), the others are sorted (value desc, item asc) and the
  // best k kept, all final. Returns, on lane e < k, the e-th output entry when fin.
  // (g is a run-time, wave-uniform group index: the loop has one compaction site, not one
  // per group and tile -- inlined copies made the kernel ~54 KB of code)
  // (an explicit conditional chain: a helper taking the array by reference kept the per-group
  // arrays in scratch memory -- private segment 128 B/lane -- instead of registers)
  static_assert(NG == 1 || NG == 2 || NG == 4, "gget's chains");
#define gget(a, g)                                                                              \
  (NG == 1   ? (a)[0]                                                                           \
   : NG == 2 ? ((g) ? (a)[1 % NG] : (a)[0])                                                     \
             : ((g) == 0 ? (a)[0] : (g) == 1 ? (a)[1 % NG] : (g) == 2 ? (a)[2 % NG] : (a)[3 % NG]))
  // (GL: the same on the user's slab, whose entries are {key, item}; the staging list is empty
  // then -- compactions follow the user's spill -- and the slab's stores are waited first)
  auto compact_user = [&](int g, int u, int lim, bool fin, float (&ov)[M], int (&oi)[M])
      __attribute__((always_inline)) {
    const int n = __shfl(GL ? gget(gcnt, g) : gget(cnt, g), u);
    const int c0 = __shfl(gget(chk, g), u);
    int64_t pos = __shfl(gget(ex_pos, g), u);
    const int64_t hi = __shfl(gget(ex_hi, g), u);
    const float m = __shfl(gget(marg, g), u), st = __shfl(gget(sthr, g), u);
    uint32_t *ks = &lk[wave][g][u][0];
    uint16_t *ts = &lt[wave][g][u][0];
    uint2 *slab = nullptr;
    if constexpr (GL) {
      slab = gslab(g, u);
      // the spills' and the last compaction's stores have completed (in L2) before the slab is
      // read, and the reads bypass the CU's L1 (agent-scope loads): the vector L1 may still
      // hold the slab's lines from the last compaction's reads
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bool have[M], excl[M], keep[M];
    float lb[M], hb[M];
    uint32_t kbits[M];
    int item[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int ej = 64 * j + lane;
      have[j] = ej < n;
      if constexpr (GL) {
        const uint64_t e =
            have[j] ? __hip_atomic_load(reinterpret_cast<uint64_t *>(slab + ej),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : 0ull;
        kbits[j] = (uint32_t)e;
        item[j] = (int)(uint32_t)(e >> 32);
      } else {
        kbits[j] = have[j] ? ks[ej] : 0u;
        const int tix = have[j] ? (int)ts[ej] : 0;
        item[j] = (int)i0 + (tix << 4) + (int)(kbits[j] & kRowMask);
      }
    }
    // the lazy exclusion of the entries [c0, n), in registers
    if (n > c0) {
      while (pos < hi) {
        const int64_t e = pos + lane;
        const int32_t x = e < hi ? ex_col[e] : 0x7fffffff;
        LG_COUNT(4, 1);
        const int nin = __popcll(__ballot(x < lim));  // ascending: a prefix of the lanes
        if (nin == 0) break;
        exs[wave][lane] = x;
        wave_sync();
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const int ej = 64 * j + lane;
          if (ej >= c0 && ej < n) {  // (entries since the last compaction: bound entries)
            int a = 0, b = nin;  // first index with exs[] >= item
            while (a < b) {
              const int mid = (a + b) >> 1;
              if (exs[wave][mid] < item[j]) a = mid + 1;
              else b = mid;
            }
            if (a < nin && exs[wave][a] == item[j])
              kbits[j] = key_pack(mask_value, (kbits[j] & kRowMask) | kExact | kExcl);
          }
        }
        wave_sync();
        pos += nin;
        if (nin < 64) break;
      }
    }
#pragma unroll
    for (int j = 0; j < M; ++j) {
      excl[j] = (kbits[j] & kExcl) != 0;
      const float v = key_value(kbits[j]), mj = (kbits[j] & kExact) ? 0.f : m;
      lb[j] = excl[j] ? mask_value : lbound_t(v, mj);
      hb[j] = excl[j] ? mask_value : ubound_t(v, mj);
      lb[j] = lb[j] == lb[j] ? lb[j] : neg_inf<float>();       // (NaN: no lower bound)
      hb[j] = hb[j] == hb[j] ? hb[j] : __builtin_huge_valf();  // (NaN: no upper bound)
    }
    float tau = neg_inf<float>();
    if (n >= k) {  // the k-th largest LB: greatest T with k entries at or above it
      uint32_t o[M];
#pragma unroll
      for (int j = 0; j < M; ++j) o[j] = ford(lb[j]);
      uint32_t T = 0u;
#pragma unroll 4
      for (int b = 31; b >= 0; --b) {
        const uint32_t c = T | (1u << b);
        int nc = 0;
#pragma unroll
        for (int j = 0; j < M; ++j) nc += __popcll(__ballot(have[j] && o[j] >= c));
        if (nc >= k) T = c;
      }
      tau = funord(T);
    }
    uint64_t kb[M];
    int nk = 0;
#pragma unroll
    for (int j = 0; j < M; ++j) {
      keep[j] = have[j] && hb[j] >= fmaxf(tau, st);
      kb[j] = __ballot(keep[j]);
      nk += __popcll(kb[j]);
    }
    wave_sync();  // (every lane has read its entries)
    LG_COUNT(2, fin ? 0 : 1);
    // escape (make the list exact) when more entries stay than room for a tile; for the
    // 4-slab lists (k <= 128) already at k + 30: their exact k-th value then bounds the next
    // insertions (k = 100 at C5: 31.2 -> 28.2 ms; k + 18 / 24 / 36: 32.3 / 28.4 / 28.7 ms; the
    // same for k <= 64 lists was slower). GL: when the slab could not take the next spill.
    // (Measurement builds: -DLG_RING_ESC=n escapes at > n.)
    constexpr int ROOM = GL ? CAPG - CAP : CAP - 16;
#ifdef LG_RING_ESC
    const int esc = LG_RING_ESC < ROOM ? LG_RING_ESC : ROOM;
#elif defined(LG_GL_ESC)  // (measurement builds: GL slabs escape at > k + LG_GL_ESC)
    const int esc = !GL ? (M == 4 && k + 30 < ROOM ? k + 30 : ROOM)
                        : (k + LG_GL_ESC < ROOM ? k + LG_GL_ESC : ROOM);
#else
    const int esc = !GL && M == 4 && k + 30 < ROOM ? k + 30 : ROOM;
#endif
    LG_COUNT(3, (!fin && nk > esc) ? 1 : 0);
    LG_COUNT(5, fin ? nk : 0);
    LG_COUNT(6, fin ? 1 : 0);
    if (fin || nk > esc) {
      float kk[M];
      int ii[M];
      int nok = 0;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const float raw = kb[j] ? exact_entries(ubase + g * 16 + u, kb[j], item[j]) : 0.f;
        const bool ok = keep[j] && raw == raw && raw > neg_inf<float>();
        kk[j] = ok ? (excl[j] ? mask_value : raw) : neg_inf<float>();
        ii[j] = ok ? item[j] : kPadId;
        nok += __popcll(__ballot(ok));
      }
      wave_bitonic_sort<float, M>(kk, ii);
      nk = nok < k ? nok : k;
      tau = neg_inf<float>();
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const int ej = 64 * j + lane;
        if (ej < nk && !fin) {  // (an exact score equal to the mask value may pass as excluded: the same)
          const int rel = ii[j] - (int)i0;
          const uint32_t key =
              key_pack(kk[j], (uint32_t)(rel & 15) | kExact | (kk[j] == mask_value ? kExcl : 0u));
          if constexpr (GL) {
            slab[ej] = make_uint2(key, (uint32_t)ii[j]);
          } else {
            ks[ej] = key;
            ts[ej] = (uint16_t)(rel >> 4);
          }
        }
        if (nk == k && j == ((k - 1) >> 6)) tau = __shfl(kk[j], (k - 1) & 63);  // (uniform)
        ov[j] = ej < nk ? kk[j] : neg_inf<float>();
        oi[j] = ej < nk ? ii[j] : -1;
      }
    } else {
      int base = 0;
#pragma unroll
      for (int j = 0; j < M; ++j) {
        if (keep[j]) {
          const int p = base + __popcll(kb[j] & lanemask_lt());
          if constexpr (GL) {
            slab[p] = make_uint2(kbits[j], (uint32_t)item[j]);
          } else {
            ks[p] = kbits[j];
            ts[p] = (uint16_t)((item[j] - (int)i0) >> 4);
          }
        }
        base += __popcll(kb[j]);
      }
    }
    wave_sync();
    const float nthr = entry_thr(tau, st);
#pragma unroll
    for (int j = 0; j < NG; ++j)
      if (j == g && ul == u) {
        if constexpr (GL) gcnt[j] = nk;
        else cnt[j] = nk;
        chk[j] = nk;
        ex_pos[j] = pos;
        thr[j] = uvalid[j] ? nthr : __builtin_huge_valf();
        thrm[j] = thr_minus(thr[j], marg[j]);
      }
  };
  // compact every list that could overflow on the next tile (+16 entries max per tile)
  // the lists holding more than `over` entries (bit 16 g + u)
  static_assert(NG <= 4, "16 NG list bits");
  auto lists_over = [&](int over) __attribute__((always_inline)) {
    uint64_t need = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g)
      need |= (__ballot(cnt[g] > over) & 0xffffull) << (16 * g);
    return need;
  };
  auto compact_one = [&](int b, int lim) __attribute__((always_inline)) {
    float ov[M];
    int oi[M];
    compact_user(b >> 4, b & 15, lim, false, ov, oi);
  };
  // (GL) append user u's staging list to its slab (lane e: entry e) and empty it
  auto spill_user = [&](int g, int u) __attribute__((always_inline)) {
    const int n = __shfl(gget(cnt, g), u);
    const int gc = __shfl(gget(gcnt, g), u);
    if (lane < n) {
      const uint32_t kb = lk[wave][g][u][lane];
      const int it = (int)i0 + ((int)lt[wave][g][u][lane] << 4) + (int)(kb & kRowMask);
      gslab(g, u)[gc + lane] = make_uint2(kb, (uint32_t)it);
    }
#pragma unroll
    for (int j = 0; j < NG; ++j)
      if (j == g && ul == u) {
        cnt[j] = 0;
        gcnt[j] = gc + n;
      }
  };
  auto compact_over = [&](int lim) __attribute__((always_inline)) {
    uint64_t need = lists_over(CAP - 16);
    wave_sync();
    if constexpr (GL) {
      uint64_t full = 0;  // slabs that could not take the next spill
      while (need) {
        const int b = __builtin_ctzll(need);
        need &= need - 1;
        spill_user(b >> 4, b & 15);
      }
      wave_sync();  // (the staging entries are read before the next insertions overwrite them)
#ifdef LG_GL_TRIG  // (measurement builds: compact once a slab holds more than k + LG_GL_TRIG)
      const int trig = k + LG_GL_TRIG < CAPG - CAP ? k + LG_GL_TRIG : CAPG - CAP;
#else
      const int trig = CAPG - CAP;
#endif
#pragma unroll
      for (int g = 0; g < NG; ++g)
        full |= (__ballot(gcnt[g] > trig) & 0xffffull) << (16 * g);
      while (full) {
        const int b = __builtin_ctzll(full);
        full &= full - 1;
        compact_one(b, lim);
      }
    } else {
      while (need) {
        const int b = __builtin_ctzll(need);
        need &= need - 1;
        compact_one(b, lim);
      }
    }
  };
  // insertion of group g's bf16 products accb of tile t (lane (ul, gq): items 4 gq + r of the
  // tile, user ul): every item whose upper bound beats the running threshold enters with its
  // product as the key
  auto insert_bound = [&](int t, int g, const f32x4 acc) __attribute__((always_inline)) {
    const int rel = t * 16 + gq * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // (a NaN bound -- a NaN product or margin -- enters: its exact chain decides)
      const bool cand = rel + r < n_valid && above(acc[r] + marg[g], thr[g]) &&
                        (!GL || uvalid[g]);  // (GL: padding users have no slab)
      const uint64_t bal = __ballot(cand);
      LG_COUNT(0, __popcll(bal));
      if (bal) {
        const int pos = cnt[g] + __popcll(bal & same_user & lanemask_lt());
        if (cand) {
          lk[wave][g][ul][pos] = key_pack(acc[r], (uint32_t)(4 * gq + r));
          lt[wave][g][ul][pos] = (uint16_t)t;
        }
        cnt[g] += __popcll(bal & same_user);
      }
    }
  };

  const int lim_end = (int)i1;
  // the seed pass's class maxima (SEEDP only)
  f32x4 cmax[NG][SEEDP ? TPC_S : 1][SEEDP ? R : 1];  // (per class, descending)
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int tt = 0; tt < (SEEDP ? TPC_S : 1); ++tt)
#pragma unroll
      for (int l = 0; l < (SEEDP ? R : 1); ++l)
        cmax[g][tt][l] = f32x4{neg_inf<float>(), neg_inf<float>(), neg_inf<float>(),
                               neg_inf<float>()};
  {
    // The block's waves share the bf16 item fragments through LDS: chunks of CI items (CB
    // bytes, PPT 16-byte LDS-DMA pieces per thread: global_load_lds_dwordx4, no VGPRs) in a
    // ring of NBUF buffers; the 16-byte pieces of row r stored XOR-swizzled by sw(r) through
    // the SOURCE address, so the fragment reads of any 16 consecutive lanes hit distinct banks
    // (the layout of csrc/gbound.hip).
    // No block barrier: the waves drift apart, coupled only through one progress word per wave
    // in LDS, prog[w] = consumed << 16 | landed (16-bit counts, compared with wrap-around: the
    // drift is < NBUF):
    //   landed:   chunks whose pieces from wave w have landed in LDS (its own vmcnt);
    //   consumed: chunks wave w has read into registers.
    // Wave w at chunk c: (1) once every wave has consumed chunk c + LA - NBUF, issue its pieces
    // of chunk c + LA into that chunk's buffer; (2) vmcnt: its pieces up to chunk c + LA - LAG
    // have landed; (3) once every wave's pieces of chunk c + 1 have landed, read that chunk
    // (software pipeline, below) and publish both counts. Each wave writes only its own word (a
    // plain LDS store from lane 0, no atomics) and checks all WAVES words with one lane-parallel
    // LDS read (lane j reads wave j's word), issued right after its publication so that its
    // latency hides behind the chunk's MFMAs; only a failed check spins (and re-reads). The LDS
    // serves each wave's operations in order, so a wave's fragment reads have been performed
    // before any wave can see its consumed count (and DMA into that buffer), and a DMA piece has
    // landed before the landed count that covers it is published. The slowest wave never
    // waits, so the ring cannot deadlock. The DMA is inline asm with no register outputs,
    // invisible to hipcc's waits (hipcc's own __builtin_amdgcn_global_load_lds puts vmcnt(0)
    // before every LDS read, as it cannot tell the ring's buffers apart); an untracked load
    // only makes hipcc's own vmcnt waits stricter (the counter retires in order).
    auto sw = [](int r) { return (r / (128 / D)) & (PR - 1); };
    // this thread's DMA source for chunk 0 (element offset), and the last chunk whose rows all
    // lie inside the table: past it the rows are clamped per lane (harmless reads)
    int64_t src0[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int p = 64 * WAVES * j + (int)threadIdx.x, r = p / PR;
      src0[j] = (i0 + r) * D + 8 * ((p % PR) ^ sw(r));
    }
    const int64_t c_full = (n_items - i0) / CI - 1;  // chunks c <= c_full need no clamp
    // buffer b (= c % NBUF) of chunk c
    auto dma = [&](int c, int b) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < PPT; ++j) {
        const __bf16 *src;
        if (c <= c_full) {  // (wave-uniform)
          src = eib + src0[j] + (int64_t)c * CI * D;
        } else {
          const int p = 64 * WAVES * j + (int)threadIdx.x, r = p / PR;
          int64_t it = i0 + (int64_t)c * CI + r;
          it = it < n_items ? it : n_items - 1;  // (past the split or the table)
          src = eib + it * D + 8 * ((p % PR) ^ sw(r));
        }
        const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(
            __attribute__((address_space(3))) char *)(frs[b] + 1024 * (WAVES * j + wave)));
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
      }
    };
    uint32_t landed = 0u, consumed = 0u;  // this wave's counts (wave-uniform)
    uint32_t pv_ = 0u;  // the last read of every wave's progress word (lane j: wave j)
    auto publish = [&]() __attribute__((always_inline)) {
      asm volatile("" ::: "memory");  // (after the reads / the vmcnt wait before it)
      if (lane == 0)
        __hip_atomic_store(&prog[wave], (consumed << 16) | (landed & 0xffffu), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto read_prog = [&]() __attribute__((always_inline)) {
      return __hip_atomic_load(&prog[lane < WAVES ? lane : 0], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // every wave's count (bits `sh`) has reached `need` (16-bit wrap-around)
    auto all_reached = [&](uint32_t v, uint32_t need, int sh) __attribute__((always_inline)) {
#if LG_RING_LEAN
      // (bit 15 of the 16-bit difference = not yet reached; the ballot masked by a constant
      // instead of a per-lane condition: one compare, no select)
      const uint64_t nr = __ballot((((v >> sh) - need) & 0x8000u) != 0u);
      return (nr & ((WAVES >= 64 ? 0ull : (1ull << WAVES)) - 1ull)) == 0;
#else
      const int16_t d = (int16_t)(uint16_t)(((v >> sh) - need) & 0xffffu);
      return __ballot(lane < WAVES && d < 0) == 0;
#endif
    };
    auto wait_reached = [&](uint32_t &v, uint32_t need, int sh) __attribute__((always_inline)) {
      while (!all_reached(v, need, sh)) {
        __builtin_amdgcn_s_sleep(1);
        v = read_prog();
      }
      asm volatile("" ::: "memory");
    };
    typedef bf16x8 Frags[TPC][S];
    typedef f32x4 Accs[TPC][NG];
    auto read_chunk = [&](int b, Frags &fr) __attribute__((always_inline)) {
      const char *fb = frs[b];
#pragma unroll
      for (int tt = 0; tt < TPC; ++tt) {
        const int r = 16 * tt + ul;
#pragma unroll
        for (int s = 0; s < S; ++s)
          fr[tt][s] =
              *reinterpret_cast<const bf16x8 *>(fb + r * RB + 16 * ((4 * s + gq) ^ sw(r)));
      }
    };
    auto mfma_chunk = [&](const Frags &fr, Accs &acc) __attribute__((always_inline)) {
#pragma unroll
      for (int tt = 0; tt < TPC; ++tt)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          acc[tt][g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < S; ++s)
            acc[tt][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[tt][s], ub[g][s],
                                                                acc[tt][g], 0, 0, 0);
        }
    };
    // The chunk's test: per group the largest product of the chunk plus the margin against
    // the threshold, one ballot per group; returns the groups (bits) with a possible entrant.
    // Tests run against the thresholds of that moment: never above the later ones (they only
    // rise). The maxima propagate NaN (v_maximum3), and !(bound <= thr) hits on a NaN bound: a
    // NaN product or margin sends its tile down the insertion path, where the item's own bound
    // decides (the same compare) and its exact chain ranks it.
    auto test_chunk = [&](const Accs &acc) __attribute__((always_inline)) {
      uint32_t gm = 0;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
#if LG_RING_LEAN
        // a linear chain folds two values per v_maximum3_f32 (the pairwise tree left one of
        // every other instruction's three inputs duplicated)
        float m = acc[0][g][0];
#pragma unroll
        for (int e = 1; e < 4 * TPC; ++e)
          m = __builtin_elementwise_maximum(m, acc[e / 4][g][e % 4]);
#else
        float m = max4(acc[0][g]);
#pragma unroll
        for (int tt = 1; tt < TPC; ++tt)
          m = __builtin_elementwise_maximum(
              m, __builtin_elementwise_maximum(
                     __builtin_elementwise_maximum(acc[tt][g][0], acc[tt][g][1]),
                     __builtin_elementwise_maximum(acc[tt][g][2], acc[tt][g][3])));
#endif
#if LG_RING_LEAN
        if (__ballot(!(m < thrm[g])) != 0) gm |= 1u << g;  // (thrm: below)
#else
        if (__ballot(above(m + marg[g], thr[g])) != 0) gm |= 1u << g;
#endif
      }
      return gm;
    };
    // the seed pass: each lane's R largest lower bounds per class (past the range: -inf),
    // class (item mod NCLS) = 16 (tt mod TPC_S) + 4 gq + r; a value enters the class's sorted
    // R slots by a max / min chain. A NaN lower bound (NaN product or margin) is no candidate:
    // fmaxf skips it for R = 1; for R > 1 it is made -inf first (the min of the chain would
    // otherwise carry the slot's value down as a duplicate candidate)
    auto seed_chunk = [&](int c, const Accs &acc) __attribute__((always_inline)) {
      const int t0 = c * TPC;
#pragma unroll
      for (int tt = 0; tt < TPC; ++tt) {
        const int rel = (t0 + tt) * 16 + gq * 4;
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = rel + r < n_valid ? lbound(acc[tt][g][r], marg[g]) : neg_inf<float>();
            if (R > 1) v = v == v ? v : neg_inf<float>();
#pragma unroll
            for (int l = 0; l < R; ++l) {
              const float h = cmax[g][tt % TPC_S][l][r];
              cmax[g][tt % TPC_S][l][r] = fmaxf(h, v);
              if (l + 1 < R) v = fminf(h, v);
            }
          }
      }
    };
    // chunk c's hit tiles (after its chunk test hit the groups gm): per-tile tests of those
    // groups, then the insertions in tile order; when a list could overflow on the next tile,
    // the lists are compacted (one code site) and the insertion resumes after that tile. The
    // products and the tile index pass an opaque (empty) asm inside each tile's insertion:
    // otherwise hipcc hoists the insertions' set-up -- bound sums, item ids, range tests, SGPR
    // spills -- out of the tile loop to the top of this path (~100 instructions per hit chunk).
    auto process_hits = [&](int c, const Accs &acc, uint32_t gm) __attribute__((always_inline)) {
      const int t0 = c * TPC;
      uint32_t hits = 0;  // bit tt * NG + g: group g's screen hit in tile tt (wave-uniform)
#pragma unroll
      for (int tt = 0; tt < TPC; ++tt)
#pragma unroll
        for (int g = 0; g < NG; ++g)
          if (((gm >> g) & 1u) && __ballot(above(max4(acc[tt][g]) + marg[g], thr[g])) != 0)
            hits |= 1u << (tt * NG + g);
      if (t0 + TPC > n_t) hits &= (1u << ((n_t - t0) * NG)) - 1u;  // (tiles past the split)
      int tt0 = 0;
      while (hits) {
        int stop = TPC;
#pragma unroll
        for (int tt = 0; tt < TPC; ++tt) {
          const uint32_t th = (hits >> (tt * NG)) & ((1u << NG) - 1u);
          if (tt < tt0 || stop != TPC || th == 0) continue;  // (wave-uniform)
          LG_COUNT(1, __popc(th));
          LG_CLK0(t_ins);
          int t = t0 + tt;
          asm volatile("" : "+s"(t));
#pragma unroll
          for (int g = 0; g < NG; ++g)
            if ((th >> g) & 1u) {
              f32x4 a = acc[tt][g];
              asm volatile("" : "+v"(a));
              insert_bound(t, g, a);
            }
          LG_CLK1(10, t_ins);
          bool over = false;
#pragma unroll
          for (int g = 0; g < NG; ++g) over |= cnt[g] > CAP - 16;
          if (__ballot(over) != 0) stop = tt;
        }
        if (stop == TPC) break;
        const int l = (int)i0 + (t0 + stop + 1) * 16;
        LG_CLK0(t_cmp);
        compact_over(l < lim_end ? l : lim_end);
        LG_CLK1(11, t_cmp);
        tt0 = stop + 1;
        hits &= ~((1u << (tt0 * NG)) - 1u);
      }
    };
    const int n_c = (n_t + TPC - 1) / TPC;  // (block-uniform)
    if (threadIdx.x < WAVES) prog[threadIdx.x] = 0u;
    __syncthreads();  // (the only block barrier)
    for (int c = 0; c < LA; ++c) dma(c, c);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LAG * PPT) : "memory");
    landed = LA - LAG;
    publish();
    pv_ = read_prog();
    int bc = 0, bn = LA;  // the buffers of chunks c and c + LA (running, no divisions)
    for (int c = 0; c < n_c; ++c) {
      LG_CLK0(t_ring);
      {
        const int cn = c + LA, cp = cn - NBUF;  // chunk cn replaces chunk cp in its buffer
        if (cp >= 0) wait_reached(pv_, (uint32_t)(cp + 1), 16);
        LG_CLK1(14, t_ring);
        LG_CLK0(t_dma);
        dma(cn, bn);  // (chunks past the split: harmless clamped reads, published like the rest)
        bn = bn + 1 == NBUF ? 0 : bn + 1;
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LAG * PPT) : "memory");
        landed = (uint32_t)(cn - LAG + 1);
        LG_CLK1(15, t_dma);
      }
      LG_CLK0(t_arr);
      wait_reached(pv_, (uint32_t)(c + 1), 0);
      LG_CLK1(7, t_arr);
      LG_CLK1(8, t_ring);
      LG_CLK0(t_scr);
      // The chunk's TPC tiles are screened together -- every fragment read, then every bf16
      // MFMA, then the test -- so the reads and the MFMA chains of different tiles overlap
      // instead of one tile's LDS -> MFMA -> compare chain at a time.
      Frags fr;
      Accs acc;
      read_chunk(bc, fr);
      bc = bc + 1 == NBUF ? 0 : bc + 1;
      mfma_chunk(fr, acc);
      // (the fragments are in registers: the buffer is free) -- published with this chunk's
      // landed count, and the next check's read issued right away
      consumed = (uint32_t)(c + 1);
      publish();
      pv_ = read_prog();
      if constexpr (SEEDP) {
        seed_chunk(c, acc);
        LG_CLK1(9, t_scr);
        continue;
      }
      uint32_t gm = test_chunk(acc);
      LG_CLK1(9, t_scr);
#ifdef LG_SCREEN_PROBE  // measurement builds only (wrong lists): the screen and its tests alone
      asm volatile("" ::"s"(gm));
      gm = 0;
#endif
      if (gm != 0) process_hits(c, acc, gm);  // (rare: one branch otherwise)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no DMA in flight at the exit)
  }

  wave_sync();
  if constexpr (SEEDP) {
    // per user: the (k + E)-th largest of its NCLS x R candidates -- distinct items' lower
    // bounds -- (E = its excluded items in this split's range, by two binary searches of its
    // sorted exclusion row), into the K-th slot of its output row; -inf when k + E > NCLS R.
    // All 16 users of a group at once: a radix select whose counts sum each lane's candidates
    // over the user's 4 lanes (gq) by two xor shuffles.
    constexpr int NV = TPC_S * R * 4;  // candidates per lane
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int64_t user = ubase + g * 16 + ul;
      int E = 0;
      if (ex_rowptr && user < n_users) {
        const int64_t e0 = ex_rowptr[user], e1 = ex_rowptr[user + 1];
        E = (int)(lower_bound_i32(ex_col, e0, e1, (int32_t)i1) -
                  lower_bound_i32(ex_col, e0, e1, (int32_t)i0));
      }
      const int need = k + E;
      uint32_t o[NV];
#pragma unroll
      for (int tt = 0; tt < TPC_S; ++tt)
#pragma unroll
        for (int l = 0; l < R; ++l)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = cmax[g][tt][l][r];
            o[(tt * R + l) * 4 + r] = ford(x);
          }
      uint32_t T = 0u;  // the greatest T with `need` candidates at or above it
#pragma unroll 1
      for (int b = 31; b >= 0; --b) {
        const uint32_t c = T | (1u << b);
        int n = 0;
#pragma unroll
        for (int j = 0; j < NV; ++j) n += o[j] >= c ? 1 : 0;
        n += __shfl_xor(n, 16);
        n += __shfl_xor(n, 32);
        if (n >= need) T = c;
      }
      const float sv = need <= NCLS * R ? funord(T) : neg_inf<float>();
      if (gq == 0 && user < n_users) {
        if (n_splits == 1) out_val[user * k + k - 1] = sv;
        else part_val[((int64_t)split * n_users + user) * k + k - 1] = sv;
      }
    }
    return;
  }
  LG_CLK0(t_fin);
#pragma unroll 1
  for (int b = 0; b < 16 * NG; ++b) {  // (user ubase + b = group b / 16, column b % 16)
    {
      const int64_t user = ubase + b;
      if (user >= n_users) break;
      float v[M];
      int id[M];
      if constexpr (GL) {  // the staging list's entries join the slab first
        if (__shfl(gget(cnt, b >> 4), b & 15) > 0) spill_user(b >> 4, b & 15);
      }
      compact_user(b >> 4, b & 15, lim_end, true, v, id);
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const int ej = 64 * j + lane;
        if (ej < k) {
          if (n_splits == 1) {
            out_val[user * k + ej] = v[j];
            out_idx[user * k + ej] = id[j];
          } else {
            const int64_t o = ((int64_t)split * n_users + user) * k + ej;
            part_val[o] = v[j];
            part_idx[o] = id[j];
          }
        }
      }
    }
  }
#ifdef LG_TOPK_COUNT
  LG_CLK1(12, t_fin);
  LG_CLK1(13, t_all);
  if (lane == 0)
    for (int i = 0; i < 16; ++i)
      if (cnt_ev[i]) __hip_atomic_fetch_add(&g_topk_counts[i], cnt_ev[i], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
#endif
}

#undef gget

// Merge n_splits partial lists (each sorted, item ranges ascending by split) per user.
template <int M>
__global__ __launch_bounds__(256) void k_topk_merge(const float *__restrict__ part_val,
                                                    const int32_t *__restrict__ part_idx,
                                                    int64_t n_users, int k, int n_splits,
                                                    float *__restrict__ out_val,
                                                    int64_t *__restrict__ out_idx) {
  constexpr int CAP = 64 * M;
  __shared__ float cs[4][CAP];
  __shared__ int ci[4][CAP];
  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int64_t user = (int64_t)blockIdx.x * 4 + wave;
  if (user >= n_users) return;
  int cnt = 0;
  float tau = neg_inf<float>();
  int tau_id = kPadId;
  for (int s = 0; s < n_splits; ++s) {
    const int64_t base = ((int64_t)s * n_users + user) * k;
    for (int e0 = 0; e0 < k; e0 += 64) {
      const int e = e0 + lane;
      float v = neg_inf<float>();
      int id = -1;
      if (e < k) {
        v = part_val[base + e];
        id = part_idx[base + e];
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
        cnt = wave_compact<float, M>(cs[wave], ci[wave], cnt, k, tau, tau_id);
      }
    }
  }
  wave_sync();
  const int nc = wave_compact<float, M>(cs[wave], ci[wave], cnt, k, tau, tau_id);
  for (int e = lane; e < k; e += 64) {
    out_val[user * k + e] = e < nc ? cs[wave][e] : neg_inf<float>();
    out_idx[user * k + e] = e < nc ? ci[wave][e] : -1;
  }
}

// Dense masked score tile writer: G[u][i] for a 16-user x 16-item MFMA tile per step.
template <int D>
__global__ __launch_bounds__(256) void k_score_dense(
    const float *__restrict__ eu, const float *__restrict__ ei, int64_t n_users,
    int64_t n_items, const int64_t *__restrict__ ex_rowptr,
    const int32_t *__restrict__ ex_col, float mask_value, float *__restrict__ G,
    int64_t ldg, int64_t items_per_block) {
  constexpr int Q = D / 4;
  const int wave = threadIdx.x / 64;
  const int lane = lane_id();
  const int ul = lane & 15;
  const int gq = lane >> 4;
  // blockIdx.x -> (user group of 64 users = 4 waves x 16, item chunk)
  const int64_t n_chunks = (n_items + items_per_block - 1) / items_per_block;
  const int64_t ugrp = blockIdx.x / n_chunks;
  const int64_t chunk = blockIdx.x % n_chunks;
  const int64_t u = ugrp * 64 + wave * 16 + ul;
  const bool uvalid = u < n_users;
  const int64_t uu = uvalid ? u : n_users - 1;
  if (ugrp * 64 + wave * 16 >= n_users) return;
  float uf[Q];
  load_piece<Q>(eu + uu * D + gq * Q, uf);
  const int64_t i0 = chunk * items_per_block;
  int64_t i1 = i0 + items_per_block;
  if (i1 > n_items) i1 = n_items;
  // exclusion pointer: this lane's items (it + 4gq + r) increase across tiles
  int64_t lo = 0, hi = 0;
  if (ex_rowptr && uvalid) {
    lo = ex_rowptr[u];
    hi = ex_rowptr[u + 1];
    lo = lower_bound_i32(ex_col, lo, hi, (int32_t)i0);
  }
  for (int64_t it = i0; it < i1; it += 16) {
    const int64_t item_l = it + ul;
    const int64_t itc = item_l < n_items ? item_l : n_items - 1;
    float af[Q];
    load_piece<Q>(ei + itc * D + gq * Q, af);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < Q; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], uf[s], acc, 0, 0, 0);
    if (uvalid) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t item = it + gq * 4 + r;
      v[r] = acc[r];
      while (lo < hi && ex_col[lo] < (int32_t)item) ++lo;
      if (lo < hi && ex_col[lo] == (int32_t)item) v[r] = mask_value;
    }
    const int64_t c0 = it + gq * 4;
    float *row = G + u * ldg;
    if (c0 + 3 < i1 && ((ldg & 3) == 0)) {
      *reinterpret_cast<float4 *>(row + c0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (c0 + r < i1) row[c0 + r] = v[r];
    }
    }
  }
}

// Measurement knob, compiled in only with -DLG_TOPK_PROBE (make EXTRA=-DLG_TOPK_PROBE):
// LGCNHS_TOPK_PROBE=1 times the scoring loop with no candidate insertion, =2 drops the
// exclusion sets. Results are wrong under a probe; the product build always passes 0.
#ifdef LG_TOPK_PROBE
static int topk_probe() {
  const char *e = getenv("LGCNHS_TOPK_PROBE");
  return e ? atoi(e) : 0;
}
#else
static int topk_probe() { return 0; }
#endif
// seeded thresholds in the screened top-K (measurement builds may turn them off:
// -DLG_TOPK_SEED=0)
#ifndef LG_TOPK_SEED
#define LG_TOPK_SEED 1
#endif
static bool lg_topk_seeding() { return LG_TOPK_SEED != 0; }
#ifndef LG_TOPK_SEED_DIV  // the seed pass covers the first 1/LG_TOPK_SEED_DIV of the items
#define LG_TOPK_SEED_DIV 16
#endif
#ifndef LG_TOPK_SEED_DIV_HI  // ... for k > 32
#define LG_TOPK_SEED_DIV_HI 16
#endif

template <int D, int NG, int M, int WAVES>
static void launch_topk(const float *eu, const float *ei, int64_t n_users, int64_t n_items,
                        const int64_t *ex_rowptr, const int32_t *ex_col, float mask_value,
                        int k, int n_splits, int64_t items_per_split, float *out_val,
                        int64_t *out_idx, float *part_val, int32_t *part_idx,
                        hipStream_t stream) {
  const int64_t users_per_block = (int64_t)WAVES * NG * 16;
  const int64_t tiles = (n_users + users_per_block - 1) / users_per_block;
  k_score_topk<D, NG, M, WAVES><<<dim3((unsigned)(tiles * n_splits)), dim3(64 * WAVES), 0,
                                  stream>>>(eu, ei, n_users, n_items, ex_rowptr, ex_col,
                                            mask_value, k, n_splits, items_per_split,
                                            out_val, out_idx, part_val, part_idx,
                                            topk_probe());
}

template <int D>
static void dispatch_topk(int M, const float *eu, const float *ei, int64_t n_users,
                          int64_t n_items, const int64_t *ex_rowptr, const int32_t *ex_col,
                          float mask_value, int k, int n_splits, int64_t items_per_split,
                          float *out_val, int64_t *out_idx, float *part_val,
                          int32_t *part_idx, hipStream_t stream) {
  // LDS per block: WAVES * NG * 16 * CAP * 8 B = 64 KiB (+256 B per wave) in every
  // configuration: two blocks per CU.
  if (M == 1)
    launch_topk<D, 2, 1, 4>(eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, k,
                            n_splits, items_per_split, out_val, out_idx, part_val, part_idx,
                            stream);
  else if (M == 2)
    launch_topk<D, 2, 2, 2>(eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, k,
                            n_splits, items_per_split, out_val, out_idx, part_val, part_idx,
                            stream);
  else
    launch_topk<D, 1, 4, 2>(eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, k,
                            n_splits, items_per_split, out_val, out_idx, part_val, part_idx,
                            stream);
}

// the seed pass's per-split seeds (slot K - 1 of each partial row): the largest of them
__global__ __launch_bounds__(256) void k_seed_combine(const float *__restrict__ part_val,
                                                      int64_t n_users, int k, int n_splits,
                                                      float *__restrict__ out_val) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_users) return;
  float m = neg_inf<float>();
  for (int p = 0; p < n_splits; ++p) {
    const float v = part_val[((int64_t)p * n_users + u) * k + k - 1];
    m = v > m ? v : m;  // (a NaN seeds nothing)
  }
  out_val[u * k + k - 1] = m;
}

// Global-list (GL) shapes: 8 waves x 2 groups (256 users per block), staging lists of
// LG_GL_CAP entries (48 KiB at 32), LG_GL_NBUF ring buffers issued LG_GL_LA chunks ahead. The
// product uses them for k > 32 (slabs of 128 / 256 entries); k <= 32 keeps the LDS lists
// unless built with -DLG_TOPK_GL32=1 (slabs of 128). -DLG_TOPK_LDS_LISTS=1 restores the LDS
// lists for every k (measurement builds).
#ifndef LG_GL_CAP
#define LG_GL_CAP 32
#endif
#ifndef LG_GL_NBUF
#define LG_GL_NBUF 13
#endif
#ifndef LG_GL_LA
#define LG_GL_LA 7
#endif
#ifndef LG_TOPK_GL32
#define LG_TOPK_GL32 0
#endif
#ifndef LG_SEED4_NG  // the k > 32 seed pass's shape
#define LG_SEED4_NG 1
#endif
#ifndef LG_SEED4_NBUF
#define LG_SEED4_NBUF 9
#endif
#ifndef LG_SEED4_LA
#define LG_SEED4_LA 5
#endif
// one user group per wave for the 4-slab GL shape at d <= 64 (k > 64: 128 users per block,
// one split at C5): k = 100 16.9 -> 16.1 ms, k = 128 18.8 -> 17.6 ms; k = 50 / 64 keep 2 groups
// (13.1 / 14.9 ms with 1 against 12.4 / 14.6; scripts/gpu_r06_glng.sh)
#ifndef LG_GL4_NG
#define LG_GL4_NG 1
#endif
#ifndef LG_GL_NG  // user groups per wave in the GL shapes (4: 512 users per block)
#define LG_GL_NG 2
#endif
#ifndef LG_TOPK_LDS_LISTS
#define LG_TOPK_LDS_LISTS 0
#endif
// the list slabs (uint2 entries per user) of the screened kernel's main pass at this k
static int screen_slab_m(int k) {
  if (LG_TOPK_LDS_LISTS) return 0;
  if (k <= 32) return LG_TOPK_GL32 ? 2 : 0;
  return k <= 64 ? 2 : 4;
}

template <int D>
static void dispatch_topk_screen(int M, bool seedp, const float *eu, const float *ei,
                                 const __bf16 *eub, const __bf16 *eib, const float *umarg,
                                 int64_t n_users, int64_t n_items, const int64_t *ex_rowptr,
                                 const int32_t *ex_col, float mask_value, int k, int n_splits,
                                 int64_t items_per_split, float *out_val, int64_t *out_idx,
                                 float *part_val, int32_t *part_idx, const float *seed_val,
                                 uint2 *gl_list, hipStream_t stream) {
  // one block per CU: the lists (6-byte entries) + the fragment ring. k <= 32: 256 users of
  // CAP 56 (84 KiB) + 9 ring buffers; k <= 64: 128 users (8 waves x 1 group) of CAP 112
  // (84 KiB) + 9 buffers; k <= 128: 128 users of CAP 160 (120 KiB) + 4 buffers. GL (the main
  // pass at k > 32): 256 users of staging lists + LG_GL_NBUF buffers, lists in gl_list.
#define LG_RING_LAUNCH(NG, W, MM, CAP, NBUF, LA, LAG, SEEDP, GLM)                             \
  {                                                                                           \
    const int64_t upb = (int64_t)(W) * (NG) * 16;                                             \
    const int64_t tiles = (n_users + upb - 1) / upb;                                          \
    k_topk_ring<D, NG, W, MM, CAP, NBUF, LA, LAG, SEEDP, GLM>                                 \
        <<<dim3((unsigned)(tiles * n_splits)), dim3(64 * (W)), 0, stream>>>(                  \
            eu, ei, eub, eib, umarg, n_users, n_items, ex_rowptr, ex_col, mask_value, k,      \
            n_splits, items_per_split, out_val, out_idx, part_val, part_idx, seed_val,        \
            gl_list);                                                                         \
  }
  const int gm = seedp ? 0 : screen_slab_m(k);
  if (gm == 2) {
    LG_RING_LAUNCH(LG_GL_NG, 8, 2, LG_GL_CAP, LG_GL_NBUF, LG_GL_LA, 1, false, true)
  } else if (gm == 4) {
    LG_RING_LAUNCH((D <= 64 ? LG_GL4_NG : LG_GL_NG), 8, 4, LG_GL_CAP, LG_GL_NBUF, LG_GL_LA, 1,
                   false, true)
  } else if (M == 1 && seedp) {
    LG_RING_LAUNCH(LG_RING_NG, LG_RING_W, 1, LG_RING_CAP, LG_RING_NBUF, LG_RING_LA,
                   LG_RING_LAG, true, false)
  } else if (M == 1) {
    LG_RING_LAUNCH(LG_RING_NG, LG_RING_W, 1, LG_RING_CAP, LG_RING_NBUF, LG_RING_LA,
                   LG_RING_LAG, false, false)
  } else if (M == 2 && seedp) {
    LG_RING_LAUNCH(1, 8, 2, LG_RING2_CAP, LG_RING2_NBUF, LG_RING_LA, LG_RING_LAG, true, false)
  } else if (M == 2) {
    if (LG_TOPK_LDS_LISTS)
      LG_RING_LAUNCH(1, 8, 2, LG_RING2_CAP, LG_RING2_NBUF, LG_RING_LA, LG_RING_LAG, false, false)
  } else if (seedp) {
    // (k > 32: the seed pass keeps no lists, so its ring takes the LDS the lists would)
    LG_RING_LAUNCH(LG_SEED4_NG, 8, 4, 160, LG_SEED4_NBUF, LG_SEED4_LA, 1, true, false)
  } else if constexpr (D > 64) {  // (the LG_RING4_* shapes apply to d <= 64)
    if (LG_TOPK_LDS_LISTS) LG_RING_LAUNCH(1, 8, 4, 160, 4, 2, 1, false, false)
  } else {
    if (LG_TOPK_LDS_LISTS)
      LG_RING_LAUNCH(1, LG_RING4_W, 4, LG_RING4_CAP, LG_RING4_NBUF, LG_RING4_LA, 1, false, false)
  }
#undef LG_RING_LAUNCH
}

static int cap_m(int k) { return k <= 32 ? 1 : (k <= 64 ? 2 : 4); }

// the screened call's workspace: partial lists (several splits) and the GL list slabs
static size_t screened_part_bytes(int64_t n_users, int k, int ns) {
  return ns > 1 ? (size_t)ns * (size_t)n_users * (size_t)k * (sizeof(float) + sizeof(int32_t))
                : 0;
}
static size_t screened_slab_bytes(int64_t n_users, int k, int ns) {
  return (size_t)ns * (size_t)n_users * 64 * (size_t)screen_slab_m(k) * sizeof(uint2);
}

static int64_t split_len(int64_t n_items, int n_splits) {
  int64_t per = (n_items + n_splits - 1) / n_splits;
  per = (per + 15) / 16 * 16;
  return per < 16 ? 16 : per;
}

// the screened kernel's splits: at least one per 2^20 items (k_topk_ring's 16-bit tile
// indices); split_len of it is then <= 2^20 (a multiple of 16)
static int screened_splits(int64_t n_items, int n_splits) {
  const int64_t need = (n_items + ((int64_t)1 << (kTileBits + 4)) - 1) >> (kTileBits + 4);
  return n_splits > need ? n_splits : (int)need;
}

}  // namespace lg

using namespace lg;

extern "C" size_t lg_score_topk_ws_bytes(int64_t n_users, int64_t n_items, int32_t dim,
                                         int32_t k, int32_t n_splits) {
  (void)dim;
  // (either kernel: the screened one splits catalogs of more than 2^20 items at least)
  if (n_items > 0 && n_splits >= 1) n_splits = screened_splits(n_items, n_splits);
  if (n_splits <= 1 || n_users <= 0 || k <= 0) return 0;
  return (size_t)n_splits * (size_t)n_users * (size_t)k * (sizeof(float) + sizeof(int32_t));
}

extern "C" size_t lg_score_topk_screened_ws_bytes(int64_t n_users, int64_t n_items,
                                                  int32_t dim, int32_t k, int32_t n_splits) {
  (void)dim;
  if (n_users <= 0 || n_items <= 0 || n_items >= 0x7fffffff || k < 1 || k > 128 ||
      n_splits < 1)
    return 0;
  const int64_t per = split_len(n_items, screened_splits(n_items, n_splits));
  const int ns = (int)((n_items + per - 1) / per);
  return screened_part_bytes(n_users, k, ns) + screened_slab_bytes(n_users, k, ns);
}

extern "C" int lg_score_topk_f32(const float *eu, const float *ei, int64_t n_users,
                                 int64_t n_items, int32_t dim, const int64_t *ex_rowptr,
                                 const int32_t *ex_col, float mask_value, int32_t k,
                                 int32_t n_splits, float *out_val, int64_t *out_idx,
                                 void *ws, size_t ws_bytes, lg_stream_t stream) {
  LG_REQUIRE(eu && ei && out_val && out_idx, "lg_score_topk_f32: null pointer");
  LG_REQUIRE(n_users >= 0 && n_items > 0 && n_items < 0x7fffffff,
             "lg_score_topk_f32: n_items must be in [1, 2^31-1)");
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128, "lg_score_topk_f32: dim %d not in {32,64,128}",
             dim);
  LG_REQUIRE(k >= 1 && k <= 128, "lg_score_topk_f32: k=%d not in [1,128]", k);
  LG_REQUIRE(n_splits >= 1 && n_splits <= 4096, "lg_score_topk_f32: bad n_splits %d", n_splits);
  LG_REQUIRE(!ex_rowptr == !ex_col, "lg_score_topk_f32: ex_rowptr/ex_col must both be set");
  if (n_users == 0) return LG_OK;
  const int64_t per = split_len(n_items, n_splits);
  const int ns = (int)((n_items + per - 1) / per);
  float *part_val = nullptr;
  int32_t *part_idx = nullptr;
  if (ns > 1) {
    const size_t need = lg_score_topk_ws_bytes(n_users, n_items, dim, k, ns);
    if (!ws || ws_bytes < need) {
      set_error("lg_score_topk_f32: workspace %zu < %zu bytes", ws_bytes, need);
      return LG_ERR_WORKSPACE;
    }
    part_val = (float *)ws;
    part_idx = (int32_t *)((char *)ws + (size_t)ns * n_users * k * sizeof(float));
  }
  hipStream_t s = (hipStream_t)stream;
  const int M = cap_m(k);
  if (topk_probe() == 2) ex_rowptr = nullptr, ex_col = nullptr;
  switch (dim) {
    case 32: dispatch_topk<32>(M, eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, k, ns, per, out_val, out_idx, part_val, part_idx, s); break;
    case 64: dispatch_topk<64>(M, eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, k, ns, per, out_val, out_idx, part_val, part_idx, s); break;
    default: dispatch_topk<128>(M, eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, k, ns, per, out_val, out_idx, part_val, part_idx, s); break;
  }
  int st = launch_status("lg_score_topk_f32");
  if (st != LG_OK || ns == 1) return st;
  const unsigned blocks = (unsigned)((n_users + 3) / 4);
  if (k <= 64)
    k_topk_merge<2><<<dim3(blocks), dim3(256), 0, s>>>(part_val, part_idx, n_users, k, ns,
                                                        out_val, out_idx);
  else
    k_topk_merge<4><<<dim3(blocks), dim3(256), 0, s>>>(part_val, part_idx, n_users, k, ns,
                                                        out_val, out_idx);
  return launch_status("lg_score_topk_f32(merge)");
}

extern "C" int lg_score_topk_screened_f32(const float *eu, const float *ei, const void *eu_bf16,
                                          const void *ei_bf16, const float *umarg,
                                          int64_t n_users, int64_t n_items, int32_t dim,
                                          const int64_t *ex_rowptr, const int32_t *ex_col,
                                          float mask_value, int32_t k, int32_t n_splits,
                                          float *out_val, int64_t *out_idx, void *ws,
                                          size_t ws_bytes, lg_stream_t stream) {
  LG_REQUIRE(eu && ei && eu_bf16 && ei_bf16 && umarg && out_val && out_idx,
             "lg_score_topk_screened_f32: null pointer");
  LG_REQUIRE(n_users >= 0 && n_items > 0 && n_items < 0x7fffffff,
             "lg_score_topk_screened_f32: n_items must be in [1, 2^31-1)");
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128,
             "lg_score_topk_screened_f32: dim %d not in {32,64,128}", dim);
  LG_REQUIRE(k >= 1 && k <= 128, "lg_score_topk_screened_f32: k=%d not in [1,128]", k);
  LG_REQUIRE(n_splits >= 1 && n_splits <= 4096, "lg_score_topk_screened_f32: bad n_splits %d",
             n_splits);
  LG_REQUIRE(!ex_rowptr == !ex_col,
             "lg_score_topk_screened_f32: ex_rowptr/ex_col must both be set");
  LG_REQUIRE(((uintptr_t)eu_bf16 & 15) == 0 && ((uintptr_t)ei_bf16 & 15) == 0,
             "lg_score_topk_screened_f32: bf16 copies must be 16-byte aligned");
  if (n_users == 0) return LG_OK;
  // (the lists' 16-bit tile indices: splits of at most 2^20 items)
  const int64_t per = split_len(n_items, screened_splits(n_items, n_splits));
  const int ns = (int)((n_items + per - 1) / per);
  float *part_val = nullptr;
  int32_t *part_idx = nullptr;
  uint2 *gl_list = nullptr;
  {
    const size_t part = screened_part_bytes(n_users, k, ns);
    const size_t need = part + screened_slab_bytes(n_users, k, ns);
    if (need > 0 && (!ws || ws_bytes < need)) {
      set_error("lg_score_topk_screened_f32: workspace %zu < %zu bytes", ws_bytes, need);
      return LG_ERR_WORKSPACE;
    }
    if (ns > 1) {
      part_val = (float *)ws;
      part_idx = (int32_t *)((char *)ws + (size_t)ns * n_users * k * sizeof(float));
    }
    if (screen_slab_m(k)) gl_list = (uint2 *)((char *)ws + part);
  }
  hipStream_t s = (hipStream_t)stream;
  const int M = cap_m(k);
  const __bf16 *ub = (const __bf16 *)eu_bf16, *ib = (const __bf16 *)ei_bf16;
  auto pass = [&](bool seedp, int64_t n_it, int nsp, int64_t per_sp, const float *seed) {
    switch (dim) {
      case 32: dispatch_topk_screen<32>(M, seedp, eu, ei, ub, ib, umarg, n_users, n_it, ex_rowptr, ex_col, mask_value, k, nsp, per_sp, out_val, out_idx, part_val, part_idx, seed, gl_list, s); break;
      case 64: dispatch_topk_screen<64>(M, seedp, eu, ei, ub, ib, umarg, n_users, n_it, ex_rowptr, ex_col, mask_value, k, nsp, per_sp, out_val, out_idx, part_val, part_idx, seed, gl_list, s); break;
      default: dispatch_topk_screen<128>(M, seedp, eu, ei, ub, ib, umarg, n_users, n_it, ex_rowptr, ex_col, mask_value, k, nsp, per_sp, out_val, out_idx, part_val, part_idx, seed, gl_list, s); break;
    }
    int st = launch_status("lg_score_topk_screened_f32");
    if (st != LG_OK || nsp == 1) return st;
    if (seedp) {  // the splits' seeds: the largest, into the K-th slot of each output row
      k_seed_combine<<<dim3((unsigned)((n_users + 255) / 256)), dim3(256), 0, s>>>(
          part_val, n_users, k, nsp, out_val);
      return launch_status("lg_score_topk_screened_f32(seeds)");
    }
    const unsigned blocks = (unsigned)((n_users + 3) / 4);
    if (k <= 64)
      k_topk_merge<2><<<dim3(blocks), dim3(256), 0, s>>>(part_val, part_idx, n_users, k, nsp,
                                                          out_val, out_idx);
    else
      k_topk_merge<4><<<dim3(blocks), dim3(256), 0, s>>>(part_val, part_idx, n_users, k, nsp,
                                                          out_val, out_idx);
    return launch_status("lg_score_topk_screened_f32(merge)");
  };
  // the seed pass (large catalogs): the screen-only lower-bound class maxima (the R largest per
  // class for k > 32) over the first 1/16 of the items, each user's seed into the K-th slot of its out_val row (the main
  // pass reads it there before it writes anything: a user's seed and its list belong to the
  // same wave), on at most as many splits as the main pass (their seeds fit the same
  // workspace; the largest is kept)
  const int64_t n_seed = n_items / (k > 32 ? LG_TOPK_SEED_DIV_HI : LG_TOPK_SEED_DIV) / 16 * 16;
  const bool seeded = lg_topk_seeding() && n_seed >= (int64_t)k * 64;
  if (seeded) {
    const int64_t per_s = split_len(n_seed, ns);
    const int ns_s = (int)((n_seed + per_s - 1) / per_s);
    const int st = pass(true, n_seed, ns_s, per_s, nullptr);
    if (st != LG_OK) return st;
  }
  return pass(false, n_items, ns, per, seeded ? out_val : nullptr);
}

extern "C" int lg_score_dense_f32(const float *eu, const float *ei, int64_t n_users,
                                  int64_t n_items, int32_t dim, const int64_t *ex_rowptr,
                                  const int32_t *ex_col, float mask_value, float *G,
                                  int64_t ldg, lg_stream_t stream) {
  LG_REQUIRE(eu && ei && G, "lg_score_dense_f32: null pointer");
  LG_REQUIRE(n_users >= 0 && n_items >= 0 && n_items < 0x7fffffff && ldg >= n_items,
             "lg_score_dense_f32: bad sizes");
  LG_REQUIRE(dim == 32 || dim == 64 || dim == 128, "lg_score_dense_f32: dim %d not in {32,64,128}",
             dim);
  LG_REQUIRE(!ex_rowptr == !ex_col, "lg_score_dense_f32: ex_rowptr/ex_col must both be set");
  if (n_users == 0 || n_items == 0) return LG_OK;
  const int64_t ipb = 1024;
  const int64_t chunks = (n_items + ipb - 1) / ipb;
  const int64_t ugrps = (n_users + 63) / 64;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)(ugrps * chunks)), block(256);
  switch (dim) {
    case 32: k_score_dense<32><<<grid, block, 0, s>>>(eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, G, ldg, ipb); break;
    case 64: k_score_dense<64><<<grid, block, 0, s>>>(eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, G, ldg, ipb); break;
    default: k_score_dense<128><<<grid, block, 0, s>>>(eu, ei, n_users, n_items, ex_rowptr, ex_col, mask_value, G, ldg, ipb); break;
  }
  return launch_status("lg_score_dense_f32");
}

#ifdef LG_TOPK_COUNT
// measurement builds only: read and clear k_topk_ring's event counts (16 x uint64, host)
extern "C" int lg_topk_counts(unsigned long long *host16) {
  if (hipDeviceSynchronize() != hipSuccess) return LG_ERR_HIP;
  if (hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_topk_counts), 128) != hipSuccess) return LG_ERR_HIP;
  const unsigned long long z[16] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_topk_counts), z, 128) != hipSuccess) return LG_ERR_HIP;
  return LG_OK;
}
#endif
