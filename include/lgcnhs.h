/*
 * lgcnhs.h — C ABI of the MI355X (gfx950) hot path for LGCNHS
 * (Light Graph Convolutional Recommendation based on Hybrid Spreading).
 *
 * Every entry point replaces one piece of arithmetic that the reference runs inside
 * third-party kernels (PyG 2.6.1, torch 1.13.1, numpy 1.24.3/MKL). The reference has no
 * FFI of its own (it is pure Python), so the "binding" a maintainer adds is the ctypes
 * stub shown in INTEGRATION.md; the reference call site each function replaces is cited
 * on the function.
 *
 * Conventions (all functions):
 *   - Plain device pointers, sizes and a stream. No allocation, no free, no host sync:
 *     the caller owns every buffer; work is enqueued on `stream` (a hipStream_t, NULL =
 *     the default stream). Safe to capture into a hipGraph.
 *   - Return LG_OK (0) or an LG_ERR_* code; lg_last_error() gives a thread-local message.
 *     Nothing is thrown across the ABI.
 *   - Graph rows are CSR: int64 rowptr[n_rows+1] (absolute offsets), int32 column ids,
 *     columns ascending inside a row (the order of the reference's coalesced COO,
 *     utils/graph.py:32-33). Node ids cover users then items (items offset by U).
 *   - Embeddings are row-major fp32 [n, dim]; spreading matrices are row-major fp64.
 *   - Top-K output is sorted by (value desc, index asc); unused slots hold index -1.
 */
#ifndef LGCNHS_H
#define LGCNHS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *lg_stream_t; /* hipStream_t */

enum lg_status {
  LG_OK = 0,
  LG_ERR_ARG = 1,         /* bad size / null pointer / unsupported dim or k */
  LG_ERR_HIP = 2,         /* a HIP runtime call failed (launch error) */
  LG_ERR_WORKSPACE = 3,   /* workspace smaller than the *_ws_bytes() answer */
};

/* ABI version of this header (bumped on any signature change). */
#define LG_ABI_VERSION 15
int lg_abi_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char *lg_last_error(void);

/* ------------------------------------------------------------------------------------
 * Graph format and normalisation
 * ------------------------------------------------------------------------------------ */

/* rowptr[r] = lower_bound(keys, r) for r in [0, n_rows]; `keys` = the row id of each of
 * `nnz` entries, sorted ascending. Replaces the dense (U+I)^2 -> to_sparse_coo() round trip
 * of utils/graph.py:22-35 (convertEdgeIndexToAdjMatrix) as the way the graph reaches the
 * propagation kernel. */
int lg_csr_rowptr_from_sorted(const int64_t *keys, int64_t nnz, int64_t n_rows,
                              int64_t *rowptr, lg_stream_t stream);

/* dis[n] = deg(n)^-1/2 with deg(n) = rowptr[n+1]-rowptr[n] (in-degree as a target),
 * inf -> 0. PyG 2.6.1 gcn_norm(add_self_loops=False), called at
 * model/LightGCN/model.py:53 and model/LightGCNOpti/model.py:65. */
int lg_gcn_norm_f32(const int64_t *rowptr, int64_t n_nodes, float *dis,
                    lg_stream_t stream);

/* w[e] = dis[src[e]] * dis[row_offset + r] for every entry e of row r: the edge weights
 * gcn_norm returns (model/LightGCN/model.py:53, second tuple element). Only needed by
 * callers that ask for the weights; the propagation kernel recomputes them on the fly. */
int lg_gcn_edge_weight_f32(const int64_t *rowptr, const int32_t *src, const float *dis,
                           int64_t n_rows, int64_t row_offset, float *w,
                           lg_stream_t stream);

/* ------------------------------------------------------------------------------------
 * LightGCN propagation: one layer of  e^{l+1} = D^-1/2 A D^-1/2 e^l  over a row range,
 * with the layer mean of model/LightGCN/model.py:66-69 fused into the epilogue.
 * Replaces PyG propagate (index_select + message + scatter_add,
 * model/LightGCN/model.py:61-63,76-84) and torch.stack/mean (:66-69).
 *
 * For r in [0, n_rows), node g = row_offset + r:
 *   v[g] = sum_{e in row r, s = src[e]} w_e * x[s]      (w_e = w[e], or dis[s]*dis[g]
 *                                                          when w is NULL; same value)
 *   y[g] = v[g]                                   if y != NULL
 *   acc_mode FIRST: acc[g] = x0[g] + v[g]
 *            MID  : acc[g] = acc[g] + v[g]
 *            LAST : out[g] = (acc[g] + v[g]) / denom
 *            ONLY : out[g] = (x0[g] + v[g]) / denom            (a 1-layer model)
 *            NONE : nothing
 * x, y, x0, acc, out are [*, dim] arrays indexed by node id g (row-sharded callers pass
 * full-size arrays and their own row range). dim in {32, 64, 128, 256}. w (optional) is
 * the per-entry gcn_norm weight of lg_gcn_edge_weight_f32, indexed like src; passing it
 * streams 4 B/edge instead of gathering dis[s]. y must not alias x.
 * Rows with more than long_threshold entries (<= 0: none) are skipped; the caller runs
 * them through lg_spmm_long_rows_f32 (power-law hubs).
 * ------------------------------------------------------------------------------------ */
enum lg_acc_mode {
  LG_ACC_NONE = 0,
  LG_ACC_FIRST = 1,
  LG_ACC_MID = 2,
  LG_ACC_LAST = 3,
  LG_ACC_ONLY = 4,
};
int lg_spmm_layer_f32(const int64_t *rowptr, const int32_t *src, const float *dis,
                      const float *w, const float *x, float *y, const float *x0, float *acc,
                      float *out, int64_t n_rows, int64_t row_offset, int32_t dim,
                      int32_t acc_mode, float denom, int64_t long_threshold,
                      lg_stream_t stream);

/* lg_spmm_layer_f32 for a sparse input x (the backward pass of the same call sites,
 * reference model/LightGCN/train.py:150 `loss.backward()` through model.py:62): live[n]
 * (uint8, one per source node) == 0 promises that row n of x is all zero, and its gather is
 * skipped (its contribution is added as 0). Same sums as lg_spmm_layer_f32 when the
 * promise holds. Long rows (above long_threshold) are left to lg_spmm_long_rows_f32. */
int lg_spmm_layer_live_f32(const int64_t *rowptr, const int32_t *src, const float *dis,
                           const float *w, const float *x, float *y, const float *x0,
                           float *acc, float *out, int64_t n_rows, int64_t row_offset,
                           int32_t dim, int32_t acc_mode, float denom, int64_t long_threshold,
                           const uint8_t *live, lg_stream_t stream);

/* The long rows skipped above, cut into segments [seg_beg[s], seg_end[s]) of src/w
 * (seg_node[s] = node id of the segment's row): one wave per segment writes a partial sum
 * into partial[n_seg, dim] (caller-owned workspace), then long row j (node long_node[j],
 * segments seg_ptr[j] .. seg_ptr[j+1]) adds its partials in order and runs the same
 * y / acc_mode epilogue as lg_spmm_layer_f32. Deterministic (no atomics). */
int lg_spmm_long_rows_f32(const int64_t *seg_beg, const int64_t *seg_end,
                          const int32_t *seg_node, int64_t n_seg, const int32_t *long_node,
                          const int64_t *seg_ptr, int64_t n_long, const int32_t *src,
                          const float *dis, const float *w, const float *x, float *y,
                          const float *x0, float *acc, float *out, int32_t dim,
                          int32_t acc_mode, float denom, float *partial, lg_stream_t stream);

/* Output-restricted layers (the forward of one BPR training step, reference
 * model/LightGCN/train.py:30 `model.forward` + :31-45 indexing the mini-batch's rows: the loss
 * reads layer L only at the batch's rows, layer L-1 only there and at their neighbours, ...):
 * lg_spmm_layer_f32 / lg_spmm_long_rows_f32 computing only the rows r whose row_mask[r]
 * (uint8, per node id) is non-zero; every other row of y / acc / out is left untouched. Each
 * computed row is bitwise the unrestricted call's. lg_mark_neighbors_u8 sets out_mask[r] = 1
 * for every row r of in_mask and every source of its entries (the rows the layer below must
 * produce for it); out_mask is not cleared first and must not alias in_mask. */
int lg_spmm_layer_rows_f32(const int64_t *rowptr, const int32_t *src, const float *dis,
                           const float *w, const float *x, float *y, const float *x0,
                           float *acc, float *out, int64_t n_rows, int64_t row_offset,
                           int32_t dim, int32_t acc_mode, float denom, int64_t long_threshold,
                           const uint8_t *row_mask, lg_stream_t stream);
int lg_spmm_long_rows_masked_f32(const int64_t *seg_beg, const int64_t *seg_end,
                                 const int32_t *seg_node, int64_t n_seg,
                                 const int32_t *long_node, const int64_t *seg_ptr,
                                 int64_t n_long, const int32_t *src, const float *dis,
                                 const float *w, const float *x, float *y, const float *x0,
                                 float *acc, float *out, int32_t dim, int32_t acc_mode,
                                 float denom, float *partial, const uint8_t *row_mask,
                                 lg_stream_t stream);
int lg_mark_neighbors_u8(const int64_t *rowptr, const int32_t *src, int64_t n_rows,
                         const uint8_t *in_mask, uint8_t *out_mask, lg_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Full-catalog scoring with exclusion mask and top-K.
 * Replaces  score = e0_u @ e0_i^T ; score[train|val positives] = -1024 ; topk(score, k)
 * of model/LightGCN/recommend.py:83-114 (same code: LightGCNOpti/recommend.py:83-114,
 * LightGCN/evaluation.py:31-51). The U x I score matrix is never materialised.
 *
 * score(u, i) is the fp32 fused-multiply-add chain, in this element order,
 *   acc = 0; for s in [0, dim/4): for g in [0, 4): acc = fmaf(eu[u][g*dim/4+s], ei[i][g*dim/4+s], acc)
 * (what v_mfma_f32_16x16x4_f32 computes), replaced by mask_value when i is in the user's
 * exclusion row ex_col[ex_rowptr[u] .. ex_rowptr[u+1]) (sorted ascending).
 * eu = [n_users, dim] (a sharded caller passes its own user block and the matching
 * ex_rowptr slice), ei = [n_items, dim]. k in [1, 128]; dim in {32, 64, 128}.
 * n_splits >= 1 splits the item range over that many workgroup sets (for small user
 * counts); the workspace holds the partial lists.
 * ------------------------------------------------------------------------------------ */
size_t lg_score_topk_ws_bytes(int64_t n_users, int64_t n_items, int32_t dim, int32_t k,
                              int32_t n_splits);
int lg_score_topk_f32(const float *eu, const float *ei, int64_t n_users, int64_t n_items,
                      int32_t dim, const int64_t *ex_rowptr, const int32_t *ex_col,
                      float mask_value, int32_t k, int32_t n_splits, float *out_val,
                      int64_t *out_idx, void *ws, size_t ws_bytes, lg_stream_t stream);

/* lg_score_topk_f32 with a bf16 MFMA screen (csrc/topk.hip K2r): the same outputs bit
 * for bit (values, ids, order). eu_bf16 / ei_bf16: lg_bound_prep_f32's bf16 copies of eu / ei
 * (16-byte aligned). umarg[u] (fp32, per user) must bound |bf16 MFMA product - fp32 chain|
 * over every item, with slack for the fp32 roundings of the screen's own compares:
 *   umarg[u] >= (||du|| I + (||eu[u]|| + ||du||) DI + (2.01 dim 2^-24 + 2^-22) ||eu[u]|| I)
 * with du = eu[u] - bf16(eu[u]), I = max_i ||ei[i]||, DI = max_i ||ei[i] - bf16(ei[i])||
 * (lgcnhs.ops.screen_margins, from lg_bound_prep_f32's norm_up / err_up; the round-3 form
 * 0.0081 ||eu[u]|| I is larger and also valid). Any input is memory-safe and gives
 * lg_score_topk_f32's lists: a umarg[u] that is NaN, negative or +inf (non-finite
 * embeddings), and any NaN bf16 product, is no bound -- those items enter the user's list
 * and get the exact chain (NaN chain scores never rank, as in lg_score_topk_f32). One pass keeps per user the items whose bound can still reach the k-th
 * largest lower bound, and ranks those by the exact chain at the end (every k <= 128).
 * Workspace: lg_score_topk_screened_ws_bytes (the per-split partial lists as
 * lg_score_topk_f32's, plus for k > 32 the per-user list slabs of 128 / 256 8-byte entries per
 * split that the main pass keeps its lists in); splits as lg_score_topk_f32. On catalogs of
 * >= 1024 k items a
 * screen-only seed pass over the first 1/16 of the items runs first and leaves each user's
 * starting threshold in out_val[u * k + k - 1] (overwritten by the result); the outputs do
 * not depend on it. */
size_t lg_score_topk_screened_ws_bytes(int64_t n_users, int64_t n_items, int32_t dim,
                                       int32_t k, int32_t n_splits);
int lg_score_topk_screened_f32(const float *eu, const float *ei, const void *eu_bf16,
                               const void *ei_bf16, const float *umarg, int64_t n_users,
                               int64_t n_items, int32_t dim, const int64_t *ex_rowptr,
                               const int32_t *ex_col, float mask_value, int32_t k,
                               int32_t n_splits, float *out_val, int64_t *out_idx, void *ws,
                               size_t ws_bytes, lg_stream_t stream);

/* Dense masked score matrix G[u][i] (same score definition and mask as above), written
 * with leading dimension ldg. Replaces getAllocateMat's matmul + masks
 * (model/SpreadLightGCN/model.py:74-104, model/SpreadLightGCNOpti/model.py:139-169). */
int lg_score_dense_f32(const float *eu, const float *ei, int64_t n_users, int64_t n_items,
                       int32_t dim, const int64_t *ex_rowptr, const int32_t *ex_col,
                       float mask_value, float *G, int64_t ldg, lg_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Hybrid spreading (model/SpreadMethod/model.py), fp64, from the interaction matrix A
 * held sparse: user rows (user_rowptr/user_items) and item rows (item_rowptr/item_users).
 * ------------------------------------------------------------------------------------ */

/* gW[i][j] = sum_{v in users(i), ascending} [j in items(v)] * (1 / k_v), k_v = |items(v)|.
 * = np.dot(A.T / k_u, A) of getSpreadingGeneralMat (model/SpreadMethod/model.py:14-27).
 * gW is [n_items, n_items], fully written (zeros included). */
int lg_spread_general_f64(const int64_t *item_rowptr, const int32_t *item_users,
                          const int64_t *user_rowptr, const int32_t *user_items,
                          int64_t n_users, int64_t n_items, double *gW,
                          lg_stream_t stream);

/* W = lg_hybrid_weight_f64(lg_spread_general_f64(...), k_item, lambda, either transpose)
 * bit for bit, without general_W in memory (general_W is exactly symmetric): getSpreading-
 * GeneralMat + HybridS (model/SpreadMethod/model.py:14-27, 63-85) for one lambda. W is
 * [n_items, n_items], fully written; ws: lg_spread_hybrid_ws_bytes(n_items, n_users) bytes. */
size_t lg_spread_hybrid_ws_bytes(int64_t n_items, int64_t n_users);
int lg_spread_hybrid_f64(const int64_t *item_rowptr, const int32_t *item_users,
                         const int64_t *user_rowptr, const int32_t *user_items,
                         const double *k_item, int64_t n_users, int64_t n_items, double lambda,
                         double *W, void *ws, size_t ws_bytes, lg_stream_t stream);

/* W[i][j] = gWsrc[i][j] / den, den = k_i^(1-lambda) * k_j^lambda, den == 0 -> 1, with
 * gWsrc = gW (transpose_gw = 0) or gW^T (transpose_gw = 1). HybridS,
 * model/SpreadMethod/model.py:63-85 (the .T variants: SpreadMethod/recommend.py:91,101). */
int lg_hybrid_weight_f64(const double *gW, const double *k_item, int64_t n_items,
                         double lambda, int32_t transpose_gw, double *W,
                         lg_stream_t stream);

/* F[u][j] = sum_{i in items(u), ascending} W[i][j] : getResource's np.dot(A, W)
 * (model/SpreadMethod/model.py:88-99) for user rows [0, n_users). */
int lg_spread_resource_f64(const int64_t *user_rowptr, const int32_t *user_items,
                           const double *W, int64_t n_users, int64_t n_items, double *F,
                           int64_t ldf, lg_stream_t stream);

/* Per-row top-K over dense fp64 rows F[r][0..n_cols) (leading dim ldf), optionally
 * multiplied by the fp32 score G[r][j] (eu/ei non-NULL; same chain as lg_score_topk_f32,
 * promoted to fp64 before the product, as numpy's G * F does:
 * model/SpreadLightGCN/model.py:151). Exclusion rows ex_* (may be NULL):
 *   excl_mode DROP: excluded columns are removed (argsort + filter of
 *                   model/SpreadMethod/recommend.py:39-47);
 *   excl_mode NONE: nothing is removed (the unfiltered ProbS/movielens branch,
 *                   model/SpreadMethod/recommend.py:49-50).
 * With a G factor the exclusions must be DROP (G's -1024 mask is then never observable).
 * k in [1, 128]. Rows with fewer than k survivors are padded with index -1. */
enum lg_excl_mode { LG_EXCL_DROP = 0, LG_EXCL_NONE = 1 };
int lg_rows_topk_f64(const double *F, int64_t ldf, int64_t n_rows, int64_t n_cols,
                     const float *eu, const float *ei, int32_t dim,
                     const int64_t *ex_rowptr, const int32_t *ex_col, int32_t excl_mode,
                     int32_t k, double *out_val, int64_t *out_idx, lg_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Factored spreading over item tiles: the path for catalogs whose I x I general_W / W do
 * not fit (SURVEY.md §8 a9 "K3s"; C5 = 1M x 1M would need 8 TB per matrix). The values of
 * lg_spread_general_f64 -> lg_hybrid_weight_f64 -> lg_spread_resource_f64
 * (-> lg_rows_topk_f64), i.e. the reference's getSpreadingGeneralMat / HybridS /
 * getResource / recommendForAllUser (model/SpreadMethod/model.py:14-99,
 * model/SpreadMethod/recommend.py:31-50, model/SpreadLightGCN/model.py:151), without ever
 * holding an I x I or U x I matrix, as
 *   F[u][j] = rb_j * sum over the paths u -> i -> v -> j of fl(1/k_v) * ra_i
 * (ra = 1/alpha, rb = 1/beta; each term within a few ulp of the reference's W entry, the
 * summation order the walk's own, fixed). Tiles [j0, j0 + tile) of item columns are built
 * a group of <= 16 at a time: lg_spread_group_cursor -> lg_spread_group_bound ->
 * lg_spread_group_units -> (inclusive scan of the units) -> lg_spread_group_rows_f64; each
 * tile is then walked by lg_spread_tile_resource_topk_f64 (running top-K lists), with
 * lg_score_chunk_bound's score bounds when there is a G factor. The orchestration
 * (lgcnhs.ops.spread_topk_tiled) is host code; see DESIGN.md §5 K3s. The per-tile build
 * passes, the F-writing walk and the two-kernel top-K merge that these replace are kept,
 * as bitwise references for the tests, in include/lgcnhs_ref.h (lib/liblgcnhs_ref.so only).
 * ------------------------------------------------------------------------------------ */

/* ra[i] = 1 / alpha[i], rb[i] = 1 / beta[i] (a zero factor -> 1: the reference's den == 0
 * rule, model/SpreadMethod/model.py:81-82; such rows / columns hold no paths). */
int lg_hybrid_recip_f64(const double *k_item, int64_t n_items, double lambda, double *ra,
                        double *rb, lg_stream_t stream);

/* inv[v] = fl(1 / (rowptr[v+1] - rowptr[v])): the (A.T / k_u) factor of
 * model/SpreadMethod/model.py:21-25, as lg_spread_general_f64 computes it. */
int lg_inv_degree_f64(const int64_t *rowptr, int64_t n_rows, double *inv,
                      lg_stream_t stream);

/* Line format of a tile (lgcnhs_ref.h lg_spread_tile_rows_f64 builds one tile at a time):
 * row i of general_W restricted to the tile as one 128-byte line at lines + 128 i (32
 * uint32 words) plus, for rows that do not fit, a run of 16-byte units in ovf. Word 0 =
 * header: bit 31 V format, bit 30 overflow, bit 29 "slow" (V rows, P rows with a class
 * >= 512), bits 0-28 the run's first unit (whose .x = the number of data units after it).
 *   P rows (bound[i] <= vthr): one word per (user v, item j) pair behind the row, users
 *     ascending then items ascending: bits 0-15 j - item_begin, bits 16-30 user_cls[v] (a
 *     1-based class of v's degree: inv_cls[user_cls[v]] = fl(1/k_v)); 0 = padding.
 *   V rows (hub items, bound[i] > vthr): one 16-byte entry per distinct column, ascending:
 *     {0x80000000 | (j - item_begin), fp64 general_W[i][j] (lo, hi), 0}.
 * Lambda-independent (a sweep reuses the tile); line n_items (the walk's padding row) is
 * zeroed by the caller.
 *
 * Group build: n_tiles (<= 16; <= 8 for tiles wider than 4096) consecutive tiles at once, each
 * (item row, user) pair visited once per group instead of once per tile. Tile t of the group
 * is [group_begin + t tile, min(group_begin + (t + 1) tile, stop)).
 * lg_spread_group_cursor: counts[v][0..15] (16 uint16 per user, 16-byte aligned, unused
 *   tiles 0) = user v's items in each tile, end[v] = the position after the group's last
 *   (cur[v] = the first position with item >= group_begin; cur and end must not alias;
 *   positions < 2^32), rec[v] (16 bytes per user, 16-byte aligned) = the user's record for
 *   the rows pass: its class (user_cls) and up to 6 of its group items in place, else cur.
 * lg_spread_group_bound: bound[t][i] ([n_tiles][n_items] int64) = the (user, tile item)
 *   pairs behind row i of W in tile t (its paths).
 * lg_spread_group_units: units[t][i] ([n_tiles][n_items] int64) = the overflow units of
 *   row i in tile t (1 + ceil((bound - 31) / 4) for P rows with bound > 31, 1 + (min(bound,
 *   width_t) - 7) for V rows with more than 7 entries, else 0); the caller's inclusive scan
 *   of the flat array (units_incl) places every run: tile t's runs start at unit
 *   units_incl[t n_items - 1] (0 for t = 0), each row's run at its exclusive prefix.
 * lg_spread_group_rows_f64: the lines and runs of every tile t of the group, tile t's
 *   lines at lines + t (n_items + 1) 128 bytes (each tile's line n_items zeroed by the
 *   caller), its runs in ovf as units_incl places them (header pointers relative to the
 *   tile's first unit: each tile's lines and runs are the per-tile build's, bit for bit);
 *   ovf holds units_incl[n_tiles n_items - 1] + 64 units; row_len as [n_tiles][n_items];
 *   vthr in [31, 65535]; cur / counts / rec from lg_spread_group_cursor; ws:
 *   lg_spread_group_rows_ws_bytes(n_items, n_tiles) bytes. */
int lg_spread_group_cursor(const int64_t *user_rowptr, const int32_t *user_items,
                           const uint16_t *user_cls, int64_t n_users, int32_t group_begin,
                           int32_t tile, int32_t n_tiles, int32_t stop, const int64_t *cur,
                           int64_t *end, uint16_t *counts, void *rec, lg_stream_t stream);
int lg_spread_group_bound(const int64_t *item_rowptr, const int32_t *item_users,
                          int64_t n_items, const uint16_t *counts, int32_t n_tiles,
                          int64_t *bound, lg_stream_t stream);
int lg_spread_group_units(const int64_t *bound, int64_t n_items, int32_t group_begin,
                          int32_t tile, int32_t n_tiles, int32_t stop, int64_t vthr,
                          int64_t *units, lg_stream_t stream);
size_t lg_spread_group_rows_ws_bytes(int64_t n_items, int32_t n_tiles);
int lg_spread_group_rows_f64(const int64_t *item_rowptr, const int32_t *item_users,
                             const int32_t *user_items, const double *inv_deg,
                             int64_t n_items, const int64_t *cur, const uint16_t *counts,
                             const void *rec, int32_t group_begin, int32_t tile,
                             int32_t n_tiles, int32_t stop, const int64_t *bound, int64_t vthr,
                             const int64_t *units_incl, void *lines, void *ovf,
                             int32_t *row_len, void *ws, size_t ws_bytes, lg_stream_t stream);

/* cur[v] = first position of user v's item row (ascending) with item >= item_begin: the
 * cursor state for a tile walk that starts at item_begin (an item-range shard of a
 * multi-GPU run) instead of 0. */
int lg_spread_tile_seek(const int64_t *user_rowptr, const int32_t *user_items,
                        int64_t n_users, int32_t item_begin, int64_t *cur, lg_stream_t stream);

/* Merge n_lists sorted top-K lists per row, in_val/in_idx laid out [n_lists][n_rows][k]
 * (value desc, index asc; index -1 = empty), into out_val/out_idx [n_rows][k] in the same
 * order: the per-item-range lists of lg_spread_tile_resource_topk_f64 (disjoint item ranges,
 * the multi-GPU shards) give the lists
 * a single walk over all items would. k in [1, 128]. */
int lg_topk_lists_merge_f64(const double *in_val, const int64_t *in_idx, int32_t n_lists,
                            int64_t n_rows, int32_t k, double *out_val, int64_t *out_idx,
                            lg_stream_t stream);

/* The tile walk: each user's F columns [item_begin, item_begin + width) are accumulated in
 * LDS (the values of the F-writing reference walk, lgcnhs_ref.h, bit for bit) and merged
 * straight into the running top-K lists
 * io_val/io_idx [n_users][k] (first != 0: start empty); F is never written to memory. G
 * factor: eu = the rows' user embeddings, ei = all item embeddings, gb =
 * lg_score_chunk_bound's [n_users][n_chunks] bounds for this tile (n_chunks =
 * ceil(width / 64) <= 64) and optionally qb/qstride, its per-column 8-bit bounds: only
 * columns whose bound (gb * q / 255 with qb) times F can beat the K-th value get the exact
 * score chain.
 * Exclusions (dropped): ex_rowptr/ex_col as in lg_rows_topk_f64 plus a per-row cursor
 * ex_cur[n_users] positioned at the walk's first item by lg_spread_tile_seek(ex_rowptr,
 * ex_col, ...) and advanced here. Walked over tiles in ascending order, the lists equal
 * lg_rows_topk_f64 over the F rows the walk sums. k in [1, 128]; dim in
 * {32, 64, 128}. The walk keeps its stream positions in 32 bits: n_users, the interactions
 * and the exclusions must each be < 2^31; n_positions / n_ex_positions are upper bounds of
 * user_rowptr[n_users] / ex_rowptr[n_users] (the lengths of user_items / ex_col, 0 without
 * exclusions), checked here -- the library does not read device memory on the host.
 * lg_spread_tile_resource_topk_lds_bytes: LDS of one wave plus the
 * workgroup's tables (the launch fits as many waves per CU as the LDS holds). */
size_t lg_spread_tile_resource_topk_lds_bytes(int32_t tile, int32_t k, int32_t dim);
int lg_spread_tile_resource_topk_f64(const int64_t *user_rowptr, const int32_t *user_items,
                                     const double *ra_edge, int64_t n_users,
                                     const void *lines, const void *ovf, int32_t null_row,
                                     const double *rbeta,
                                     const double *inv_cls, int32_t item_begin, int32_t tile,
                                     int32_t width, const float *eu, const float *ei,
                                     int32_t dim, const float *gb, int32_t n_chunks,
                                     const uint8_t *qb, int32_t qstride,
                                     const int64_t *ex_rowptr, const int32_t *ex_col,
                                     int64_t *ex_cur, int32_t k, int32_t first,
                                     double *io_val, int64_t *io_idx, int64_t n_positions,
                                     int64_t n_ex_positions, lg_stream_t stream);

/* x_bf16[r] = bf16(x[r]) (round to nearest even), norm_up[r] = ||x[r]||_2 rounded up to
 * fp32: the operands of lg_score_chunk_bound (csrc/gbound.hip). err_up (optional, may be
 * NULL): err_up[r] = ||x[r] - x_bf16[r]||_2 rounded up, the rounding-error norms the
 * screened top-K's margin umarg is built from (lgcnhs.ops.screen_margins). */
int lg_bound_prep_f32(const float *x, int64_t n_rows, int32_t dim, void *x_bf16,
                      float *norm_up, float *err_up, lg_stream_t stream);

/* Widest item tile lg_score_chunk_bound accepts (64 chunks of 64 columns). */
#define LG_BOUND_MAX_WIDTH 4096

/* gb[u][c] (fp32, [n_users][ceil(width / 64)]) >= the fp32 score chain e0_u . e0_j of every
 * column j of chunk c = [item_begin + 64c, item_begin + 64c + 64) of the tile: the bf16 MFMA
 * product's chunk maximum plus a rigorous rounding margin (csrc/gbound.hip). u/i from
 * lg_bound_prep_f32 of the users' rows and of all items. dim in {32, 64, 128}. qb (optional,
 * [n_users][qstride] bytes, qstride >= width rounded up to 256): per column j,
 * q = ceil(255 (G_bf16 + margin) / gb) in [0, 255], so gb * q / 255 >= the chain score too
 * (csrc/gbound.hip). width <= LG_BOUND_MAX_WIDTH (LG_ERR_ARG otherwise). */
int lg_score_chunk_bound(const void *u_bf16, const float *u_norm, int64_t n_users,
                         const void *i_bf16, const float *i_norm, int32_t dim,
                         int32_t item_begin, int32_t width, float *gb, uint8_t *qb,
                         int32_t qstride, lg_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Recommendation-list metrics (reference metrics/accurate.py and
 * metrics/diversity.py). recs is a [n_rows][k] int64 list matrix (recommendDictToTensor,
 * utils/trans.py:82-92); entries < 0 are padding and match nothing.
 * ------------------------------------------------------------------------------------ */

/* hit[q * k + p] = 1 if recs[eval_rows[q]][p] is in test row q (pos_rowptr/pos_col: one
 * sorted row per evaluated user, in eval_rows order), else 0: the `item in items` labels of
 * calPrecisionAndRecall / calNDCG (metrics/accurate.py:24-31, :69-76). */
int lg_rec_hits(const int64_t *recs, int64_t n_rows, int32_t k, const int64_t *eval_rows,
                int64_t n_eval, const int64_t *pos_rowptr, const int32_t *pos_col,
                uint8_t *hit, lg_stream_t stream);

/* *total = sum over ordered pairs of rows u != v of |set(recs[u]) & set(recs[v])|, computed
 * exactly as sum_i c_i (c_i - 1) over the per-item list counts c_i (written to counts[n_items],
 * items >= n_items ignored): calHammingDistance (metrics/diversity.py:15-63) is
 * 1 - total / (k n_rows (n_rows - 1)). */
int lg_rec_pair_overlap(const int64_t *recs, int64_t n_rows, int32_t k, int64_t n_items,
                        int32_t *counts, uint64_t *total, lg_stream_t stream);

/* part[r * k + p] = sum over q > p with recs[r][q] != recs[r][p], both items of nonzero
 * item_degree, of co(a, b) / sqrt(deg_a * deg_b), co = |users(a) & users(b)| over the item
 * columns item_rowptr/item_users (sorted) of the binary interaction matrix:
 * calInternalSimilarity (metrics/diversity.py:66-115) is 2 * sum(part) / (n_rows k (k-1)). */
int lg_rec_intra_similarity_f64(const int64_t *recs, int64_t n_rows, int32_t k,
                                const int64_t *item_rowptr, const int32_t *item_users,
                                const int64_t *item_degree, int64_t n_items, double *part,
                                lg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* LGCNHS_H */
