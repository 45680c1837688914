/*
 * lgcnhs_ref.h — test-reference entry points of the factored spreading (K3s), exported ONLY
 * by lib/liblgcnhs_ref.so (the same sources built with -DLG_REFERENCE_PATHS=1). The product
 * library lib/liblgcnhs.so does not carry them: they are the per-tile forms that the
 * product's group build (lg_spread_group_*) and fused walk (lg_spread_tile_resource_topk_f64)
 * replace, kept so the tests can check those bit for bit (tests/_ref_paths.py). Conventions
 * and the tile line format: include/lgcnhs.h.
 */
#ifndef LGCNHS_REF_H
#define LGCNHS_REF_H

#include "lgcnhs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* end[v] = first position p >= cur[v] of user v's item row (user_rowptr/user_items, items
 * ascending) with user_items[p] >= item_end (or the row end), count[v] = end[v] - cur[v].
 * With cur = the row starts (first tile) or the previous tile's end,
 * user_items[cur[v] .. end[v]) are v's items in the tile. cur and end must not alias;
 * item_end - (the tile's first item) <= 8192 (count is 16-bit). */
int lg_spread_tile_cursor(const int64_t *user_rowptr, const int32_t *user_items,
                          int64_t n_users, int32_t item_end, const int64_t *cur,
                          int64_t *end, uint16_t *count, lg_stream_t stream);

/* bound[i] = sum over users v of item i (item_rowptr/item_users) of count[v]: the number of
 * (user, tile item) pairs behind W's row i in the tile (its paths). */
int lg_spread_tile_bound(const int64_t *item_rowptr, const int32_t *item_users,
                         int64_t n_items, const uint16_t *count, int64_t *bound,
                         lg_stream_t stream);

/* Row i of general_W restricted to the tile, for every item i, as one 128-byte line at
 * lines + 128 i (32 uint32 words) plus, for rows that do not fit, a run of 16-byte units in
 * ovf. Word 0 = header: bit 31 V format, bit 30 overflow, bits 0-28 the run's first unit
 * (whose .x = the number of data units after it).
 *   P rows (bound[i] <= vthr): one word per (user v, item j) pair behind the row, users
 *     ascending then items ascending: bits 0-15 j - item_begin, bits 16-30 user_cls[v] (a
 *     1-based class of v's degree, < 0x8000: inv_cls[user_cls[v]] = fl(1/k_v)); 0 =
 *     padding; bit 31 clear. Line words 1-31 then 4 per data unit.
 *   V rows (hub items, bound[i] > vthr): one 16-byte entry per distinct column, ascending:
 *     {0x80000000 | (j - item_begin), fp64 general_W[i][j] (lo, hi), 0}. Line units 1-7 then
 *     1 per data unit.
 * ovf_ptr[i] = the caller's exclusive prefix over rows of their overflow units:
 * 1 + ceil((bound - 31) / 4) for P rows with bound > 31, 1 + (min(bound, tile) - 7) for V
 * rows with min(bound, tile) > 7, else 0; ovf must hold that total + 64 units (the walk
 * reads 64 units per run). row_len[i] (optional) = the row's pairs (P) or entries (V).
 * Header bit 29 ("slow") marks V rows and P rows with a class >= 512 (the walk's general
 * decode); the overflow pointer has 29 bits. Lambda-independent (a sweep reuses the tile).
 * Line n_items (the walk's padding row) is never written: the caller zeroes it. cur/count from lg_spread_tile_cursor, bound
 * from lg_spread_tile_bound, inv_deg from lg_inv_degree_f64 over the user rows (V rows).
 * ws: lg_spread_tile_rows_ws_bytes(n_items) bytes of scratch. tile in [1, 8192];
 * vthr >= 31; every item of the tile lies in [item_begin, item_begin + tile). */
size_t lg_spread_tile_rows_ws_bytes(int64_t n_items);
int lg_spread_tile_rows_f64(const int64_t *item_rowptr, const int32_t *item_users,
                            const int32_t *user_items, const uint16_t *user_cls,
                            const double *inv_deg, int64_t n_items, const int64_t *cur,
                            const uint16_t *count, int32_t item_begin, int32_t tile,
                            const int64_t *bound, int64_t vthr, const int64_t *ovf_ptr,
                            void *lines, void *ovf, int32_t *row_len, void *ws,
                            size_t ws_bytes, lg_stream_t stream);

/* F[u][j - item_begin] = rb[j] * sum over the paths of u's items of the tile's rows (see the
 * section comment) for the n_users rows of user_rowptr (pass user_rowptr + u0 for a block)
 * and j in [item_begin, item_begin + tile) (columns >= item_begin + width are 0); F
 * row-major with leading dim ldf >= tile. ra_edge[p] = ra[user_items[p]] (aligned with
 * user_items, at least one entry), rbeta = rb of all items, inv_cls the class table;
 * lines / ovf from lg_spread_tile_rows_f64, with line null_row (= n_items: lines holds
 * n_items + 1) all zero. */
int lg_spread_tile_resource_f64(const int64_t *user_rowptr, const int32_t *user_items,
                                const double *ra_edge, int64_t n_users, const void *lines,
                                const void *ovf, int32_t null_row, const double *rbeta,
                                const double *inv_cls,
                                int32_t item_begin, int32_t tile, int32_t width, double *F,
                                int64_t ldf, lg_stream_t stream);

/* Merge columns [item_begin, item_begin + n_cols) of (G *) F (F[r][0..n_cols), leading dim
 * ldf; G as in lg_rows_topk_f64 with eu = the rows' user embeddings and ei = all item
 * embeddings) into running top-K lists io_val/io_idx [n_rows][k] (sorted by value desc,
 * index asc; index -1 = empty). first != 0 ignores their contents. Exclusions as in
 * lg_rows_topk_f64 (ex_rowptr indexed by r). Applied over all tiles in ascending order the
 * lists equal lg_rows_topk_f64 over the full rows. k in [1, 128]. */
int lg_tile_topk_f64(const double *F, int64_t ldf, int64_t n_rows, int32_t item_begin,
                     int32_t n_cols, const float *eu, const float *ei, int32_t dim,
                     const int64_t *ex_rowptr, const int32_t *ex_col, int32_t excl_mode,
                     int32_t k, int32_t first, double *io_val, int64_t *io_idx,
                     lg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* LGCNHS_REF_H */
