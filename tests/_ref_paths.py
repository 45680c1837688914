"""Test-only reference paths of the factored spreading (K3s), on lib/liblgcnhs_ref.so (the
product library built with -DLG_REFERENCE_PATHS=1, include/lgcnhs_ref.h): the per-tile build
passes (lg_spread_tile_cursor / _bound / _rows_f64), the F-writing walk
(lg_spread_tile_resource_f64) and the two-kernel top-K merge (lg_tile_topk_f64). The product
(lgcnhs.ops) builds tiles a group at a time and walks them fused; these are the bitwise
references it is tested against. Not product code: the product library does not export
them."""
import torch

from lgcnhs import _native as N
from lgcnhs import ops


class PerTileWeights(ops.TileWeights):
    """ops.TileWeights whose tiles come from the per-tile reference passes, one tile per
    build (their overflow-run placement by torch ops, as the reference build did)."""

    def __init__(self, A, lam, tile, vthr=None):
        super().__init__(A, lam, tile, vthr=vthr, group=1)
        self.count1 = torch.empty(A.n_users, dtype=torch.uint16, device=self.dev)
        R = N.ref_lib()
        self.ws = torch.empty(max(1, R.lg_spread_tile_rows_ws_bytes(A.n_items)),
                              dtype=torch.uint8, device=self.dev)

    def _build_group(self, j0, stop, widths):
        A, I, R = self.A, self.A.n_items, N.ref_lib()
        strm = N.stream_handle(self.dev)
        N.ref_check(R.lg_spread_tile_cursor(N.ptr(A.by_user.rowptr), N.ptr(A.by_user.col),
                                            A.n_users, j0 + widths[0], N.ptr(self.cur),
                                            N.ptr(self.end), N.ptr(self.count1), strm),
                    "lg_spread_tile_cursor")
        N.ref_check(R.lg_spread_tile_bound(N.ptr(A.by_item.rowptr), N.ptr(A.by_item.col), I,
                                           N.ptr(self.count1), N.ptr(self.g_bound), strm),
                    "lg_spread_tile_bound")
        b = self.g_bound[0]
        hub = b > self.vthr
        units = ops._run_units(torch.where(hub, torch.clamp(b, max=widths[0]), b), hub)
        cum = torch.cumsum(units, 0)
        ovf_ptr = cum - units
        total = int(cum[-1]) if I else 0
        self._grow_ovf(total)
        N.ref_check(R.lg_spread_tile_rows_f64(
            N.ptr(A.by_item.rowptr), N.ptr(A.by_item.col), N.ptr(A.by_user.col),
            N.ptr(self.user_cls), N.ptr(self.inv_deg), I, N.ptr(self.cur), N.ptr(self.count1),
            j0, widths[0], N.ptr(self.g_bound), self.vthr, N.ptr(ovf_ptr), N.ptr(self.g_lines),
            N.ptr(self.g_ovf), N.ptr(self.g_row_len), N.ptr(self.ws), self.ws.numel(), strm),
            "lg_spread_tile_rows_f64")
        self._grp = (j0, widths, [0], [total])


def resource(tw, u0, u1, out, scale=None):
    """out[u - u0][j - j0] = F[u][j] for users [u0, u1) and tw's current tile (the
    F-writing reference walk)."""
    A = tw.A
    sc = scale if scale is not None else tw.scale
    N.ref_check(N.ref_lib().lg_spread_tile_resource_f64(
        N.ptr(A.by_user.rowptr[u0:]), N.ptr(A.by_user.col), N.ptr(sc.ra_edge), u1 - u0,
        N.ptr(tw.lines), N.ptr(tw.ovf), A.n_items, N.ptr(sc.rb), N.ptr(tw.inv_cls), tw.j0,
        tw.tile, tw.width, N.ptr(out), out.stride(0), N.stream_handle(tw.dev)),
        "lg_spread_tile_resource_f64")
    return out


def tile_topk(F, j0, n_cols, k, vals, idxs, first, excl=None, drop=True, eu=None, ei=None):
    """Merge columns [j0, j0 + n_cols) of (G *) F into the running lists vals/idxs."""
    d = 0 if eu is None else eu.shape[1]
    N.ref_check(N.ref_lib().lg_tile_topk_f64(
        N.ptr(F), F.stride(0), F.shape[0], j0, n_cols, N.ptr(eu), N.ptr(ei), d,
        N.ptr(excl.rowptr if excl else None), N.ptr(excl.col if excl else None),
        N.LG_EXCL_DROP if drop else N.LG_EXCL_NONE, int(k), int(bool(first)), N.ptr(vals),
        N.ptr(idxs), N.stream_handle(F.device)), "lg_tile_topk_f64")


def spread_topk_two_kernel(A, lam, k, excl, drop=True, eu=None, ei=None, users=None,
                           tile=2048, scratch_bytes=4 << 30, items=None, stats=None,
                           count_paths=False):
    """ops.spread_topk_tiled in the two-kernel form: F of a span of tiles written to a
    [users, span] scratch of scratch_bytes by the reference walk, then lg_tile_topk_f64 --
    the same F values, so the same lists, bit for bit."""
    u0, u1 = (0, A.n_users) if users is None else (users.start, users.stop)
    i0, i1 = (0, A.n_items) if items is None else (max(0, items.start),
                                                   min(A.n_items, items.stop))
    n = u1 - u0
    dev = A.k_item.device
    vals = torch.full((n, k), float("-inf"), dtype=torch.float64, device=dev)
    idxs = torch.full((n, k), -1, dtype=torch.int64, device=dev)
    if n == 0 or i1 <= i0:
        return vals, idxs
    tile = min(int(tile), i1 - i0, 4096 if eu is not None else 8192)
    tw = ops.TileWeights(A, lam, tile)
    if i0:
        tw.seek(i0)
    ex = excl.slice_rows(u0, u1) if excl is not None else None
    eu_r = None if eu is None else eu[u0:u1].contiguous()
    ei = None if ei is None else ei.contiguous()
    if stats is not None and count_paths:
        ops._count_rows(tw, A, u0, u1)
    span = max(tile, scratch_bytes // (n * 8) // tile * tile)
    span = min(span, -(-(i1 - i0) // tile) * tile)
    F = torch.empty((n, span), dtype=torch.float64, device=dev)
    for s0 in range(i0, i1, span):
        s1 = min(i1, s0 + span)
        for j0 in range(s0, s1, tile):
            tw.build(j0, stop=i1)
            resource(tw, u0, u1, F[:, j0 - s0:])
        tile_topk(F, s0, s1 - s0, k, vals, idxs, s0 == i0, ex, drop, eu_r, ei)
    if stats is not None and count_paths:
        stats["w_paths"] = stats.get("w_paths", 0) + int(tw.paths_read)
        stats["w_bytes"] = stats.get("w_bytes", 0) + int(tw.bytes_read)
    return vals, idxs
