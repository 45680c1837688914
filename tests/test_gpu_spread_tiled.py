"""GPU parity of the factored (item-tiled) spreading path, K3s: its
general_W tiles bitwise equal to lg_spread_general_f64's columns, its F within 1e-12
relative of the dense path (lg_spread_general_f64 -> lg_hybrid_weight_f64 ->
lg_spread_resource_f64, itself pinned to the reference's numpy results in
test_gpu_spread.py; the walk sums each column's paths in its own fixed order), its top-k
lists equal to the dense path's except rounding-level ties; plus the reference fixture for
the LGCNHS recommendation. Tiled-vs-tiled properties (user / item shards, fused vs the
two-kernel reference of tests/_ref_paths.py, lambda sweep) are bitwise."""
import numpy as np
import pytest
import torch

from _compare import compare_lists_close, compare_topk_sets
import _ref_paths as RP

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inter(U, I, n, seed, zipf=False):
    from lgcnhs import ops
    from lgcnhs.synth import synth_interactions
    u, i = synth_interactions(U, I, n, seed=seed, dist="zipf" if zipf else "uniform")
    return ops.Interactions.from_pairs(torch.as_tensor(u), torch.as_tensor(i), U, I, DEV)


def _dense_tile(tw, I):
    """The current tile of general_W as a dense [I, width] matrix (zeros where no entry),
    decoded from the line format (TileWeights.dense checks the format invariants: headers,
    zero padding, ascending hub entries, row lengths)."""
    out = tw.dense()
    assert out.shape == (I, tw.width)
    return out


def _close(got, ref, rtol=1e-12):
    """Equal zeros, and within rtol elsewhere (the factored walk's own summation order)."""
    assert np.array_equal(got == 0, ref == 0)
    nz = ref != 0
    err = np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])
    assert err.size == 0 or err.max() <= rtol, err.max()
    return float(err.max()) if err.size else 0.0


@pytest.mark.parametrize("zipf", [False, True])
@pytest.mark.parametrize("lam", [0.0, 0.5, 0.85, 1.0])
def test_tile_weights_and_resource(zipf, lam):
    """Every tile of general_W equals the dense matrix's columns bit for bit (P slots summed
    in slot order = users ascending; the hub rows of the zipf graph exceed the tile width and
    are merged by the block-wide path), and every tile of F is within 1e-12 of the dense F."""
    from lgcnhs import ops
    U, I = 700, 900
    A = _inter(U, I, 30000 if zipf else 12000, seed=5, zipf=zipf)
    gW = ops.spread_general(A)
    W = ops.hybrid_weight(gW, A.k_item, lam)
    F = ops.spread_resource(A, W).cpu().numpy()
    gW = gW.cpu().numpy()
    tile = 256
    tw = ops.TileWeights(A, lam, tile)
    Fb = torch.empty((U, tile), dtype=torch.float64, device=DEV)
    hub_seen = ovf_seen = False
    for j0 in range(0, I, tile):
        tw.build(j0)
        hub_seen |= bool(tw.is_hub.any())
        ovf_seen |= bool(((tw.bound > 31) & ~tw.is_hub).any())
        Wt = _dense_tile(tw, I)
        assert np.array_equal(Wt.view(np.uint64), gW[:, j0:j0 + tw.width].view(np.uint64))
        RP.resource(tw, 0, U, Fb)
        _close(Fb[:, :tw.width].cpu().numpy(), F[:, j0:j0 + tw.width])
    assert ovf_seen, "the graph should exercise P rows with overflow runs"
    if zipf:
        assert hub_seen, "the zipf graph should exercise the hub-row path"


@pytest.mark.parametrize("zipf,tile,group,vthr", [(False, 64, 8, None), (True, 100, 3, None),
                                                  (True, 256, 8, None), (True, 128, 5, 40),
                                                  (False, 1000, 8, None), (False, 40, 16, None),
                                                  (True, 50, 11, None), (True, 33, 16, 35)])
def test_group_build_equals_per_tile(zipf, tile, group, vthr):
    """The group build (lg_spread_group_*: each (item, user) pair visited once per group of
    tiles) writes every tile's lines, overflow runs, bounds and row lengths bit for bit as the
    per-tile passes do, including hub (V) rows, overflow runs, a partial last group and a
    stop inside a tile."""
    from lgcnhs import ops
    U, I = 700, 900
    A = _inter(U, I, 30000 if zipf else 12000, seed=5, zipf=zipf)
    stop = I - 37
    a = RP.PerTileWeights(A, 0.5, tile, vthr=vthr)
    b = ops.TileWeights(A, 0.5, tile, vthr=vthr, group=group)
    hub_seen = ovf_seen = False
    for j0 in range(0, stop, tile):
        a.build(j0, stop)
        b.build(j0, stop)
        assert (a.j0, a.width, a.n_units) == (b.j0, b.width, b.n_units)
        assert torch.equal(a.lines, b.lines)
        assert torch.equal(a.bound, b.bound) and torch.equal(a.row_len, b.row_len)
        # the runs themselves (a hub row's run may end before its allocated units, whose
        # words are never read: compared through the decoder, which walks the headers)
        assert np.array_equal(a.dense().view(np.uint64), b.dense().view(np.uint64))
        hub_seen |= bool(a.is_hub.any())
        ovf_seen |= a.n_units > 0
    assert ovf_seen
    if zipf:
        assert hub_seen


def test_group_build_halves_default_group_on_overflow(monkeypatch):
    """A default-size group whose overflow units pass the 29-bit pointer limit is rebuilt
    with half as many tiles (16 -> 8 -> ...) instead of raising; its tiles are the per-tile
    build's bit for bit. An explicit group still raises. (The limit is lowered to a few
    hundred units so a small Zipf graph reaches it.)"""
    from lgcnhs import ops
    U, I, tile = 700, 900, 64
    A = _inter(U, I, 30000, seed=5, zipf=True)
    a = RP.PerTileWeights(A, 0.5, tile, vthr=8)
    sizes = []
    for j0 in range(0, I, tile):
        a.build(j0)
        sizes.append(a.n_units)
    # a limit every pair of tiles fits under and the first 16 tiles do not
    lim = max(sizes[t] + sizes[t + 1] for t in range(len(sizes) - 1)) + 65
    assert sum(sizes[:16]) + 64 >= lim
    monkeypatch.setattr(ops, "OVF_UNITS_MAX", lim)
    b = ops.TileWeights(A, 0.5, tile, vthr=8)
    assert b.group == 16 or b.group == -(-I // tile)
    for j0 in range(0, I, tile):
        a.build(j0)
        b.build(j0)
        assert (a.j0, a.width, a.n_units) == (b.j0, b.width, b.n_units)
        assert torch.equal(a.lines, b.lines)
        assert torch.equal(a.bound, b.bound) and torch.equal(a.row_len, b.row_len)
        assert np.array_equal(a.dense().view(np.uint64), b.dense().view(np.uint64))
    assert b.group < 16
    c = ops.TileWeights(A, 0.5, tile, vthr=8, group=16)
    with pytest.raises(ValueError, match="29-bit"):
        c.build(0)


@pytest.mark.parametrize("k", [1, 10, 33, 100])
@pytest.mark.parametrize("tile", [64, 333, 4096])
@pytest.mark.parametrize("mode", ["G_drop", "drop", "none"])
def test_spread_topk_tiled_equals_dense(k, tile, mode):
    from lgcnhs import ops
    U, I, d = 300, 1000, 64
    A = _inter(U, I, 9000, seed=11, zipf=True)
    g = torch.Generator(device=DEV).manual_seed(3)
    eu = torch.randn(U, d, device=DEV, generator=g) * 0.1
    ei = torch.randn(I, d, device=DEV, generator=g) * 0.1
    use_g = mode == "G_drop"
    drop = mode != "none"
    lam = 0.4
    W = ops.hybrid_weight(ops.spread_general(A), A.k_item, lam)
    kw = dict(eu=eu if use_g else None, ei=ei if use_g else None)
    v0, i0 = ops.spread_topk(A, W, k, A.by_user, drop=drop, **kw)
    # the fused walk; the two-kernel reference (tests/_ref_paths.py: F written by the
    # reference walk, then lg_tile_topk_f64) with scratch for one tile (span = tile) and for
    # several tiles per top-k merge gives the same lists bit for bit
    vf, if_ = ops.spread_topk_tiled(A, lam, k, A.by_user, drop=drop, tile=tile, **kw)
    compare_lists_close(vf.cpu().numpy(), if_.cpu().numpy(), v0.cpu().numpy(), i0.cpu().numpy(),
                        label=f"tiled vs dense k={k} tile={tile} {mode}")
    for scratch in (1, 3 * U * 8 * tile):
        v1, i1 = RP.spread_topk_two_kernel(A, lam, k, A.by_user, drop=drop, tile=tile,
                                           scratch_bytes=scratch, **kw)
        assert torch.equal(i1, if_), scratch
        assert torch.equal(v1.view(torch.int64), vf.view(torch.int64)), scratch


def test_spread_topk_tiled_user_shards():
    """users= slices (the multi-GPU shard) give the rows of the full run."""
    from lgcnhs import ops
    U, I = 500, 700
    A = _inter(U, I, 10000, seed=2)
    v, i = ops.spread_topk_tiled(A, 0.5, 20, A.by_user, tile=200)
    for a, b in ((0, 130), (130, 131), (131, 500)):
        vs, is_ = ops.spread_topk_tiled(A, 0.5, 20, A.by_user, users=slice(a, b), tile=200)
        assert torch.equal(is_, i[a:b]) and torch.equal(vs, v[a:b])


def test_spread_lightgcn_tiled_vs_reference(golden):
    """The tiled LGCNHS recommendation against the reference fixture (getResourceMat +
    recommendForAllUser of model/SpreadLightGCN)."""
    import pandas as pd
    from lgcnhs import ops
    from model.LightGCN.model import LightGCN
    g = golden("lightgcn_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, 3).to(DEV)
    both = np.concatenate([g["train"], g["val"]], axis=1).astype(np.int64)
    A = ops.Interactions.from_pairs(torch.as_tensor(both[0]), torch.as_tensor(both[1]), U, I,
                                    DEV)
    eu = m.users_emb.weight.detach().float().contiguous()
    ei = m.items_emb.weight.detach().float().contiguous()
    _, idx = ops.spread_topk_tiled(A, float(g["slgcn_lambda"]), k, A.by_user, eu=eu, ei=ei,
                                   tile=512)
    gaps = g["slgcn_gaps"]
    compare_topk_sets(idx.cpu().numpy(), g["slgcn_recs"], gaps,
                      tol=1e-6 * np.nanmax(np.abs(gaps)))


def test_tile_api_errors():
    from lgcnhs import ops
    A = _inter(50, 60, 500, seed=1)
    with pytest.raises(ValueError):
        ops.TileWeights(A, 0.5, 0)
    with pytest.raises(ValueError):  # groups of more than 8 tiles: tiles <= 4096 wide
        ops.TileWeights(A, 0.5, 5000, group=16)
    with pytest.raises(ValueError):
        ops.TileWeights(A, 0.5, 16, group=17)
    tw = ops.TileWeights(A, 0.5, 16)
    tw.build(0)
    with pytest.raises(ValueError):
        tw.build(48)  # not the next tile


@pytest.mark.parametrize("zipf", [False, True])
def test_general_w_exactly_symmetric(zipf):
    """general_W[i][j] and [j][i] are the same sum (common users ascending, fl(1/k_v)), so
    the reference's general_W.T overrides need no transposed tile path."""
    from lgcnhs import ops
    A = _inter(400, 600, 20000 if zipf else 8000, seed=9, zipf=zipf)
    gW = ops.spread_general(A)
    assert torch.equal(gW.view(torch.int64), gW.t().contiguous().view(torch.int64))


@pytest.mark.parametrize("method,dataset", [("ProbS", "movielens"), ("HeatS", "douban"),
                                            ("HybridS", "douban"), ("ProbS", "douban")])
def test_spread_method_tiled_dispatch_equals_dense(method, dataset):
    """spread_method_topk through the tile path (forced) = the dense path within rounding
    (values 1e-12, lists except near-ties), including the lambda / general_W.T overrides and
    the unfiltered ML-ProbS branch."""
    from lgcnhs.synth import synth_dataframes
    from model.SpreadMethod.recommend import spread_method_topk
    _, tr, va, _ = synth_dataframes(150, 400, 6000, seed=7, dist="zipf")
    unf = method == "ProbS" and dataset == "movielens"
    out = [spread_method_topk(150, 400, tr, va, method, 0.35, dataset, 15, unfiltered=unf,
                              tiled=t) for t in (False, True)]
    compare_lists_close(out[1][0].cpu().numpy(), out[1][1].cpu().numpy(),
                        out[0][0].cpu().numpy(), out[0][1].cpu().numpy(),
                        label=f"{method}/{dataset} tiled vs dense")


def _np_merge(vals, idxs, k):
    L, n, _ = vals.shape
    ov = np.full((n, k), -np.inf)
    oi = np.full((n, k), -1, np.int64)
    for r in range(n):
        v, i = vals[:, r].reshape(-1), idxs[:, r].reshape(-1)
        v, i = v[i >= 0], i[i >= 0]
        o = np.lexsort((i, -v))[:k]
        ov[r, :o.size], oi[r, :o.size] = v[o], i[o]
    return ov, oi


@pytest.mark.parametrize("k", [1, 7, 64, 100, 128])
@pytest.mark.parametrize("L", [1, 3, 8])
def test_topk_lists_merge_vs_oracle(k, L):
    """lg_topk_lists_merge_f64 = lexsort (value desc, item asc) of the union, including
    ties across lists, partially empty and fully empty lists."""
    from lgcnhs import ops
    rng = np.random.default_rng(k * 31 + L)
    n = 300
    vals = np.full((L, n, k), -np.inf)
    idxs = np.full((L, n, k), -1, np.int64)
    for l in range(L):
        for r in range(n):
            m = int(rng.integers(0, k + 1)) if r % 5 else (0 if r % 2 else k)
            ids = rng.choice(np.arange(l * 1000, (l + 1) * 1000), size=m, replace=False)
            v = rng.integers(0, 6, size=m).astype(np.float64) * 0.25  # many ties
            o = np.lexsort((ids, -v))
            vals[l, r, :m], idxs[l, r, :m] = v[o], ids[o]
    ov, oi = ops.merge_topk_lists(torch.as_tensor(vals).to(DEV), torch.as_tensor(idxs).to(DEV))
    ev, ei = _np_merge(vals, idxs, k)
    assert np.array_equal(oi.cpu().numpy(), ei)
    assert np.array_equal(ov.cpu().numpy(), ev)


def test_tile_seek_matches_searchsorted():
    from lgcnhs import ops
    A = _inter(400, 900, 9000, seed=4, zipf=True)
    rp, col = A.by_user.rowptr.cpu().numpy(), A.by_user.col.cpu().numpy()
    for j0 in (0, 1, 333, 899, 900):
        tw = ops.TileWeights(A, 0.5, 128)
        tw.seek(j0)
        want = [rp[v] + np.searchsorted(col[rp[v]:rp[v + 1]], j0) for v in range(400)]
        assert np.array_equal(tw.cur.cpu().numpy(), np.array(want))


@pytest.mark.parametrize("mode", ["G_drop", "none"])
@pytest.mark.parametrize("world,tile", [(2, 128), (3, 100), (8, 64), (5, 1000)])
def test_item_range_shards_merge_to_full(mode, world, tile):
    """The item-range shards of dist.sharded_spread_topk (each rank's tiles only, all
    users), merged, equal the single walk over all items bit for bit."""
    from lgcnhs import ops
    from lgcnhs.dist import item_range
    U, I, d, k = 260, 900, 64, 20
    A = _inter(U, I, 12000, seed=8, zipf=True)
    g = torch.Generator(device=DEV).manual_seed(5)
    eu = torch.randn(U, d, device=DEV, generator=g) * 0.1
    ei = torch.randn(I, d, device=DEV, generator=g) * 0.1
    kw = dict(eu=eu, ei=ei) if mode == "G_drop" else {}
    drop = mode != "none"
    v0, i0 = ops.spread_topk_tiled(A, 0.3, k, A.by_user, drop=drop, tile=tile, **kw)
    parts = [ops.spread_topk_tiled(A, 0.3, k, A.by_user, drop=drop, tile=tile,
                                   items=slice(*item_range(I, tile, r, world)), **kw)
             for r in range(world)]
    mv, mi = ops.merge_topk_lists(torch.stack([p[0] for p in parts]),
                                  torch.stack([p[1] for p in parts]))
    assert torch.equal(mi, i0)
    assert torch.equal(mv.view(torch.int64), v0.view(torch.int64))


@pytest.mark.parametrize("d", [32, 128])
@pytest.mark.parametrize("k", [5, 128])
def test_fused_dims_and_wide_k(d, k):
    """The fused path at the other embedding widths and at k = 128 (CAP 256 lists), users
    with fewer than k surviving columns (-1 padding), over an item sub-range."""
    from lgcnhs import ops
    U, I = 200, 600
    A = _inter(U, I, 4000, seed=12, zipf=True)
    g = torch.Generator(device=DEV).manual_seed(9)
    eu = torch.randn(U, d, device=DEV, generator=g) * 0.1
    ei = torch.randn(I, d, device=DEV, generator=g) * 0.1
    for items in (None, slice(130, 470)):
        ref = RP.spread_topk_two_kernel(A, 0.6, k, A.by_user, eu=eu, ei=ei, tile=128,
                                        scratch_bytes=1, items=items)
        got = ops.spread_topk_tiled(A, 0.6, k, A.by_user, eu=eu, ei=ei, tile=128,
                                    items=items)
        assert torch.equal(got[1], ref[1])
        assert torch.equal(got[0].view(torch.int64), ref[0].view(torch.int64))


@pytest.mark.parametrize("fused", [False, True])
def test_spread_stats_count_path_updates(fused):
    """stats["w_paths"] = sum over the users' items of the row lengths inside each tile of
    the item range: a P row holds one slot per (user, item) pair behind it (the co-occurrence
    counts of the row, A^T A), a hub row (more pairs than the tile width) one entry per
    distinct column; stats["w_bytes"] = 128 bytes per (user, item, tile) line plus 16 per
    overflow unit (run header + data; a dense hub row -- more than width / 2 + 8 entries --
    ceil(width / 2) data units)."""
    from lgcnhs import ops
    U, I = 150, 400
    A = _inter(U, I, 3000, seed=3, zipf=True)
    Ad = np.zeros((U, I))
    rp, col = A.by_user.rowptr.cpu().numpy(), A.by_user.col.cpu().numpy()
    for u in range(U):
        Ad[u, col[rp[u]:rp[u + 1]]] = 1
    C = Ad.T @ Ad  # pairs behind general_W[i][j]
    tile = 64
    for users, items in ((slice(0, U), slice(0, I)), (slice(20, 90), slice(77, 301))):
        st = {}
        fn = ops.spread_topk_tiled if fused else RP.spread_topk_two_kernel
        fn(A, 0.5, 10, A.by_user, tile=tile, users=users, items=items, stats=st,
           count_paths=True)
        uses = Ad[users].sum(0)
        paths = nbytes = 0
        for j0 in range(items.start, items.stop, tile):
            blk = C[:, j0:min(items.stop, j0 + tile)]
            pairs = blk.sum(1)
            hub = pairs > tile
            ln = np.where(hub, (blk != 0).sum(1), pairs)
            units = np.where(hub, np.where(ln > 7, 1 + ln - 7, 0),
                             np.where(ln > 31, 1 + (ln - 31 + 3) // 4, 0))
            w = blk.shape[1]
            units = np.where(hub & (ln > w // 2 + 8), 1 + (w + 1) // 2, units)
            paths += int((uses * ln).sum())
            nbytes += int((uses * (128 + 16 * units)).sum())
        assert st["w_paths"] == paths
        assert st["w_bytes"] == nbytes
        # the untimed accounting the bench uses: the same counts from the tiles alone
        assert ops.tile_traffic(A, tile, users=users, items=items) == (paths, nbytes)
    assert (C.sum(1) > tile).any(), "the zipf graph should have hub rows"


@pytest.mark.parametrize("zipf", [False, True])
def test_tile_resource_persistent_waves(zipf):
    """More users than resident waves (each persistent wave walks several users, the next
    users' row pointers and item ids prefetched), users with no items and users with more
    than 128 items (extra row batches): every F tile within 1e-12 of the dense F, and a user
    sub-range's rows bitwise those of the full walk."""
    from lgcnhs import ops
    from lgcnhs.synth import synth_interactions
    U, I = 6000, 300
    u, i = synth_interactions(U, I, 60000 if zipf else 30000, seed=21,
                              dist="zipf" if zipf else "uniform")
    keep = (u % 997) != 5                     # a few users with no items at all
    u, i = u[keep], i[keep]
    heavy = np.repeat(np.arange(3, 3000, 500), 200)
    hi = np.tile(np.arange(200) + 50, heavy.size // 200)
    u, i = np.concatenate([u, heavy]), np.concatenate([i, hi])
    A = ops.Interactions.from_pairs(torch.as_tensor(u), torch.as_tensor(i), U, I, DEV)
    assert int(A.by_user.degrees().max()) > 128 and int((A.by_user.degrees() == 0).sum()) > 0
    W = ops.hybrid_weight(ops.spread_general(A), A.k_item, 0.5)
    F = ops.spread_resource(A, W).cpu().numpy()
    tile = 128
    tw = ops.TileWeights(A, 0.5, tile)
    Fb = torch.empty((U, tile), dtype=torch.float64, device=DEV)
    first = None
    for j0 in range(0, I, tile):
        tw.build(j0)
        RP.resource(tw, 0, U, Fb)
        Ft = Fb[:, :tw.width].cpu().numpy()
        _close(Ft, F[:, j0:j0 + tw.width])
        if first is None:
            first = Ft
    # a user sub-range (the resource pass of a user block)
    Fb2 = torch.empty((2500, tile), dtype=torch.float64, device=DEV)
    tw2 = ops.TileWeights(A, 0.5, tile)
    tw2.build(0)
    RP.resource(tw2, 1000, 3500, Fb2)
    assert np.array_equal(Fb2[:, :tw2.width].cpu().numpy().view(np.uint64),
                          first[1000:3500].view(np.uint64))


@pytest.mark.parametrize("tiled", [False, True])
def test_lambda_sweep_equals_per_lambda_recommend(tiled):
    """spread_lambda_sweep (findLambda.py's loop with general_W / the W tiles and score
    bounds built once) gives, for every lambda, spread_recommend's lists bit for bit; the
    tiled sweep also with a cache too small to hold the tiles (rebuild per lambda)."""
    from lgcnhs import ops
    U, I, d = 240, 700, 64
    A = _inter(U, I, 9000, seed=13, zipf=True)
    g = torch.Generator(device=DEV).manual_seed(4)
    eu = torch.randn(U, d, device=DEV, generator=g) * 0.1
    ei = torch.randn(I, d, device=DEV, generator=g) * 0.1
    lams = [0.0, 0.31, 0.5, 0.85, 1.0]
    caches = (None, 1) if tiled else (None,)
    for cache in caches:
        got = list(ops.spread_lambda_sweep(A, lams, 12, A.by_user, True, eu, ei, tiled=tiled,
                                           tile=128, cache_bytes=cache))
        assert [g_[0] for g_ in got] == lams
        for lam, v, i in got:
            rv, ri = (ops.spread_topk_tiled(A, lam, 12, A.by_user, True, eu, ei, tile=128)
                      if tiled else ops.spread_recommend(A, lam, 12, A.by_user, True, eu, ei,
                                                         tiled=False))
            assert torch.equal(i, ri), (lam, cache)
            assert torch.equal(v.view(torch.int64), rv.view(torch.int64)), (lam, cache)


def test_find_lambda_api_rows(tmp_path):
    """findLambda.sweep_lambdas: one metrics row per lambda with the reference's columns."""
    import pandas as pd
    from lgcnhs.synth import synth_dataframes
    from model.LightGCN.model import LightGCN
    from findLambda import sweep_lambdas
    _, tr, va, te = synth_dataframes(150, 300, 5000, seed=6, dist="zipf")
    torch.manual_seed(42)
    m = LightGCN(150, 300, 64, 3).to(DEV)
    df = sweep_lambdas(m, 150, 300, tr, va, te, 10, lambdas=[0.0, 0.5, 1.0])
    assert list(df.columns) == ["lambda", "precision", "recall", "f1", "ndcg", "H", "I"]
    assert list(df["lambda"]) == [0.0, 0.5, 1.0]
    assert df[["precision", "recall", "H", "I"]].notna().all().all()
    del pd


@pytest.mark.parametrize("d", [32, 64, 128])
def test_score_bounds_cover_chain_scores_many_blocks(d):
    """lg_score_chunk_bound at a launch of many blocks (65,536 users, a full 2048-column
    tile of 32 chunks: the block's waves hand every chunk's item fragments over through
    LDS): gb and gb * q / 255 cover the exact chain score of 384 sampled users (the first
    and last blocks and random ones) on every column."""
    from lgcnhs import ops
    from oracle import lgcn_oracle as O
    g = torch.Generator().manual_seed(100 + d)
    U, W, j0 = 65536, 2048, 1000
    eu = torch.randn(U, d, generator=g) * 0.1
    ei = torch.randn(j0 + W + 7, d, generator=g) * 0.1
    ub, un = ops.bound_operands(eu.to(DEV))
    ib, inn = ops.bound_operands(ei.to(DEV))
    q = torch.zeros((U, W), dtype=torch.uint8, device=DEV)
    gb, q = ops.chunk_bounds(ub, un, ib, inn, d, j0, W, qout=q)
    rs = np.random.default_rng(d)
    users = np.unique(np.concatenate([np.arange(128), np.arange(U - 128, U),
                                      rs.choice(U, 128, replace=False)]))
    G = O.chain_scores(eu[users].numpy(), ei[j0:j0 + W].numpy()).astype(np.float64)
    gbn = gb.cpu().numpy()[users].astype(np.float64)
    qn = q.cpu().numpy()[users].astype(np.float64)
    chunk = np.arange(W) // 64
    assert np.all(gbn[:, chunk] >= G)
    colb = gbn[:, chunk] * qn / 255.0
    bad = colb < G
    assert not bad.any(), (np.argwhere(bad)[:5], colb[bad][:5], G[bad][:5])
    assert np.mean(colb - G) < np.mean(gbn[:, chunk] - G)
    # the kernel's waits leave the chunk's own stores in flight (named counts, gbound.hip):
    # gb alone (no q stores) and an odd chunk count (a lone last chunk) give the same gb bits
    gb_only = ops.chunk_bounds(ub, un, ib, inn, d, j0, W)
    assert torch.equal(gb_only.view(torch.int32), gb.view(torch.int32))
    W3 = W - 64 * 3  # 29 chunks
    q3 = torch.zeros((U, W), dtype=torch.uint8, device=DEV)
    gb3, q3 = ops.chunk_bounds(ub, un, ib, inn, d, j0, W3, qout=q3)
    assert torch.equal(gb3[:, :28].view(torch.int32), gb[:, :28].view(torch.int32))
    assert torch.equal(q3[:, :64 * 28], q[:, :64 * 28])


@pytest.mark.parametrize("W", [333, 300, 64, 1])
@pytest.mark.parametrize("d", [32, 64, 128])
def test_score_bounds_cover_chain_scores(d, W):
    """lg_score_chunk_bound: the chunk bound gb and the per-column 8-bit bounds
    gb * q / 255 are >= the exact fp32 chain score (the C chain of oracle/score_chain.c) of
    every column, including a partial last chunk and users / items with large norms. Widths:
    an even and an odd number of chunks (the q bytes go out per chunk pair, a lone last chunk
    alone), one whole chunk, one column."""
    from lgcnhs import ops
    from oracle import lgcn_oracle as O
    g = torch.Generator().manual_seed(d + W)
    U, j0 = 70, 40
    eu = torch.randn(U, d, generator=g) * 0.1
    ei = torch.randn(j0 + W + 5, d, generator=g) * 0.1
    eu[3] *= 40.0
    ei[j0 + min(7, W - 1)] *= 25.0
    ub, un = ops.bound_operands(eu.to(DEV))
    ib, inn = ops.bound_operands(ei.to(DEV))
    qs = -(-W // 256) * 256
    q = torch.zeros((U, qs), dtype=torch.uint8, device=DEV)
    gb, q = ops.chunk_bounds(ub, un, ib, inn, d, j0, W, qout=q)
    G = O.chain_scores(eu.numpy(), ei[j0:j0 + W].numpy()).astype(np.float64)  # [U, W]
    gbn = gb.cpu().numpy().astype(np.float64)
    qn = q.cpu().numpy()[:, :W].astype(np.float64)
    chunk = np.arange(W) // 64
    assert np.all(gbn[:, chunk] >= G)
    colb = gbn[:, chunk] * qn / 255.0
    bad = colb < G
    assert not bad.any(), (np.argwhere(bad)[:5], colb[bad][:5], G[bad][:5])
    # and tight: the column bound is within a few % of the chunk bound's scale of the score
    # (one column: the column bound is the chunk bound)
    if W >= 64:
        assert np.mean(colb - G) < np.mean(gbn[:, chunk] - G)
