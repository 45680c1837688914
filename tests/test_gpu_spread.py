"""GPU parity of the hybrid-spreading path (K3 general_W / HybridS / F, K4 row top-k with
the G factor) against the reference's own numpy results (golden fixtures) and the oracle.
fp64 tolerance: 1e-12 relative (only the summation order differs)."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O
from _compare import compare_topk_sets

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 1e-12


def _A(g):
    U, I = int(g["n_users"]), int(g["n_items"])
    both = np.concatenate([g["train"], g["val"]], axis=1).astype(np.int64)
    return U, I, O.interaction_matrix(U, I, both[0], both[1])


@pytest.mark.parametrize("name", ["spread_toy", "spread_edge"])
def test_numpy_api_matches_reference(golden, name):
    from model.SpreadMethod import model as sm
    g = golden(name)
    U, I, A = _A(g)
    gW = sm.getSpreadingGeneralMat(A)
    np.testing.assert_allclose(gW, g["gW"], rtol=RTOL, atol=0)
    assert np.array_equal(gW, gW.T)  # ascending-order sums: exactly symmetric
    for j, lam in enumerate(g["lambdas"]):
        W = sm.HybridS(A, g["gW"], float(lam))
        np.testing.assert_allclose(W, g[f"W_{j}"], rtol=RTOL, atol=0)
        F = sm.getResource(A, W)
        np.testing.assert_allclose(F, g[f"F_{j}"], rtol=RTOL, atol=1e-300)
    if "probs_W" in g:
        np.testing.assert_allclose(sm.ProbS(A, g["gW"]), g["probs_W"], rtol=RTOL, atol=0)
        np.testing.assert_allclose(sm.HeatS(A, g["gW"]), g["heats_W"], rtol=RTOL, atol=0)
        np.testing.assert_allclose(sm.HybridS(A, g["gW"], 1), g["W_int1"], rtol=RTOL, atol=0)


def test_hybrid_transpose_and_rows_topk_exact():
    from lgcnhs import ops
    rng = np.random.default_rng(3)
    n = 77
    gW = rng.random((n, n))
    k_item = rng.integers(0, 5, n).astype(np.float64)
    Wt = ops.hybrid_weight(torch.as_tensor(gW).to(DEV), torch.as_tensor(k_item).to(DEV), 0.3,
                           transpose=True).cpu().numpy()
    np.testing.assert_allclose(Wt, O.hybrid_s(np.ones((1, n)) * k_item, gW.T, 0.3), rtol=1e-15)
    # rows_topk is exact selection: identical to the oracle on the same F, incl. ties
    F = np.round(rng.random((40, 300)) * 8) / 8  # many exact ties
    rp, col = O.exclusion_csr(40, 300, (rng.integers(0, 40, 900), rng.integers(0, 300, 900)))
    from lgcnhs.graph import RowSets
    ex = RowSets(torch.as_tensor(rp).to(DEV), torch.as_tensor(col).to(DEV), 40, 300)
    for k in (1, 7, 64, 65, 128):
        for drop in (True, False):
            v, i = ops.rows_topk(torch.as_tensor(F).to(DEV), k, ex, drop=drop)
            ov, oi = O.rows_topk(F, k, rp, col, drop=drop)
            np.testing.assert_array_equal(i.cpu().numpy(), oi)
            np.testing.assert_array_equal(v.cpu().numpy(), ov)
    # rows of >= 4096 columns: 8 waves per row, their lists merged (ties across the waves'
    # column ranges: the smaller column first, as in one ascending scan)
    F = np.round(rng.random((12, 5001)) * 4) / 4
    F[3, :] = 0.5  # one row all ties
    rp, col = O.exclusion_csr(12, 5001, (rng.integers(0, 12, 3000), rng.integers(0, 5001, 3000)))
    ex = RowSets(torch.as_tensor(rp).to(DEV), torch.as_tensor(col).to(DEV), 12, 5001)
    for k in (1, 20, 64, 100, 128):
        v, i = ops.rows_topk(torch.as_tensor(F).to(DEV), k, ex, drop=True)
        ov, oi = O.rows_topk(F, k, rp, col, drop=True)
        np.testing.assert_array_equal(i.cpu().numpy(), oi)
        np.testing.assert_array_equal(v.cpu().numpy(), ov)
    # and with the G factor: the fp32 chain score (oracle/score_chain.c) times F, in fp64
    eu = (rng.standard_normal((12, 64)) * 0.1).astype(np.float32)
    ei = (rng.standard_normal((5001, 64)) * 0.1).astype(np.float32)
    GF = O.chain_scores(eu, ei).astype(np.float64) * F
    v, i = ops.rows_topk(torch.as_tensor(F).to(DEV), 20, ex, drop=True,
                         eu=torch.as_tensor(eu).to(DEV), ei=torch.as_tensor(ei).to(DEV))
    ov, oi = O.rows_topk(GF, 20, rp, col, drop=True)
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    np.testing.assert_array_equal(v.cpu().numpy(), ov)


@pytest.mark.parametrize("tag", ["hybrid", "hybrid85", "probs_ml", "heats_db"])
def test_recommend_spread_method_vs_reference(golden, tag):
    import pandas as pd
    from const import cfg
    from model.SpreadMethod.recommend import recommendSpreadMethod
    g = golden("spread_ml100k")
    U, I, A = _A(g)
    method, dataset = {"hybrid": ("HybridS", "movielens"), "hybrid85": ("HybridS", "movielens"),
                       "probs_ml": ("ProbS", "movielens"), "heats_db": ("HeatS", "douban")}[tag]
    tr = pd.DataFrame({"user_id": g["train"][0].astype(np.int64), "item_id": g["train"][1].astype(np.int64)})
    va = pd.DataFrame({"user_id": g["val"][0].astype(np.int64), "item_id": g["val"][1].astype(np.int64)})
    cfg.DATA_SET, cfg.MODEL["name"] = dataset, method
    cfg.MODEL["HyperParameter"] = {"lambda": float(g[f"{tag}_lambda"])}
    cfg.RECOMMEND["k"] = int(g["k"])
    try:
        recs = recommendSpreadMethod(U, I, tr, va, method)
    finally:
        cfg.DATA_SET = "movielens"
    got = np.array([recs[u] for u in range(U)])
    gaps = g[f"{tag}_gaps"]
    compare_topk_sets(got, g[f"{tag}_recs"], gaps, tol=RTOL * np.nanmax(np.abs(gaps)))


def test_spread_lightgcn_vs_reference(golden):
    """The fused LGCNHS path (F blocks x fp32 e0 score inside the top-k kernel) against
    the reference's getResourceMat + recommendForAllUser (fixture)."""
    import pandas as pd
    from model.LightGCN.model import LightGCN
    from model.SpreadLightGCN.recommend import spread_lightgcn_topk
    g = golden("lightgcn_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, 3).to(DEV)
    tr = pd.DataFrame({"user_id": g["train"][0].astype(np.int64), "item_id": g["train"][1].astype(np.int64)})
    va = pd.DataFrame({"user_id": g["val"][0].astype(np.int64), "item_id": g["val"][1].astype(np.int64)})
    _, idx = spread_lightgcn_topk(m, U, I, tr, va, float(g["slgcn_lambda"]), k)
    gaps = g["slgcn_gaps"]
    compare_topk_sets(idx.cpu().numpy(), g["slgcn_recs"], gaps,
                      tol=1e-6 * np.nanmax(np.abs(gaps)))


def test_dense_api_G_times_F_path(golden):
    """getAllocateMat-style G (dense, masked) times getHybridSResourceMat F through the
    numpy API, then recommendForAllUser: same recs as the fused path."""
    import pandas as pd
    from model.LightGCN.model import LightGCN
    from model.SpreadLightGCN.model import allocate_from_model, getHybridSResourceMat
    from model.SpreadLightGCN.recommend import recommendForAllUser, spread_lightgcn_topk
    from model.SpreadMethod.model import getSpreadingGeneralMat
    from utils.graph import convertEdgeIndexToAdjMatrix
    g = golden("lightgcn_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, 3).to(DEV)
    trp, vap = g["train"].astype(np.int64), g["val"].astype(np.int64)
    G = allocate_from_model(m, U, I, convertEdgeIndexToAdjMatrix(U, I, torch.as_tensor(trp)),
                            convertEdgeIndexToAdjMatrix(U, I, torch.as_tensor(vap))).cpu().numpy()
    Gref = O.chain_masked_matrix(g["e0_u"], g["e0_i"], *O.exclusion_csr(U, I, trp, vap))
    assert np.array_equal(G.view(np.uint32), Gref.view(np.uint32))
    A = O.interaction_matrix(U, I, np.concatenate([trp[0], vap[0]]), np.concatenate([trp[1], vap[1]]))
    F = getHybridSResourceMat(A, getSpreadingGeneralMat(A), float(g["slgcn_lambda"]))
    tr = pd.DataFrame({"user_id": trp[0], "item_id": trp[1]})
    va = pd.DataFrame({"user_id": vap[0], "item_id": vap[1]})
    recs = recommendForAllUser(G * F, U, tr, va, k)
    _, idx = spread_lightgcn_topk(m, U, I, tr, va, float(g["slgcn_lambda"]), k)
    np.testing.assert_array_equal(np.array([recs[u] for u in range(U)]), idx.cpu().numpy())


@pytest.mark.parametrize("zipf,U,I,n,heavy", [(False, 300, 900, 9000, 0),
                                              (True, 400, 9000, 40000, 0),
                                              (True, 50, 4096, 3000, 0), (False, 20, 4097, 200, 0),
                                              (False, 200, 9000, 20000, 3)])
def test_spread_hybrid_equals_general_then_hybrid(zipf, U, I, n, heavy):
    """lg_spread_hybrid_f64 (general_W and HybridS in one pass, the dense recommend path)
    writes W bit for bit as lg_spread_general_f64 -> lg_hybrid_weight_f64 does, transposed
    or not (general_W is exactly symmetric), over several 4096-column ranges, with items no
    user holds (k = 0: den == 0 -> 1) and at lambda 0 and 1. `heavy` users hold more than 256
    items inside one 4096-column range (Douban-style heavy users: k_spread_hybrid's strided
    loop past the block's 256 threads): 300, 1000 and 3000 items of range 0 and 700 of
    range 1."""
    from lgcnhs import ops
    rng = np.random.default_rng(U + I)
    items = (rng.zipf(1.3, n) - 1) % I if zipf else rng.integers(0, I - I // 10, n)
    users = rng.integers(0, U, n)
    for h, cnt in enumerate((300, 1000, 3000)[:heavy]):
        users = np.concatenate([users, np.full(cnt, h)])
        items = np.concatenate([items, rng.choice(4096, cnt, replace=False)])
    if heavy:
        users = np.concatenate([users, np.full(700, 0)])
        items = np.concatenate([items, 4096 + rng.choice(4096, 700, replace=False)])
    key = np.unique(users.astype(np.int64) * I + items)
    if heavy:  # the strided loop is reached: some user has > 256 items in one range
        ku, ki = key // I, key % I
        assert max(int(((ku == h) & (ki < 4096)).sum()) for h in range(heavy)) > 256
    A = ops.Interactions.from_pairs(torch.as_tensor(key // I), torch.as_tensor(key % I), U, I,
                                    DEV)
    assert bool((A.k_item == 0).any())
    gW = ops.spread_general(A)
    for lam in (0.0, 0.37, 1.0):
        W = ops.spread_hybrid(A, lam)
        for tr in (False, True):
            ref = ops.hybrid_weight(gW, A.k_item, lam, transpose=tr)
            assert torch.equal(W.view(torch.int64), ref.view(torch.int64)), (lam, tr)
