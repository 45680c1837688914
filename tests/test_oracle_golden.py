"""Pin the CPU oracle (oracle/) to the golden vectors produced by the reference's own code
(tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O
from _compare import compare_topk_sets

LG_CASES = ["lightgcn_toy", "lightgcn_edge", "lightgcn_mid"]


@pytest.mark.parametrize("name", LG_CASES)
def test_coo_format_matches_reference(golden, name):
    g = golden(name)
    U, I = int(g["n_users"]), int(g["n_items"])
    coo = O.coo_adjacency(U, I, g["train"][0], g["train"][1])
    np.testing.assert_array_equal(coo, g["train_coo"])
    np.testing.assert_array_equal(O.coo_to_interactions(U, I, coo), g["train_back"])


@pytest.mark.parametrize("name", LG_CASES)
def test_gcn_norm_and_init(golden, name):
    g = golden(name)
    U, I = int(g["n_users"]), int(g["n_items"])
    _, w = O.gcn_norm(torch.as_tensor(g["train_coo"]).long())
    np.testing.assert_array_equal(w.numpy(), g["gcn_w"])
    eu, ei = O.lightgcn_init(U, I, 64, seed=42)
    np.testing.assert_array_equal(eu.numpy(), g["e0_u"])
    np.testing.assert_array_equal(ei.numpy(), g["e0_i"])


@pytest.mark.parametrize("name", LG_CASES)
@pytest.mark.parametrize("L", [1, 2, 3])
def test_forward_matches_reference(golden, name, L):
    g = golden(name)
    uf, itf = O.lightgcn_forward(torch.as_tensor(g["train_coo"]).long(),
                                 torch.as_tensor(g["e0_u"]), torch.as_tensor(g["e0_i"]), L)
    np.testing.assert_allclose(uf.numpy(), g[f"out_u_L{L}"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(itf.numpy(), g[f"out_i_L{L}"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("name", LG_CASES)
def test_torch_recommend_matches_reference(golden, name):
    g = golden(name)
    k = int(g["k"])
    _, idx, _ = O.recommend_topk_torch(torch.as_tensor(g["e0_u"]), torch.as_tensor(g["e0_i"]),
                                       g["train"], g["val"], k)
    compare_topk_sets(idx.numpy(), g["recs"], g["rec_gaps"], tol=0.0)


@pytest.mark.parametrize("name", LG_CASES + ["recommend_ml100k"])
def test_chain_topk_vs_reference(golden, name):
    """The exact fp32 fma-chain scores (what the GPU computes) give the reference's top-k
    sets except at near-ties (score rounding differs by ~1e-8)."""
    g = golden(name)
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    if "e0_u" in g:
        eu, ei = g["e0_u"], g["e0_i"]
    else:
        a, b = O.lightgcn_init(U, I, 64, seed=int(g["e0_seed"]))
        e0 = torch.cat([a, b]).numpy()
        assert np.array_equal(e0[:4], g["e0_head"]), "torch RNG stream changed"
        assert abs(e0.astype(np.float64).sum() - float(g["e0_sum"])) < 1e-9
        eu, ei = a.numpy(), b.numpy()
    rp, col = O.exclusion_csr(U, I, g["train"], g["val"])
    _, idx = O.chain_topk(eu, ei, rp, col, k)
    compare_topk_sets(idx, g["recs"], g["rec_gaps"], tol=1e-6)


def _spread_case(g):
    U, I = int(g["n_users"]), int(g["n_items"])
    both = np.concatenate([g["train"], g["val"]], axis=1)
    return U, I, O.interaction_matrix(U, I, both[0], both[1])


@pytest.mark.parametrize("name", ["spread_toy", "spread_edge"])
def test_spreading_matrices(golden, name):
    g = golden(name)
    U, I, A = _spread_case(g)
    np.testing.assert_array_equal(A, g["A"])
    gW = O.spreading_general_mat(A.copy())
    np.testing.assert_allclose(gW, g["gW"], rtol=1e-13, atol=0)
    for j, lam in enumerate(g["lambdas"]):
        W = O.hybrid_s(A, g["gW"], float(lam))
        np.testing.assert_allclose(W, g[f"W_{j}"], rtol=1e-13, atol=0)
        np.testing.assert_allclose(O.get_resource(A, W), g[f"F_{j}"], rtol=1e-12, atol=1e-300)
    if "probs_W" in g:
        np.testing.assert_allclose(O.prob_s(A, g["gW"]), g["probs_W"], rtol=1e-13, atol=0)
        np.testing.assert_allclose(O.heat_s(A, g["gW"]), g["heats_W"], rtol=1e-13, atol=0)
        np.testing.assert_array_equal(O.hybrid_s(A, g["gW"], 1), g["W_int1"])
        np.testing.assert_array_equal(O.prob_s(A, g["gW"]), O.hybrid_s(A, g["gW"], 1.0))


def test_spread_edge_recs(golden):
    g = golden("spread_edge")
    U, I, A = _spread_case(g)
    F = O.get_resource(A, O.hybrid_s(A, O.spreading_general_mat(A.copy()), 0.5))
    excl = {u: np.nonzero(A[u])[0].tolist() for u in range(U)}
    recs = O.recommend_all_user(F, U, excl, int(g["k"]))
    got = np.full((U, int(g["k"])), -1)
    for u, lst in recs.items():
        got[u, :len(lst)] = lst
    # the toy has exact ties (many F == 0 items): compare as sets of tie groups
    for u in range(U):
        r = g["recs"][u][g["recs"][u] >= 0]
        gg = got[u][got[u] >= 0]
        assert len(r) == len(gg)
        np.testing.assert_array_equal(np.sort(F[u, r])[::-1], np.sort(F[u, gg])[::-1])


@pytest.mark.parametrize("tag", ["hybrid", "hybrid85", "probs_ml", "heats_db"])
def test_spread_method_recs(golden, tag):
    g = golden("spread_ml100k")
    U, I, A = _spread_case(g)
    lam = float(g[f"{tag}_lambda"])
    method, dataset = {"hybrid": ("HybridS", "movielens"), "hybrid85": ("HybridS", "movielens"),
                       "probs_ml": ("ProbS", "movielens"), "heats_db": ("HeatS", "douban")}[tag]
    gW = O.spreading_general_mat(A.copy())
    lam, gWx = O.spread_overrides(method, dataset, lam, gW)
    F = O.get_resource(A, O.hybrid_s(A, gWx, lam))
    excl = {u: np.nonzero(A[u])[0].tolist() for u in range(U)}
    recs = O.recommend_all_user(F, U, excl, int(g["k"]), unfiltered=(tag == "probs_ml"))
    got = np.array([recs[u] for u in range(U)])
    gaps = g[f"{tag}_gaps"]
    compare_topk_sets(got, g[f"{tag}_recs"], gaps, tol=1e-12 * np.nanmax(np.abs(gaps)))


def test_spread_lightgcn_recs(golden):
    g = golden("lightgcn_mid")
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    both = np.concatenate([g["train"], g["val"]], axis=1)
    A = O.interaction_matrix(U, I, both[0], both[1])
    G = O.masked_scores_torch(torch.as_tensor(g["e0_u"]), torch.as_tensor(g["e0_i"]),
                              g["train"], g["val"]).numpy()
    F = O.get_resource(A, O.hybrid_s(A, O.spreading_general_mat(A.copy()),
                                     float(g["slgcn_lambda"])))
    excl = {u: np.nonzero(A[u])[0].tolist() for u in range(U)}
    recs = O.recommend_all_user(G * F, U, excl, k)
    got = np.array([recs[u] for u in range(U)])
    gaps = g["slgcn_gaps"]
    compare_topk_sets(got, g["slgcn_recs"], gaps, tol=1e-12 * np.nanmax(np.abs(gaps)))


@pytest.mark.parametrize("lam", [0.0, 0.5, 1.0])
def test_spread_rows_sparse_equals_dense_restatement(golden, lam):
    """The oracle's list-based F rows (the C5-scale checker of test_gpu_configs.py) equal
    the dense numpy restatement pinned to the reference fixtures, to fp64 rounding."""
    g = golden("spread_ml100k")
    U, I, A = _spread_case(g)
    F = O.get_resource(A, O.hybrid_s(A, O.spreading_general_mat(A.copy()), lam))
    uu, ii = np.nonzero(A)
    urp = np.searchsorted(uu, np.arange(U + 1))
    order = np.lexsort((uu, ii))
    irp = np.searchsorted(ii[order], np.arange(I + 1))
    users = np.array([0, 5, 17, U - 1])
    Fs = O.spread_rows_sparse(urp, ii, irp, uu[order], I, users, lam)
    np.testing.assert_allclose(Fs, F[users], rtol=1e-12, atol=1e-15 * np.abs(F).max())


@pytest.mark.parametrize("name", ["spread_toy", "spread_edge"])
def test_spread_row_paths_equals_reference_F(golden, name):
    """The path-order restatement behind the C5 LGCNHS parity (spread_row_paths) against
    the reference's own F matrices (the fixtures' F_j, every lambda of the file)."""
    g = golden(name)
    U, I, A = _spread_case(g)
    uu, ii = np.nonzero(A)
    urp = np.searchsorted(uu, np.arange(U + 1))
    order = np.lexsort((uu, ii))
    irp = np.searchsorted(ii[order], np.arange(I + 1))
    for j, lam in enumerate(g["lambdas"]):
        F = np.stack([O.spread_row_paths(urp, ii, irp, uu[order], I, u, float(lam))
                      for u in range(U)])
        np.testing.assert_allclose(F, g[f"F_{j}"], rtol=1e-12,
                                   atol=1e-15 * np.abs(g[f"F_{j}"]).max())


@pytest.mark.parametrize("name", ["spread_toy", "spread_edge", "spread_ml100k"])
def test_spread_rows_spmv_equals_reference_F(golden, name):
    """The regrouped restatement for hub-heavy graphs (spread_rows_spmv: two sparse products,
    the checker of the Zipf LGCNHS parity) against the reference's own F matrices where the
    fixture holds them, and against the path-order rows (spread_row_paths) everywhere."""
    g = golden(name)
    U, I, A = _spread_case(g)
    uu, ii = np.nonzero(A)
    urp = np.searchsorted(uu, np.arange(U + 1))
    order = np.lexsort((uu, ii))
    irp = np.searchsorted(ii[order], np.arange(I + 1))
    users = np.arange(U) if U <= 64 else np.array([0, 1, 5, 17, 100, U - 1])
    lams = [float(x) for x in g["lambdas"]] if "lambdas" in g else [0.0, 0.5, 1.0]
    for j, lam in enumerate(lams):
        Fm = O.spread_rows_spmv(urp, ii, irp, uu[order], I, users, lam)
        Fp = np.stack([O.spread_row_paths(urp, ii, irp, uu[order], I, u, lam) for u in users])
        np.testing.assert_allclose(Fm, Fp, rtol=1e-13, atol=1e-16 * max(1.0, np.abs(Fp).max()))
        if f"F_{j}" in g:
            ref = g[f"F_{j}"][users]
            np.testing.assert_allclose(Fm, ref, rtol=1e-12, atol=1e-15 * np.abs(ref).max())


@pytest.mark.parametrize("method", ["paths", "spmv"])
def test_spread_parity_counts_reference_lists(golden, method):
    """spread_parity on lists taken from the dense restatement (G * F, interactions
    dropped): every user identical; a corrupted list is counted as mismatched -- with F from
    the path enumeration and from the regrouped sparse products."""
    g = golden("spread_ml100k")
    U, I, A = _spread_case(g)
    F = O.get_resource(A, O.hybrid_s(A, O.spreading_general_mat(A.copy()), 0.5))
    rng = np.random.default_rng(3)
    eu = (rng.normal(size=(U, 64)) * 0.1).astype(np.float32)
    ei = (rng.normal(size=(I, 64)) * 0.1).astype(np.float32)
    S = (eu.astype(np.float64) @ ei.astype(np.float64).T) * F
    S[A != 0] = -np.inf
    ref = np.argsort(-S, axis=1, kind="stable")[:, :10]
    uu, ii = np.nonzero(A)
    urp = np.searchsorted(uu, np.arange(U + 1))
    order = np.lexsort((uu, ii))
    irp = np.searchsorted(ii[order], np.arange(I + 1))
    users = np.arange(0, U, 7)
    r = O.spread_parity(ref[users], users, urp, ii, irp, uu[order], I, 0.5, eu, ei, 10,
                        method=method)
    assert r["identical"] == users.size and r["mismatched"] == 0
    bad = ref[users].copy()
    bad[0, 3] = int(np.argsort(S[users[0]])[I // 2])  # a mid-ranked item
    assert O.spread_parity(bad, users, urp, ii, irp, uu[order], I, 0.5, eu, ei,
                           10, method=method)["mismatched"] == 1
