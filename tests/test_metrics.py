"""Recommendation metrics (reference metrics/accurate.py,
metrics/diversity.py). CPU: the oracle's restatement against the reference's own outputs
(tests/golden/metrics_*.npz from make_golden_metrics.py). GPU: the reference-signature
mirror (metrics/accurate.py, metrics/diversity.py of the package) on the HIP kernels
against the same fixtures and the oracle, and the exact-integer Hamming closed form at a
size the reference's O(U^2) loop cannot reach."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O

CASES = ["ml100k_lgcn", "ml100k_hybrid", "mid_k50", "mid_k100", "edge"]


def _inputs(g):
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    tr, va, te = (g[n].astype(np.int64) for n in ("train", "val", "test"))
    test_d, train_d, val_d = O.pos_dict(te), O.pos_dict(tr), O.pos_dict(va)
    A = O.interaction_matrix(U, I, np.concatenate([tr[0], va[0]]), np.concatenate([tr[1], va[1]]))
    return U, I, k, g["recs"].astype(np.int64), test_d, O.item_degrees(train_d, val_d), A


@pytest.mark.parametrize("name", ["ml100k_lgcn", "mid_k50", "edge"])
def test_oracle_metrics_vs_reference(golden, name):
    g = golden(f"metrics_{name}")
    U, I, k, recs, test_d, deg, A = _inputs(g)
    p, r = O.precision_recall(test_d, recs, k)
    assert (p, r) == (float(g["P"]), float(g["R"]))
    assert O.f1_score(p, r) == float(g["F1"])
    assert O.ndcg(test_d, recs, k) == float(g["NDCG"])
    assert O.internal_similarity(recs, deg, A, k) == float(g["I"])
    if U <= 300:  # the O(U^2) pair loop; the ML-100K shape takes ~10 s in Python
        assert O.hamming_distance(recs, k) == float(g["H"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_metrics_vs_reference(golden, name):
    """The package's getAccurateMetrics / getDiversityMetrics on the HIP kernels give the
    reference's rounded values (P/R/F1/NDCG through the reference's own fp32 reductions of
    the device labels; H exact in integers; I per term bit-exact, fp64 sum order)."""
    from metrics.accurate import getAccurateMetrics
    from metrics.diversity import getDiversityMetrics
    g = golden(f"metrics_{name}")
    U, I, k, recs, test_d, deg, A = _inputs(g)
    rt = torch.as_tensor(recs).cuda()
    P, R, F1, NDCG = getAccurateMetrics(test_d, rt, k)
    assert (P, R, F1, NDCG) == tuple(float(g[n]) for n in ("P", "R", "F1", "NDCG"))
    H, Is = getDiversityMetrics(rt, deg, A, k)
    assert H == float(g["H"])
    assert Is == float(g["I"])


@pytest.mark.gpu
def test_gpu_pair_overlap_exact_and_hamming_large():
    """sum_{u != v} |R_u & R_v| by the item-count closed form equals a direct count (dense
    0/1 incidence product) on 3000 users, including lists with repeated items and -1 pads."""
    from lgcnhs import metrics as M
    rng = np.random.default_rng(3)
    U, I, k = 3000, 400, 30
    recs = rng.integers(0, I, size=(U, k))
    recs[::7, 5] = recs[::7, 4]     # repeated items count once (set semantics)
    recs[::11, -3:] = -1            # padding matches nothing
    B = np.zeros((U, I), np.int64)
    for u in range(U):
        r = recs[u][recs[u] >= 0]
        B[u, np.unique(r)] = 1
    G = B @ B.T
    want = int(G.sum() - np.trace(G))
    got = M.pair_overlap(torch.as_tensor(recs).cuda(), I)
    assert got == want
    h = M.hamming(torch.as_tensor(recs).cuda(), k, I)
    assert abs(h - (U * (U - 1) - want / k) / (U * (U - 1))) < 1e-15


@pytest.mark.gpu
def test_gpu_intra_similarity_parts_vs_oracle():
    """Per (user, position) partial sums: each pair term equals the reference's arithmetic
    bit for bit; hub columns (> 2048 users, global-memory path) included."""
    from lgcnhs import metrics as M
    from lgcnhs.graph import RowSets
    rng = np.random.default_rng(5)
    U, I, k = 5000, 60, 12
    # items 0..2 are hubs held by most users
    A = (rng.random((U, I)) < 0.05).astype(np.float64)
    A[:, :3] = (rng.random((U, 3)) < 0.8)
    deg = A.sum(0).astype(np.int64)
    deg[7] = 0  # a zero-degree item is skipped (reference: item_degree_dict.get(i, 0))
    recs = np.stack([rng.choice(I, size=k, replace=False) for _ in range(64)])
    recs[:, 0] = rng.integers(0, 3, size=64)
    users, items = np.nonzero(A)
    by_item = RowSets.from_pairs(torch.as_tensor(items), torch.as_tensor(users), I, U, "cuda")
    part = M.intra_similarity_parts(torch.as_tensor(recs).cuda(), by_item,
                                    torch.as_tensor(deg)).cpu().numpy().reshape(64, k)
    for r in range(64):
        for p in range(k):
            a, s = recs[r, p], 0.0
            for q in range(p + 1, k):
                b = recs[r, q]
                if a == b or deg[a] == 0 or deg[b] == 0:
                    continue
                s += np.dot(A[:, a], A[:, b]) / np.sqrt(int(deg[a]) * int(deg[b]))
            assert part[r, p] == s, (r, p)


@pytest.mark.gpu
def test_gpu_metric_api_errors():
    from metrics.accurate import calF1Score, calPrecisionAndRecall
    from metrics.diversity import calHammingDistance, calInternalSimilarity
    with pytest.raises(ZeroDivisionError):
        calF1Score(0.0, 0.0)
    with pytest.raises(ZeroDivisionError):
        calHammingDistance(torch.zeros((1, 3), dtype=torch.int64).cuda(), 3)
    with pytest.raises(ZeroDivisionError):
        calInternalSimilarity(torch.zeros((4, 1), dtype=torch.int64).cuda(), {0: 1},
                              np.ones((2, 3)), 1)
    with pytest.raises(IndexError):
        calPrecisionAndRecall({9: [1]}, torch.zeros((4, 3), dtype=torch.int64).cuda(), 3)
