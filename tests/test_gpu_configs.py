"""Parity at the BASELINE.json configurations' own sizes (VERDICT r01 "what's weak" 1).

C2  ML-1M shape (6040 x 3706, 1,000,209 ratings, 80/10/10): the full 3-layer forward
    against the oracle's PyG op sequence (1e-4), and the all-user top-20 against the
    reference's torch.matmul + -1024 + topk op sequence, judged by exact fp64 scores.
C4  200K x 200K, 20M interactions, d=64: the full 3-layer forward of EVERY row against a
    fp64 scipy restatement of the same operator (1e-4).
C5  1M x 1M, 100M interactions, d=128: sampled rows of the full 3-layer forward against
    fp64 three-hop sums (1e-4); the top-20 of 512 users over all 1M items against
    torch.matmul + topk; the LGCNHS (SpreadLightGCN) top-20 of sampled users against the
    oracle's fp64 sparse restatement of F = A @ HybridS(general_W) and exact G.
Zipf  the power-law input of SURVEY.md §8(d): Zipf(1.1) item popularity, uniform users. C4
    shape (200K x 200K, 20M): every row of the forward against fp64; C5 shape (1M x 1M,
    100M, d=64: hub items of ~10^6 interactions run the long-row pass): sampled rows (the
    8 highest-degree item rows among them) against fp64 three-hop sums, and the top-20 of
    512 users against torch.matmul + topk.
C3 (Douban-shape SpreadLightGCNOpti, lambda = 0.5) is pinned to the reference's own run in
test_opti_golden.py (fixture spread_opti_douban.npz).

Tie-affected users (top-k sets that differ only by items whose exact scores lie within
the two methods' rounding bounds of the k-th score) are counted and printed."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O
from _compare import compare_topk_exact

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4
U32 = 2.0 ** -24


def _gamma(n):
    return n * U32 / (1 - n * U32)


def _dot_tols(eu_row, ei, items, d):
    """|fp32 chain or BLAS dot - exact| <= gamma_d * sum |u_k i_k|, for either method."""
    return 2.0 * _gamma(d) * (np.abs(ei[items].astype(np.float64)) @
                              np.abs(eu_row.astype(np.float64))) + 1e-30


def _csr_fp64(rowptr, src, n):
    """A_hat = D^-1/2 A D^-1/2 of a symmetric CSR as scipy fp64."""
    import scipy.sparse as sp
    rp = rowptr.cpu().numpy()
    s = src.cpu().numpy()
    deg = np.diff(rp).astype(np.float64)
    dis = np.where(deg > 0, 1.0 / np.sqrt(np.maximum(deg, 1)), 0.0)
    rows = np.repeat(np.arange(n), np.diff(rp))
    w = dis[rows] * dis[s]
    return sp.csr_matrix((w, s, rp), shape=(n, n))


# -------------------------------------------------------------------------------- C2
@pytest.fixture(scope="module")
def c2():
    from lgcnhs.synth import synth_dataframes
    from model.LightGCN.model import LightGCN
    from model.LightGCN.recommend import buildGraph
    U, I = 6040, 3706
    rating_df, tr, va, te = synth_dataframes(U, I, 1_000_209, seed=1, dist="zipf")
    _, tr_coo, va_coo, _ = buildGraph(U, I, rating_df, tr, va, te)
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, 3).to(DEV)
    return U, I, tr, va, tr_coo, va_coo, m


def test_c2_forward_full(c2):
    U, I, tr, va, tr_coo, _, m = c2
    assert tr_coo.shape[1] == 2 * len(tr) and len(tr) == 800_167
    with torch.no_grad():
        uf, _, itf, _ = m.forward(tr_coo)
    ou, oi = O.lightgcn_forward(tr_coo.cpu(), m.users_emb.weight.detach().cpu(),
                                m.items_emb.weight.detach().cpu(), 3)
    np.testing.assert_allclose(uf.cpu().numpy(), ou.numpy(), rtol=0, atol=TOL)
    np.testing.assert_allclose(itf.cpu().numpy(), oi.numpy(), rtol=0, atol=TOL)


def test_c2_all_user_top20_vs_reference_ops(c2):
    from model.LightGCN.recommend import recommendForAllUser
    U, I, tr, va, tr_coo, va_coo, m = c2
    k = 20
    recs = recommendForAllUser(m, U, I, tr_coo, va_coo, None, k)
    got = np.full((U, k), -1)
    for u, lst in recs.items():
        got[u, :len(lst)] = lst
    eu = m.users_emb.weight.detach().cpu()
    ei = m.items_emb.weight.detach().cpu()
    tp = (tr.user_id.to_numpy(), tr.item_id.to_numpy())
    vp = (va.user_id.to_numpy(), va.item_id.to_numpy())
    _, ref, _ = O.recommend_topk_torch(eu, ei, tp, vp, k)
    eun, ein = eu.numpy(), ei.numpy()
    ex64 = lambda u, it: ein[it].astype(np.float64) @ eun[u].astype(np.float64)  # noqa: E731
    tol = lambda u, it: _dot_tols(eun[u], ein, it, 64)  # noqa: E731
    ties, n = compare_topk_exact(got, ref.numpy(), ex64, tol, "C2 top-20")
    assert ties <= n // 100
    # and bit-exact against the kernel's own fp32 chain order (C oracle)
    rp, col = O.exclusion_csr(U, I, tp, vp)
    _, oi = O.chain_topk(eun, ein, rp, col, k)
    np.testing.assert_array_equal(got, oi)


# -------------------------------------------------------------------------------- C4
def test_c4_forward_every_row():
    """20M interactions (40M directed nnz): every row of the 3-layer mean against fp64."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    from lgcnhs.synth import synth_graph_device
    U = I = 200_000
    rowptr, src, keys = synth_graph_device(U, I, 20_000_000, seed=4, device=DEV)
    n = U + I
    assert int(src.numel()) == 40_000_000
    adj = Adjacency(rowptr, src, n, n_users=U, symmetric=True)
    e0 = torch.randn(n, 64, device=DEV, generator=torch.Generator(DEV).manual_seed(3)) * 0.1
    out = ops.propagate(adj, e0, 3).cpu().numpy()
    assert np.array_equal(out, ops.propagate(adj, e0, 3).cpu().numpy())  # deterministic
    A = _csr_fp64(rowptr, src, n)
    x = e0.cpu().numpy().astype(np.float64)
    acc, cur = x.copy(), x
    for _ in range(3):
        cur = A @ cur
        acc += cur
    np.testing.assert_allclose(out, acc / 4, rtol=0, atol=TOL)


# -------------------------------------------------------------------------------- C5
@pytest.fixture(scope="module")
def c5():
    from lgcnhs.synth import synth_graph_device
    U = I = 1_000_000
    rowptr, src, keys = synth_graph_device(U, I, 100_000_000, seed=0, device=DEV)
    e0 = torch.randn(U + I, 128, device=DEV, generator=torch.Generator(DEV).manual_seed(42)) * 0.1
    return U, I, rowptr, src, keys, e0


def test_c5_forward_sampled_rows_d128(c5):
    """The full C5 forward (d=128); 24 sampled rows against fp64 three-hop sums
    (x + A x + A^2 x + A^3 x)/4 restricted to each row's neighbourhood."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    U, I, rowptr, src, _, e0 = c5
    n = U + I
    adj = Adjacency(rowptr, src, n, n_users=U, symmetric=True)
    out = ops.propagate(adj, e0, 3)
    rows = np.random.default_rng(5).choice(n, 24, replace=False)
    got = out[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    del out
    A = _csr_fp64(rowptr, src, n)
    x = e0.cpu().numpy().astype(np.float64)
    import scipy.sparse as sp
    for t, r in enumerate(rows):
        v = sp.csr_matrix(([1.0], ([0], [r])), shape=(1, n))
        acc = x[r].copy()
        for _ in range(3):
            v = v @ A
            acc += (v @ x).ravel()
        np.testing.assert_allclose(got[t], acc / 4, rtol=0, atol=TOL)


@pytest.mark.parametrize("k", [20, 100])
def test_c5_topk_512_users_vs_reference_ops(c5, k):
    """The product top-K dispatch (ops.score_topk's default) over all 1M items for 512 users (train|val =
    every interaction masked) against torch.matmul + -1024 index-put + torch.topk on the
    host, at k = 20 and at the reference's production k = 100 (const.py:433)."""
    from lgcnhs import ops
    from lgcnhs.graph import RowSets
    U, I, _, _, keys, e0 = c5
    nu = 512
    eu, ei = e0[:nu].contiguous(), e0[U:].contiguous()
    ku = keys[keys < nu * I]
    excl = RowSets.from_pairs(ku // I, ku % I, nu, I, DEV)
    _, got = ops.score_topk(eu, ei, k, excl)
    kc = ku.cpu().numpy()
    _, ref, _ = O.recommend_topk_torch(eu.cpu(), ei.cpu(), (kc // I, kc % I), None, k)
    eun, ein = eu.cpu().numpy(), ei.cpu().numpy()
    ex64 = lambda u, it: ein[it].astype(np.float64) @ eun[u].astype(np.float64)  # noqa: E731
    tol = lambda u, it: _dot_tols(eun[u], ein, it, 128)  # noqa: E731
    ties, n = compare_topk_exact(got.cpu().numpy(), ref.numpy(), ex64, tol,
                                 f"C5 top-{k} (512 users x 1M items)")
    assert ties <= max(2, n // 100)


def _lgcnhs_sample(A, U, n=512, top=32, seed=11):
    """512 users spread over the whole range: the `top` highest-degree users, the first and
    last user, the rest uniform at random (seeded)."""
    deg = A.by_user.degrees().cpu().numpy()
    fixed = np.unique(np.concatenate([np.argsort(-deg, kind="stable")[:top], [0, U - 1]]))
    rng = np.random.default_rng(seed)
    rest = rng.choice(np.setdiff1d(np.arange(U), fixed), n - fixed.size, replace=False)
    return np.sort(np.concatenate([fixed, rest]))


@pytest.mark.parametrize("dim", [128, 64])
def test_c5_lgcnhs_sampled_users_vs_oracle(c5, dim):
    """SpreadLightGCN at C5 (lambda 0.5, k 20, train|val dropped) for ALL 1M users through
    the tiled K3s walk (the bench's path), then 512 users spread over the range -- the 32
    highest-degree users, the first and the last, and random ones -- against the oracle's
    fp64 path-order restatement of F = A @ HybridS(general_W) (model/SpreadMethod/model.py:
    14-99) times the exact e0 dot product (model/SpreadLightGCN/model.py:151), every
    interaction dropped (recommend.py:18-52). Judged by exact scores with the rounding bounds
    of both methods (G: fp32 dot, F: fp64 sums): 0 mismatched, tie-affected <= 1 %."""
    from lgcnhs import ops
    U, I, _, _, keys, e0 = c5
    lam, k = 0.5, 20
    A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, DEV)
    eu, ei = e0[:U, :dim].contiguous(), e0[U:, :dim].contiguous()
    _, got = ops.spread_topk_tiled(A, lam, k, A.by_user, True, eu, ei)
    users = _lgcnhs_sample(A, U)
    got = got[torch.as_tensor(users, device=DEV)].cpu().numpy()
    r = O.spread_parity(got, users, A.by_user.rowptr.cpu().numpy(), A.by_user.col.cpu().numpy(),
                        A.by_item.rowptr.cpu().numpy(), A.by_item.col.cpu().numpy(), I, lam,
                        eu.cpu().numpy(), ei.cpu().numpy(), k)
    print(f"[C5 LGCNHS top-20 d={dim}] {len(users)} users: identical {r['identical']}, "
          f"tie-affected {r['tie_affected']}, mismatched {r['mismatched']}")
    assert r["mismatched"] == 0, r["first_mismatch"]
    assert r["tie_affected"] <= max(1, len(users) // 100)


# ------------------------------------------------------------------------- Zipf(1.1)
def test_c4_zipf_forward_every_row():
    """Zipf(1.1) items (hubs up to ~2e5 interactions, over half of the edges on rows past the
    long-row threshold): every row of the 3-layer mean against fp64."""
    from lgcnhs import ops
    from lgcnhs.graph import LONG_ROW_THRESHOLD, Adjacency
    from lgcnhs.synth import synth_graph_device
    U = I = 200_000
    rowptr, src, _ = synth_graph_device(U, I, 20_000_000, seed=6, device=DEV, dist="zipf")
    n = U + I
    deg = (rowptr[1:] - rowptr[:-1]).cpu().numpy()
    assert int(src.numel()) == 40_000_000 and deg.max() > 40 * LONG_ROW_THRESHOLD
    adj = Adjacency(rowptr, src, n, n_users=U, symmetric=True)
    e0 = torch.randn(n, 64, device=DEV, generator=torch.Generator(DEV).manual_seed(7)) * 0.1
    out = ops.propagate(adj, e0, 3).cpu().numpy()
    assert np.array_equal(out, ops.propagate(adj, e0, 3).cpu().numpy())  # deterministic
    A = _csr_fp64(rowptr, src, n)
    x = e0.cpu().numpy().astype(np.float64)
    acc, cur = x.copy(), x
    for _ in range(3):
        cur = A @ cur
        acc += cur
    np.testing.assert_allclose(out, acc / 4, rtol=0, atol=TOL)


def test_c4_zipf_lgcnhs_sampled_users_vs_oracle():
    """SpreadLightGCN on the power-law graph (c4-zipf: 200K x 200K, 20M Zipf(1.1)
    interactions; the top items are held by most users, so their W rows are dense V rows in
    every tile and carry most of the 3-hop paths) for ALL users through the tiled walk, then
    256 users -- the 16 highest-degree, the first and the last, random ones -- against the
    oracle (its regrouped sparse-product F, spread_rows_spmv, where a user's paths run into
    the 10^9) times the exact e0 dot product, every interaction dropped: 0 mismatched,
    tie-affected <= 1 %."""
    from lgcnhs import ops
    from lgcnhs.synth import synth_graph_device
    U = I = 200_000
    lam, k = 0.5, 20
    _, _, keys = synth_graph_device(U, I, 20_000_000, seed=6, device=DEV, dist="zipf")
    A = ops.Interactions.from_pairs(keys // I, keys % I, U, I, DEV)
    g = torch.Generator(DEV).manual_seed(43)
    eu = torch.randn(U, 64, device=DEV, generator=g) * 0.1
    ei = torch.randn(I, 64, device=DEV, generator=g) * 0.1
    _, got = ops.spread_topk_tiled(A, lam, k, A.by_user, True, eu, ei)
    users = _lgcnhs_sample(A, U, n=256, top=16)
    got = got[torch.as_tensor(users, device=DEV)].cpu().numpy()
    deg_i = A.k_item.cpu().numpy()
    assert deg_i.max() > 0.5 * U  # hub items held by most users
    r = O.spread_parity(got, users, A.by_user.rowptr.cpu().numpy(), A.by_user.col.cpu().numpy(),
                        A.by_item.rowptr.cpu().numpy(), A.by_item.col.cpu().numpy(), I, lam,
                        eu.cpu().numpy(), ei.cpu().numpy(), k)
    print(f"[c4-zipf LGCNHS top-20] {len(users)} users: identical {r['identical']}, "
          f"tie-affected {r['tie_affected']}, mismatched {r['mismatched']}")
    assert r["mismatched"] == 0, r["first_mismatch"]
    assert r["tie_affected"] <= max(1, len(users) // 100)


@pytest.fixture(scope="module")
def c5zipf():
    from lgcnhs.synth import synth_graph_device
    U = I = 1_000_000
    rowptr, src, keys = synth_graph_device(U, I, 100_000_000, seed=3, device=DEV, dist="zipf")
    e0 = torch.randn(U + I, 64, device=DEV, generator=torch.Generator(DEV).manual_seed(43)) * 0.1
    return U, I, rowptr, src, keys, e0


def test_c5_zipf_forward_sampled_rows(c5zipf):
    """The C5-shape Zipf forward (d=64): the 8 highest-degree item rows (each ~10^6 edges:
    the long-row pass) and 16 random rows against fp64 three-hop sums."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    U, I, rowptr, src, _, e0 = c5zipf
    n = U + I
    adj = Adjacency(rowptr, src, n, n_users=U, symmetric=True)
    out = ops.propagate(adj, e0, 3)
    deg = (rowptr[1:] - rowptr[:-1]).cpu().numpy()
    hubs = U + np.argsort(-deg[U:], kind="stable")[:8]
    rows = np.concatenate([hubs, np.random.default_rng(8).choice(n, 16, replace=False)])
    got = out[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    del out
    A = _csr_fp64(rowptr, src, n)
    x = e0.cpu().numpy().astype(np.float64)
    print(f"[C5 Zipf] hub degrees {deg[hubs].tolist()}")
    import scipy.sparse as sp
    for t, r in enumerate(rows):
        v = sp.csr_matrix(([1.0], ([0], [r])), shape=(1, n))
        acc = x[r].copy()
        for _ in range(3):
            v = v @ A
            acc += (v @ x).ravel()
        np.testing.assert_allclose(got[t], acc / 4, rtol=0, atol=TOL)


def test_c5_zipf_top20_512_users_vs_reference_ops(c5zipf):
    """The screened top-K over all 1M items for 512 users whose histories hold the hub items
    (every interaction masked) against torch.matmul + -1024 index-put + torch.topk."""
    from lgcnhs import ops
    from lgcnhs.graph import RowSets
    U, I, _, _, keys, e0 = c5zipf
    nu, k = 512, 20
    eu, ei = e0[:nu].contiguous(), e0[U:].contiguous()
    ku = keys[keys < nu * I]
    excl = RowSets.from_pairs(ku // I, ku % I, nu, I, DEV)
    _, got = ops.score_topk(eu, ei, k, excl)
    kc = ku.cpu().numpy()
    _, ref, _ = O.recommend_topk_torch(eu.cpu(), ei.cpu(), (kc // I, kc % I), None, k)
    eun, ein = eu.cpu().numpy(), ei.cpu().numpy()
    ex64 = lambda u, it: ein[it].astype(np.float64) @ eun[u].astype(np.float64)  # noqa: E731
    tol = lambda u, it: _dot_tols(eun[u], ein, it, 64)  # noqa: E731
    ties, n = compare_topk_exact(got.cpu().numpy(), ref.numpy(), ex64, tol,
                                 "C5 Zipf top-20 (512 users x 1M items)")
    assert ties <= max(2, n // 100)
    # bit-exact against the kernel's fp32 chain (C oracle) for the first 128 users as well
    m = kc < 128 * I
    rp, col = O.exclusion_csr(128, I, (kc[m] // I, kc[m] % I))
    _, oi = O.chain_topk(eun[:128], ein, rp, col, k)
    np.testing.assert_array_equal(got[:128].cpu().numpy(), oi)
