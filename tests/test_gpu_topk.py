"""GPU parity of K2 (e0 scoring + -1024 mask + top-k) and of the dense masked score matrix:
bit-exact against the C oracle's fp32 fma chain (values AND indices, ties by item id), and
tie-aware against the reference's own torch.topk results (golden fixtures)."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O
from _compare import compare_topk_sets

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _excl(U, I, density, seed):
    rng = np.random.default_rng(seed)
    n = int(U * I * density)
    u = rng.integers(0, U, n)
    i = rng.integers(0, I, n)
    return O.exclusion_csr(U, I, (u, i))


def _rowsets(rp, col, U, I):
    from lgcnhs.graph import RowSets
    return RowSets(torch.as_tensor(rp).to(DEV), torch.as_tensor(col).to(DEV), U, I)


def _emb(n, d, seed, scale=0.1):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, d, generator=g) * scale).float()


def test_mfma_chain_is_bit_exact():
    """score_dense (MFMA 16x16x4 f32) == the C fmaf chain, bit for bit, incl. subnormal-
    and large-magnitude inputs."""
    from lgcnhs import ops
    eu, ei = _emb(37, 64, 1), _emb(53, 64, 2)
    eu[0, :5] = torch.tensor([1e-39, -3e-40, 1e30, -1e30, 7.0])
    G = ops.score_dense(eu.to(DEV), ei.to(DEV)).cpu().numpy()
    ref = O.chain_scores(eu.numpy(), ei.numpy())
    assert np.array_equal(G.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("d", [32, 64, 128])
def test_score_dense_masked(d):
    from lgcnhs import ops
    U, I = 150, 333
    eu, ei = _emb(U, d, 3), _emb(I, d, 4)
    rp, col = _excl(U, I, 0.05, 5)
    G = ops.score_dense(eu.to(DEV), ei.to(DEV), _rowsets(rp, col, U, I)).cpu().numpy()
    ref = O.chain_masked_matrix(eu.numpy(), ei.numpy(), rp, col)
    assert np.array_equal(G.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("screen", [True, False])
@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("k", [1, 5, 20, 32, 33, 64, 100, 128])
def test_score_topk_bit_exact(d, k, screen):
    """lg_score_topk_screened_f32 (bf16 screen, the default) and lg_score_topk_f32: both
    bit-exact against the C chain oracle."""
    from lgcnhs import ops
    U, I = 301, 2047
    eu, ei = _emb(U, d, 10 + k), _emb(I, d, 20 + d)
    rp, col = _excl(U, I, 0.03, k)
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    for ns in (1, None, 7):
        v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I), n_splits=ns,
                              screen=screen)
        np.testing.assert_array_equal(i.cpu().numpy(), oi)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


@pytest.mark.parametrize("k", [20, 64, 100, 128])
def test_screened_topk_near_ties_and_wide_norms(k):
    """The bf16 screen's margin under stress: items that differ below bf16 resolution (their
    bf16 products tie, the fp32 chain orders them), scaled items and users over 1e-3..1e2,
    a zero user row: the screened lists equal the plain kernel's and the oracle's bit for
    bit (k = 64 / 100 / 128: lists of 2 and 4 slabs per lane, escapes among the near-copies)."""
    from lgcnhs import ops
    U, I, d = 96, 5000, 64
    eu, ei = _emb(U, d, 31), _emb(I, d, 32)
    base = ei[:40].clone()
    for r in range(1, 8):  # 7 near-copies of 40 items, each off by a sub-bf16 perturbation
        ei[40 * r:40 * r + 40] = base * (1 + r * 2.0 ** -14)
    g = torch.Generator().manual_seed(33)
    ei *= torch.exp(torch.randn(I, 1, generator=g) * 1.5)
    eu *= torch.exp(torch.randn(U, 1, generator=g) * 1.5)
    eu[5] = 0.0
    rp, col = _excl(U, I, 0.01, 34)
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I), screen=True)
    v0, i0 = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I), screen=False)
    assert torch.equal(i, i0) and torch.equal(v.view(torch.int32), v0.view(torch.int32))
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


@pytest.mark.parametrize("I", [3000, 40000])
def test_screened_topk_non_finite_rows(I):
    """A NaN item row makes every user's screen margin NaN and a NaN user row its own: the
    screened path then hands the call to the plain kernel (non-finite margins are outside the
    screened kernel's contract), so the lists stay the plain kernel's bit for bit (NaN scores
    never enter), and finite items still fill them."""
    from lgcnhs import ops
    U, d, k = 64, 64, 20
    eu, ei = _emb(U, d, 41), _emb(I, d, 42)
    ei[1234] = float("nan")
    eu[7] = float("nan")
    rp, col = _excl(U, I, 0.01, 43)
    ex = _rowsets(rp, col, U, I)
    v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, ex, screen=True)
    v0, i0 = ops.score_topk(eu.to(DEV), ei.to(DEV), k, ex, screen=False)
    assert torch.equal(i, i0) and torch.equal(v.view(torch.int32), v0.view(torch.int32))
    i = i.cpu().numpy()
    assert (i[np.arange(U) != 7] >= 0).all() and not (i == 1234).any()


@pytest.mark.parametrize("k", [1, 20, 32, 64, 100])
def test_seeded_topk_exclusions_in_seed_range(k):
    """The screened kernel's seed pass (catalogs of >= 1024 k items): every user's threshold
    starts at the (k + E)-th largest of the lower bounds kept per item class over the first
    1/16 of the items (the class maximum for k <= 32, the 4 largest per class above), E = its
    excluded items there. Users whose best items of that range are excluded (E from 0 to 60:
    the seed must skip them, and there is none once k + E exceeds the candidates), items tied
    in bf16 and exactly inside the range, a zero user, users scaled over 1e-2..1e2: the lists
    equal the plain kernel's and the C oracle's bit for bit."""
    from lgcnhs import ops
    U, d = 200, 64
    I = 65536 if k <= 64 else 131072
    eu, ei = _emb(U, d, 51 + k), _emb(I, d, 52)
    ei[100:140] = ei[60:100]  # exact ties inside the seed range
    g = torch.Generator().manual_seed(53)
    eu *= torch.exp(torch.randn(U, 1, generator=g) * 1.5)
    eu[9] = 0.0
    n_seed = I // 16
    G = O.chain_scores(eu.numpy(), ei[:n_seed].numpy())
    us, its = [], []
    for u in range(U):
        e = (u * 7) % 61  # 0..60 of the user's best seed-range items excluded
        top = np.argsort(-G[u], kind="stable")[:e]
        us += [u] * e
        its += top.tolist()
    rng = np.random.default_rng(54)
    extra = rng.integers(0, I, 2000)
    us += rng.integers(0, U, 2000).tolist()
    its += extra.tolist()
    rp, col = O.exclusion_csr(U, I, (np.array(us), np.array(its)))
    ex = _rowsets(rp, col, U, I)
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    for ns in (1, None):
        v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, ex, n_splits=ns, screen=True)
        v0, i0 = ops.score_topk(eu.to(DEV), ei.to(DEV), k, ex, n_splits=ns, screen=False)
        assert torch.equal(i, i0) and torch.equal(v.view(torch.int32), v0.view(torch.int32))
        np.testing.assert_array_equal(i.cpu().numpy(), oi)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


def test_score_topk_edge_cases():
    from lgcnhs import ops
    # fewer items than k (padding), all-excluded user (mask values surface), ties (equal
    # item rows), one user
    U, I, k = 5, 7, 10
    eu, ei = _emb(U, 64, 1), _emb(I, 64, 2)
    ei[3] = ei[1]  # exact ties between items 1 and 3
    rp, col = O.exclusion_csr(U, I, (np.array([0] * 7 + [2, 2]), np.array(list(range(7)) + [1, 5])))
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I))
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    assert (oi[:, 7:] == -1).all() and np.isinf(ov[:, 7:]).all()
    assert (ov[0] [:7] == -1024.0).all()  # every item of user 0 excluded
    v1, i1 = ops.score_topk(eu[:1].to(DEV), ei.to(DEV), 3)
    np.testing.assert_array_equal(i1.cpu().numpy(), O.chain_topk(eu[:1].numpy(), ei.numpy(),
                                                                  None, None, 3)[1])


@pytest.mark.parametrize("k", [20, 100])
def test_score_topk_large_catalog_sample(k):
    """1M-item catalog (the C5 item count), 256 users: bit-exact vs the C oracle."""
    from lgcnhs import ops
    U, I = 256, 1_000_000
    eu, ei = _emb(U, 64, 7), _emb(I, 64, 8)
    rp, col = _excl(U, I, 1e-4, 9)
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I))
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))


@pytest.mark.parametrize("name", ["lightgcn_toy", "lightgcn_edge", "lightgcn_mid",
                                  "recommend_ml100k"])
def test_recommend_for_all_user_vs_reference(golden, name):
    """model.LightGCN.recommend.recommendForAllUser == the reference's dict (fixture),
    tie-aware at 1e-6, and == the C chain oracle exactly."""
    from model.LightGCN.model import LightGCN
    from model.LightGCN.recommend import recommendForAllUser
    from utils.graph import convertEdgeIndexToAdjMatrix
    g = golden(name)
    U, I, k = int(g["n_users"]), int(g["n_items"]), int(g["k"])
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, 3).to(DEV)
    tr = convertEdgeIndexToAdjMatrix(U, I, torch.as_tensor(g["train"].astype(np.int64)))
    va = convertEdgeIndexToAdjMatrix(U, I, torch.as_tensor(g["val"].astype(np.int64)))
    recs = recommendForAllUser(m, U, I, tr, va, None, k)
    got = np.full((U, k), -1)
    for u, lst in recs.items():
        got[u, :len(lst)] = lst
    compare_topk_sets(got, g["recs"], g["rec_gaps"], tol=1e-6)
    rp, col = O.exclusion_csr(U, I, g["train"], g["val"])
    _, oi = O.chain_topk(m.users_emb.weight.detach().cpu().numpy(),
                         m.items_emb.weight.detach().cpu().numpy(), rp, col, k)
    np.testing.assert_array_equal(got, oi)


@pytest.mark.parametrize("d,n", [(32, 1001), (64, 4099), (128, 777), (48, 300)])
def test_bound_prep_rounds_and_bounds(d, n):
    """lg_bound_prep_f32 (the screen's operands): the bf16 copy is round-to-nearest-even of
    every element (torch's conversion), and the fp32 norms ||x|| and ||x - bf16(x)|| are
    rounded up -- >= the fp64 norms, within 1e-6 of them -- for the vectorised dims (32, 64,
    128) and the general kernel (48), row counts that leave partial waves."""
    from lgcnhs import ops
    g = torch.Generator().manual_seed(d + n)
    x = torch.randn(n, d, generator=g) * torch.exp(torch.randn(n, 1, generator=g) * 2)
    x[3] = 0.0
    xb, nu, ne = ops.bound_operands(x.to(DEV), with_err=True)
    assert torch.equal(xb.cpu().view(torch.int16), x.to(torch.bfloat16).view(torch.int16))
    x64 = x.double()
    n64 = x64.norm(dim=1)
    e64 = (x64 - x.to(torch.bfloat16).double()).norm(dim=1)
    for got, ref in ((nu.cpu().double(), n64), (ne.cpu().double(), e64)):
        assert (got >= ref).all()
        assert ((got - ref) <= 1e-6 * ref + 1e-38).all()


def test_screened_topk_catalog_over_2_20_items():
    """The screened kernel's list entries hold a 16-bit tile index, so lg_score_topk_screened_f32
    splits a catalog of more than 2^20 items (here 1,100,017: two splits even when one is asked
    for, the workspace sized by lg_score_topk_ws_bytes for it): bit-exact vs the C oracle, with
    a 20-user block whose best items sit past item 2^20."""
    from lgcnhs import _native as N
    from lgcnhs import ops
    U, I, k = 96, 1_100_017, 20
    assert N.lib().lg_score_topk_ws_bytes(U, I, 64, k, 1) == 2 * U * k * 8
    eu, ei = _emb(U, 64, 61), _emb(I, 64, 62)
    ei[(1 << 20) + 5:(1 << 20) + 25] = eu[:20] * 3.0  # user u's best item: 2^20 + 5 + u
    rp, col = _excl(U, I, 2e-5, 63)
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    for ns in (1, None):
        v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I), n_splits=ns,
                              screen=True)
        np.testing.assert_array_equal(i.cpu().numpy(), oi)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ov.view(np.uint32))
    assert (oi[:20, 0] >= (1 << 20)).all()

