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


def _screened_direct(eu, ei, k, ex, umarg, n_splits=1):
    """lg_score_topk_screened_f32 through the C ABI with caller-chosen margins (no host
    routing of any kind between the inputs and the kernel)."""
    from lgcnhs import _native as N
    from lgcnhs import ops
    nu, d = eu.shape
    ni = ei.shape[0]
    ub, _ = ops.bound_operands(eu)
    ib, _ = ops.bound_operands(ei)
    ws_bytes = N.lib().lg_score_topk_screened_ws_bytes(nu, ni, d, k, n_splits)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=eu.device)
    val = torch.empty((nu, k), dtype=torch.float32, device=eu.device)
    idx = torch.empty((nu, k), dtype=torch.int64, device=eu.device)
    N.check(N.lib().lg_score_topk_screened_f32(
        N.ptr(eu), N.ptr(ei), N.ptr(ub), N.ptr(ib), N.ptr(umarg), nu, ni, d,
        N.ptr(ex.rowptr), N.ptr(ex.col), float(O.MASK), int(k), int(n_splits), N.ptr(val),
        N.ptr(idx), N.ptr(ws), ws_bytes, N.stream_handle(eu.device)),
        "lg_score_topk_screened_f32")
    return val, idx


@pytest.mark.parametrize("I,k", [(3000, 20), (40000, 20), (70000, 64), (3000, 100),
                                 (120000, 100)])
def test_screened_topk_non_finite_rows(I, k):
    """lg_score_topk_screened_f32 on non-finite inputs, called directly: a NaN item row, an item
    with an +inf element, a NaN user row, a user with a -inf element, under three margin sets --
    the host's (every margin NaN: the item norms are), the margins of the finite inputs (NaN
    and infinite products under finite margins), and those with NaN / negative / +inf margins
    forced on users with finite rows. Every item of a no-bound user and every NaN-bound item
    enters and gets the exact chain, so the lists equal lg_score_topk_f32's bit for bit (NaN
    scores never rank), on one split and on several, with and without the seed pass (40,000
    items and more). 70 users: the last block has padding users, whose clamped rows are NaN."""
    from lgcnhs import ops
    U, d = 70, 64
    eu, ei = _emb(U, d, 41), _emb(I, d, 42)
    clean_u, clean_i = eu.clone(), ei.clone()
    ei[1234] = float("nan")
    ei[2000, 5] = float("inf")
    eu[7] = float("nan")
    eu[11, 3] = -float("inf")
    eu[U - 1] = float("nan")  # the row padding users clamp to
    rp, col = _excl(U, I, 0.01, 43)
    ex = _rowsets(rp, col, U, I)
    eu, ei = eu.to(DEV), ei.to(DEV)
    v0, i0 = ops.score_topk(eu, ei, k, ex, n_splits=1, screen=False)
    _, un, ue = ops.bound_operands(eu, with_err=True)
    _, inorm, ierr = ops.bound_operands(ei, with_err=True)
    host = ops.screen_margins(un, ue, inorm, ierr, d)
    assert torch.isnan(host).all()
    _, cun, cue = ops.bound_operands(clean_u.to(DEV), with_err=True)
    _, cin, cie = ops.bound_operands(clean_i.to(DEV), with_err=True)
    clean = ops.screen_margins(cun, cue, cin, cie, d)
    assert torch.isfinite(clean).all()
    forced = clean.clone()
    forced[3], forced[4], forced[5] = float("nan"), -1.0, float("inf")
    for name, m in (("host", host), ("clean", clean), ("forced", forced)):
        for ns in (1, 3):
            v, i = _screened_direct(eu, ei, k, ex, m, n_splits=ns)
            assert torch.equal(i, i0), (name, ns)
            assert torch.equal(v.view(torch.int32), v0.view(torch.int32)), (name, ns)
    i0 = i0.cpu().numpy()
    ok = np.ones(U, bool)
    ok[[7, 11, U - 1]] = False
    assert (i0[ok] >= 0).all() and not (i0 == 1234).any()
    # the +inf item ranks first wherever its chain is +inf
    assert (i0[:, 0] == 2000).sum() > 0
    # the product path: ops.score_topk's screened default on the same inputs, no host sync
    v, i = ops.score_topk(eu, ei, k, ex, screen=True)
    assert np.array_equal(i.cpu().numpy(), i0)


@pytest.mark.parametrize("d,k", [(64, 1), (64, 20), (64, 32), (64, 64), (64, 100), (64, 128),
                                 (32, 20), (32, 64), (32, 128), (128, 20), (128, 32),
                                 (128, 64), (128, 100), (128, 128)])
def test_seeded_topk_exclusions_in_seed_range(d, k):
    """The screened kernel's seed pass (catalogs of >= 1024 k items): every user's threshold
    starts at the (k + E)-th largest of the lower bounds kept per item class over the first
    1/16 of the items (the class maximum for k <= 32, the 4 largest per class above), E = its
    excluded items there. Users whose best items of that range are excluded (E from 0 to 60:
    the seed must skip them, and there is none once k + E exceeds the candidates), items tied
    in bf16 and exactly inside the range, a zero user, users scaled over 1e-2..1e2: the lists
    equal the plain kernel's and the C oracle's bit for bit. Every seed shape: d = 32 / 64
    (64 classes: R = 1 for k <= 32, 4 above) and d = 128 (32 classes: R = 2 for k <= 32,
    4 above through its own k <= 128 launch)."""
    from lgcnhs import ops
    U = 200
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


@pytest.mark.parametrize("d,k", [(64, 20), (64, 100), (32, 20), (32, 128), (128, 20),
                                 (128, 100), (128, 128)])
def test_score_topk_large_catalog_sample(d, k):
    """1M-item catalog (the C5 item count), 256 users: bit-exact vs the C oracle (seeded
    screened kernel, every width and list size)."""
    from lgcnhs import ops
    U, I = 256, 1_000_000
    eu, ei = _emb(U, d, 7), _emb(I, d, 8)
    rp, col = _excl(U, I, 1e-4, 9)
    ov, oi = O.chain_topk(eu.numpy(), ei.numpy(), rp, col, k)
    v, i = ops.score_topk(eu.to(DEV), ei.to(DEV), k, _rowsets(rp, col, U, I), screen=True)
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


@pytest.mark.parametrize("k", [20, 100])
def test_screened_topk_catalog_over_2_20_items(k):
    """The screened kernel's list entries hold a 16-bit tile index, so lg_score_topk_screened_f32
    splits a catalog of more than 2^20 items (here 1,100,017: two splits even when one is asked
    for, the workspace sized by lg_score_topk_ws_bytes for it): bit-exact vs the C oracle, with
    a 20-user block whose best items sit past item 2^20."""
    from lgcnhs import _native as N
    from lgcnhs import ops
    U, I = 96, 1_100_017
    assert N.lib().lg_score_topk_ws_bytes(U, I, 64, k, 1) == 2 * U * k * 8
    assert N.lib().lg_score_topk_screened_ws_bytes(U, I, 64, k, 1) == \
        2 * U * k * 8 + (0 if k <= 32 else 2 * U * 256 * 8)
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

