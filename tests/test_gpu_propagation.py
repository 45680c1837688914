"""GPU parity of the propagation path (K0 gcn_norm, K1 SpMM + fused layer mean) against
the golden vectors of the reference and the CPU oracle. Tolerance: 1e-4 absolute on fp32
embeddings (BASELINE.json north_star); observed differences are ~1e-7."""
import numpy as np
import pytest
import torch

from oracle import lgcn_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = "cuda"


def _adj_from_coo(coo, n):
    from lgcnhs.graph import Adjacency
    return Adjacency.from_edge_index(torch.as_tensor(coo).long().to(DEV), n)


@pytest.mark.parametrize("name", ["lightgcn_toy", "lightgcn_edge", "lightgcn_mid"])
def test_gcn_norm_weights_match_reference(golden, name):
    g = golden(name)
    U, I = int(g["n_users"]), int(g["n_items"])
    adj = _adj_from_coo(g["train_coo"], U + I)
    w = adj.edge_weight().cpu().numpy()
    # the fixture COO is (row=source, col=target) sorted by row; the CSR is target-major.
    coo = g["train_coo"].astype(np.int64)
    order = np.lexsort((coo[0], coo[1]))  # by (target, source)
    # torch-CPU pow(-0.5) is a vectorised rsqrt (differs from IEEE 1/sqrt in the last bit
    # for ~0.5% of degrees, CPU-ISA dependent); the kernel computes 1/sqrt, so each dis is
    # <= 1 ulp off and the product dis[s]*dis[t] <= 3 ulp.
    np.testing.assert_array_max_ulp(w, g["gcn_w"][order], maxulp=3)


@pytest.mark.parametrize("name", ["lightgcn_toy", "lightgcn_edge", "lightgcn_mid"])
@pytest.mark.parametrize("L", [1, 2, 3])
def test_forward_matches_reference(golden, name, L):
    from model.LightGCN.model import LightGCN
    g = golden(name)
    U, I = int(g["n_users"]), int(g["n_items"])
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, L)
    assert np.array_equal(m.users_emb.weight.detach().numpy(), g["e0_u"])  # same init stream
    m = m.to(DEV)
    with torch.no_grad():
        uf, u0, itf, i0 = m.forward(torch.as_tensor(g["train_coo"]).long())
    np.testing.assert_allclose(uf.cpu().numpy(), g[f"out_u_L{L}"], rtol=0, atol=TOL)
    np.testing.assert_allclose(itf.cpu().numpy(), g[f"out_i_L{L}"], rtol=0, atol=TOL)
    err = max(np.abs(uf.cpu().numpy() - g[f"out_u_L{L}"]).max(),
              np.abs(itf.cpu().numpy() - g[f"out_i_L{L}"]).max())
    assert err < 1e-6, err


def _synth_graph(U, I, E, seed, dist="uniform"):
    from lgcnhs.synth import synth_interactions
    return synth_interactions(U, I, E, seed=seed, dist=dist)


@pytest.mark.parametrize("dim", [32, 64, 128, 256])
@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_forward_vs_oracle_synthetic(dim, dist):
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    U, I, E = 3000, 2000, 60000
    users, items = _synth_graph(U, I, E, seed=7, dist=dist)
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items), U, I, DEV)
    coo = torch.as_tensor(O.coo_adjacency(U, I, users, items))
    assert torch.equal(adj.edge_index().cpu(), coo)
    gen = torch.Generator().manual_seed(1)
    e0 = (torch.randn(U + I, dim, generator=gen) * 0.1).float()
    uf, itf = O.lightgcn_forward(coo, e0[:U], e0[U:], 3)
    out = ops.propagate(adj, e0.to(DEV), 3).cpu()
    np.testing.assert_allclose(out.numpy(), torch.cat([uf, itf]).numpy(), rtol=0, atol=TOL)


def test_forward_deterministic_and_layers0():
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    users, items = _synth_graph(5000, 5000, 200000, seed=3)
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items),
                                      5000, 5000, DEV)
    e0 = torch.randn(10000, 64, device=DEV) * 0.1
    a = ops.propagate(adj, e0, 3)
    b = ops.propagate(adj, e0, 3)
    assert torch.equal(a, b)  # no atomics: bitwise reproducible
    assert torch.equal(ops.propagate(adj, e0, 0), e0)


def test_backward_matches_autograd_oracle():
    """grad of sum(out * R) through the HIP op == torch autograd through the PyG-style
    restatement (symmetric graph: backward is the same operator)."""
    from model.LightGCN.model import LightGCN
    users, items = _synth_graph(400, 600, 8000, seed=11)
    U, I = 400, 600
    coo = torch.as_tensor(O.coo_adjacency(U, I, users, items))
    torch.manual_seed(42)
    m = LightGCN(U, I, 64, 3)
    wu = m.users_emb.weight.detach().clone().requires_grad_(True)
    wi = m.items_emb.weight.detach().clone().requires_grad_(True)
    R = torch.randn(U + I, 64)
    uf, itf = O.lightgcn_forward(coo, wu, wi, 3)
    (torch.cat([uf, itf]) * R).sum().backward()
    m = m.to(DEV)
    uf2, _, itf2, _ = m.forward(coo)
    (torch.cat([uf2, itf2]) * R.to(DEV)).sum().backward()
    np.testing.assert_allclose(m.users_emb.weight.grad.cpu().numpy(), wu.grad.numpy(),
                               rtol=0, atol=TOL)
    np.testing.assert_allclose(m.items_emb.weight.grad.cpu().numpy(), wi.grad.numpy(),
                               rtol=0, atol=TOL)


def test_asymmetric_graph_forward_backward():
    """A directed edge_index (PyG semantics: deg from targets, messages source->target)."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    rng = np.random.default_rng(5)
    n = 500
    ei = torch.as_tensor(np.unique(rng.integers(0, n, (2, 6000)), axis=1)).long()
    adj = Adjacency.from_edge_index(ei.to(DEV), n)
    assert adj.symmetric is False
    x = (torch.randn(n, 64) * 0.1).requires_grad_(True)
    ein, w = O.gcn_norm(ei, n)
    ref = [x]
    cur = x
    for _ in range(2):
        cur = O.propagate(ein, w, cur)
        ref.append(cur)
    ref = torch.stack(ref, 1).mean(1)
    R = torch.randn(n, 64)
    (ref * R).sum().backward()
    xg = x.detach().to(DEV).requires_grad_(True)
    out = ops.propagate(adj, xg, 2)
    (out * R.to(DEV)).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=TOL, rtol=0)
    np.testing.assert_allclose(xg.grad.cpu().numpy(), x.grad.numpy(), atol=TOL, rtol=0)


def test_large_graph_properties():
    """At a C4-like scale (200K x 200K, 4M interactions): layer-1 rows against an exact
    fp64 gather on sampled rows, and linearity of the whole 3-layer operator."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    U = I = 200_000
    users, items = _synth_graph(U, I, 4_000_000, seed=21)
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items), U, I, DEV)
    n = U + I
    x = torch.randn(n, 64, device=DEV) * 0.1
    y = torch.empty_like(x)
    from lgcnhs import _native as N
    ops.spmm_layer(adj, x, y, None, None, None, N.LG_ACC_NONE, 1.0)
    y2 = torch.empty_like(x)
    ops.spmm_layer(adj, x, y2, None, None, None, N.LG_ACC_NONE, 1.0, stream_weights=False)
    assert torch.equal(y, y2)  # streamed weights == recomputed dis[s]*dis[g], bitwise
    rowptr, src, dis = adj.rowptr.cpu().numpy(), adj.src.cpu().numpy(), adj.dis().cpu().numpy()
    xc = x.cpu().numpy().astype(np.float64)
    yc = y.cpu().numpy()
    for r in np.random.default_rng(0).integers(0, n, 64):
        s = src[rowptr[r]:rowptr[r + 1]]
        exact = ((dis[s].astype(np.float64) * dis[r]) [:, None] * xc[s]).sum(0)
        np.testing.assert_allclose(yc[r], exact, rtol=0, atol=1e-5)
    z = torch.randn(n, 64, device=DEV) * 0.1
    lhs = ops.propagate(adj, 2.0 * x + z, 3)
    rhs = 2.0 * ops.propagate(adj, x, 3) + ops.propagate(adj, z, 3)
    assert (lhs - rhs).abs().max().item() < 1e-5


def test_power_law_hub_rows_segmented():
    """Zipf(1.1) items: hub rows above the long-row threshold go through the segmented
    path; the result matches the oracle and the one-wave-per-row path, and repeats bitwise."""
    from lgcnhs import ops, _native as N
    from lgcnhs import graph as G
    from lgcnhs.graph import Adjacency
    U, I, E = 60_000, 5_000, 600_000
    users, items = _synth_graph(U, I, E, seed=9, dist="zipf")
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items), U, I, DEV)
    deg = (adj.rowptr[1:] - adj.rowptr[:-1]).cpu()
    assert int(deg.max()) > 4 * G.LONG_ROW_THRESHOLD  # real hubs
    plan = adj.long_plan()
    assert plan.n_long > 0 and plan.n_seg > plan.n_long
    e0 = (torch.randn(U + I, 64, generator=torch.Generator().manual_seed(3)) * 0.1)
    out = ops.propagate(adj, e0.to(DEV), 2)
    assert torch.equal(out, ops.propagate(adj, e0.to(DEV), 2))
    coo = torch.as_tensor(O.coo_adjacency(U, I, users, items))
    uf, itf = O.lightgcn_forward(coo, e0[:U], e0[U:], 2)
    np.testing.assert_allclose(out.cpu().numpy(), torch.cat([uf, itf]).numpy(), rtol=0, atol=TOL)
    x = e0.to(DEV)
    y1, y2 = torch.empty_like(x), torch.empty_like(x)
    ops.spmm_layer(adj, x, y1, None, None, None, N.LG_ACC_NONE, 1.0, long_rows=True)
    ops.spmm_layer(adj, x, y2, None, None, None, N.LG_ACC_NONE, 1.0, long_rows=False)
    np.testing.assert_allclose(y1.cpu().numpy(), y2.cpu().numpy(), rtol=0, atol=1e-6)


def test_captured_graph_replay_matches_eager():
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    users, items = _synth_graph(943, 1682, 80000, seed=1)
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items),
                                      943, 1682, DEV)
    pg = ops.PropagationGraph(adj, 64, 3)
    for seed in (0, 1):
        e0 = torch.randn(943 + 1682, 64, device=DEV, generator=torch.Generator(device=DEV).manual_seed(seed)) * 0.1
        assert torch.equal(pg.run(e0).clone(), ops.propagate(adj, e0, 3))


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("cls", ["rows", "bipartite"])
def test_sharded_layouts_single_rank_equal_propagate(cls, chunks):
    """The multi-GPU drivers (lgcnhs.dist) on the HIP layer at world 1: the chunk-major and
    the bipartite segment layouts (users / items sharded separately, half order alternating
    per layer) give exactly ops.propagate's result."""
    from lgcnhs import ops
    from lgcnhs.dist import (BipartitePropagation, RowShard, SegmentShard,
                             ShardedPropagation)
    from lgcnhs.graph import Adjacency
    from lgcnhs.synth import synth_interactions
    U, I, d, L = 3000, 2000, 64, 3
    u, i = synth_interactions(U, I, 40000, seed=6, dist="zipf")
    adj = Adjacency.from_interactions(torch.as_tensor(u), torch.as_tensor(i), U, I, "cuda")
    e0 = torch.randn(U + I, d, device="cuda", generator=torch.Generator("cuda").manual_seed(1)) * 0.1
    want = ops.propagate(adj, e0, L)
    w = adj.edge_weight()
    if cls == "rows":
        sh = RowShard(adj.rowptr, adj.src, U + I, 0, 1, "cuda", weight=w, chunks=chunks)
        prop = ShardedPropagation(sh, sh.permute_rows(adj.dis()), d, L, "cuda")
    else:
        sh = SegmentShard(adj.rowptr, adj.src, [0, U, U + I], 0, 1, "cuda", weight=w,
                          chunks=chunks)
        assert sh.is_bipartite()
        prop = BipartitePropagation(sh, sh.permute_rows(adj.dis()), d, L, "cuda")
    got = sh.unpermute_rows(prop.forward(sh.permute_rows(e0)))
    assert torch.equal(got, want)


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
@pytest.mark.parametrize("dim", [64, 128])
def test_live_mask_backward_equals_dense(dist, dim):
    """The backward of a mini-batch loss: the input gradient is non-zero on a few rows, so
    the sparse-input layers (lg_spmm_layer_live_f32) skip the dead rows' gathers. The sums
    equal the dense kernel's bitwise (zero rows add 0), including hub rows on the segmented
    path, and the autograd gradient equals the dense propagate of the same gradient."""
    from lgcnhs import ops, _native as N
    from lgcnhs.graph import Adjacency
    U, I, E = (60_000, 5_000, 600_000) if dist == "zipf" else (40_000, 30_000, 800_000)
    users, items = _synth_graph(U, I, E, seed=5, dist=dist)
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items), U, I, DEV)
    n = U + I
    g = torch.zeros(n, dim, device=DEV)
    rows = torch.randint(0, n, (700,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    g[rows] = torch.randn(rows.numel(), dim, device=DEV)
    live = ops.live_rows(g)
    assert int(live.sum()) == int(torch.unique(rows).numel())
    y1, y2 = torch.empty_like(g), torch.empty_like(g)
    ops.spmm_layer(adj, g, y1, None, None, None, N.LG_ACC_NONE, 1.0)
    ops.spmm_layer(adj, g, y2, None, None, None, N.LG_ACC_NONE, 1.0, live=live)
    assert torch.equal(y1, y2)
    dense = ops.propagate_mean(adj, g, 3)
    sparse = ops.propagate_mean(adj, g, 3, sparse_input=True)
    assert torch.equal(dense, sparse)
    e0 = (torch.randn(n, dim, device=DEV) * 0.1).requires_grad_(True)
    out = ops.propagate(adj, e0, 3)
    (out * g).sum().backward()
    assert torch.equal(e0.grad, dense)
    with pytest.raises(ValueError):
        ops.spmm_layer(adj, g, y2, None, None, None, N.LG_ACC_NONE, 1.0,
                       live=live.to(torch.int32))


@pytest.mark.parametrize("dist,force", [("uniform", False), ("uniform", True), ("zipf", False),
                                        ("zipf", True)])
@pytest.mark.parametrize("L", [1, 2, 3, 4])
def test_restricted_forward_rows_equal_full_forward(dist, force, L):
    """The training step's forward (ops.propagate_rows: each layer only at the rows the
    mini-batch's final embeddings depend on, lg_spmm_layer_rows_f32 / the masked segmented
    path for hub rows / lg_mark_neighbors_u8) gives the full forward's rows bit for bit, with
    duplicate nodes, under the default layer plan (full below the restricted layers) and with
    every layer masked; its gradient equals the full forward + gather's."""
    from lgcnhs import ops
    from lgcnhs.graph import Adjacency
    U, I, E = (60_000, 5_000, 600_000) if dist == "zipf" else (40_000, 30_000, 300_000)
    users, items = _synth_graph(U, I, E, seed=7, dist=dist)
    adj = Adjacency.from_interactions(torch.as_tensor(users), torch.as_tensor(items), U, I, DEV)
    if dist == "zipf":
        assert adj.long_plan().n_long > 0
    n, d = U + I, 64
    gen = torch.Generator(device=DEV).manual_seed(L)
    e0 = torch.randn(n, d, device=DEV, generator=gen) * 0.1
    nodes = torch.cat([torch.randint(0, U, (300,), device=DEV, generator=gen),
                       U + torch.randint(0, I, (600,), device=DEV, generator=gen)])
    nodes[5] = nodes[17]  # a duplicate
    if dist == "zipf":  # the hub items' rows (segmented path) among the nodes
        deg = adj.rowptr[1:] - adj.rowptr[:-1]
        nodes[:8] = torch.topk(deg, 8).indices
    full = ops.propagate(adj, e0, L)
    got = ops.propagate_rows_mean(adj, e0, L, nodes, force_masks=force)
    assert torch.equal(got, full[nodes])
    masks = ops.row_masks(adj, nodes.long(), L, force=force)
    assert masks[L - 1] is not None and int(masks[L - 1].sum()) == int(torch.unique(nodes).numel())
    if force or L == 1:
        assert all(m is not None for m in masks)
    # autograd: the restricted rows' gradient = the full forward's + the gather's (distinct
    # nodes: no accumulation order in between)
    nd = torch.unique(nodes)
    w = torch.randn(nd.numel(), d, device=DEV, generator=gen)
    a = e0.clone().requires_grad_(True)
    (ops.propagate_rows(adj, a, L, nd) * w).sum().backward()
    b = e0.clone().requires_grad_(True)
    (ops.propagate(adj, b, L)[nd] * w).sum().backward()
    assert torch.equal(a.grad, b.grad)
