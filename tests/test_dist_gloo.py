"""World-size-2 (and 3) CPU run of the row-sharded propagation bookkeeping with the gloo
backend: shard ranges, padding, per-layer all-gather and the fused layer-mean modes. The
per-shard layer is the oracle's restatement (HIP kernels need a GPU), so this checks
lgcnhs.dist exactly as bench.py drives it on RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import lgcn_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cpu_layer(shard, piece, dis, x, y, x0, acc, out, mode, denom):
    """Oracle stand-in for lg_spmm_layer_f32 over one sub-chunk of the shard's rows (all
    ids in the chunk-major layout)."""
    lb, le, off = piece
    rp = shard.rowptr.numpy()
    src = shard.src.numpy().astype(np.int64)
    for r in range(lb, le):
        g = off + (r - lb)
        s = src[rp[r]:rp[r + 1]]
        w = dis[s] * dis[g]
        v = (w[:, None] * x[s]).sum(0) if s.size else torch.zeros(x.shape[1])
        if y is not None:
            y[g] = v
        if mode == 1:
            acc[g] = x0[g] + v
        elif mode == 2:
            acc[g] = acc[g] + v
        elif mode == 3:
            out[g] = (acc[g] + v) / denom
        elif mode == 4:
            out[g] = (x0[g] + v) / denom


def _worker(rank, world, port, U, I, users, items, layers, chunks, q, bipartite=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lgcnhs.dist import RowShard, ShardedPropagation
        n = U + I
        coo = O.coo_adjacency(U, I, users, items)
        # target-major CSR (symmetric graph: same as row-major)
        rowptr = torch.as_tensor(np.searchsorted(coo[0], np.arange(n + 1)))
        src = torch.as_tensor(coo[1].astype(np.int32))
        deg = (rowptr[1:] - rowptr[:-1]).float()
        dis = deg.pow(-0.5)
        dis.masked_fill_(dis == float("inf"), 0)
        torch.manual_seed(0)
        if bipartite:
            from lgcnhs.dist import BipartitePropagation, SegmentShard
            shard = SegmentShard(rowptr, src, [0, U, n], rank, world, "cpu", chunks=chunks)
            assert shard.is_bipartite()
            e0 = shard.permute_rows(torch.randn(n, 8) * 0.1)
            prop = BipartitePropagation(shard, shard.permute_rows(dis), 8, layers, "cpu",
                                        layer_fn=cpu_layer)
        else:
            shard = RowShard(rowptr, src, n, rank, world, "cpu", chunks=chunks)
            e0 = shard.permute_rows(torch.randn(n, 8) * 0.1)
            prop = ShardedPropagation(shard, shard.permute_rows(dis), 8, layers, "cpu",
                                      layer_fn=cpu_layer)
        out = prop.forward(e0, gather_out=True)
        if rank == 0:
            q.put(shard.unpermute_rows(out).numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,layers,chunks,bipartite",
                         [(2, 3, 1, False), (2, 1, 1, False), (3, 2, 1, False),
                          (2, 3, 3, False), (3, 3, 2, False), (1, 3, 4, False),
                          (2, 3, 1, True), (3, 4, 1, True), (2, 2, 3, True), (4, 3, 2, True),
                          (1, 3, 1, True)])
def test_sharded_propagation_gloo(world, layers, chunks, bipartite):
    U, I = 13, 17
    users, items = O.coo_to_interactions(U, I, O.coo_adjacency(U, I, *np.random.default_rng(1).integers(0, [U, I], (60, 2)).T))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, U, I, users, items, layers, chunks, q, bipartite))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    torch.manual_seed(0)
    n = U + I
    e0 = torch.randn(n, 8) * 0.1
    coo = torch.as_tensor(O.coo_adjacency(U, I, users, items))
    uf, itf = O.lightgcn_forward(coo, e0[:U], e0[U:], layers)
    np.testing.assert_allclose(got, torch.cat([uf, itf]).numpy(), atol=1e-6, rtol=0)


def _worker_zipf(rank, world, port, U, I, users, items, layers, chunks, q, balance):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lgcnhs.dist import BipartitePropagation, SegmentShard
        n = U + I
        coo = O.coo_adjacency(U, I, users, items)
        rowptr = torch.as_tensor(np.searchsorted(coo[0], np.arange(n + 1)))
        src = torch.as_tensor(coo[1].astype(np.int32))
        deg = (rowptr[1:] - rowptr[:-1]).float()
        dis = deg.pow(-0.5)
        dis.masked_fill_(dis == float("inf"), 0)
        torch.manual_seed(0)
        shard = SegmentShard(rowptr, src, [0, U, n], rank, world, "cpu", chunks=chunks,
                             balance=balance)
        e0 = shard.permute_rows(torch.randn(n, 8) * 0.1)
        prop = BipartitePropagation(shard, shard.permute_rows(dis), 8, layers, "cpu",
                                    layer_fn=cpu_layer)
        out = prop.forward(e0, gather_out=True)
        q.put((rank, shard.nnz, shard.unpermute_rows(out).numpy().copy() if rank == 0 else None,
               shard.pad_ratio))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_nnz_balanced_shards_zipf(world):
    """Zipf item popularity (s = 0.5: hub item rows up to ~0.8 % of the edges): the
    bipartite shards cut each segment by cumulative non-zeros, so every rank's edge count
    is within 5 % of the mean (equal-row cuts are not: the popular items sit in the first
    rows of the item segment), and the sharded forward still equals the oracle's."""
    from lgcnhs.synth import synth_interactions
    U, I = 4000, 4000
    users, items = synth_interactions(U, I, 80_000, seed=3, dist="zipf", zipf_s=0.5)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_zipf,
                         args=(r, world, port, U, I, users, items, 3, 2, q, "nnz"))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    nnz = np.array([g[1] for g in sorted(got, key=lambda g: g[0])], np.float64)
    assert nnz.sum() == 2 * users.size
    assert np.abs(nnz - nnz.mean()).max() <= 0.05 * nnz.mean(), nnz
    # the pieces are capped at 2x the mean piece length: padding (replicated tables and
    # all-gathered rows beyond n) stays bounded
    assert max(g[3] for g in got) <= 2.0 + 2 * world * 2 / (U + I), [g[3] for g in got]
    out = [g[2] for g in got if g[0] == 0][0]
    torch.manual_seed(0)
    e0 = torch.randn(U + I, 8) * 0.1
    coo = torch.as_tensor(O.coo_adjacency(U, I, users, items))
    uf, itf = O.lightgcn_forward(coo, e0[:U], e0[U:], 3)
    np.testing.assert_allclose(out, torch.cat([uf, itf]).numpy(), atol=1e-6, rtol=0)


def test_piece_bounds_cap_bounds_padding():
    """A power-law row range whose heavy rows come first: uncapped nnz cuts give the last
    piece most of the rows (padding ~parts-fold); the cap holds every piece to max_rows x the
    mean length and still covers the range monotonically."""
    from lgcnhs.dist import piece_bounds
    deg = np.concatenate([np.full(50, 2000), np.ones(9950, np.int64)])
    rowptr = torch.as_tensor(np.concatenate([[0], np.cumsum(deg)]))
    for parts in (4, 8, 16):
        free = piece_bounds(rowptr, 0, deg.size, parts, max_rows=0)
        capped = piece_bounds(rowptr, 0, deg.size, parts)
        lf = np.diff(free)
        lc = np.diff(capped)
        assert lf.max() > 2 * deg.size / parts  # the pathology the cap removes
        assert capped[0] == 0 and capped[-1] == deg.size and (lc >= 0).all()
        assert lc.max() <= -(-int(2.0 * deg.size) // parts)


def test_piece_bounds_balance_and_rows():
    """piece_bounds: nnz cuts hold every piece within one row's edges of the ideal share;
    'rows' reproduces the equal-row cuts."""
    from lgcnhs.dist import piece_bounds
    rng = np.random.default_rng(0)
    deg = rng.zipf(1.5, 5000).clip(max=300)
    rowptr = torch.as_tensor(np.concatenate([[0], np.cumsum(deg)]))
    for parts in (1, 2, 7, 16):
        b = piece_bounds(rowptr, 0, 5000, parts)
        assert b[0] == 0 and b[-1] == 5000 and all(x <= y for x, y in zip(b, b[1:]))
        sizes = np.diff(rowptr.numpy()[b])
        assert np.abs(sizes - deg.sum() / parts).max() <= deg.max()
        r = piece_bounds(rowptr, 100, 5000, parts, balance="rows")
        S = -(-4900 // parts)
        assert r == [min(5000, 100 + p * S) for p in range(parts)] + [5000]
    with pytest.raises(ValueError):
        piece_bounds(rowptr, 0, 10, 2, balance="bogus")
