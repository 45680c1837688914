"""World-size 2/3 CPU run (gloo) of the item-sharded spreading exchange
(lgcnhs.dist.sharded_spread_topk): item ranges per rank, the all-to-all of per-range top-k
lists to the owners of each user block, and the merge. The per-range lists come from the
oracle's dense restatement (the HIP kernels need a GPU); the merged rows must equal the
oracle's top-k over all items. The GPU side (same lists from ops.spread_topk_tiled, merged by
lg_topk_lists_merge_f64) is tests/test_gpu_spread_tiled.py."""
import os
import socket
import types

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


def _problem(U, I, n, seed, lam):
    rng = np.random.default_rng(seed)
    keys = np.unique(rng.integers(0, U, n) * I + rng.integers(0, I, n))
    A = O.interaction_matrix(U, I, keys // I, keys % I)
    W = O.hybrid_s(A, O.spreading_general_mat(A), lam)
    return A, O.get_resource(A, W)


def _cpu_local(F, ex_rowptr, ex_col):
    def local(A, lam, k, excl, drop, eu, ei, tile, items):
        Fm = np.full_like(F, -np.inf)
        Fm[:, items.start:items.stop] = F[:, items.start:items.stop]
        v, i = O.rows_topk(Fm, k, ex_rowptr, ex_col, drop)
        i = np.where(np.isneginf(v), -1, i)  # columns outside the range never surface
        return torch.as_tensor(v), torch.as_tensor(i)
    return local


def _cpu_merge(vals, idxs):
    L, n, k = vals.shape
    ov = np.full((n, k), -np.inf)
    oi = np.full((n, k), -1, np.int64)
    for r in range(n):
        v = vals[:, r].reshape(-1).numpy()
        i = idxs[:, r].reshape(-1).numpy()
        keep = i >= 0
        v, i = v[keep], i[keep]
        o = np.lexsort((i, -v))[:k]
        ov[r, :o.size], oi[r, :o.size] = v[o], i[o]
    return torch.as_tensor(ov), torch.as_tensor(oi)


def _worker(rank, world, port, U, I, n, k, tile, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lgcnhs.dist import sharded_spread_topk
        A, F = _problem(U, I, n, 4, 0.5)
        rp, col = O.exclusion_csr(U, I, np.nonzero(A))
        Ans = types.SimpleNamespace(n_users=U, n_items=I)
        (u0, u1), v, i = sharded_spread_topk(Ans, 0.5, k, None, True, rank=rank, world=world,
                                             tile=tile, local_fn=_cpu_local(F, rp, col),
                                             merge_fn=_cpu_merge)
        q.put((rank, u0, u1, v.numpy().copy(), i.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,tile", [(2, 16), (3, 7), (3, 64), (8, 5)])
def test_sharded_spread_gloo(world, tile):
    U, I, n, k = 23, 50, 300, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, U, I, n, k, tile, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    A, F = _problem(U, I, n, 4, 0.5)
    rp, col = O.exclusion_csr(U, I, np.nonzero(A))
    ev, ei = O.rows_topk(F, k, rp, col, True)
    rows = np.zeros(U, int)
    for rank, u0, u1, v, i in got:
        assert np.array_equal(i, ei[u0:u1])
        assert np.array_equal(v, ev[u0:u1])
        rows[u0:u1] += 1
    assert np.all(rows == 1), "user blocks must tile the users exactly once"
