"""Row-sharded multi-GPU propagation: one process per GPU, RCCL all-gather over xGMI,
overlapped with the SpMM.

SURVEY.md §8(e). Rank r owns the contiguous original rows [r*C*S, (r+1)*C*S) of A_hat
(equal row counts; the benchmark's uniform graphs are nnz-balanced that way), cut into C
sub-chunks of S rows. Every rank keeps a full replica of the layer input x. Per layer it
runs the SpMM kernel on one sub-chunk at a time and, as soon as sub-chunk c is done,
starts an asynchronous ``all_gather_into_tensor`` of it (RCCL runs on its own stream)
while the kernel works on sub-chunk c+1; the next layer waits for all C gathers. Only the
last gather of a layer is exposed.

For the gathers to land in place, node ids live in a *chunk-major* layout:
    new(g) = c*(W*S) + r*S + i      for original g = r*(C*S) + c*S + i
so sub-chunk c of every rank is one contiguous block of W*S rows in rank order, which is
exactly what ``all_gather_into_tensor`` writes. ``src`` ids, dis and e0 are permuted into
that layout once; the output is permuted back on demand. C = 1 is the plain row shard.

The per-shard layer is pluggable so the bookkeeping can run on CPU with gloo
(tests/test_dist_gloo.py); on GPUs it is lg_spmm_layer_f32.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


def acc_mode(l: int, layers: int) -> int:
    first, last = l == 0, l == layers - 1
    if first and last:
        return 4  # LG_ACC_ONLY
    if first:
        return 1  # LG_ACC_FIRST
    if last:
        return 3  # LG_ACC_LAST
    return 2  # LG_ACC_MID


class RowShard:
    """This rank's rows of a CSR over n_nodes nodes, in the chunk-major layout."""

    def __init__(self, rowptr: torch.Tensor, src: torch.Tensor, n_nodes: int, rank: int,
                 world: int, device=None, weight: torch.Tensor | None = None,
                 chunks: int = 1):
        self.n_nodes, self.rank, self.world, self.chunks = int(n_nodes), rank, world, chunks
        self.S = math.ceil(self.n_nodes / (world * chunks))
        self.n_pad = self.S * world * chunks
        dev = device if device is not None else rowptr.device
        self.device = dev
        g0 = min(rank * chunks * self.S, self.n_nodes)
        g1 = min(self.n_nodes, g0 + chunks * self.S)
        b, e = int(rowptr[g0]), int(rowptr[g1])
        self.g0, self.g1 = g0, g1
        self.rowptr = (rowptr[g0:g1 + 1] - b).to(dev)
        src_local = src[b:e].to(dev)
        self.src = self.to_layout(src_local.to(torch.int64)).to(torch.int32) if (world > 1 or chunks > 1) else src_local
        self.weight = None if weight is None else weight[b:e].to(dev)
        self.nnz = e - b
        # (local row begin, local row end, output row offset) per sub-chunk
        self.pieces = []
        for c in range(chunks):
            lb = min(c * self.S, g1 - g0)
            le = min((c + 1) * self.S, g1 - g0)
            self.pieces.append((lb, le, c * world * self.S + rank * self.S))

    @property
    def n_rows(self) -> int:
        return self.g1 - self.g0

    # ------------------------------------------------------------------ layout maps
    def to_layout(self, g: torch.Tensor) -> torch.Tensor:
        """original node id -> chunk-major id."""
        CS = self.chunks * self.S
        r, o = g // CS, g % CS
        c, i = o // self.S, o % self.S
        return c * (self.world * self.S) + r * self.S + i

    def permute_rows(self, t: torch.Tensor) -> torch.Tensor:
        """[n_nodes, ...] in original order -> [n_pad, ...] chunk-major (zero padding)."""
        out = torch.zeros((self.n_pad,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        out[self.to_layout(torch.arange(self.n_nodes, device=t.device))] = t
        return out

    def unpermute_rows(self, t: torch.Tensor) -> torch.Tensor:
        return t[self.to_layout(torch.arange(self.n_nodes, device=t.device))]


def hip_layer(shard: RowShard, piece, dis, x, y, x0, acc, out, mode, denom):
    from .graph import LONG_ROW_SEGMENT, LONG_ROW_THRESHOLD, LongRowPlan
    from .ops import run_layer
    lb, le, off = piece
    if le <= lb:
        return
    plans = shard.__dict__.setdefault("_plans", {})
    if piece not in plans:
        plans[piece] = LongRowPlan(shard.rowptr[lb:le + 1], off, LONG_ROW_THRESHOLD,
                                   LONG_ROW_SEGMENT)
    run_layer(shard.rowptr[lb:], shard.src, dis, shard.weight, x, y, x0, acc, out, le - lb,
              off, mode, denom, plans[piece])


def _gather_block(buf: torch.Tensor, shard: RowShard, c: int, group=None, async_op=True):
    W, S = shard.world, shard.S
    blk = buf[c * W * S:(c + 1) * W * S]
    mine = blk[shard.rank * S:(shard.rank + 1) * S]
    if dist.get_backend(group) == "gloo":
        return dist.all_gather([blk[r * S:(r + 1) * S] for r in range(W)], mine.clone(),
                               group=group, async_op=async_op)
    return dist.all_gather_into_tensor(blk, mine, group=group, async_op=async_op)


class ShardedPropagation:
    """mean_{l<=L} A_hat^l e0 on this rank's rows, all-gathers overlapped with the SpMM."""

    def __init__(self, shard: RowShard, dis_layout: torch.Tensor, dim: int, layers: int,
                 device, layer_fn=hip_layer, group=None):
        self.shard, self.dis, self.layers, self.group = shard, dis_layout, layers, group
        self.layer_fn = layer_fn
        n_pad = shard.n_pad
        self.bufs = [torch.zeros(n_pad, dim, device=device),
                     torch.zeros(n_pad, dim, device=device) if layers > 2 else None]
        self.out = torch.zeros(n_pad, dim, device=device)
        self.events = None  # optional list of (start, end) event pairs around each layer

    def forward(self, e0_layout: torch.Tensor, gather_out: bool = False) -> torch.Tensor:
        """e0_layout: [n_pad, d] layer-0 embeddings in the chunk-major layout (replicated).
        Returns the [n_pad, d] output (chunk-major); rows of other ranks are valid only
        with gather_out."""
        sh = self.shard
        x = e0_layout
        L = self.layers
        for l in range(L):
            last = l == L - 1
            y = None if last else self.bufs[l % 2]
            mode = acc_mode(l, L)
            handles = []
            if self.events is not None:
                s = torch.cuda.Event(enable_timing=True)
                s.record()
            for c, piece in enumerate(sh.pieces):
                self.layer_fn(sh, piece, self.dis, x, y, e0_layout, self.out, self.out, mode,
                              L + 1)
                if not last and sh.world > 1:
                    handles.append(_gather_block(y, sh, c, self.group))
            if self.events is not None:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                self.events.append((s, e))
            for h in handles:
                h.wait()
            x = y
        if gather_out and sh.world > 1:
            for c in range(sh.chunks):
                _gather_block(self.out, sh, c, self.group, async_op=False)
        return self.out


# ------------------------------------------------------------------ spreading (K3s)
def item_range(n_items: int, tile: int, rank: int, world: int) -> tuple[int, int]:
    """Rank r's contiguous run of whole item tiles (the last tile may be short)."""
    n_tiles = -(-n_items // tile) if n_items else 0
    t0, t1 = rank * n_tiles // world, (rank + 1) * n_tiles // world
    return min(n_items, t0 * tile), min(n_items, t1 * tile)


def user_block(n_users: int, rank: int, world: int) -> tuple[int, int]:
    return rank * n_users // world, (rank + 1) * n_users // world


def exchange_topk(vals: torch.Tensor, idxs: torch.Tensor, rank: int, world: int,
                  group=None):
    """[U, k] lists over this rank's item range, all users -> [world, n_own, k] lists of this
    rank's user block, one per item range (rank order): one all-to-all (RCCL over xGMI)."""
    U, k = vals.shape
    sizes = [user_block(U, r, world)[1] - user_block(U, r, world)[0] for r in range(world)]
    own = sizes[rank]
    dev = vals.device
    if dist.get_backend(group) == "gloo":  # rehearsal backend: host tensors only
        vals, idxs = vals.cpu(), idxs.cpu()
    ov = torch.empty((world * own, k), dtype=vals.dtype, device=vals.device)
    oi = torch.empty((world * own, k), dtype=idxs.dtype, device=idxs.device)
    dist.all_to_all_single(ov, vals.contiguous(), [own] * world, sizes, group=group)
    dist.all_to_all_single(oi, idxs.contiguous(), [own] * world, sizes, group=group)
    return ov.view(world, own, k).to(dev), oi.view(world, own, k).to(dev)


def sharded_spread_topk(A, lam: float, k: int, excl, drop: bool = True, eu=None, ei=None,
                        rank: int = 0, world: int = 1, group=None, tile: int = 2048,
                        scratch_bytes: int = 16 << 30, local_fn=None, merge_fn=None):
    """The LGCNHS recommendation (model/SpreadLightGCN/model.py:122-153 + recommend.py:18-52)
    over `world` GPUs, sharded by ITEM range: rank r builds only its own tiles of W
    (user-independent work is never repeated across ranks) and scores every user on them;
    an all-to-all hands each rank the per-range lists of its user block, which are merged.
    Returns ((u0, u1), values [n_own, k] fp64, items [n_own, k] int64), bitwise the rows
    [u0, u1) of the single-GPU ops.spread_topk_tiled.

    local_fn / merge_fn default to the HIP path (ops.spread_topk_tiled /
    ops.merge_topk_lists); tests substitute CPU stand-ins to run the exchange on gloo."""
    from . import ops
    local_fn = local_fn or ops.spread_topk_tiled
    merge_fn = merge_fn or ops.merge_topk_lists
    i0, i1 = item_range(A.n_items, tile, rank, world)
    v, i = local_fn(A, lam, k, excl, drop, eu, ei, tile=tile, scratch_bytes=scratch_bytes,
                    items=slice(i0, i1))
    u0, u1 = user_block(A.n_users, rank, world)
    if world == 1:
        return (u0, u1), v, i
    pv, pi = exchange_topk(v, i, rank, world, group)
    del v, i
    mv, mi = merge_fn(pv, pi)
    return (u0, u1), mv, mi
