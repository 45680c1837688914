"""Row-sharded multi-GPU propagation: one process per GPU, RCCL all-gather over xGMI.

SURVEY.md §8(e): the N = U+I rows of A_hat are split into `world` contiguous ranges of
`chunk = ceil(N / world)` rows; rank r owns rows [r*chunk, (r+1)*chunk) of the CSR and
of every embedding buffer. Each rank keeps a full (padded) replica of the layer input x;
per layer it runs the SpMM kernel on its own rows, writing them into its slice of the next
layer's buffer, then ``all_gather_into_tensor`` rebuilds the full buffer on every rank
(the only exchange step of the path). The layer-mean accumulator stays local. Equal row
counts keep node ids unchanged (no relabelling); the uniform synthetic graphs of the
benchmark are nnz-balanced under equal row counts.

The per-shard layer is pluggable so that the bookkeeping can be exercised on CPU with
the gloo backend (tests/test_dist_gloo.py); on GPUs it is lg_spmm_layer_f32.
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
    """Rows [r0, r1) of a CSR held by one rank, with rowptr rebased to the local src."""

    def __init__(self, rowptr: torch.Tensor, src: torch.Tensor, n_nodes: int, rank: int,
                 world: int, device=None, weight: torch.Tensor | None = None):
        self.n_nodes, self.rank, self.world = int(n_nodes), rank, world
        self.chunk = math.ceil(self.n_nodes / world)
        self.n_pad = self.chunk * world
        self.r0 = min(rank * self.chunk, self.n_nodes)
        self.r1 = min(self.n_nodes, self.r0 + self.chunk)
        dev = device if device is not None else rowptr.device
        b = int(rowptr[self.r0])
        e = int(rowptr[self.r1])
        self.rowptr = (rowptr[self.r0:self.r1 + 1] - b).to(dev)
        self.src = src[b:e].to(dev)
        self.weight = None if weight is None else weight[b:e].to(dev)
        self.nnz = e - b

    @property
    def n_rows(self) -> int:
        return self.r1 - self.r0


def hip_layer(shard: RowShard, dis, x, y, x0, acc, out, mode, denom):
    from . import _native as N
    N.check(N.lib().lg_spmm_layer_f32(
        N.ptr(shard.rowptr), N.ptr(shard.src), N.ptr(dis), N.ptr(shard.weight), N.ptr(x),
        N.ptr(y), N.ptr(x0),
        N.ptr(acc), N.ptr(out), shard.n_rows, shard.r0, x.shape[1], mode, float(denom),
        N.stream_handle(x.device)), "lg_spmm_layer_f32")


def all_gather_rows(buf: torch.Tensor, shard: RowShard, group=None) -> None:
    """Rebuild the full [n_pad, d] buffer from every rank's [chunk, d] slice, in place."""
    c = shard.chunk
    mine = buf[shard.rank * c:(shard.rank + 1) * c]
    if dist.get_backend(group) == "gloo":
        dist.all_gather([buf[r * c:(r + 1) * c] for r in range(shard.world)], mine.clone(),
                        group=group)
    else:
        dist.all_gather_into_tensor(buf, mine, group=group)


class ShardedPropagation:
    """mean_{l<=L} A_hat^l e0 for this rank's rows, with a per-layer all-gather."""

    def __init__(self, shard: RowShard, dis: torch.Tensor, dim: int, layers: int,
                 device, layer_fn=hip_layer, group=None):
        self.shard, self.dis, self.layers, self.group = shard, dis, layers, group
        self.layer_fn = layer_fn
        n_pad = shard.n_pad
        self.bufs = [torch.zeros(n_pad, dim, device=device),
                     torch.zeros(n_pad, dim, device=device) if layers > 2 else None]
        self.out = torch.zeros(n_pad, dim, device=device)
        self.events = None  # optional list of (start, end) event pairs around each layer

    def forward(self, e0: torch.Tensor, gather_out: bool = False) -> torch.Tensor:
        """e0: full [n_pad, d] layer-0 embeddings (replicated). Returns the [n_pad, d]
        output buffer; rows outside this rank's range are valid only with gather_out."""
        x = e0
        L = self.layers
        for l in range(L):
            last = l == L - 1
            y = None if last else self.bufs[l % 2]
            if self.events is not None:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
            self.layer_fn(self.shard, self.dis, x, y, e0, self.out, self.out,
                          acc_mode(l, L), L + 1)
            if self.events is not None:
                e.record()
                self.events.append((s, e))
            if not last and self.shard.world > 1:
                all_gather_rows(y, self.shard, self.group)
            x = y
        if gather_out and self.shard.world > 1:
            all_gather_rows(self.out, self.shard, self.group)
        return self.out
