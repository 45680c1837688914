"""Device-resident graph structures for the hot path.

* :class:`Adjacency` — the propagation graph as target-major CSR (int64 rowptr, int32
  source ids, fp32 ``dis`` = deg^-1/2), i.e. what the reference's symmetric coalesced COO
  (utils/graph.py:12-35, consumed by model/LightGCN/model.py:53-62) means to PyG's
  ``gcn_norm`` + ``propagate``: messages flow ``edge_index[0] -> edge_index[1]``, degrees
  count ``edge_index[1]``.
* :class:`RowSets` — per-row sorted column sets (user -> items), used for the exclusion
  masks of the recommenders (train|val positives, model/LightGCN/recommend.py:93-111,
  model/SpreadMethod/recommend.py:31-44) and for the sparse interaction matrix A of the
  spreading path (utils/trans.py:13-29).

Sorting/dedup of index arrays is torch glue on the device; row pointers and the
normalisation are computed by the HIP library (lg_csr_rowptr_from_sorted, lg_gcn_norm_f32).
"""
from __future__ import annotations

import torch

from . import _native as N


def _rowptr_from_sorted(keys: torch.Tensor, n_rows: int) -> torch.Tensor:
    N.require_gpu(keys, "keys")
    rowptr = torch.empty(n_rows + 1, dtype=torch.int64, device=keys.device)
    keys = keys.contiguous()
    N.check(N.lib().lg_csr_rowptr_from_sorted(N.ptr(keys), keys.numel(), n_rows, N.ptr(rowptr),
                                              N.stream_handle(keys.device)),
            "lg_csr_rowptr_from_sorted")
    return rowptr


def _sorted_unique_keys(rows: torch.Tensor, cols: torch.Tensor, n_cols: int,
                        dedup: bool) -> torch.Tensor:
    keys = rows.to(torch.int64) * n_cols + cols.to(torch.int64)
    if keys.numel() > 1 and not bool((keys[1:] > keys[:-1]).all()):
        keys = torch.unique(keys) if dedup else torch.sort(keys).values
    return keys


LONG_ROW_THRESHOLD = 4096   # rows with more entries go through the segmented path
LONG_ROW_SEGMENT = 2048     # entries per segment (one wave each)


class LongRowPlan:
    """Segments of the rows of a CSR slice longer than the threshold (power-law hubs),
    for lg_spmm_long_rows_f32. Node ids are ``row_offset + local row``."""

    def __init__(self, rowptr: torch.Tensor, row_offset: int, threshold: int, seg_len: int):
        self.threshold, self.seg_len = int(threshold), int(seg_len)
        deg = rowptr[1:] - rowptr[:-1]
        long_r = torch.nonzero(deg > threshold).flatten()
        self.n_long = int(long_r.numel())
        dev = rowptr.device
        if self.n_long == 0:
            self.n_seg = 0
            return
        beg, end = rowptr[long_r], rowptr[long_r + 1]
        nseg = (end - beg + seg_len - 1) // seg_len
        self.seg_ptr = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev),
                                  torch.cumsum(nseg, 0)])
        self.n_seg = int(self.seg_ptr[-1])
        owner = torch.repeat_interleave(torch.arange(self.n_long, device=dev), nseg)
        k = torch.arange(self.n_seg, device=dev) - self.seg_ptr[owner]
        self.seg_beg = beg[owner] + k * seg_len
        self.seg_end = torch.minimum(self.seg_beg + seg_len, end[owner])
        nodes = (long_r + row_offset).to(torch.int32)
        self.long_node = nodes
        self.seg_node = nodes[owner].contiguous()

    def partial(self, dim: int, device) -> torch.Tensor:
        return torch.empty((max(self.n_seg, 1), dim), dtype=torch.float32, device=device)


class Adjacency:
    """Target-major CSR of a message-passing graph over ``n_nodes`` nodes."""

    def __init__(self, rowptr: torch.Tensor, src: torch.Tensor, n_nodes: int,
                 n_users: int | None = None, symmetric: bool | None = None):
        self.rowptr = rowptr
        self.src = src
        self.n_nodes = int(n_nodes)
        self.n_users = n_users
        self.symmetric = symmetric
        self._dis = None
        self._transpose = None
        self._edge_weight = None
        self._long_plan = None

    @property
    def device(self):
        return self.rowptr.device

    @property
    def nnz(self) -> int:
        return int(self.src.numel())

    # ---------------------------------------------------------------- builders
    @classmethod
    def from_edge_index(cls, edge_index: torch.Tensor, num_nodes: int,
                        device=None) -> "Adjacency":
        """From a PyG-style ``[2, nnz]`` edge index (row = source, col = target), e.g. the
        reference's ``convertEdgeIndexToAdjMatrix`` output. Duplicate edges are kept (PyG
        counts them twice too)."""
        dev = torch.device(device) if device is not None else (
            edge_index.device if edge_index.is_cuda else torch.device("cuda"))
        ei = edge_index.to(dev, torch.int64)
        n = int(num_nodes)
        keys = _sorted_unique_keys(ei[1], ei[0], n, dedup=False)  # by (target, source)
        tgt, src = keys // n, keys % n
        rowptr = _rowptr_from_sorted(tgt, n)
        sym = None
        if ei.numel():
            tkeys = _sorted_unique_keys(ei[0], ei[1], n, dedup=False)
            sym = bool(torch.equal(tkeys, keys))
        return cls(rowptr, src.to(torch.int32), n, symmetric=sym)

    @classmethod
    def from_interactions(cls, users: torch.Tensor, items: torch.Tensor, n_users: int,
                          n_items: int, device=None) -> "Adjacency":
        """The symmetric bipartite graph of convertEdgeIndexToAdjMatrix
        (utils/graph.py:22-33): user u <-> node U + i, duplicates collapse."""
        dev = torch.device(device) if device is not None else (
            users.device if users.is_cuda else torch.device("cuda"))
        u = torch.as_tensor(users, device=dev).to(torch.int64)
        i = torch.as_tensor(items, device=dev).to(torch.int64) + n_users
        n = n_users + n_items
        rows = torch.cat([u, i])
        cols = torch.cat([i, u])
        keys = torch.unique(rows * n + cols)
        rowptr = _rowptr_from_sorted(keys // n, n)
        return cls(rowptr, (keys % n).to(torch.int32), n, n_users=n_users, symmetric=True)

    # ---------------------------------------------------------------- views
    def edge_index(self) -> torch.Tensor:
        """The reference's coalesced COO ``[2, nnz]`` (row = source, col = target), sorted
        by (row, col) like ``to_sparse_coo().indices()``."""
        deg = self.rowptr[1:] - self.rowptr[:-1]
        tgt = torch.repeat_interleave(torch.arange(self.n_nodes, device=self.device), deg)
        src = self.src.to(torch.int64)
        keys = torch.sort(src * self.n_nodes + tgt).values
        return torch.stack([keys // self.n_nodes, keys % self.n_nodes])

    def dis(self) -> torch.Tensor:
        """deg^-1/2 per node (gcn_norm), computed once per graph."""
        if self._dis is None:
            dis = torch.empty(self.n_nodes, dtype=torch.float32, device=self.device)
            N.check(N.lib().lg_gcn_norm_f32(N.ptr(self.rowptr), self.n_nodes, N.ptr(dis),
                                            N.stream_handle(self.device)), "lg_gcn_norm_f32")
            self._dis = dis
        return self._dis

    def long_plan(self) -> LongRowPlan:
        if self._long_plan is None:
            self._long_plan = LongRowPlan(self.rowptr, 0, LONG_ROW_THRESHOLD, LONG_ROW_SEGMENT)
        return self._long_plan

    def edge_weight(self) -> torch.Tensor:
        """gcn_norm's per-edge weight in this CSR's entry order."""
        if self._edge_weight is None:
            w = torch.empty(self.nnz, dtype=torch.float32, device=self.device)
            N.check(N.lib().lg_gcn_edge_weight_f32(N.ptr(self.rowptr), N.ptr(self.src),
                                                   N.ptr(self.dis()), self.n_nodes, 0,
                                                   N.ptr(w), N.stream_handle(self.device)),
                    "lg_gcn_edge_weight_f32")
            self._edge_weight = w
        return self._edge_weight

    def transpose(self) -> "Adjacency":
        """Source-major CSR (for the backward pass A^T g); itself when symmetric. Keeps the
        forward graph's ``dis`` (the weights are dis[s]*dis[t] either way)."""
        if self.symmetric:
            return self
        if self._transpose is None:
            deg = self.rowptr[1:] - self.rowptr[:-1]
            tgt = torch.repeat_interleave(torch.arange(self.n_nodes, device=self.device), deg)
            keys = torch.sort(self.src.to(torch.int64) * self.n_nodes + tgt).values
            rowptr = _rowptr_from_sorted(keys // self.n_nodes, self.n_nodes)
            t = Adjacency(rowptr, (keys % self.n_nodes).to(torch.int32), self.n_nodes,
                          self.n_users, symmetric=False)
            t._dis = self.dis()
            t._transpose = self
            self._transpose = t
        return self._transpose


class RowSets:
    """Sorted, de-duplicated column sets per row: (rowptr int64 [n_rows+1], col int32)."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, n_rows: int, n_cols: int):
        if col.numel() == 0 and col.data_ptr() == 0:
            # an empty set still passes a valid device pointer: the C ABI refuses NULL columns
            col = torch.empty(1, dtype=col.dtype, device=col.device)[:0]
        self.rowptr, self.col = rowptr, col
        self.n_rows, self.n_cols = int(n_rows), int(n_cols)

    @classmethod
    def from_pairs(cls, rows, cols, n_rows: int, n_cols: int, device=None) -> "RowSets":
        dev = torch.device(device) if device is not None else torch.device("cuda")
        r = torch.as_tensor(rows).to(dev, torch.int64)
        c = torch.as_tensor(cols).to(dev, torch.int64)
        if r.numel():
            keys = torch.unique(r * n_cols + c)
        else:
            keys = torch.zeros(0, dtype=torch.int64, device=dev)
        rowptr = _rowptr_from_sorted(keys // n_cols, n_rows)
        return cls(rowptr, (keys % n_cols).to(torch.int32), n_rows, n_cols)

    @classmethod
    def union(cls, *sets: "RowSets") -> "RowSets":
        base = sets[0]
        dev = base.rowptr.device
        rows, cols = [], []
        for s in sets:
            deg = s.rowptr[1:] - s.rowptr[:-1]
            rows.append(torch.repeat_interleave(torch.arange(s.n_rows, device=dev), deg))
            cols.append(s.col.to(torch.int64))
        return cls.from_pairs(torch.cat(rows), torch.cat(cols), base.n_rows, base.n_cols, dev)

    def transpose(self) -> "RowSets":
        deg = self.rowptr[1:] - self.rowptr[:-1]
        rows = torch.repeat_interleave(torch.arange(self.n_rows, device=self.rowptr.device), deg)
        return RowSets.from_pairs(self.col, rows, self.n_cols, self.n_rows, self.rowptr.device)

    def degrees(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]

    def slice_rows(self, r0: int, r1: int) -> "RowSets":
        """Rows [r0, r1) keeping absolute offsets into ``col`` (no copy of col)."""
        return RowSets(self.rowptr[r0:r1 + 1], self.col, r1 - r0, self.n_cols)


_ADJ_CACHE: dict = {}


def as_adjacency(edge_index, n_nodes: int, device=None) -> Adjacency:
    """The cached device CSR of a reference-style COO ``edge_index`` (or pass-through of an
    :class:`Adjacency`). Keyed by the tensor's storage, shape and version counter, so the
    per-epoch ``model.forward(train_edge_index)`` of the reference's training loop
    (model/LightGCN/train.py:45) converts the graph once, not every call."""
    if isinstance(edge_index, Adjacency):
        return edge_index
    t = torch.as_tensor(edge_index)
    key = (t.data_ptr(), tuple(t.shape), str(t.device), t._version, int(n_nodes), str(device))
    hit = _ADJ_CACHE.get(key)
    # the cache holds a reference to the keyed tensor, so its storage (and data_ptr) can
    # not be recycled for another tensor while the entry lives
    if hit is not None and hit[0] is t:
        return hit[1]
    if t.numel() and (int(t.min()) < 0 or int(t.max()) >= n_nodes):
        raise ValueError(f"edge_index has node ids outside [0, {n_nodes})")
    adj = Adjacency.from_edge_index(t, n_nodes, device=device)
    if len(_ADJ_CACHE) >= 8:
        _ADJ_CACHE.pop(next(iter(_ADJ_CACHE)))
    _ADJ_CACHE[key] = (t, adj)
    return adj
