"""Row-sharded multi-GPU propagation: one process per GPU, RCCL all-gather over xGMI,
overlapped with the SpMM.

SURVEY.md §8(e). The rows of A_hat are cut into W*C contiguous pieces balanced by
NON-ZEROS (cumulative rowptr search: every piece holds ~nnz/(W*C) edges, so a Zipf graph's
hub rows do not pile onto one rank); rank r owns pieces r*C .. r*C+C-1, i.e. a contiguous
run of rows, worked as C sub-chunks. Every rank keeps a full replica of the layer input x.
Per layer it runs the SpMM kernel on one sub-chunk at a time and, as soon as sub-chunk c is
done, starts an asynchronous ``all_gather_into_tensor`` of it (RCCL runs on its own stream)
while the kernel works on sub-chunk c+1; the next layer waits for all C gathers. Only the
last gather of a layer is exposed.

For the gathers to land in place, node ids live in a *chunk-major* layout where every piece
is padded to the longest piece's S rows:
    new(g) = c*(W*S) + r*S + (g - start(r, c))      for g in piece (r, c)
so sub-chunk c of every rank is one contiguous block of W*S rows in rank order, which is
exactly what ``all_gather_into_tensor`` writes. ``src`` ids, dis and e0 are permuted into
that layout once; the output is permuted back on demand. C = 1 is the plain row shard;
``balance="rows"`` restores equal row counts (S = ceil(n / (W*C))).

The per-shard layer is pluggable so the bookkeeping can run on CPU with gloo
(tests/test_dist_gloo.py); on GPUs it is lg_spmm_layer_f32.
"""
from __future__ import annotations

import math
import time

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


def piece_bounds(rowptr: torch.Tensor, lo: int, hi: int, parts: int,
                 balance: str = "nnz", max_rows: float = 2.0) -> list:
    """parts+1 row boundaries cutting rows [lo, hi) into contiguous pieces: by cumulative
    non-zeros (piece p ends at the first row whose prefix reaches (p+1)/parts of the
    range's edges) or, with balance="rows", into pieces of ceil((hi-lo)/parts) rows.

    The nnz cuts are capped at ``max_rows`` times the mean piece length: every piece is
    padded to the longest one in the chunk-major layout (its replicated tables and the
    per-layer all-gather are n_pad = longest piece x pieces rows), so on a power-law graph
    whose hub rows sit at low ids an uncapped cut would hand the tail piece many short rows
    and inflate n_pad up to parts-fold; the cap bounds n_pad at ~max_rows x the rows. A capped
    piece gives up some of its nnz balance instead (at max_rows = 1.5 a Zipf(0.5) item
    segment cut 16 ways pads 1.26x instead of 1.43x but its ranks' nnz spread 8 % instead of
    0.4 %; the default 2.0 only stops pathological padding)."""
    lo, hi = int(lo), int(hi)
    if balance == "rows":
        S = -(-(hi - lo) // parts) if hi > lo else 0
        return [min(hi, lo + p * S) for p in range(parts)] + [hi]
    if balance != "nnz":
        raise ValueError(f"balance must be 'nnz' or 'rows', got {balance!r}")
    rp = rowptr[lo:hi + 1].to(torch.int64).cpu()
    total = int(rp[-1] - rp[0])
    if total == 0:
        return piece_bounds(rowptr, lo, hi, parts, "rows")
    targets = torch.tensor([int(rp[0]) + (p * total + parts - 1) // parts
                            for p in range(1, parts)], dtype=torch.int64)
    cuts = torch.searchsorted(rp, targets).tolist()
    cap = max(1, -(-int(max_rows * (hi - lo)) // parts)) if max_rows else hi - lo
    b = [lo]
    for p in range(1, parts):
        t = lo + int(cuts[p - 1])
        t = min(t, b[-1] + cap)                    # this piece at most cap rows
        t = max(t, hi - (parts - p) * cap, b[-1])  # the rest must fit in cap-row pieces
        b.append(min(t, hi))
    b.append(hi)
    return b


class _Layout:
    """Piece table of a chunk-major layout: piece P covers original rows
    [start[P], start[P] + len) and lands at layout row offset[P]."""

    def __init__(self, starts: list, offsets: list):
        self.starts = torch.tensor(starts, dtype=torch.int64)
        self.offsets = torch.tensor(offsets, dtype=torch.int64)

    def map(self, g: torch.Tensor) -> torch.Tensor:
        st, off = self.starts.to(g.device), self.offsets.to(g.device)
        P = torch.searchsorted(st, g, right=True) - 1
        return off[P] + (g - st[P])


class RowShard:
    """This rank's rows of a CSR over n_nodes nodes, in the chunk-major layout."""

    def __init__(self, rowptr: torch.Tensor, src: torch.Tensor, n_nodes: int, rank: int,
                 world: int, device=None, weight: torch.Tensor | None = None,
                 chunks: int = 1, balance: str = "nnz"):
        self.n_nodes, self.rank, self.world, self.chunks = int(n_nodes), rank, world, chunks
        W, C = world, chunks
        self.bounds = piece_bounds(rowptr, 0, self.n_nodes, W * C, balance)
        lens = [self.bounds[p + 1] - self.bounds[p] for p in range(W * C)]
        self.S = max(1, max(lens))
        self.n_pad = self.S * W * C
        dev = device if device is not None else rowptr.device
        self.device = dev
        starts, offsets, piece_off = [], [], []
        for p in range(W * C):
            r, c = p // C, p % C
            piece_off.append(c * W * self.S + r * self.S)
            if lens[p]:
                starts.append(self.bounds[p])
                offsets.append(piece_off[p])
        self._layout = _Layout(starts or [0], offsets or [0])
        g0, g1 = self.bounds[rank * C], self.bounds[(rank + 1) * C]
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
            p = rank * C + c
            self.pieces.append((self.bounds[p] - g0, self.bounds[p + 1] - g0, piece_off[p]))

    @property
    def n_rows(self) -> int:
        return self.g1 - self.g0

    @property
    def pad_ratio(self) -> float:
        """n_pad / n_nodes: the chunk-major layout's padding (replicated tables, gathers)."""
        return self.n_pad / max(1, self.n_nodes)

    # ------------------------------------------------------------------ layout maps
    def to_layout(self, g: torch.Tensor) -> torch.Tensor:
        """original node id -> chunk-major id."""
        return self._layout.map(g)

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


class _WaitTimer:
    """Times one batch of gather waits into `log` (a list, or None: no timing) as
    (layer, interval). On a GPU the wait is a stream-side dependency (Work.wait() makes the
    compute stream wait for RCCL's), so the interval is a pair of events recorded on the
    compute stream around it: their distance is how long that stream stalled on the
    exchange, i.e. the part of the gather the overlap did not hide (elapsed_time, ms). On
    the CPU (gloo) wait() blocks the host: host seconds."""

    def __init__(self, log, layer, like):
        self.log, self.layer = log, layer
        self.cuda = like is not None and like.is_cuda

    def __enter__(self):
        if self.log is not None:
            if self.cuda:
                self.a = torch.cuda.Event(enable_timing=True)
                self.a.record()
            else:
                self.t = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.log is not None:
            if self.cuda:
                b = torch.cuda.Event(enable_timing=True)
                b.record()
                self.log.append((self.layer, (self.a, b)))
            else:
                self.log.append((self.layer, (time.perf_counter() - self.t) * 1e3))
        return False


def exposed_wait_ms(waits, layers: int, steps: int) -> list:
    """Per layer, the mean over `steps` forwards of the compute stream's stall on the gathers
    (ms; from BipartitePropagation.waits / ShardedPropagation.waits after a synchronize)."""
    per = [0.0] * layers
    for layer, iv in waits:
        per[layer] += iv[0].elapsed_time(iv[1]) if isinstance(iv, tuple) else float(iv)
    return [v / max(steps, 1) for v in per]


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
        self.waits = None  # optional list of (layer, interval): the stall on the gathers

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
            if handles:
                with _WaitTimer(self.waits, l, y):
                    for h in handles:
                        h.wait()
            x = y
        if gather_out and sh.world > 1:
            for c in range(sh.chunks):
                _gather_block(self.out, sh, c, self.group, async_op=False)
        return self.out


# ------------------------------------------------------- bipartite-ordered propagation
class SegmentShard:
    """This rank's rows when the node ids form contiguous segments that are sharded
    separately: for LightGCN, users [0, U) and items [U, U+I). Each segment is cut into
    W*C pieces balanced by non-zeros (piece_bounds) and padded to its longest piece's S_s
    rows; rank r owns pieces r*C .. r*C+C-1 of every segment (a share of the users' edges AND
    of the items' edges). Layout: segment-major, then chunk-major inside a segment,
        new(g) = base_s + c*(W*S_s) + r*S_s + (g - start_s(r, c)),
    so piece (s, c) of every rank is one contiguous block that all_gather_into_tensor writes
    in place. Exposes the interface of RowShard (rowptr/src/weight/pieces, to_layout,
    permute_rows) plus ``seg_pieces[s]``."""

    def __init__(self, rowptr: torch.Tensor, src: torch.Tensor, bounds: list, rank: int,
                 world: int, device=None, weight: torch.Tensor | None = None,
                 chunks: int = 1, balance: str = "nnz"):
        self.bounds = [int(b) for b in bounds]
        self.n_nodes = self.bounds[-1]
        self.rank, self.world, self.chunks = rank, world, chunks
        dev = device if device is not None else rowptr.device
        self.device = dev
        W, C = world, chunks
        nseg = len(self.bounds) - 1
        self.S, self.base, self.cuts = [], [], []
        starts, offsets = [], []
        base = 0
        for s in range(nseg):
            cuts = piece_bounds(rowptr, self.bounds[s], self.bounds[s + 1], W * C, balance)
            lens = [cuts[p + 1] - cuts[p] for p in range(W * C)]
            S_s = max(lens) if self.bounds[s + 1] > self.bounds[s] else 0
            self.S.append(S_s)
            self.base.append(base)
            self.cuts.append(cuts)
            for p in range(W * C):
                if lens[p]:
                    starts.append(cuts[p])
                    offsets.append(base + (p % C) * W * S_s + (p // C) * S_s)
            base += W * C * S_s
        self.n_pad = base
        self._layout = _Layout(starts or [0], offsets or [0])
        rp_parts, src_parts, w_parts = [], [], []
        self.seg_pieces, self.ranges = [], []
        lrow, lent = 0, 0
        for s in range(nseg):
            cuts, S_s = self.cuts[s], self.S[s]
            g0, g1 = cuts[rank * C], cuts[(rank + 1) * C]
            self.ranges.append((g0, g1))
            b, e = int(rowptr[g0]), int(rowptr[g1])
            rp_parts.append((rowptr[g0:g1] - b + lent) if g1 > g0 else rowptr[:0])
            src_parts.append(src[b:e])
            if weight is not None:
                w_parts.append(weight[b:e])
            pieces = []
            for c in range(C):
                p = rank * C + c
                pieces.append((lrow + cuts[p] - g0, lrow + cuts[p + 1] - g0,
                               self.base[s] + c * W * S_s + rank * S_s))
            self.seg_pieces.append(pieces)
            lrow += g1 - g0
            lent += e - b
        self.rowptr = torch.cat(rp_parts + [torch.tensor([lent], dtype=rowptr.dtype,
                                                         device=rowptr.device)]).to(dev)
        self.nnz = lent
        src_local = torch.cat(src_parts).to(dev)
        self.src = self.to_layout(src_local.to(torch.int64)).to(torch.int32)
        self.weight = None if weight is None else torch.cat(w_parts).to(dev)
        self.pieces = [p for ps in self.seg_pieces for p in ps]
        self._n_rows = lrow

    @property
    def n_rows(self) -> int:
        return self._n_rows

    @property
    def pad_ratio(self) -> float:
        """n_pad / n_nodes: the layout's padding (replicated tables, gathers)."""
        return self.n_pad / max(1, self.n_nodes)

    def to_layout(self, g: torch.Tensor) -> torch.Tensor:
        """original node id -> layout id."""
        return self._layout.map(g)

    def permute_rows(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.zeros((self.n_pad,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        out[self.to_layout(torch.arange(self.n_nodes, device=t.device))] = t
        return out

    def unpermute_rows(self, t: torch.Tensor) -> torch.Tensor:
        return t[self.to_layout(torch.arange(self.n_nodes, device=t.device))]

    def is_bipartite(self) -> bool:
        """True when the rows of each of two segments only reference the other segment."""
        if len(self.bounds) != 3:
            return False
        split = self.base[1]  # layout ids below this belong to segment 0
        for s, pieces in enumerate(self.seg_pieces):
            lb, le = pieces[0][0], pieces[-1][1]
            if le <= lb:
                continue
            ids = self.src[int(self.rowptr[lb]):int(self.rowptr[le])]
            if ids.numel() and bool(((ids < split) if s == 0 else (ids >= split)).any()):
                return False
        return True


def _gather_piece(buf: torch.Tensor, shard: SegmentShard, s: int, c: int, group=None,
                  async_op=True):
    W, S, base = shard.world, shard.S[s], shard.base[s]
    blk = buf[base + c * W * S:base + (c + 1) * W * S]
    mine = blk[shard.rank * S:(shard.rank + 1) * S]
    if dist.get_backend(group) == "gloo":
        return dist.all_gather([blk[r * S:(r + 1) * S] for r in range(W)], mine.clone(),
                               group=group, async_op=async_op)
    return dist.all_gather_into_tensor(blk, mine, group=group, async_op=async_op)


class BipartitePropagation:
    """mean_{l<=L} A_hat^l e0 over a SegmentShard of the user-item graph, with the
    all-gathers overlapped ACROSS layer boundaries. User rows read only item rows and vice
    versa, so a layer computes one half, starts its gathers, and computes the other half;
    the next layer starts with the half whose input was gathered first:
        layer 0: items, users      layer 1: users, items      layer 2: items, users ...
    Before computing a half only the gathers of its input half are awaited, so the
    exchange of one half hides behind the computation of the other and the chain of
    gathers never waits for a whole layer. (Graphs that are not bipartite over the two
    segments wait for every pending gather.)"""

    def __init__(self, shard: SegmentShard, dis_layout: torch.Tensor, dim: int, layers: int,
                 device, layer_fn=hip_layer, group=None):
        self.shard, self.dis, self.layers, self.group = shard, dis_layout, layers, group
        self.layer_fn = layer_fn
        n_pad = shard.n_pad
        self.bufs = [torch.zeros(n_pad, dim, device=device),
                     torch.zeros(n_pad, dim, device=device) if layers > 2 else None]
        self.out = torch.zeros(n_pad, dim, device=device)
        self.bipartite = shard.is_bipartite()
        self.events = None  # optional list of (start, end) event pairs: one per layer half
        # optional list of (layer, interval) -- the compute stream's stall on the gathers it
        # awaits before each half (see _WaitTimer): the exchange the overlap did NOT hide
        self.waits = None

    def forward(self, e0_layout: torch.Tensor, gather_out: bool = False) -> torch.Tensor:
        sh = self.shard
        x = e0_layout
        L = self.layers
        nseg = len(sh.seg_pieces)
        pending = {}
        for l in range(L):
            last = l == L - 1
            y = None if last else self.bufs[l % 2]
            mode = acc_mode(l, L)
            order = [1, 0] if (l % 2 == 0 and nseg == 2) else list(range(nseg))
            fresh = {}
            for s in order:
                need = [1 - s] if (self.bipartite and nseg == 2) else list(pending)
                hs = [h for q in need for h in pending.pop(q, [])]
                if hs:
                    with _WaitTimer(self.waits, l, x):
                        for h in hs:
                            h.wait()
                if self.events is not None:
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev0.record()
                for c, piece in enumerate(sh.seg_pieces[s]):
                    self.layer_fn(sh, piece, self.dis, x, y, e0_layout, self.out, self.out,
                                  mode, L + 1)
                    if not last and sh.world > 1:
                        fresh.setdefault(s, []).append(_gather_piece(y, sh, s, c, self.group))
                if self.events is not None:
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record()
                    self.events.append((ev0, ev1))
            hs = [h for q in pending.values() for h in q]  # (non-bipartite leftovers)
            if hs:
                with _WaitTimer(self.waits, l, x):
                    for h in hs:
                        h.wait()
            pending = fresh
            x = y
        if gather_out and sh.world > 1:
            for s, pieces in enumerate(sh.seg_pieces):
                for c in range(len(pieces)):
                    _gather_piece(self.out, sh, s, c, self.group, async_op=False)
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
                        local_fn=None, merge_fn=None,
                        stats: dict | None = None):
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
    kw = {} if stats is None else {"stats": stats}
    v, i = local_fn(A, lam, k, excl, drop, eu, ei, tile=tile, items=slice(i0, i1), **kw)
    u0, u1 = user_block(A.n_users, rank, world)
    if world == 1:
        return (u0, u1), v, i
    pv, pi = exchange_topk(v, i, rank, world, group)
    del v, i
    mv, mi = merge_fn(pv, pi)
    return (u0, u1), mv, mi
