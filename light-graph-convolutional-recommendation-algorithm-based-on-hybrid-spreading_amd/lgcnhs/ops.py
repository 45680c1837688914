"""Torch-facing wrappers of the HIP hot path (no CPU fallback: GPU tensors only).

propagate        LightGCN layers + layer mean      model/LightGCN/model.py:53-74
score_topk       e0 scores, -1024 mask, top-k      model/LightGCN/recommend.py:83-114
score_dense      masked dense score matrix G       model/SpreadLightGCN/model.py:74-104
spread_general   general_W                         model/SpreadMethod/model.py:14-27
hybrid_weight    HybridS W                         model/SpreadMethod/model.py:63-85
spread_resource  F = A @ W                         model/SpreadMethod/model.py:88-99
rows_topk        argsort + filter + [:k], G * F    model/SpreadMethod/recommend.py:31-50,
                                                   model/SpreadLightGCN/model.py:151
spread_topk_tiled  the above over item tiles,      (same; for catalogs whose I x I W
                   never holding an I x I matrix    does not fit)
spread_recommend   dense or tiled, whichever fits  model/SpreadMethod/recommend.py:59-115
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as N
from .graph import Adjacency, RowSets

MASK_VALUE = float(-(1 << 10))  # model/LightGCN/recommend.py:101,111


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    N.require_gpu(t, name)
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    return t.contiguous()


# ------------------------------------------------------------------------------ propagation
def run_layer(rowptr, src, dis, w, x, y, x0, acc, out, n_rows: int, row_offset: int,
              mode: int, denom: float, plan=None, live=None, row_mask=None) -> None:
    """One propagation layer over a CSR slice: lg_spmm_layer_f32 for the ordinary rows (or
    lg_spmm_layer_live_f32 when a uint8 per-node ``live`` mask marks x's non-zero rows, or
    lg_spmm_layer_rows_f32 computing only the rows a uint8 per-node ``row_mask`` marks)
    and, when the slice has rows above the long-row threshold, lg_spmm_long_rows_f32 (its
    masked form with row_mask)."""
    dim = x.shape[1]
    thr = plan.threshold if (plan is not None and plan.n_long) else 0
    strm = N.stream_handle(x.device)
    if row_mask is not None:
        if live is not None:
            raise ValueError("row_mask and live are exclusive")
        N.check(N.lib().lg_spmm_layer_rows_f32(
            N.ptr(rowptr), N.ptr(src), N.ptr(dis), N.ptr(w), N.ptr(x), N.ptr(y), N.ptr(x0),
            N.ptr(acc), N.ptr(out), n_rows, row_offset, dim, mode, float(denom), thr,
            N.ptr(row_mask), strm), "lg_spmm_layer_rows_f32")
    elif live is not None:
        if live.dtype != torch.uint8 or live.numel() != x.shape[0] or live.device != x.device:
            raise ValueError("live must be a uint8 mask with one entry per row of x")
        N.check(N.lib().lg_spmm_layer_live_f32(
            N.ptr(rowptr), N.ptr(src), N.ptr(dis), N.ptr(w), N.ptr(x), N.ptr(y), N.ptr(x0),
            N.ptr(acc), N.ptr(out), n_rows, row_offset, dim, mode, float(denom), thr,
            N.ptr(live), strm), "lg_spmm_layer_live_f32")
    else:
        N.check(N.lib().lg_spmm_layer_f32(
            N.ptr(rowptr), N.ptr(src), N.ptr(dis), N.ptr(w), N.ptr(x), N.ptr(y), N.ptr(x0),
            N.ptr(acc), N.ptr(out), n_rows, row_offset, dim, mode, float(denom), thr, strm),
            "lg_spmm_layer_f32")
    if thr:
        part = plan.partial(dim, x.device)
        args = (N.ptr(plan.seg_beg), N.ptr(plan.seg_end), N.ptr(plan.seg_node), plan.n_seg,
                N.ptr(plan.long_node), N.ptr(plan.seg_ptr), plan.n_long, N.ptr(src),
                N.ptr(dis), N.ptr(w), N.ptr(x), N.ptr(y), N.ptr(x0), N.ptr(acc), N.ptr(out),
                dim, mode, float(denom), N.ptr(part))
        if row_mask is not None:
            N.check(N.lib().lg_spmm_long_rows_masked_f32(*args, N.ptr(row_mask), strm),
                    "lg_spmm_long_rows_masked_f32")
        else:
            N.check(N.lib().lg_spmm_long_rows_f32(*args, strm), "lg_spmm_long_rows_f32")


def spmm_layer(adj: Adjacency, x: torch.Tensor, y, x0, acc, out, mode: int, denom: float,
               stream_weights: bool = True, long_rows: bool = True, live=None,
               row_mask=None) -> None:
    """One layer over all rows of ``adj`` (or the rows ``row_mask`` marks); with
    stream_weights the precomputed gcn_norm edge weights are streamed (else recomputed from
    dis; identical values); with long_rows, hub rows go through the segmented path."""
    w = adj.edge_weight() if stream_weights else None
    run_layer(adj.rowptr, adj.src, adj.dis(), w, x, y, x0, acc, out, adj.n_nodes, 0, mode,
              denom, adj.long_plan() if long_rows else None, live, row_mask)


LIVE_FRACTION = 0.25  # below this share of non-zero input rows, skip the dead rows' gathers


def live_rows(x: torch.Tensor) -> torch.Tensor:
    """uint8 [rows]: 1 where row of x has a non-zero entry."""
    return (x != 0).any(dim=1).to(torch.uint8)


def propagate_mean(adj: Adjacency, e0: torch.Tensor, layers: int,
                   sparse_input: bool = False) -> torch.Tensor:
    """mean_{l=0..L} A_hat^l e0 with A_hat = D^-1/2 A D^-1/2 (no autograd). With
    sparse_input (the backward pass: e0 = dL/d(e_final), non-zero on a mini-batch's rows),
    each layer whose input has < LIVE_FRACTION non-zero rows gathers only those rows
    (lg_spmm_layer_live_f32; same sums)."""
    e0 = _f32(e0, "e0")
    if e0.shape[0] != adj.n_nodes:
        raise ValueError(f"e0 has {e0.shape[0]} rows, graph has {adj.n_nodes} nodes")
    if layers <= 0:
        return e0.clone()
    out = torch.empty_like(e0)
    bufs = [torch.empty_like(e0), torch.empty_like(e0) if layers > 2 else None]
    x = e0
    for l in range(layers):
        first, last = l == 0, l == layers - 1
        if first and last:
            mode = N.LG_ACC_ONLY
        elif first:
            mode = N.LG_ACC_FIRST
        elif last:
            mode = N.LG_ACC_LAST
        else:
            mode = N.LG_ACC_MID
        y = None if last else bufs[l % 2]
        live = None
        if sparse_input:
            live = live_rows(x)
            frac = int(live.sum()) / max(1, live.numel())
            if frac >= LIVE_FRACTION:
                live = None
            # the next input's non-zero rows are this one's neighbours: stop checking once
            # they are expected to pass the threshold (a mask pass + sync saved per layer)
            sparse_input = frac * adj.nnz / max(1, adj.n_nodes) < LIVE_FRACTION
        spmm_layer(adj, x, y, e0, out, out, mode, layers + 1, live=live)
        x = y
    return out


RESTRICT_FRACTION = 0.5  # a layer whose needed rows may exceed this share runs in full


def row_masks(adj: Adjacency, nodes: torch.Tensor, layers: int, force: bool = False) -> list:
    """Per layer l (0-based) the uint8 mask of the rows whose layer-l output the final
    embeddings at ``nodes`` depend on, or None for a full layer: layer L-1 at the nodes, each
    layer below also at the sources of the rows above it (lg_mark_neighbors_u8). A layer
    runs in full once its rows may exceed RESTRICT_FRACTION of the graph (estimated without a
    host sync: |nodes| times (1 + mean degree) per layer down), and so does every layer below
    it. ``force`` masks every layer (tests)."""
    n = adj.n_nodes
    masks = [None] * layers
    if layers == 0:
        return masks
    est = min(n, int(nodes.numel()))
    m = torch.zeros(n, dtype=torch.uint8, device=nodes.device)
    m[nodes] = 1
    strm = N.stream_handle(nodes.device)
    for l in range(layers - 1, -1, -1):
        if not force and est > RESTRICT_FRACTION * n:
            break
        masks[l] = m
        if l > 0:
            m2 = torch.zeros_like(m)
            N.check(N.lib().lg_mark_neighbors_u8(N.ptr(adj.rowptr), N.ptr(adj.src), n,
                                                 N.ptr(m), N.ptr(m2), strm),
                    "lg_mark_neighbors_u8")
            m = m2
            est = min(n, est * (1 + -(-adj.nnz // max(1, n))))
    return masks


def propagate_rows_mean(adj: Adjacency, e0: torch.Tensor, layers: int, nodes: torch.Tensor,
                        force_masks: bool = False) -> torch.Tensor:
    """propagate_mean's output at the rows ``nodes`` (int64, duplicates allowed), each row
    bitwise the full forward's: layer l computes only the rows row_masks marks (the training
    step's forward: the BPR loss reads the final embeddings at the mini-batch's <= 3 x batch
    rows only, reference model/LightGCN/train.py:30-45)."""
    e0 = _f32(e0, "e0")
    if e0.shape[0] != adj.n_nodes:
        raise ValueError(f"e0 has {e0.shape[0]} rows, graph has {adj.n_nodes} nodes")
    nodes = nodes.to(device=e0.device, dtype=torch.int64)
    if layers <= 0:
        return e0[nodes]
    masks = row_masks(adj, nodes, layers, force_masks)
    out = torch.empty_like(e0)
    bufs = [torch.empty_like(e0), torch.empty_like(e0) if layers > 2 else None]
    x = e0
    for l in range(layers):
        first, last = l == 0, l == layers - 1
        if first and last:
            mode = N.LG_ACC_ONLY
        elif first:
            mode = N.LG_ACC_FIRST
        elif last:
            mode = N.LG_ACC_LAST
        else:
            mode = N.LG_ACC_MID
        y = None if last else bufs[l % 2]
        spmm_layer(adj, x, y, e0, out, out, mode, layers + 1, row_mask=masks[l])
        x = y
    return out[nodes]


class _PropagateRows(torch.autograd.Function):
    """Forward: the final embeddings at ``nodes`` (output-restricted layers). Backward: the
    full operator's, grad_e0 = mean_l (A_hat^T)^l g with g scattered to the nodes' rows --
    what the full forward followed by the gather gives."""

    @staticmethod
    def forward(ctx, e0, adj, layers, nodes):
        ctx.adj, ctx.layers, ctx.n = adj, layers, e0.shape[0]
        ctx.save_for_backward(nodes)
        return propagate_rows_mean(adj, e0.detach(), layers, nodes)

    @staticmethod
    def backward(ctx, g):
        (nodes,) = ctx.saved_tensors
        gfull = torch.zeros((ctx.n, g.shape[1]), dtype=g.dtype, device=g.device)
        gfull.index_add_(0, nodes, g)
        gin = propagate_mean(ctx.adj.transpose(), gfull, ctx.layers, sparse_input=True)
        return gin, None, None, None


def propagate_rows(adj: Adjacency, e0: torch.Tensor, layers: int,
                   nodes: torch.Tensor) -> torch.Tensor:
    """propagate(adj, e0, layers)[nodes], computing only the rows it needs."""
    nodes = nodes.to(device=e0.device, dtype=torch.int64)
    if e0.requires_grad and torch.is_grad_enabled():
        return _PropagateRows.apply(e0, adj, layers, nodes)
    return propagate_rows_mean(adj, e0, layers, nodes)


class PropagationGraph:
    """The L-layer forward captured once into a hipGraph (torch.cuda.CUDAGraph on ROCm) and
    replayed: for small graphs (ML-100K/ML-1M shapes) the three layer kernels run for tens
    of microseconds and host launch overhead dominates. ``run(e0)`` copies e0 into the
    captured input buffer, replays, and returns the captured output buffer (overwritten by
    the next replay)."""

    def __init__(self, adj: Adjacency, dim: int, layers: int, device=None):
        dev = device or adj.device
        adj.dis()
        adj.edge_weight()
        adj.long_plan()  # host-side planning (syncs) must happen before capture
        self.e0 = torch.zeros(adj.n_nodes, dim, dtype=torch.float32, device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):  # warm the allocator outside the capture
            propagate_mean(adj, self.e0, layers)
        torch.cuda.current_stream(dev).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = propagate_mean(adj, self.e0, layers)

    def run(self, e0: torch.Tensor) -> torch.Tensor:
        self.e0.copy_(e0)
        self.graph.replay()
        return self.out


class _Propagate(torch.autograd.Function):
    """Forward: mean of the L+1 layer embeddings. Backward: the same operator with A_hat^T
    (A_hat itself for the symmetric LightGCN graph): grad_e0 = mean_l (A_hat^T)^l g."""

    @staticmethod
    def forward(ctx, e0, adj, layers):
        ctx.adj, ctx.layers = adj, layers
        return propagate_mean(adj, e0.detach(), layers)

    @staticmethod
    def backward(ctx, g):
        gin = propagate_mean(ctx.adj.transpose(), g.contiguous(), ctx.layers,
                             sparse_input=True)
        return gin, None, None


def propagate(adj: Adjacency, e0: torch.Tensor, layers: int) -> torch.Tensor:
    if e0.requires_grad and torch.is_grad_enabled():
        return _Propagate.apply(e0, adj, layers)
    return propagate_mean(adj, e0, layers)


# ------------------------------------------------------------------------------ scoring
def _resident_blocks(device, k: int = 64, screen: bool = False) -> int:
    """Workgroups resident at once: lg_score_topk_f32's take 64 KiB of LDS -> 2 per CU; the
    screened kernel's (k_topk_ring: 84-120 KiB of lists + the fragment ring) -> 1 per CU."""
    per_cu = 1 if screen else 2
    return per_cu * torch.cuda.get_device_properties(device).multi_processor_count


def _users_per_block(k: int, screen: bool = False, d: int = 64) -> int:
    """Users per workgroup of csrc/topk.hip's launches (dispatch_topk / _screen)."""
    if screen:  # (8 waves x 2 groups; k > 64 at d <= 64: 1 group, LG_GL4_NG)
        return 128 if k > 64 and d <= 64 else 256
    return 128 if k <= 32 else (64 if k <= 64 else 32)


def _splits_for(n_users: int, n_items: int, k: int, resident: int = 512,
                screen: bool = False, d: int = 64) -> int:
    """Item-range splits for lg_score_topk_f32: the fewest splits that keep every CU busy.

    Each split restarts every user's candidate list from an empty threshold (the warm-up
    inserts ~k*ln(items/k) candidates), so more splits cost work; too few leave CUs idle
    in the last round of workgroups. Minimise rounds/splits (the makespan in units of one
    unsplit block) with a 2 % penalty per split."""
    per_block = _users_per_block(k, screen, d)
    tiles = (n_users + per_block - 1) // per_block
    best, best_cost = 1, None
    for s in range(1, min(64, max(1, n_items // 256)) + 1):
        rounds = -(-tiles * s // resident)
        cost = rounds / s * (1 + 0.02 * s)
        if best_cost is None or cost < best_cost - 1e-12:
            best, best_cost = s, cost
    return best


# |bf16 MFMA product - fp32 chain| <= 0.00785 ||u|| ||i|| (csrc/gbound.hip); 3 % slack for
# the fp32 roundings of the margin and of the screen's compare. The worst case of bf16
# rounding; the screened top-K uses the tighter screen_margins (below), this form remains the
# bound of lg_score_chunk_bound.
SCREEN_MARGIN = 0.0081
SCREEN_DEFAULT = True  # measured: 26.8 vs 31.9 ms (d=64), 45.8 vs 59.7 ms (d=128) at C5
# The screened kernel's fixed costs (bf16 operands, margins, seed pass) lose to the plain
# kernel below these user x item counts (profiles/r06_topk_guard.log, d = 64, 22 shapes from
# 1024 x 2000 to 2048 x 1M: at k = 20 the two meet near 6e8 -- 2048 x 300K 1.39 vs 1.41 ms --,
# the screen loses at 512 x 1M and wins at 4096 x 200K; at k = 100 near 1e9 -- it loses at
# 8192 x 100K and 16384 x 50K, wins at 32768 x 30K and 2048 x 1M)
SCREEN_MIN_WORK = {32: 6e8, 128: 1e9}  # k <= key -> least users x items for the screen


def screen_pays(n_users: int, n_items: int, k: int) -> bool:
    """Whether the default top-K dispatch takes the screened kernel for this shape."""
    for kmax, work in SCREEN_MIN_WORK.items():
        if k <= kmax:
            return float(n_users) * float(n_items) >= work
    return False  # (k > 128: the screened kernel does not take it)


def screen_margins(un: torch.Tensor, ue: torch.Tensor, inorm: torch.Tensor,
                   ierr: torch.Tensor, dim: int) -> torch.Tensor:
    """Per-user fp32 margins m_u >= |bf16 MFMA product - fp32 chain score| for every item
    (the contract of lg_score_topk_screened_f32's umarg, include/lgcnhs.h).

    With du = u - bf16(u) and di = i - bf16(i) (both exact in fp32):
      u.i - bf16(u).bf16(i) = du.i + bf16(u).di, so |.| <= ||du|| ||i|| + (||u|| + ||du||) ||di||
    (Cauchy-Schwarz, ||bf16(u)|| <= ||u|| + ||du||); the MFMA's and the chain's fp32
    accumulations add gamma_dim (||bf16(u)|| ||bf16(i)|| + ||u|| ||i||) <= 2.01 dim 2^-24 ||u|| ||i||,
    and 2^-22 ||u|| ||i|| covers the rounding of the screen's own fp32 sum fl(b + m_u) (|b + m_u|
    <= 1.02 ||u|| ||i||). With I = max ||i||, DI = max ||di|| (norms rounded up by
    lg_bound_prep_f32), times (1 + 2^-20), plus 1e-30 for flushed subnormal products, in fp64,
    rounded up to fp32. On N(0, 0.1^2) embeddings this is ~0.45x the worst-case 0.0081 ||u|| I
    of SCREEN_MARGIN (bf16 rounding errors are not all at their maximum), and the observed
    error stays below 0.37 of it. Non-finite norms give non-finite margins: the kernel then
    ranks every item of those users by the exact chain."""
    I = inorm.max().double()
    DI = ierr.max().double()
    u, e = un.double(), ue.double()
    m = (e * I + (u + e) * DI + (2.01 * dim * 2.0 ** -24 + 2.0 ** -22) * u * I) \
        * (1.0 + 2.0 ** -20) + 1e-30
    m32 = m.float()
    return torch.where(m32.double() < m, torch.nextafter(m32, torch.full_like(m32, float("inf"))),
                       m32)


def score_topk(eu: torch.Tensor, ei: torch.Tensor, k: int, excl: RowSets | None = None,
               mask_value: float = MASK_VALUE, n_splits: int | None = None,
               screen: bool | None = None):
    """Top-k items per user by the masked e0 score; returns (values fp32 [U,k],
    indices int64 [U,k]) sorted by (score desc, item asc). screen=True runs
    lg_score_topk_screened_f32: a bf16 MFMA bound decides which 16-item tiles get the exact
    fp32 chain; the results are lg_score_topk_f32's (screen=False) bit for bit. Default:
    SCREEN_DEFAULT where it pays for the shape (screen_pays)."""
    eu, ei = _f32(eu, "eu"), _f32(ei, "ei")
    nu, d = eu.shape
    ni = ei.shape[0]
    if screen is None:
        screen = SCREEN_DEFAULT and screen_pays(nu, ni, k)
    if ei.shape[1] != d:
        raise ValueError("eu/ei dims differ")
    if excl is not None and excl.n_rows != nu:
        raise ValueError(f"exclusion rows {excl.n_rows} != users {nu}")
    ns = (_splits_for(nu, ni, k, _resident_blocks(eu.device, k, screen), screen, d)
          if n_splits is None else int(n_splits))
    ws_fn = (N.lib().lg_score_topk_screened_ws_bytes if screen and nu > 0
             else N.lib().lg_score_topk_ws_bytes)
    ws_bytes = ws_fn(nu, ni, d, k, ns)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=eu.device)
    val = torch.empty((nu, k), dtype=torch.float32, device=eu.device)
    idx = torch.empty((nu, k), dtype=torch.int64, device=eu.device)
    ex_rp = N.ptr(excl.rowptr if excl else None)
    ex_c = N.ptr(excl.col if excl else None)
    if screen and nu > 0:
        ub, un, ue = bound_operands(eu, with_err=True)
        ib, inorm, ierr = bound_operands(ei, with_err=True)
        # (no host sync: a non-finite embedding gives non-finite margins, and the kernel then
        # ranks those users' items by the exact chain -- include/lgcnhs.h)
        umarg = screen_margins(un, ue, inorm, ierr, d)
        N.check(N.lib().lg_score_topk_screened_f32(
            N.ptr(eu), N.ptr(ei), N.ptr(ub), N.ptr(ib), N.ptr(umarg), nu, ni, d, ex_rp, ex_c,
            float(mask_value), int(k), ns, N.ptr(val), N.ptr(idx), N.ptr(ws), ws_bytes,
            N.stream_handle(eu.device)), "lg_score_topk_screened_f32")
        return val, idx
    N.check(N.lib().lg_score_topk_f32(
        N.ptr(eu), N.ptr(ei), nu, ni, d, ex_rp, ex_c, float(mask_value), int(k), ns,
        N.ptr(val), N.ptr(idx), N.ptr(ws), ws_bytes, N.stream_handle(eu.device)),
        "lg_score_topk_f32")
    return val, idx


def score_dense(eu: torch.Tensor, ei: torch.Tensor, excl: RowSets | None = None,
                mask_value: float = MASK_VALUE) -> torch.Tensor:
    eu, ei = _f32(eu, "eu"), _f32(ei, "ei")
    nu, d = eu.shape
    ni = ei.shape[0]
    G = torch.empty((nu, ni), dtype=torch.float32, device=eu.device)
    N.check(N.lib().lg_score_dense_f32(
        N.ptr(eu), N.ptr(ei), nu, ni, d, N.ptr(excl.rowptr if excl else None),
        N.ptr(excl.col if excl else None), float(mask_value), N.ptr(G), ni,
        N.stream_handle(eu.device)), "lg_score_dense_f32")
    return G


# ------------------------------------------------------------------------------ spreading
class Interactions:
    """The 0/1 interaction matrix A held sparse both ways, with degrees as fp64."""

    def __init__(self, by_user: RowSets):
        self.by_user = by_user
        self.by_item = by_user.transpose()
        self.n_users, self.n_items = by_user.n_rows, by_user.n_cols
        self.k_user = by_user.degrees().to(torch.float64)
        self.k_item = self.by_item.degrees().to(torch.float64)

    @classmethod
    def from_pairs(cls, users, items, n_users, n_items, device=None):
        return cls(RowSets.from_pairs(users, items, n_users, n_items, device))

    @classmethod
    def from_dense(cls, A: torch.Tensor):
        """From a dense [U, I] matrix (nonzero = interaction), e.g. the reference's A."""
        N.require_gpu(A, "A")
        nz = torch.nonzero(A != 0)
        return cls.from_pairs(nz[:, 0], nz[:, 1], A.shape[0], A.shape[1], A.device)


def spread_general(A: Interactions) -> torch.Tensor:
    gW = torch.empty((A.n_items, A.n_items), dtype=torch.float64, device=A.k_item.device)
    N.check(N.lib().lg_spread_general_f64(
        N.ptr(A.by_item.rowptr), N.ptr(A.by_item.col), N.ptr(A.by_user.rowptr),
        N.ptr(A.by_user.col), A.n_users, A.n_items, N.ptr(gW),
        N.stream_handle(gW.device)), "lg_spread_general_f64")
    return gW


def hybrid_weight(gW: torch.Tensor, k_item: torch.Tensor, lam: float,
                  transpose: bool = False) -> torch.Tensor:
    N.require_gpu(gW, "gW")
    gW = gW.contiguous().to(torch.float64)
    k_item = k_item.contiguous().to(torch.float64)
    W = torch.empty_like(gW)
    N.check(N.lib().lg_hybrid_weight_f64(N.ptr(gW), N.ptr(k_item), gW.shape[0], float(lam),
                                         int(bool(transpose)), N.ptr(W),
                                         N.stream_handle(gW.device)), "lg_hybrid_weight_f64")
    return W


def spread_hybrid(A: Interactions, lam: float) -> torch.Tensor:
    """hybrid_weight(spread_general(A), A.k_item, lam) (either transpose: general_W is
    exactly symmetric) bit for bit, without general_W in memory (lg_spread_hybrid_f64)."""
    dev = A.k_item.device
    I = A.n_items
    W = torch.empty((I, I), dtype=torch.float64, device=dev)
    ws = torch.empty(max(1, N.lib().lg_spread_hybrid_ws_bytes(I, A.n_users)),
                     dtype=torch.uint8, device=dev)
    N.check(N.lib().lg_spread_hybrid_f64(
        N.ptr(A.by_item.rowptr), N.ptr(A.by_item.col), N.ptr(A.by_user.rowptr),
        N.ptr(A.by_user.col), N.ptr(A.k_item), A.n_users, I, float(lam), N.ptr(W), N.ptr(ws),
        ws.numel(), N.stream_handle(dev)), "lg_spread_hybrid_f64")
    return W


def spread_resource(A: Interactions, W: torch.Tensor, users: slice | None = None,
                    out: torch.Tensor | None = None) -> torch.Tensor:
    """F rows for users [u0, u1) (all by default)."""
    u0, u1 = (0, A.n_users) if users is None else (users.start, users.stop)
    W = W.contiguous()
    F = out if out is not None else torch.empty((u1 - u0, A.n_items), dtype=torch.float64,
                                                device=W.device)
    N.check(N.lib().lg_spread_resource_f64(
        N.ptr(A.by_user.rowptr[u0:]), N.ptr(A.by_user.col), N.ptr(W), u1 - u0, A.n_items,
        N.ptr(F), F.stride(0), N.stream_handle(W.device)), "lg_spread_resource_f64")
    return F


def rows_topk(F: torch.Tensor, k: int, excl: RowSets | None = None, drop: bool = True,
              eu: torch.Tensor | None = None, ei: torch.Tensor | None = None):
    """Per-row top-k of F (optionally times the fp32 score G = eu . ei), excluded columns
    dropped (drop=True) or kept (drop=False). Returns (values fp64, indices int64, -1 pad)."""
    N.require_gpu(F, "F")
    if F.dtype != torch.float64:
        raise TypeError("F must be float64")
    if F.stride(1) != 1:
        F = F.contiguous()
    n, m = F.shape
    d = 0
    if eu is not None:
        eu, ei = _f32(eu, "eu"), _f32(ei, "ei")
        d = eu.shape[1]
    val = torch.empty((n, k), dtype=torch.float64, device=F.device)
    idx = torch.empty((n, k), dtype=torch.int64, device=F.device)
    N.check(N.lib().lg_rows_topk_f64(
        N.ptr(F), F.stride(0), n, m, N.ptr(eu), N.ptr(ei), d,
        N.ptr(excl.rowptr if excl else None), N.ptr(excl.col if excl else None),
        N.LG_EXCL_DROP if drop else N.LG_EXCL_NONE, int(k), N.ptr(val), N.ptr(idx),
        N.stream_handle(F.device)), "lg_rows_topk_f64")
    return val, idx


def spread_topk(A: Interactions, W: torch.Tensor, k: int, excl: RowSets | None,
                drop: bool = True, eu: torch.Tensor | None = None,
                ei: torch.Tensor | None = None, block_users: int | None = None):
    """F = A @ W computed block by block and reduced to per-user top-k without ever
    holding all of F (the fused recommend path of SpreadMethod / SpreadLightGCN)."""
    U, I = A.n_users, A.n_items
    if block_users is None:
        block_users = max(1, min(U, (1 << 30) // max(1, I * 8)))  # ~1 GiB of F per block
    vals = torch.empty((U, k), dtype=torch.float64, device=W.device)
    idxs = torch.empty((U, k), dtype=torch.int64, device=W.device)
    buf = torch.empty((min(block_users, U), I), dtype=torch.float64, device=W.device)
    for u0 in range(0, U, block_users):
        u1 = min(U, u0 + block_users)
        Fb = spread_resource(A, W, slice(u0, u1), out=buf[: u1 - u0])
        ex = excl.slice_rows(u0, u1) if excl is not None else None
        v, i = rows_topk(Fb, k, ex, drop, None if eu is None else eu[u0:u1], ei)
        vals[u0:u1], idxs[u0:u1] = v, i
    return vals, idxs


# ------------------------------------------------------------------- factored spreading
INV_TAB = 512      # degree classes cached in LDS by the walk (csrc/spread_tiled.hip)
MAX_CLASSES = 0x7FFF   # P slot words keep bit 31 clear (it marks V entries)
LINE_SLOTS, LINE_ENTS = 31, 7   # P slots / V entries in a row's 128-byte line
GROUP_MAX, GROUP_WIDE = 16, 8   # tiles per group build (tiles wider than 4096: 8)
OVF_UNITS_MAX = 1 << 29  # a group's overflow units (the rows' 29-bit overflow pointers)


def hybrid_recip(k_item: torch.Tensor, lam: float):
    """(ra, rb) = (1 / k_i^(1-lambda), 1 / k_i^lambda), a zero factor -> 1: the walk's
    HybridS factors (lg_hybrid_recip_f64)."""
    k_item = k_item.contiguous().to(torch.float64)
    n = k_item.shape[0]
    ra = torch.empty(n, dtype=torch.float64, device=k_item.device)
    rb = torch.empty_like(ra)
    N.check(N.lib().lg_hybrid_recip_f64(N.ptr(k_item), n, float(lam), N.ptr(ra), N.ptr(rb),
                                        N.stream_handle(k_item.device)), "lg_hybrid_recip_f64")
    return ra, rb


class HybridScale:
    """The lambda-dependent side of the factored spreading: rb = 1/beta per item and
    ra_edge = 1/alpha of the item of every interaction, aligned with A.by_user.col (so the
    walk reads a user's factors contiguously with its item ids)."""

    def __init__(self, A: "Interactions", lam: float):
        self.lam = float(lam)
        ra, self.rb = hybrid_recip(A.k_item, lam)
        # one entry past the interactions: the walk's padding rows read it (never used)
        self.ra_edge = torch.cat([ra[A.by_user.col.to(torch.int64)], ra.new_zeros(1)])


def degree_classes(deg: torch.Tensor):
    """(1-based class of each row's degree as uint16, fp64 table inv[c] = fl(1/k) of class
    c, inv[0] = 0): the slot code of the P rows of csrc/spread_tiled.hip. Classes are
    numbered by how many rows have the degree, so the common ones fall in the walk's LDS
    table (c < 512). Rows of degree 0 get class 0 (they are in no pair)."""
    dev = deg.device
    pos = deg[deg > 0]
    if pos.numel() == 0:
        return (torch.zeros(deg.numel(), dtype=torch.int16, device=dev).view(torch.uint16),
                torch.zeros(INV_TAB, dtype=torch.float64, device=dev))
    uniq, counts = torch.unique(pos, return_counts=True)
    if uniq.numel() >= MAX_CLASSES:
        raise ValueError(f"{uniq.numel()} distinct user degrees: the tile format encodes at "
                         f"most {MAX_CLASSES - 1} (use the dense spreading path)")
    order = torch.argsort(counts, descending=True, stable=True)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(order.numel(), device=dev)
    cls = torch.zeros(deg.numel(), dtype=torch.int32, device=dev)
    m = deg > 0
    cls[m] = (rank[torch.searchsorted(uniq, deg[m])] + 1).to(torch.int32)
    inv = torch.zeros(max(INV_TAB, uniq.numel() + 1), dtype=torch.float64, device=dev)
    inv[1:uniq.numel() + 1] = 1.0 / uniq[order].to(torch.float64)
    return cls.to(torch.int16).view(torch.uint16), inv


def _run_units(length: torch.Tensor, hub: torch.Tensor) -> torch.Tensor:
    """Overflow units (run header + data) of rows with `length` pairs (P) / entries (V)."""
    p = torch.where(length > LINE_SLOTS, 1 + (length - LINE_SLOTS + 3) // 4,
                    torch.zeros_like(length))
    v = torch.where(length > LINE_ENTS, 1 + (length - LINE_ENTS), torch.zeros_like(length))
    return torch.where(hub, v, p)


class TileWeights:
    """general_W restricted to one item tile, in the line format of csrc/spread_tiled.hip
    (lg_spread_tile_rows_f64: one 128-byte line per item row at 128 * i, plus overflow runs;
    P rows = the (user, item) pairs behind the row as 4-byte slots, V rows = the merged fp64
    general_W values of hub items). The tile itself is lambda-independent; ``lam`` sets the
    HybridScale the walk applies. build() moves to the next tile; the buffers are
    reused and grown on demand. ``vthr``: rows with more pairs are V rows (default: the tile
    width).

    Tiles are built ``group`` at a time (1..16, default 16; at most 8 for tiles wider than
    4096): lg_spread_group_cursor / _bound / _units / _rows_f64 visit each (item row, user)
    pair once per group instead of once per tile and write the group's tiles side by side; build(j0) of a tile inside the built
    group only selects it. Every tile's words are those of the per-tile reference build
    (include/lgcnhs_ref.h) bit for bit (tests/test_gpu_spread_tiled.py)."""

    def __init__(self, A: Interactions, lam: float, tile: int, vthr: int | None = None,
                 group: int | None = None):
        if not 1 <= tile <= 8192:
            raise ValueError(f"tile {tile} not in [1, 8192]")
        self.A, self.tile, self.lam = A, int(tile), float(lam)
        dev = A.k_item.device
        self.dev = dev
        if vthr is None:
            vthr = self.tile
        self.vthr = max(LINE_SLOTS, int(vthr))
        gmax = GROUP_MAX if self.tile <= 4096 else GROUP_WIDE
        self._auto_group = group is None  # (a default group halves itself when too large)
        if group is None:
            group = gmax
        if not 1 <= group <= gmax:
            raise ValueError(f"group {group} not in [1, {gmax}] (tile {self.tile})")
        if self.vthr > 65535:
            raise ValueError(f"vthr {self.vthr} > 65535 (the group build counts 16-bit)")
        I = A.n_items
        self.group = int(min(group, max(1, -(-I // self.tile))))
        S = self.group
        self.cur = A.by_user.rowptr[:-1].contiguous().clone()
        self.end = torch.empty_like(self.cur)
        # 16 uint16 per user (two 16-byte halves: tiles 0-7, 8-15) + the rows pass's 16-byte
        # records
        if int(A.by_user.rowptr[-1]) >= 1 << 32:
            raise ValueError("more than 2^32 interactions: the group build's positions are "
                             "32-bit")
        self.counts = torch.empty((A.n_users, GROUP_MAX), dtype=torch.uint16, device=dev)
        self.rec = torch.empty((A.n_users, 4), dtype=torch.int32, device=dev)
        self.inv_deg = torch.empty(A.n_users, dtype=torch.float64, device=dev)
        N.check(N.lib().lg_inv_degree_f64(N.ptr(A.by_user.rowptr), A.n_users,
                                          N.ptr(self.inv_deg), N.stream_handle(dev)),
                "lg_inv_degree_f64")
        self.user_cls, self.inv_cls = degree_classes(A.by_user.degrees())
        self.g_bound = torch.empty((S, I), dtype=torch.int64, device=dev)
        # run units per (tile, row), their flat inclusive scan, the tiles' ends
        self.g_units = torch.empty(S * I, dtype=torch.int64, device=dev)
        self.g_incl = torch.empty(max(1, S * I), dtype=torch.int64, device=dev)
        self._tile_ends = torch.arange(1, S + 1, dtype=torch.int64, device=dev) * I - 1
        self._ends_host = torch.empty(S, dtype=torch.int64).pin_memory()
        self._ends_ev = torch.cuda.Event()
        # I + 1 lines per tile: line I (the walk's padding row) stays all zero
        self.g_lines = torch.empty((S, (I + 1) * 32), dtype=torch.int32, device=dev)
        self.g_lines[:, I * 32:].zero_()
        self.g_row_len = torch.empty((S, max(1, I)), dtype=torch.int32, device=dev)
        ws = N.lib().lg_spread_group_rows_ws_bytes(I, S)
        self.ws = torch.empty(max(1, ws), dtype=torch.uint8, device=dev)
        self.g_ovf = torch.zeros(64 * 4, dtype=torch.int32, device=dev)
        self._grp = None  # (first item, [widths], [ovf bases], [overflow units]) built
        self.j0 = None
        self.width = 0
        self._seek_at = None
        self._scale = None
        self.row_uses = None  # set by spread_topk_tiled(stats=...)

    @property
    def scale(self) -> HybridScale:
        if self._scale is None:
            self._scale = HybridScale(self.A, self.lam)
        return self._scale

    @property
    def is_hub(self) -> torch.Tensor:
        """True for V (merged-value) rows of the current tile."""
        return self.bound > self.vthr

    def dense(self) -> torch.Tensor:
        """general_W of the current tile as a dense [I, width] fp64 matrix (host, test
        helper), decoded from the lines with the format invariants checked: P slots summed in
        slot order (users ascending: lg_spread_general_f64's order), V values as stored."""
        I = self.A.n_items
        lines = self.lines[:I * 32].cpu().numpy().view(np.uint32).reshape(I, 32)
        ovf = self.ovf.cpu().numpy().view(np.uint32)
        inv = self.inv_cls.cpu().numpy()
        rl = self.row_len.cpu().numpy()
        hub = self.is_hub.cpu().numpy()
        out = np.zeros((I, self.width))
        for i in range(I):
            h = int(lines[i, 0])
            isv, has, slow, ou = h >> 31, (h >> 30) & 1, (h >> 29) & 1, h & 0x1FFFFFFF
            assert bool(isv) == bool(hub[i]) and (slow or not isv)
            run = np.zeros((0, 4), np.uint32)
            if has and not (isv and int(ovf[4 * ou]) >> 31):
                n = int(ovf[4 * ou])
                assert np.all(ovf[4 * ou + 1:4 * ou + 4] == 0)
                run = ovf[4 * (ou + 1):4 * (ou + 1 + n)].reshape(n, 4)
            if isv and has and int(ovf[4 * ou]) >> 31:  # a dense V row
                nd = int(ovf[4 * ou]) & 0x7FFFFFFF
                assert nd == (self.width + 1) // 2 and np.all(lines[i, 1:] == 0)
                run = ovf[4 * (ou + 1):4 * (ou + 1 + nd)].reshape(nd, 4)
                vals = run.reshape(-1).view(np.uint64).view(np.float64)  # (lo, hi) pairs
                assert np.all(vals[self.width:] == 0) and int((vals != 0).sum()) == rl[i]
                assert rl[i] > self.width // 2 + 8
                out[i, :] = vals[:self.width]
                continue
            if isv:
                assert rl[i] <= self.width // 2 + 8
                assert np.all(lines[i, 1:4] == 0)
                units = np.concatenate([lines[i, 4:].reshape(7, 4), run])
                units = units[units[:, 0] != 0]
                assert units.shape[0] == rl[i] and np.all(units[:, 0] >> 31 == 1)
                col = (units[:, 0] & 0xFFFF).astype(np.int64)
                assert np.all(np.diff(col) > 0) and np.all(col < self.width)
                out[i, col] = (units[:, 1].astype(np.uint64) |
                               (units[:, 2].astype(np.uint64) << 32)).view(np.float64)
                continue
            words = np.concatenate([lines[i, 1:], run.reshape(-1)])
            n = int(rl[i])
            assert np.all(words[:n] != 0) and np.all(words[n:] == 0)
            col = (words[:n] & 0xFFFF).astype(np.int64)
            cls = (words[:n] >> 16).astype(np.int64)
            assert np.all(col < self.width) and np.all(cls > 0)
            assert bool(slow) == bool(np.any(cls >= INV_TAB))
            for c, q in zip(col, cls):
                out[i, c] += inv[q]
        return out

    def seek(self, j0: int) -> None:
        """Start the tile walk at item j0 instead of 0 (an item-range shard): the next
        build() must be build(j0)."""
        A = self.A
        if not 0 <= j0 <= A.n_items:
            raise ValueError(f"seek({j0}) outside [0, {A.n_items}]")
        N.check(N.lib().lg_spread_tile_seek(N.ptr(A.by_user.rowptr), N.ptr(A.by_user.col),
                                            A.n_users, j0, N.ptr(self.cur),
                                            N.stream_handle(self.dev)), "lg_spread_tile_seek")
        self._seek_at = j0

    def build(self, j0: int, stop: int | None = None) -> None:
        """Build the tile [j0, min(j0 + tile, stop)); tiles come in ascending order from 0
        (or from the item given to seek()). Builds the group starting at j0 unless j0 is the
        next tile of the group already built."""
        I = self.A.n_items
        stop = I if stop is None else min(int(stop), I)
        g = self._grp
        if (g is not None and self._seek_at is None and self.j0 is not None
                and j0 == self.j0 + self.width and j0 < g[0] + sum(g[1])):
            self._select((j0 - g[0]) // self.tile)
            return
        if self._seek_at is not None and j0 == self._seek_at:
            pass  # cursors placed by seek()
        elif j0 == 0:
            self.cur.copy_(self.A.by_user.rowptr[:-1])
        elif self.j0 is None or j0 != self.j0 + self.width:
            raise ValueError("tiles must be built in ascending order")
        else:
            self.cur, self.end = self.end, self.cur
        self._seek_at = None
        if stop - j0 <= 0:
            raise ValueError(f"empty tile at {j0} (stop {stop})")
        widths = [min(self.tile, stop - t0) for t0 in
                  range(j0, min(stop, j0 + self.group * self.tile), self.tile)]
        self._build_group(j0, stop, widths)
        self._select(0)

    def _build_group(self, j0: int, stop: int, widths: list) -> None:
        A, I, L = self.A, self.A.n_items, N.lib()
        strm = N.stream_handle(self.dev)
        nt = len(widths)
        # group: cursors, bounds, run units and their inclusive scan all on the device; one
        # event wait for the tiles' unit totals (to size ovf), then the rows
        N.check(L.lg_spread_group_cursor(N.ptr(A.by_user.rowptr), N.ptr(A.by_user.col),
                                         N.ptr(self.user_cls), A.n_users, j0, self.tile, nt,
                                         stop, N.ptr(self.cur), N.ptr(self.end),
                                         N.ptr(self.counts), N.ptr(self.rec), strm),
                "lg_spread_group_cursor")
        N.check(L.lg_spread_group_bound(N.ptr(A.by_item.rowptr), N.ptr(A.by_item.col), I,
                                        N.ptr(self.counts), nt, N.ptr(self.g_bound), strm),
                "lg_spread_group_bound")
        if I:
            units = self.g_units[:nt * I]
            N.check(L.lg_spread_group_units(N.ptr(self.g_bound), I, j0, self.tile, nt, stop,
                                            self.vthr, N.ptr(units), strm),
                    "lg_spread_group_units")
            incl = self.g_incl[:nt * I]
            torch.cumsum(units, 0, out=incl)
            ends = torch.index_select(incl, 0, self._tile_ends[:nt])
            self._ends_host[:nt].copy_(ends, non_blocking=True)
            self._ends_ev.record()
            self._ends_ev.synchronize()  # the tiles' last units (not the whole stream's work)
            ends = self._ends_host[:nt].tolist()
        else:
            ends = [0] * nt
        bases = [0] + ends[:-1]
        totals = [e - b for e, b in zip(ends, bases)]
        if ends[-1] + 64 >= OVF_UNITS_MAX:
            if self._auto_group and nt > 1:
                # the default group size: retry this group (and build the later ones) with
                # half as many tiles -- the cursor kernel reads cur and rewrites only end
                self.group = nt // 2
                self._build_group(j0, stop, widths[:self.group])
                return
            raise ValueError("tile group too large for the 29-bit overflow pointers (use a "
                             "smaller tile or group)")
        self._grow_ovf(ends[-1])
        N.check(L.lg_spread_group_rows_f64(
            N.ptr(A.by_item.rowptr), N.ptr(A.by_item.col), N.ptr(A.by_user.col),
            N.ptr(self.inv_deg), I, N.ptr(self.cur), N.ptr(self.counts), N.ptr(self.rec),
            j0, self.tile, nt, stop, N.ptr(self.g_bound), self.vthr,
            N.ptr(self.g_incl), N.ptr(self.g_lines), N.ptr(self.g_ovf),
            N.ptr(self.g_row_len), N.ptr(self.ws), self.ws.numel(), strm),
            "lg_spread_group_rows_f64")
        self._grp = (j0, widths, bases, totals)

    def _grow_ovf(self, units: int) -> None:
        need = (units + 64) * 4
        if need > self.g_ovf.numel():
            self.g_ovf = torch.zeros(max(need, int(self.g_ovf.numel() * 1.25)),
                                     dtype=torch.int32, device=self.dev)

    def _select(self, t: int) -> None:
        """Make tile t of the built group the current tile (lines / ovf / bound / row_len
        views, j0, width, n_units)."""
        g0, widths, bases, totals = self._grp
        I = self.A.n_items
        self.j0, self.width = g0 + t * self.tile, widths[t]
        self.lines = self.g_lines[t]
        self.ovf = self.g_ovf[bases[t] * 4:]
        self.bound = self.g_bound[t]
        self.row_len = self.g_row_len[t]
        self.n_units = totals[t]
        if self.row_uses is not None:
            hub = self.is_hub
            ln = self.row_len[:I].to(torch.int64)
            self.paths_read += (self.row_uses * ln).sum()
            self.paths_hub += (self.row_uses * ln * hub[:I]).sum()  # (V rows' share)
            used = _run_units(ln, hub)
            # (dense V rows: ceil(width / 2) data units + the header, whatever their entries)
            used = torch.where(hub[:I] & (ln > self.width // 2 + 8),
                               torch.full_like(used, 1 + (self.width + 1) // 2), used)
            self.bytes_read += 128 * self.row_uses.sum() + 16 * (self.row_uses * used).sum()

def spread_topk_tiled(A: Interactions, lam: float, k: int, excl: RowSets | None,
                      drop: bool = True, eu: torch.Tensor | None = None,
                      ei: torch.Tensor | None = None, users: slice | None = None,
                      tile: int = 2048, items: slice | None = None,
                      stats: dict | None = None, count_paths: bool = False,
                      col_bounds: bool = True, **_):
    """Per-user top-k of (G *) F, F = A @ HybridS(A, general_W, lam), over item tiles:
    never holds general_W, W (I x I) or F (U x I). The values of spread_topk(A,
    hybrid_weight(spread_general(A), A.k_item, lam), ...) within a few ulp (the walk's
    summation order), the lists equal except near-ties.

    Each tile of general_W (user-independent) is built once and walked by every user
    (lg_spread_tile_resource_topk_f64): the user's F columns are summed in LDS and merged
    into its running top-k list in the same pass. With a G factor (SpreadLightGCN) the
    per-(user, 64-column chunk) score bounds of lg_score_chunk_bound (bf16 MFMA) screen the
    columns, so only those whose bound times F can beat the list's k-th value get the exact
    fp32 score chain. ``users`` restricts the output to a row range; ``items`` restricts the
    candidates to an item range (the lists of disjoint item ranges merge, with
    merge_topk_lists, into the full lists: the multi-GPU item shard). (The two-kernel form
    -- F written per tile, then a top-K merge -- is a test reference, tests/_ref_paths.py.)
    ``stats`` (optional dict) receives the HIP-event times of the tile
    builds / score bounds / walk launches (t_*_ms, walk_launches) and the walk's (user, item)
    rows per launch; with ``count_paths`` also "w_paths": the paths the walk adds (sum over
    tiles and users u of sum_{i in items(u)} the pairs (P) / entries (V) of row i in the
    tile) and "w_bytes": the row bytes it gathers (one 128-byte line per (user, item) and
    tile, plus 16 bytes per overflow unit) -- extra GPU work per tile, so timed runs leave it
    off and take the counts from tile_traffic()."""
    u0, u1 = (0, A.n_users) if users is None else (users.start, users.stop)
    i0, i1 = (0, A.n_items) if items is None else (max(0, items.start),
                                                   min(A.n_items, items.stop))
    n = u1 - u0
    dev = A.k_item.device
    vals = torch.full((n, k), float("-inf"), dtype=torch.float64, device=dev)
    idxs = torch.full((n, k), -1, dtype=torch.int64, device=dev)
    if n == 0 or i1 <= i0:
        return vals, idxs
    tile = min(int(tile), i1 - i0, 4096 if eu is not None else 8192)  # G: <= 64 chunk bounds
    tw = TileWeights(A, lam, tile)
    if i0:
        tw.seek(i0)
    ex = excl.slice_rows(u0, u1) if excl is not None else None
    eu_r = None if eu is None else eu[u0:u1]
    if stats is not None and count_paths:
        _count_rows(tw, A, u0, u1)
    walk = TileWalk(A, u0, u1, i0, k, ex if drop else None, eu_r, ei, tile, col_bounds)
    evs = [] if stats is not None else None
    for j0 in range(i0, i1, tile):
        if evs is not None:  # per-tile HIP events on the launch stream: build / bounds / walk
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            e[0].record()
        tw.build(j0, stop=i1)
        if evs is not None:
            e[1].record()
        bnd = walk.bounds(j0, tw.width, tw.scale)
        if evs is not None:
            e[2].record()
        walk.step(tw.lines, tw.ovf, tw.inv_cls, tw.scale, j0, tile, tw.width, j0 == i0, bnd)
        if evs is not None:
            e[3].record()
            evs.append(e)
    vals.copy_(walk.vals)
    idxs.copy_(walk.idxs)
    if evs:
        torch.cuda.synchronize(dev)
        stats["t_build_ms"] = stats.get("t_build_ms", 0.0) + sum(e[0].elapsed_time(e[1]) for e in evs)
        stats["t_bounds_ms"] = stats.get("t_bounds_ms", 0.0) + sum(e[1].elapsed_time(e[2]) for e in evs)
        stats["t_walk_ms"] = stats.get("t_walk_ms", 0.0) + sum(e[2].elapsed_time(e[3]) for e in evs)
        stats["walk_launches"] = stats.get("walk_launches", 0) + len(evs)
        stats["walk_ms_list"] = stats.get("walk_ms_list", []) + [e[2].elapsed_time(e[3]) for e in evs]
        stats["user_items"] = stats.get("user_items", 0) + len(evs) * int(
            A.by_user.rowptr[u1] - A.by_user.rowptr[u0])
        stats["users"] = n
        stats["qstride"] = 0 if walk.d == 0 or walk.qbuf is None else walk.qbuf.shape[1]
        stats["nch"] = -(-tile // 64) if walk.d else 0
    if stats is not None and count_paths:
        stats["w_paths"] = stats.get("w_paths", 0) + int(tw.paths_read)
        stats["w_paths_hub"] = stats.get("w_paths_hub", 0) + int(tw.paths_hub)
        stats["w_bytes"] = stats.get("w_bytes", 0) + int(tw.bytes_read)
    return vals, idxs


def _count_rows(tw: "TileWeights", A: Interactions, u0: int, u1: int) -> None:
    """Make tw accumulate the walk's paths / row bytes for users [u0, u1) as tiles are
    selected (the times each item's row is gathered per tile = its users in the range)."""
    cols = A.by_user.col[int(A.by_user.rowptr[u0]):int(A.by_user.rowptr[u1])]
    tw.row_uses = torch.bincount(cols, minlength=A.n_items).to(torch.int64)
    tw.paths_read = torch.zeros((), dtype=torch.int64, device=A.k_item.device)
    tw.paths_hub = torch.zeros((), dtype=torch.int64, device=A.k_item.device)
    tw.bytes_read = torch.zeros((), dtype=torch.int64, device=A.k_item.device)


def tile_traffic(A: Interactions, tile: int = 2048, users: slice | None = None,
                 items: slice | None = None, hub: bool = False) -> tuple:
    """(paths, row bytes) the tile walk of users / items gathers (the stats of
    spread_topk_tiled(count_paths=True)), from the tiles alone: builds every tile, no walk;
    with ``hub`` also the paths that come from V (hub) rows: (paths, row bytes, V paths)."""
    u0, u1 = (0, A.n_users) if users is None else (users.start, users.stop)
    i0, i1 = (0, A.n_items) if items is None else (max(0, items.start),
                                                   min(A.n_items, items.stop))
    if i1 <= i0 or u1 <= u0:
        return (0, 0, 0) if hub else (0, 0)
    tw = TileWeights(A, 0.5, min(int(tile), i1 - i0))
    if i0:
        tw.seek(i0)
    _count_rows(tw, A, u0, u1)
    for j0 in range(i0, i1, tw.tile):
        tw.build(j0, stop=i1)
    if hub:
        return int(tw.paths_read), int(tw.bytes_read), int(tw.paths_hub)
    return int(tw.paths_read), int(tw.bytes_read)


def bound_operands(x: torch.Tensor, with_err: bool = False):
    """(bf16 copy as int16 storage, fp32 row norms rounded up) of an fp32 [n, d] matrix:
    the operands of lg_score_chunk_bound; with_err also the rounded-up norms of
    x - bf16(x) (screen_margins' operand)."""
    x = _f32(x, "x")
    xb = torch.empty(x.shape, dtype=torch.int16, device=x.device)
    nrm = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    err = torch.empty(x.shape[0], dtype=torch.float32, device=x.device) if with_err else None
    N.check(N.lib().lg_bound_prep_f32(N.ptr(x), x.shape[0], x.shape[1], N.ptr(xb), N.ptr(nrm),
                                      N.ptr(err), N.stream_handle(x.device)),
            "lg_bound_prep_f32")
    return (xb, nrm, err) if with_err else (xb, nrm)


def chunk_bounds(ub, un, ib, inorm, dim: int, j0: int, width: int,
                 out: torch.Tensor | None = None, qout: torch.Tensor | None = None):
    """[users, ceil(width/64)] fp32 upper bounds of the fp32 score chain over each 64-column
    chunk of items [j0, j0 + width) (lg_score_chunk_bound); with qout ([users, qstride]
    uint8, qstride >= width rounded up to 256) also the per-column 8-bit bounds. Returns gb,
    or (gb, q) with qout. width <= 4096 (LG_BOUND_MAX_WIDTH; the library refuses wider
    tiles)."""
    n = ub.shape[0]
    nch = -(-width // 64)
    if out is None or out.numel() < n * nch:
        out = torch.empty(n * nch, dtype=torch.float32, device=ub.device)
    gb = out[:n * nch].view(n, nch)
    qs = 0 if qout is None else qout.shape[1]
    N.check(N.lib().lg_score_chunk_bound(N.ptr(ub), N.ptr(un), n, N.ptr(ib), N.ptr(inorm),
                                         int(dim), int(j0), int(width), N.ptr(gb),
                                         N.ptr(qout), int(qs),
                                         N.stream_handle(ub.device)),
            "lg_score_chunk_bound")
    return gb if qout is None else (gb, qout)


class TileWalk:
    """The fused top-K walk of users [u0, u1) over general_W tiles
    (lg_spread_tile_resource_topk_f64 per tile, with lg_score_chunk_bound screening when
    there is a G factor). Holds the running lists (vals fp64 / idxs int64 [n, k]), the
    per-user exclusion cursors and the bf16 score operands, so several walks (a lambda sweep)
    can share them."""

    def __init__(self, A: Interactions, u0: int, u1: int, i0: int, k: int,
                 ex: RowSets | None, eu=None, ei=None, tile: int = 2048,
                 col_bounds: bool = True):
        self.A, self.u0, self.u1, self.i0, self.k, self.ex = A, u0, u1, i0, int(k), ex
        # the walk keeps its stream positions in 32 bits
        if A.by_user.col.numel() >= 2**31 or (ex is not None and ex.col.numel() >= 2**31):
            raise ValueError("the tile walk needs fewer than 2^31 interactions / exclusions")
        self.n = u1 - u0
        self.dev = A.k_item.device
        self.vals = torch.full((self.n, self.k), float("-inf"), dtype=torch.float64,
                               device=self.dev)
        self.idxs = torch.full((self.n, self.k), -1, dtype=torch.int64, device=self.dev)
        self.d = 0
        self.eu = self.ei = None
        if eu is not None:
            self.eu, self.ei = _f32(eu, "eu"), _f32(ei, "ei")
            self.d = self.eu.shape[1]
            self.ub, self.un = bound_operands(self.eu)
            self.ib, self.inorm = bound_operands(self.ei)
            self.gbuf = torch.empty(self.n * -(-int(tile) // 64), dtype=torch.float32,
                                    device=self.dev)
            # per-column 8-bit bounds (col_bounds=False: chunk bounds only)
            self.qbuf = None
            if col_bounds:
                self.qbuf = torch.empty((self.n, -(-int(tile) // 256) * 256),
                                        dtype=torch.uint8, device=self.dev)
        self.ex_cur = None
        if ex is not None:
            self.ex_cur = torch.empty(self.n, dtype=torch.int64, device=self.dev)
        self.reset()

    def reset(self) -> None:
        """Empty lists; exclusion cursors back at the walk's first item."""
        self.vals.fill_(float("-inf"))
        self.idxs.fill_(-1)
        if self.ex is not None:
            N.check(N.lib().lg_spread_tile_seek(N.ptr(self.ex.rowptr), N.ptr(self.ex.col),
                                                self.n, self.i0, N.ptr(self.ex_cur),
                                                N.stream_handle(self.dev)),
                    "lg_spread_tile_seek")

    def bounds(self, j0: int, width: int, scale: "HybridScale | None" = None):
        """(gb, q) score bounds of tile [j0, j0 + width) (q None: chunk bounds only)."""
        if not self.d:
            return None
        if self.qbuf is None:
            return chunk_bounds(self.ub, self.un, self.ib, self.inorm, self.d, j0, width,
                                self.gbuf), None
        return chunk_bounds(self.ub, self.un, self.ib, self.inorm, self.d, j0, width,
                            self.gbuf, self.qbuf)

    def step(self, lines, ovf, inv_cls, scale: HybridScale, j0: int, tile: int, width: int,
             first: bool, bnd=None) -> None:
        """Merge tile [j0, j0 + width) (its rows: lines / ovf) into the lists; bnd = the
        tile's bounds() (computed here when None)."""
        A, ex = self.A, self.ex
        if self.d and bnd is None:
            bnd = self.bounds(j0, width, scale)
        gb, q = bnd if bnd is not None else (None, None)
        nch = gb.shape[1] if gb is not None else 0
        N.check(N.lib().lg_spread_tile_resource_topk_f64(
            N.ptr(A.by_user.rowptr[self.u0:]), N.ptr(A.by_user.col), N.ptr(scale.ra_edge),
            self.n, N.ptr(lines), N.ptr(ovf), A.n_items, N.ptr(scale.rb), N.ptr(inv_cls), int(j0),
            int(tile), int(width), N.ptr(self.eu), N.ptr(self.ei), self.d, N.ptr(gb), nch,
            N.ptr(q), 0 if q is None else q.shape[1],
            N.ptr(ex.rowptr if ex is not None else None),
            N.ptr(ex.col if ex is not None else None), N.ptr(self.ex_cur), self.k,
            int(bool(first)), N.ptr(self.vals), N.ptr(self.idxs), A.by_user.col.numel(),
            ex.col.numel() if ex is not None else 0, N.stream_handle(self.dev)),
            "lg_spread_tile_resource_topk_f64")


def spread_lambda_sweep(A: Interactions, lams, k: int, excl: RowSets | None,
                        drop: bool = True, eu: torch.Tensor | None = None,
                        ei: torch.Tensor | None = None, tiled: bool | None = None,
                        tile: int = 2048, cache_bytes: int | None = None):
    """Yield (lam, values [U, k] fp64, items [U, k] int64) of spread_recommend for every
    lam of ``lams`` (the loop of findLambda.py:93-114: HybridS -> A @ W -> G * F -> top-k per
    lambda), reusing what does not depend on lambda:
      dense  general_W (lg_spread_general_f64) once; per lambda W (lg_hybrid_weight_f64) and
             the fused F / top-k.
      tiled  the general_W tiles (lambda-independent: ra / rb are applied by the walk) are
             built once and cached on the device while they fit ``cache_bytes`` (default:
             half the free memory); per lambda only the HybridScale (ra per interaction, rb
             per item) changes and the score bounds are recomputed (cheap; the per-column
             bounds of every tile would not fit). If the cache does not fit, each lambda
             rebuilds the tiles.
    Every result is bitwise the one spread_recommend(A, lam, ...) returns."""
    lams = [float(x) for x in lams]
    dev = A.k_item.device
    if tiled is None:
        tiled = not dense_spread_fits(A.n_items, dev)
    if not tiled:
        gW = spread_general(A)
        for lam in lams:
            W = hybrid_weight(gW, A.k_item, lam)
            v, i = spread_topk(A, W, k, excl, drop, eu, ei)
            del W
            yield lam, v, i
        return
    if cache_bytes is None:
        cache_bytes = torch.cuda.mem_get_info(dev)[0] // 2
    U, I = A.n_users, A.n_items
    tile = min(int(tile), I, 4096 if eu is not None else 8192) if I else 1
    ex = excl if drop else None
    walk = TileWalk(A, 0, U, 0, k, ex, eu, ei, tile)
    cache, used, cached = [], 0, True
    inv_cls = None
    for n, lam in enumerate(lams):
        scale = HybridScale(A, lam)
        walk.reset()
        if n > 0 and cached:
            for (j0, width, lines, ovf) in cache:
                walk.step(lines, ovf, inv_cls, scale, j0, tile, width, j0 == 0)
        else:
            tw = TileWeights(A, lam, tile)
            inv_cls = tw.inv_cls
            for j0 in range(0, I, tile):
                tw.build(j0)
                walk.step(tw.lines, tw.ovf, inv_cls, scale, j0, tile, tw.width, j0 == 0)
                if n == 0 and cached and len(lams) > 1:
                    nov = (tw.n_units + 64) * 4
                    need = tw.lines.numel() * 4 + nov * 4
                    if used + need <= cache_bytes:
                        cache.append((j0, tw.width, tw.lines.clone(), tw.ovf[:nov].clone()))
                        used += need
                    else:
                        cached = False
                        cache.clear()
            del tw
        yield lam, walk.vals.clone(), walk.idxs.clone()


def merge_topk_lists(vals: torch.Tensor, idxs: torch.Tensor):
    """[L, n, k] sorted lists (index -1 = empty) -> the [n, k] top-k of their union, same
    order (value desc, index asc)."""
    N.require_gpu(vals, "vals")
    if vals.dtype != torch.float64 or idxs.dtype != torch.int64 or vals.shape != idxs.shape \
            or vals.dim() != 3:
        raise ValueError("merge_topk_lists: vals fp64 / idxs int64 of one [L, n, k] shape")
    L, n, k = vals.shape
    vals, idxs = vals.contiguous(), idxs.contiguous()
    ov = torch.empty((n, k), dtype=torch.float64, device=vals.device)
    oi = torch.empty((n, k), dtype=torch.int64, device=vals.device)
    N.check(N.lib().lg_topk_lists_merge_f64(N.ptr(vals), N.ptr(idxs), L, n, k, N.ptr(ov),
                                            N.ptr(oi), N.stream_handle(vals.device)),
            "lg_topk_lists_merge_f64")
    return ov, oi


def dense_spread_fits(n_items: int, device, fraction: float = 0.25) -> bool:
    """True when general_W and W (two fp64 I x I matrices) fit in ``fraction`` of the free
    device memory: the dense path; otherwise the factored tile path."""
    free, _ = torch.cuda.mem_get_info(device)
    return 2 * 8 * n_items * n_items <= fraction * free


def spread_recommend(A: Interactions, lam: float, k: int, excl: RowSets | None,
                     drop: bool = True, eu: torch.Tensor | None = None,
                     ei: torch.Tensor | None = None, transpose: bool = False,
                     tiled: bool | None = None):
    """Per-user top-k of (G *) A @ HybridS(A, general_W(^T), lam), dense (I x I matrices on
    the device) or factored over item tiles (tiled=None: dense when it fits). The two
    paths give the same values within a few ulp (the factored walk sums each column's paths
    in its own order) and the same lists except near-ties. general_W is exactly symmetric (entry (i, j) and (j, i) are
    the same sum, over the common users ascending, of the same fl(1/k_v)), so the
    reference's general_W.T overrides (model/SpreadMethod/recommend.py:89-91, :99-101)
    are served by either path unchanged."""
    if tiled is None:
        tiled = not dense_spread_fits(A.n_items, A.k_item.device)
    if tiled:
        return spread_topk_tiled(A, lam, k, excl, drop, eu, ei)
    W = spread_hybrid(A, lam)  # (= hybrid_weight(spread_general(A), ..., transpose))
    return spread_topk(A, W, k, excl, drop, eu, ei)
