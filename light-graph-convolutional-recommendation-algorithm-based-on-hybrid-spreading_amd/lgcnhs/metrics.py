"""Recommendation-list metrics on the device: the expensive parts of the
reference's metrics/accurate.py and metrics/diversity.py as HIP kernels (csrc/metrics.hip).

hit_flags           `item in items` labels (accurate.py:24-31, :69-76)   lg_rec_hits
accuracy            P / R / NDCG, fp64 on the device (accurate.py:11-102)
pair_overlap        sum_{u != v} |R_u & R_v|, exact (diversity.py:15-63)  lg_rec_pair_overlap
hamming             calHammingDistance's value, unrounded
intra_similarity    calInternalSimilarity's value, unrounded             lg_rec_intra_similarity_f64
                    (diversity.py:66-115)

The reference-signature wrappers (dicts, numpy matrices, 5-decimal rounding, float32 torch
reductions) are metrics/accurate.py and metrics/diversity.py of this package.
No CPU fallback: GPU tensors only.
"""
from __future__ import annotations

import torch

from . import _native as N
from .graph import RowSets


def _recs(recs: torch.Tensor) -> torch.Tensor:
    N.require_gpu(recs, "recs")
    if recs.dim() != 2:
        raise ValueError(f"recs must be [n_users, k], got shape {tuple(recs.shape)}")
    return recs.to(torch.int64).contiguous()


def hit_flags(recs: torch.Tensor, eval_rows: torch.Tensor, pos: RowSets) -> torch.Tensor:
    """uint8 [n_eval, k]: recs[eval_rows[q]][p] in row q of ``pos`` (one row per evaluated
    user, in eval_rows order)."""
    recs = _recs(recs)
    eval_rows = eval_rows.to(recs.device, torch.int64).contiguous()
    n_eval, k = int(eval_rows.numel()), recs.shape[1]
    if pos.n_rows != n_eval:
        raise ValueError(f"pos has {pos.n_rows} rows for {n_eval} evaluated users")
    if n_eval and (int(eval_rows.min()) < 0 or int(eval_rows.max()) >= recs.shape[0]):
        raise IndexError("evaluated user outside the recommendation matrix")
    hit = torch.empty((n_eval, k), dtype=torch.uint8, device=recs.device)
    N.check(N.lib().lg_rec_hits(N.ptr(recs), recs.shape[0], k, N.ptr(eval_rows), n_eval,
                                N.ptr(pos.rowptr), N.ptr(pos.col), N.ptr(hit),
                                N.stream_handle(recs.device)), "lg_rec_hits")
    return hit


def accuracy(recs: torch.Tensor, test: RowSets, k: int | None = None) -> dict:
    """Precision, recall and NDCG over the users with at least one test item (``test``: one
    sorted row per user of recs), in fp64 (the reference computes them in fp32 torch).
    NDCG keeps the reference's ideal DCG of k ones (accurate.py:80-89)."""
    recs = _recs(recs)
    k = recs.shape[1] if k is None else int(k)
    deg = test.degrees()
    eval_rows = torch.nonzero(deg > 0).flatten()
    # the non-empty rows ascending: their compacted row pointers are rowptr[eval_rows] + end
    pos = RowSets(torch.cat([test.rowptr[eval_rows], test.rowptr[-1:]]), test.col,
                  int(eval_rows.numel()), test.n_cols)
    hit = hit_flags(recs, eval_rows, pos).to(torch.float64)
    w = 1.0 / torch.log2(torch.arange(2, recs.shape[1] + 2, dtype=torch.float64,
                                      device=recs.device))
    n = hit.sum(1)
    idcg = float(w[:min(k, recs.shape[1])].sum())  # ones in the first min(len, k) slots
    return {"precision": float(n.mean()) / k, "recall": float((n / deg[eval_rows]).mean()),
            "ndcg": float(((hit * w).sum(1) / (idcg if idcg else 1.0)).mean()),
            "n_eval": int(eval_rows.numel())}


def pair_overlap(recs: torch.Tensor, n_items: int | None = None) -> int:
    """sum over ordered user pairs u != v of |set(R_u) & set(R_v)| (exact integer)."""
    recs = _recs(recs)
    if n_items is None:
        n_items = int(recs.max()) + 1 if recs.numel() else 0
    counts = torch.empty(max(1, n_items), dtype=torch.int32, device=recs.device)
    total = torch.zeros(1, dtype=torch.int64, device=recs.device)
    N.check(N.lib().lg_rec_pair_overlap(N.ptr(recs), recs.shape[0], recs.shape[1], n_items,
                                        N.ptr(counts), N.ptr(total),
                                        N.stream_handle(recs.device)), "lg_rec_pair_overlap")
    return int(total.item())


def hamming(recs: torch.Tensor, k: int, n_items: int | None = None) -> float:
    """calHammingDistance's mean over ordered user pairs of 1 - overlap / k (unrounded)."""
    U = recs.shape[0]
    pairs = U * (U - 1)
    s = pair_overlap(recs, n_items)
    return (pairs - s / k) / pairs  # ZeroDivisionError for one user, as the reference


def intra_similarity_parts(recs: torch.Tensor, by_item: RowSets,
                           item_degree: torch.Tensor) -> torch.Tensor:
    """fp64 [n_users * k]: per (user, position p) the sum over later positions of the
    item-pair similarity co(a, b) / sqrt(k_a k_b)."""
    recs = _recs(recs)
    item_degree = item_degree.to(recs.device, torch.int64).contiguous()
    if item_degree.numel() != by_item.n_rows:
        raise ValueError("item_degree must have one entry per item column")
    part = torch.empty(recs.numel(), dtype=torch.float64, device=recs.device)
    N.check(N.lib().lg_rec_intra_similarity_f64(
        N.ptr(recs), recs.shape[0], recs.shape[1], N.ptr(by_item.rowptr), N.ptr(by_item.col),
        N.ptr(item_degree), by_item.n_rows, N.ptr(part), N.stream_handle(recs.device)),
        "lg_rec_intra_similarity_f64")
    return part


def intra_similarity(recs: torch.Tensor, by_item: RowSets, item_degree: torch.Tensor,
                     k: int) -> float:
    """calInternalSimilarity (unrounded): every unordered pair counted twice, as the
    reference's ordered double loop does."""
    total = 2.0 * float(intra_similarity_parts(recs, by_item, item_degree).sum())
    return total / (recs.shape[0] * k * (k - 1))

