"""Host-side glue shared by the recommend modules: exclusion sets in, dicts out.

Replaces the per-edge Python loops around the reference's top-k
(utils/trans.py:65-80 getUserItemsDictByEdgeIndex + the extend/index-put loops of
model/LightGCN/recommend.py:93-111; the dict building of :116-119 and of
model/SpreadMethod/recommend.py:33-47) with device CSR construction and one
device->host copy of the [U, k] index matrix.
"""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import torch

from .graph import RowSets


def gpu_device(*tensors) -> torch.device:
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
    if not torch.cuda.is_available():
        raise RuntimeError("lgcnhs: no GPU visible; the hot path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def interactions_from_coo(user_num: int, item_num: int, coo: torch.Tensor):
    """(users, items) of the user->item block of a symmetric COO (any device)."""
    coo = torch.as_tensor(coo)
    r, c = coo[0].to(torch.int64), coo[1].to(torch.int64)
    m = (r < user_num) & (c >= user_num)
    return r[m], c[m] - user_num


def exclusion_from_coo(user_num: int, item_num: int, *coos, device=None) -> RowSets:
    """Union of the user->item positives of symmetric COO adjacencies (train, val, ...)."""
    dev = device or gpu_device(*coos)
    us, its = [], []
    for coo in coos:
        u, i = interactions_from_coo(user_num, item_num, coo)
        us.append(u.to(dev))
        its.append(i.to(dev))
    return RowSets.from_pairs(torch.cat(us), torch.cat(its), user_num, item_num, dev)


def exclusion_from_dfs(user_num: int, item_num: int, *dfs: pd.DataFrame, device=None) -> RowSets:
    dev = device or gpu_device()
    df = pd.concat(dfs)
    u = torch.from_numpy(df["user_id"].to_numpy(np.int64))
    i = torch.from_numpy(df["item_id"].to_numpy(np.int64))
    return RowSets.from_pairs(u, i, user_num, item_num, dev)


def topk_to_dict(idx: torch.Tensor, n_rows: int | None = None, factory=dict) -> dict:
    """[U, k] indices (-1 = trailing padding) -> {uid: [item, ...]} with one device->host
    copy and one tolist(); only rows that are padded get trimmed (the
    reference builds these dicts per user and per item in Python)."""
    a = idx.cpu().numpy()
    if n_rows is not None:
        a = a[:n_rows]
    rows = a.tolist()
    if a.size:
        counts = (a >= 0).sum(1)
        for u in np.nonzero(counts < a.shape[1])[0].tolist():
            rows[u] = rows[u][:counts[u]]
    out = factory()
    out.update(enumerate(rows))
    return out


def save_recs(recs: dict, path: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.save(path, recs)
