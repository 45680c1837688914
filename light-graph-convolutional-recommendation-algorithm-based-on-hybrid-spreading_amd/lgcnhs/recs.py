"""Host-side glue shared by the recommend modules: exclusion sets in, dicts out.

Replaces the per-edge Python loops around the reference's top-k
(utils/trans.py:65-80 getUserItemsDictByEdgeIndex + the extend/index-put loops of
model/LightGCN/recommend.py:93-111; the dict building of :116-119 and of
model/SpreadMethod/recommend.py:33-47) with device CSR construction and one
device->host copy of the [U, k] index matrix.
"""
from __future__ import annotations

import os
import zipfile

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


def lists_path(path: str) -> str:
    """The pickle-free sidecar of a saved recommendation dict: '<name>.npy' ->
    '<name>.lists.npz'."""
    return (path[:-4] if path.endswith(".npy") else path) + ".lists.npz"


def save_recs(recs: dict, path: str) -> None:
    """The reference's format (np.save of the dict, read back by its evaluationMetrics.py with
    allow_pickle=True) plus a pickle-free sidecar (lists_path: uids + [U, k] int64 lists,
    -1 padded) that this package's main.py reads instead, so a cache file is never unpickled
    here."""
    os.makedirs(os.path.dirname(path), exist_ok=True)
    side = lists_path(path)
    if os.path.exists(side):  # (a failed write below never leaves an older run's lists)
        os.remove(side)
    np.save(path, recs)
    uids = np.fromiter(recs.keys(), dtype=np.int64, count=len(recs))
    width = max((len(v) for v in recs.values()), default=0)
    lists = np.full((len(recs), width), -1, dtype=np.int64)
    lens = np.zeros(len(recs), dtype=np.int64)
    for r, v in enumerate(recs.values()):
        lists[r, :len(v)] = v
        lens[r] = len(v)
    tmp = side + ".tmp.npz"  # (np.savez appends .npz to names without it)
    np.savez(tmp, uids=uids, lists=lists, lens=lens)
    os.replace(tmp, side)  # atomic: the sidecar exists only whole, and after its .npy


# what load_recs raises on a missing, truncated, corrupt or foreign cache file
CACHE_ERRORS = (OSError, ValueError, KeyError, EOFError, zipfile.BadZipFile)


def load_recs(path: str) -> dict:
    """The dict save_recs wrote, from its pickle-free sidecar only (allow_pickle=False).
    The '.npy' it is named after must exist and be no newer than the sidecar: deleting the
    '.npy' -- the reference's way to force a recompute -- invalidates the cache, and so does a
    '.npy' rewritten after it. Raises one of CACHE_ERRORS on a missing, stale, truncated,
    corrupt or foreign file."""
    side = lists_path(path)
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path}: no recommendation cache (its sidecar is ignored)")
    if os.path.getmtime(path) > os.path.getmtime(side):
        raise ValueError(f"{side}: older than {path} (stale sidecar)")
    with np.load(side, allow_pickle=False) as z:
        uids, lists, lens = z["uids"], z["lists"], z["lens"]
    if uids.ndim != 1 or lists.shape[0] != uids.shape[0] or lens.shape != uids.shape:
        raise ValueError(f"{lists_path(path)}: inconsistent recommendation lists")
    return {int(u): lists[r, :int(n)].tolist() for r, (u, n) in enumerate(zip(uids, lens))}
