"""Synthetic bipartite interaction data (SURVEY.md §8d "Synthetic inputs").

The reference's datasets (MovieLens-100K, Douban) are not in the image, so every parity
case and benchmark runs on synthetic graphs of the configs' shapes:

* ``uniform``: users and items uniform, duplicates removed, topped up to exactly E;
* ``zipf``: item popularity Zipf(s) truncated to I (rank r has weight r^-s), users uniform.

Every user and every item appears at least once, so ``len(rating_df.user_id.unique())``
equals U as the reference's ``main.py:48-50`` computes it. The 80/10/10 split is by a
seeded permutation of the interaction index, as ``processing/handleData.py:86-99`` splits
by index (sklearn's ``train_test_split`` is not reproduced bit for bit; the fixtures store
the split itself).
"""
from __future__ import annotations

import numpy as np


def _unique_keys(keys: np.ndarray) -> np.ndarray:
    return np.unique(keys)


def synth_interactions(n_users: int, n_items: int, n_edges: int, seed: int = 0,
                       dist: str = "uniform", zipf_s: float = 1.1):
    """Return (users, items) int64 arrays of exactly ``n_edges`` unique pairs, sorted by
    (user, item)."""
    U, I, E = int(n_users), int(n_items), int(n_edges)
    if E < max(U, I) or E > U * I:
        raise ValueError(f"need max(U,I) <= E <= U*I, got U={U} I={I} E={E}")
    rng = np.random.default_rng(seed)
    if dist == "zipf":
        w = np.arange(1, I + 1, dtype=np.float64) ** (-zipf_s)
        p = w / w.sum()

        def draw_items(n):
            return rng.choice(I, size=n, p=p)
    elif dist == "uniform":
        def draw_items(n):
            return rng.integers(0, I, size=n, dtype=np.int64)
    else:
        raise ValueError(f"unknown dist {dist!r}")
    # coverage: every user and every item at least once
    cov = np.concatenate([
        np.arange(U, dtype=np.int64) * I + draw_items(U),
        rng.integers(0, U, size=I, dtype=np.int64) * I + np.arange(I, dtype=np.int64),
    ])
    cov = _unique_keys(cov)
    if cov.size > E:
        raise ValueError("E too small for full user/item coverage")
    keys = cov
    while keys.size < E:
        need = E - keys.size
        n = int(need * 1.05) + 64
        extra = rng.integers(0, U, size=n, dtype=np.int64) * I + draw_items(n)
        keys = _unique_keys(np.concatenate([keys, extra]))
    if keys.size > E:
        rest = np.setdiff1d(keys, cov, assume_unique=True)
        pick = rng.choice(rest.size, size=E - cov.size, replace=False)
        keys = np.sort(np.concatenate([cov, rest[pick]]))
    return keys // I, keys % I


def synth_graph_device(n_users: int, n_items: int, n_edges: int, seed: int, device,
                       dist: str = "uniform", zipf_s: float = 1.1):
    """Exactly n_edges unique (user, item) pairs drawn on the device (the C4/C5 scale, where
    numpy's unique over 10^8 keys is too slow): users uniform; items uniform, or with
    ``dist="zipf"`` Zipf(zipf_s) popularity (rank r drawn with weight r^-s by inverse-CDF
    sampling; ranks mapped to a seeded random permutation of the item ids, so the hubs are
    spread over the id range as in real catalogs). A popular item saturates at n_users
    interactions (pairs are unique), so the draws are topped up until E pairs exist.
    Returns the symmetric CSR over U+I nodes (rowptr int64, src int32; users then items, each
    row ascending) and the sorted interaction keys user * I + item (int64)."""
    import torch

    from .graph import _rowptr_from_sorted
    U, I, E = int(n_users), int(n_items), int(n_edges)
    if E > U * I:
        raise ValueError(f"E={E} > U*I")
    g = torch.Generator(device=device).manual_seed(seed)
    if dist == "zipf":
        cdf = torch.cumsum(torch.arange(1, I + 1, dtype=torch.float64, device=device)
                           .pow(-float(zipf_s)), 0)
        cdf /= cdf[-1].clone()
        perm = torch.randperm(I, device=device, generator=g)

        def draw_items(n):
            r = torch.searchsorted(cdf, torch.rand(n, dtype=torch.float64, device=device,
                                                   generator=g))
            return perm[r.clamp_(max=I - 1)]
    elif dist == "uniform":
        def draw_items(n):
            return torch.randint(0, I, (n,), device=device, generator=g)
    else:
        raise ValueError(f"unknown dist {dist!r}")
    keys = torch.empty(0, dtype=torch.int64, device=device)
    over = 1.02  # draws per missing pair, re-estimated from each round's yield
    while keys.numel() < E:
        have = keys.numel()
        n = int((E - have) * over) + 1024
        u = torch.randint(0, U, (n,), device=device, generator=g)
        keys = torch.unique(torch.cat([keys, u * I + draw_items(n)]))
        del u
        gained = keys.numel() - have
        over = min(8.0, max(1.02, 1.05 * n / max(gained, 1)))
    if keys.numel() > E:
        pick = torch.randperm(keys.numel(), device=device, generator=g)[:E]
        keys = torch.sort(keys[pick]).values
    users = keys // I
    items = keys % I
    ikeys = torch.sort(items * U + users).values
    rows = torch.cat([users, (ikeys // U) + U])          # users then items: sorted
    src = torch.cat([items + U, ikeys % U]).to(torch.int32)
    del ikeys, items
    rowptr = _rowptr_from_sorted(rows, U + I)
    return rowptr, src, keys


def split_indices(n: int, seed: int = 42, fractions=(0.8, 0.1, 0.1)):
    """Seeded 80/10/10 split of interaction indices (train, val, test)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n)
    n_tr = int(round(n * fractions[0]))
    n_va = int(round(n * fractions[1]))
    return np.sort(perm[:n_tr]), np.sort(perm[n_tr:n_tr + n_va]), np.sort(perm[n_tr + n_va:])


def synth_dataframes(n_users: int, n_items: int, n_edges: int, seed: int = 0,
                     dist: str = "uniform"):
    """(rating_df, train_df, val_df, test_df) with the reference's column names."""
    import pandas as pd

    users, items = synth_interactions(n_users, n_items, n_edges, seed=seed, dist=dist)
    rng = np.random.default_rng(seed + 1)
    rating_df = pd.DataFrame({
        "user_id": users,
        "item_id": items,
        "rating": rng.integers(1, 6, size=users.size),
        "rating_time": rng.integers(874724710, 893286638, size=users.size),
    })
    tr, va, te = split_indices(users.size, seed=42)
    return rating_df, rating_df.loc[tr], rating_df.loc[va], rating_df.loc[te]
