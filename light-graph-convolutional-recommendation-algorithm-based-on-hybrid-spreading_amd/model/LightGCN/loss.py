"""BPR loss and mini-batch sampling with the reference's interface
(reference model/LightGCN/loss.py:12-70), sampling on the device."""
import torch


def BPRLoss(users_emb_final, users_emb_0, pos_items_emb_final, pos_items_emb_0,
            neg_items_emb_final, neg_items_emb_0, lambda_val: float):
    """reg + bpr with the reference's sign: bpr = -mean(softplus(pos - neg))
    (reference :12-43)."""
    reg_loss = lambda_val * (users_emb_0.norm(2).pow(2) + pos_items_emb_0.norm(2).pow(2)
                             + neg_items_emb_0.norm(2).pow(2))
    pos_scores = torch.sum(users_emb_final * pos_items_emb_final, dim=-1)
    neg_scores = torch.sum(users_emb_final * neg_items_emb_final, dim=-1)
    return -torch.mean(torch.nn.functional.softplus(pos_scores - neg_scores)) + reg_loss


def _sorted_keys(u: torch.Tensor, p: torch.Tensor, num_items: int) -> torch.Tensor:
    keys = u * num_items + p
    if keys.numel() > 1 and not bool((keys[1:] >= keys[:-1]).all()):
        keys = torch.sort(keys).values   # edge lists from the CSR builders come sorted
    return keys


REJECTION_ROUNDS = 64


def _is_positive(u: torch.Tensor, items: torch.Tensor, keys: torch.Tensor, num_items: int):
    q = u * num_items + items
    if keys.numel() == 0:
        return torch.zeros_like(q, dtype=torch.bool)
    pos = torch.searchsorted(keys, q).clamp_max(keys.numel() - 1)
    return keys[pos] == q


def _exact_free_items(u: torch.Tensor, keys: torch.Tensor, num_items: int, generator=None):
    """For each entry of ``u``: a uniform draw from the items that are NOT positives of that
    user, by rank (the r-th free item, r uniform over the free count). Raises ValueError for
    a user who has interacted with every item (no valid negative exists)."""
    uu = u.to(keys.device)
    lo = torch.searchsorted(keys, uu * num_items)
    hi = torch.searchsorted(keys, (uu + 1) * num_items)
    n_pos = hi - lo
    free = num_items - n_pos
    if bool((free <= 0).any()):
        bad = int(uu[free <= 0][0])
        raise ValueError(f"user {bad} has interacted with every item: no negative to sample")
    r = (torch.rand(uu.shape, device=uu.device, generator=generator) * free).long()
    r = torch.minimum(r, free - 1)
    # The r-th free item is r + j, j = the number of the user's positives p_i (ascending,
    # i = 0, 1, ...) with p_i - i <= r (p_i - i = the free items below p_i, non-decreasing
    # in i). All entries at once on the device: their positives gathered as segments, the
    # count by one searchsorted over (entry, p_i - i) keys (two host syncs in all).
    n = uu.numel()
    total = int(n_pos.sum())
    excl = torch.cumsum(n_pos, 0) - n_pos
    seg = torch.repeat_interleave(torch.arange(n, device=uu.device), n_pos)
    offs = torch.arange(total, device=uu.device) - excl[seg]
    g = keys[lo[seg] + offs] - uu[seg] * num_items - offs
    skey = seg * (num_items + 1) + g
    j = torch.searchsorted(skey, torch.arange(n, device=uu.device) * (num_items + 1) + r,
                           right=True) - excl
    return (r + j).to(device=u.device, dtype=torch.int64)


def _negatives(u: torch.Tensor, keys: torch.Tensor, num_items: int, generator=None):
    """One uniform item per entry of ``u`` that is not a positive of that user: rejection
    against the sorted (user, item) keys on the device; entries still rejected after
    REJECTION_ROUNDS rounds (users with few free items) are drawn exactly from their
    complement, so a positive is never returned as a negative."""
    neg = torch.randint(0, num_items, u.shape, device=u.device, generator=generator)
    bad = _is_positive(u, neg, keys, num_items)
    for _ in range(REJECTION_ROUNDS):
        if not bool(bad.any()):
            return neg
        neg = torch.where(bad, torch.randint(0, num_items, u.shape, device=u.device,
                                             generator=generator), neg)
        bad = _is_positive(u, neg, keys, num_items)
    if bool(bad.any()):
        idx = torch.nonzero(bad).flatten()
        neg = neg.clone()
        neg[idx] = _exact_free_items(u[idx], keys, num_items, generator)
    return neg


def structured_negative_sampling(edge_index: torch.Tensor, num_items: int, generator=None):
    """(users, pos, neg) with neg uniform over items and (user, neg) not an edge
    (PyG structured_negative_sampling semantics, rejection on the device; negatives are
    drawn from the item range)."""
    u, p = edge_index[0].long(), edge_index[1].long()
    return u, p, _negatives(u, _sorted_keys(u, p, num_items), num_items, generator)


def sampleMiniBatch(batch_size: int, edge_index: torch.Tensor, num_items: int = None,
                    generator=None):
    """Reference :46-70: negative-sample every edge, then draw batch_size edges with
    replacement. Each drawn edge's negative is an independent uniform non-positive item
    either way, so only the drawn edges are negative-sampled: the same distribution of
    (user, pos, neg) triples at O(batch_size) instead of O(edges) sampling work. (Joint
    difference: an edge drawn twice in one batch gets two independent negatives here, one
    shared negative in the reference.)"""
    if num_items is None:
        num_items = int(edge_index[1].max()) + 1
    u, p = edge_index[0].long(), edge_index[1].long()
    keys = _sorted_keys(u, p, num_items)
    idx = torch.randint(0, u.numel(), (batch_size,), device=u.device, generator=generator)
    bu, bp = u[idx], p[idx]
    return bu, bp, _negatives(bu, keys, num_items, generator)
