"""Diversity metrics with the reference's interface (reference metrics/diversity.py:15-135).

calHammingDistance: the reference's O(users^2) pair loop is replaced by its exact closed
form, sum_{u != v} |R_u & R_v| = sum_i c_i (c_i - 1) over per-item list counts
(lg_rec_pair_overlap, integer arithmetic). calInternalSimilarity: the per-user item-pair
co-occurrences run on the GPU (lg_rec_intra_similarity_f64) with the reference's per-term
arithmetic; only the summation order differs (fp64, within rounding; results are rounded to
5 decimals as in the reference).
"""
import numpy as np
import torch

from lgcnhs import metrics as M
from lgcnhs.graph import RowSets
from lgcnhs.recs import gpu_device


def calHammingDistance(recommendations: torch.Tensor, k: int) -> float:
    """Reference :15-63."""
    recs = torch.as_tensor(recommendations)
    user_num = recs.shape[0]
    if user_num * (user_num - 1) == 0:
        raise ZeroDivisionError("float division by zero")
    H = round(M.hamming(recs.to(gpu_device(recs)), k), 5)
    return round(H, 5)


def calInternalSimilarity(recommendations: torch.Tensor, item_degree_dict: dict,
                          interaction_mat: np.ndarray, k: int) -> float:
    """Reference :66-115. interaction_mat is the binary user x item matrix of
    getInteractionMatrixByDataframe (its column dot products are co-occurrence counts), or
    the same interactions as a user-major lgcnhs RowSets (the training loop's form: no
    dense U x I matrix)."""
    recs = torch.as_tensor(recommendations)
    dev = gpu_device(recs)
    if isinstance(interaction_mat, RowSets):
        n_items = interaction_mat.n_cols
        by_item = interaction_mat.transpose()
        A = None
    else:
        A = np.asarray(interaction_mat)
        n_items = A.shape[1]
        if not np.all((A == 0) | (A == 1)):
            raise ValueError("calInternalSimilarity: interaction_mat must be 0/1")
    deg = np.zeros(n_items, np.int64)
    outside = set()
    for it, d in item_degree_dict.items():
        if 0 <= int(it) < n_items:
            deg[int(it)] = int(d)
        elif d:
            outside.add(int(it))
    if outside and np.isin(recs.cpu().numpy(), list(outside)).any():
        raise IndexError("recommended item with a degree lies outside interaction_mat")
    if A is not None:
        users, items = np.nonzero(A)
        by_item = RowSets.from_pairs(torch.from_numpy(items), torch.from_numpy(users),
                                     n_items, A.shape[0], dev)
    user_num = recs.shape[0]
    if user_num * k * (k - 1) == 0:
        raise ZeroDivisionError("float division by zero")
    I = M.intra_similarity(recs.to(dev), by_item, torch.from_numpy(deg), k)
    return round(I, 5)


def getDiversityMetrics(recommendations: torch.Tensor, item_degree_dict: dict,
                        interaction_mat: np.ndarray, k: int) -> tuple:
    """Reference :117-135."""
    H = calHammingDistance(recommendations, k)
    I = calInternalSimilarity(recommendations, item_degree_dict, interaction_mat, k)
    return H, I
