"""Accuracy metrics with the reference's interface (reference metrics/accurate.py:11-124).

The per-entry test-set membership (the reference's `item in items` over Python lists, the
whole cost of these functions) runs on the GPU (lg_rec_hits via lgcnhs.metrics.hit_flags);
the O(users x k) reductions that follow are the reference's own float32 torch ops on the
0/1 label matrix, so P / R / NDCG come out as the reference computes them.
"""
import numpy as np
import torch

from lgcnhs import metrics as M
from lgcnhs.graph import RowSets
from lgcnhs.recs import gpu_device


def _labels(user_pos_items_dict: dict, recommendations: torch.Tensor):
    """(float32 [n_eval, len] 0/1 labels on the host, float32 [n_eval] positive counts) for
    the users of the dict, in its iteration order (reference :24-37, :69-76)."""
    recs = torch.as_tensor(recommendations)
    dev = gpu_device(recs)
    uids = np.fromiter((int(u) for u in user_pos_items_dict.keys()), np.int64,
                       len(user_pos_items_dict))
    lists = [np.asarray(list(v), np.int64).reshape(-1) for v in user_pos_items_dict.values()]
    lens = np.array([len(v) for v in user_pos_items_dict.values()], np.float64)
    if uids.size == 0:
        return torch.Tensor(np.array([]).astype("float")), torch.Tensor(lens)
    if uids.min() < -recs.shape[0] or uids.max() >= recs.shape[0]:
        raise IndexError("user id outside the recommendation matrix")
    uids = uids % recs.shape[0]  # python indexing of recommendations[uid]
    cols = np.concatenate(lists) if lists else np.zeros(0, np.int64)
    rows = np.repeat(np.arange(uids.size), [v.size for v in lists])
    n_cols = int(max(cols.max() + 1 if cols.size else 1,
                     int(recs.max()) + 1 if recs.numel() else 1))
    keep = cols >= 0  # a negative test id never matches a recommended id
    pos = RowSets.from_pairs(torch.from_numpy(rows[keep]), torch.from_numpy(cols[keep]),
                             uids.size, n_cols, dev)
    hit = M.hit_flags(recs.to(dev), torch.from_numpy(uids), pos)
    return hit.cpu().float(), torch.Tensor(lens)


def calPrecisionAndRecall(user_pos_items_dict: dict, recommendations: torch.Tensor,
                          k: int) -> tuple:
    """Reference :11-46."""
    recommend_interaction_list, user_num_liked_list = _labels(user_pos_items_dict,
                                                              recommendations)
    num_correct_pred = torch.sum(recommend_interaction_list, dim=-1)
    precision = torch.mean(num_correct_pred) / k
    recall = torch.mean(num_correct_pred / user_num_liked_list)
    return round(precision.item(), 5), round(recall.item(), 5)


def calF1Score(precision: float, recall: float) -> float:
    """Reference :48-56 (ZeroDivisionError when both are 0, as there)."""
    f1 = 2 * (precision * recall) / (precision + recall)
    return round(f1, 5)


def calNDCG(user_pos_items_dict: dict, recommendations: torch.Tensor, k: int) -> float:
    """Reference :58-102, including its ideal DCG of min(len, k) ones per user."""
    recommend_interaction_list, _ = _labels(user_pos_items_dict, recommendations)
    tmp_matrix = torch.zeros((len(recommend_interaction_list), k))
    if recommend_interaction_list.dim() == 2:
        tmp_matrix[:, :min(recommend_interaction_list.shape[1], k)] = 1
    max_r = tmp_matrix
    idcg = torch.sum(max_r * 1. / torch.log2(torch.arange(2, k + 2)), axis=1)
    dcg = recommend_interaction_list * (1. / torch.log2(torch.arange(2, k + 2)))
    dcg = torch.sum(dcg, axis=1)
    idcg[idcg == 0.] = 1.
    ndcg = dcg / idcg
    ndcg[torch.isnan(ndcg)] = 0.
    ndcg = torch.mean(ndcg)
    return round(ndcg.item(), 5)


def getAccurateMetrics(user_pos_items_dict: dict, recommendations: torch.Tensor,
                       k: int) -> tuple:
    """Reference :104-124."""
    precision, recall = calPrecisionAndRecall(user_pos_items_dict, recommendations, k)
    f1 = calF1Score(precision, recall)
    ndcg = calNDCG(user_pos_items_dict, recommendations, k)
    return precision, recall, f1, ndcg
