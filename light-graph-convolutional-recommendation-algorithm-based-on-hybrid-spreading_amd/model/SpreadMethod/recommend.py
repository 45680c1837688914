"""Spreading recommenders with the reference's interface
(reference model/SpreadMethod/recommend.py:18-115).

recommendSpreadMethod runs entirely on the GPU from the DataFrames: sparse A, general_W,
W (with the reference's per-method lambda / transpose overrides), then F = A @ W block by
block fused into the filtered top-k — F is never brought to the host. Ties are ordered
(value desc, item asc) where the reference's np.argsort leaves them unspecified.
"""
from collections import defaultdict

import numpy as np
import pandas as pd
import torch

from const import cfg
from lgcnhs import ops
from lgcnhs.recs import topk_to_dict, exclusion_from_dfs, gpu_device, save_recs


def _save(recs: dict) -> None:
    save_recs(recs, cfg.RECOMMEND["save_path"] + "all_user_recommend_dict_" + cfg.MODEL["name"]
              + "_" + str(cfg.RECOMMEND["k"]) + ".npy")


def _unfiltered() -> bool:
    # reference :49-50: movielens + ProbS returns sorted_items[:k] without the filter
    return cfg.DATA_SET == "movielens" and cfg.MODEL["name"] == "ProbS"


def _to_dict(idx: torch.Tensor, user_num: int) -> dict:
    return topk_to_dict(idx, user_num, defaultdict)


def recommendForAllUser(F_new: np.ndarray, user_num: int, train_data_df: pd.DataFrame,
                        val_data_df: pd.DataFrame, k: int) -> dict:
    """Per user: the k best items by F_new not in train|val (reference :18-56)."""
    dev = gpu_device()
    F = torch.as_tensor(np.ascontiguousarray(F_new[:user_num]), dtype=torch.float64).to(dev)
    excl = exclusion_from_dfs(user_num, F.shape[1], train_data_df, val_data_df, device=dev)
    _, idx = ops.rows_topk(F, k, excl, drop=not _unfiltered())
    recs = _to_dict(idx, user_num)
    _save(recs)
    return recs


def spread_method_topk(user_num: int, item_num: int, train_data_df: pd.DataFrame,
                       val_data_df: pd.DataFrame, method: str, lambda_val: float,
                       dataset: str, k: int, unfiltered: bool = False, device=None,
                       tiled: bool | None = None):
    """Device (values, items) of the whole spreading recommendation."""
    dev = device or gpu_device()
    both = pd.concat([train_data_df, val_data_df])
    inter = ops.Interactions.from_pairs(
        torch.from_numpy(both["user_id"].to_numpy(np.int64)),
        torch.from_numpy(both["item_id"].to_numpy(np.int64)), user_num, item_num, dev)
    transpose = False
    if method == "ProbS" and dataset == "movielens":  # reference :87-91
        lambda_val, transpose = 0.01, True
    elif method == "HeatS" and dataset == "douban":  # reference :97-101
        lambda_val, transpose = 0.99, True
    excl = inter.by_user  # train|val positives == the nonzeros of A
    # dense I x I general_W / W when they fit, else the factored tile path (same values within a few ulp)
    return ops.spread_recommend(inter, lambda_val, k, excl, drop=not unfiltered,
                                transpose=transpose, tiled=tiled)


def recommendSpreadMethod(user_num: int, item_num: int, train_data_df: pd.DataFrame,
                          val_data_df: pd.DataFrame, method: str,
                          lambda_val: float = 0) -> dict:
    """Reference :59-115 (lambda from cfg, as the reference reads it at :74)."""
    k = cfg.RECOMMEND["k"]
    lambda_val = cfg.MODEL["HyperParameter"]["lambda"]
    if method not in ["ProbS", "HeatS", "HybridS"]:
        raise ValueError(f"Invalid parameter: method={method}，必须为 ProbS | HeatS | HybridS")
    _, idx = spread_method_topk(user_num, item_num, train_data_df, val_data_df, method,
                                lambda_val, cfg.DATA_SET, k, unfiltered=_unfiltered())
    recs = _to_dict(idx, user_num)
    _save(recs)
    return recs
