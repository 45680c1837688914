"""LGCNHS-e recommendation with the reference's interface
(reference model/SpreadLightGCN/recommend.py:18-75).

recommendSpreadLightGCN runs fused on the GPU: F = A @ W per user block, multiplied by the
fp32 e0 score (promoted to fp64 as numpy's G * F does) inside the top-k kernel, train|val
items dropped. Neither G nor F is materialised for all users.
"""
from collections import defaultdict

import numpy as np
import pandas as pd
import torch

from const import cfg
from lgcnhs import ops
from lgcnhs.recs import topk_to_dict, exclusion_from_dfs, gpu_device, save_recs


def _to_dict(idx: torch.Tensor, user_num: int) -> dict:
    return topk_to_dict(idx, user_num, defaultdict)


def _save(recs: dict) -> None:
    save_recs(recs, cfg.RECOMMEND["save_path"] + "all_user_recommend_dict_" + cfg.MODEL["name"]
              + "_" + str(cfg.RECOMMEND["k"]) + ".npy")


def recommendForAllUser(F_new: np.ndarray, user_num: int, train_data_df: pd.DataFrame,
                        val_data_df: pd.DataFrame, k: int) -> dict:
    """Top-k by F_new without train|val items (reference :18-52)."""
    dev = gpu_device()
    F = torch.as_tensor(np.ascontiguousarray(F_new[:user_num]), dtype=torch.float64).to(dev)
    excl = exclusion_from_dfs(user_num, F.shape[1], train_data_df, val_data_df, device=dev)
    _, idx = ops.rows_topk(F, k, excl, drop=True)
    recs = _to_dict(idx, user_num)
    _save(recs)
    return recs


def spread_lightgcn_topk(model, user_num: int, item_num: int, train_data_df: pd.DataFrame,
                         val_data_df: pd.DataFrame, lambda_val: float, k: int, device=None,
                         tiled: bool | None = None):
    """Device (values fp64, items int64) of the whole LGCNHS recommendation."""
    dev = device or gpu_device(model.users_emb.weight)
    both = pd.concat([train_data_df, val_data_df])
    inter = ops.Interactions.from_pairs(
        torch.from_numpy(both["user_id"].to_numpy(np.int64)),
        torch.from_numpy(both["item_id"].to_numpy(np.int64)), user_num, item_num, dev)
    eu = model.users_emb.weight.detach().to(dev, torch.float32).contiguous()
    ei = model.items_emb.weight.detach().to(dev, torch.float32).contiguous()
    # dense I x I general_W / W when they fit, else the factored tile path (same values within a few ulp)
    return ops.spread_recommend(inter, lambda_val, k, inter.by_user, drop=True, eu=eu, ei=ei,
                                tiled=tiled)


def recommendSpreadLightGCN(user_num: int, item_num: int, rating_df: pd.DataFrame,
                            train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                            test_data_df: pd.DataFrame) -> dict:
    """Reference :55-75."""
    from model.SpreadLightGCN.model import getLightGCNModel

    k = cfg.RECOMMEND["k"]
    model = getLightGCNModel(user_num, item_num, rating_df, train_data_df, val_data_df,
                             test_data_df, k)[0]
    _, idx = spread_lightgcn_topk(model, user_num, item_num, train_data_df, val_data_df,
                                  cfg.MODEL["HyperParameter"]["lambda"], k)
    recs = _to_dict(idx, user_num)
    _save(recs)
    return recs
