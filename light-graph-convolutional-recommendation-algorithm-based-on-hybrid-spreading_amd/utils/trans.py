"""Conversions between DataFrames, edge lists, dicts and the interaction matrix, with the
reference's signatures and results (reference utils/trans.py:13-115), vectorised.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import pandas as pd
import torch


def _df_pairs(data_df: pd.DataFrame):
    return (data_df["user_id"].to_numpy(np.int64), data_df["item_id"].to_numpy(np.int64))


def getInteractionMatrixByDataframe(user_num: int, item_num: int,
                                    data_df: pd.DataFrame) -> np.ndarray:
    """Dense fp64 A with A[u, i] = 1 (reference utils/trans.py:13-29)."""
    A = np.zeros((user_num, item_num))
    u, i = _df_pairs(data_df)
    A[u, i] = 1
    return A


def getInteractionMatrixByEdgeIndex(user_num: int, item_num: int,
                                    edge_index: torch.Tensor) -> np.ndarray:
    """Reference utils/trans.py:31-49."""
    A = np.zeros((user_num, item_num))
    ei = torch.as_tensor(edge_index).cpu().numpy().astype(np.int64)
    A[ei[0], ei[1]] = 1
    return A


def getUserItemsDictByDataframe(data_df: pd.DataFrame) -> dict:
    """user -> list of items in row order (reference utils/trans.py:51-63)."""
    d = defaultdict(list)
    u, i = _df_pairs(data_df)
    for uu, ii in zip(u.tolist(), i.tolist()):
        d[uu].append(ii)
    return d


def getUserItemsDictByEdgeIndex(edge_index: torch.Tensor) -> dict:
    """Reference utils/trans.py:65-80."""
    ei = torch.as_tensor(edge_index).cpu().numpy()
    d = {}
    for uu, ii in zip(ei[0].tolist(), ei[1].tolist()):
        d.setdefault(uu, []).append(ii)
    return d


def recommendDictToTensor(recommend_dict: dict) -> torch.Tensor:
    """Reference utils/trans.py:82-92."""
    rows = [recommend_dict[uid] for uid in sorted(recommend_dict.keys())]
    return torch.tensor(np.array(rows))


def getItemDegreeByUserPosItemDict(*user_pos_items_dict_list: dict) -> dict:
    """Reference utils/trans.py:94-115."""
    deg = {}
    for d in user_pos_items_dict_list:
        for items in d.values():
            for it in items:
                deg[it] = deg.get(it, 0) + 1
    return deg
