"""Lambda sweep of the LGCNHS recommendation with the reference's interface (reference
findLambda.py:25-138): for lambda = 0, 0.01, ..., 1 the SpreadLightGCNOpti lists (e0 score G
times the HybridS resource F, train|val dropped) are evaluated against the test split.

The reference recomputes HybridS, A @ W, G * F and a Python argsort per user for every
lambda (:93-114) on dense U x I / I x I fp64 matrices. Here the sweep runs fused on the GPU
(lgcnhs.ops.spread_lambda_sweep): general_W (dense path) or the W tiles and the score
bounds (tiled path) are built once and reused, and each lambda's lists equal
recommendSpreadLightGCNOpti's for that lambda bit for bit. Plots are not drawn; the metrics
table is written to the reference's lambda_evaluation_<k>.csv."""
from __future__ import annotations

import os

import numpy as np
import pandas as pd
import torch

from const import cfg
from lgcnhs import ops
from lgcnhs.recs import gpu_device
from metrics.accurate import getAccurateMetrics
from metrics.diversity import getDiversityMetrics
from utils.log import logger
from utils.trans import getItemDegreeByUserPosItemDict, getUserItemsDictByDataframe


def evaluation(test_user_pos_items_dict: dict, item_degree_dict: dict, interaction_mat,
               recommendations: torch.Tensor, k: int):
    """Reference :25-47: (precision, recall, f1, ndcg, H, I) of one set of lists.
    interaction_mat: the dense 0/1 matrix or the same interactions as a RowSets."""
    precision, recall, f1, ndcg = getAccurateMetrics(test_user_pos_items_dict,
                                                     recommendations, k)
    H, I = getDiversityMetrics(recommendations, item_degree_dict, interaction_mat, k)
    return precision, recall, f1, ndcg, H, I


def sweep_lambdas(model, user_num: int, item_num: int, train_data_df: pd.DataFrame,
                  val_data_df: pd.DataFrame, test_data_df: pd.DataFrame, k: int,
                  lambdas=None, tiled: bool | None = None) -> pd.DataFrame:
    """The loop of reference :87-114 for a trained (or given) LightGCN(Opti) model: one row of
    metrics per lambda (default 0..1 step 0.01, the reference's list)."""
    if lambdas is None:
        lambdas = np.arange(0, 1 + 0.01, 0.01).tolist()
    dev = gpu_device(model.users_emb.weight)
    both = pd.concat([train_data_df, val_data_df])
    A = ops.Interactions.from_pairs(torch.from_numpy(both["user_id"].to_numpy(np.int64)),
                                    torch.from_numpy(both["item_id"].to_numpy(np.int64)),
                                    user_num, item_num, dev)
    eu = model.users_emb.weight.detach().to(dev, torch.float32).contiguous()
    ei = model.items_emb.weight.detach().to(dev, torch.float32).contiguous()
    test_pos = getUserItemsDictByDataframe(test_data_df)
    deg = getItemDegreeByUserPosItemDict(getUserItemsDictByDataframe(train_data_df),
                                         getUserItemsDictByDataframe(val_data_df))
    rows = []
    for lam, _, idx in ops.spread_lambda_sweep(A, lambdas, k, A.by_user, True, eu, ei,
                                               tiled=tiled):
        p, r, f1, ndcg, H, I = evaluation(test_pos, deg, A.by_user, idx, k)
        rows.append({"lambda": lam, "precision": p, "recall": r, "f1": f1, "ndcg": ndcg,
                     "H": H, "I": I})
        logger.info(f"Lambda: {lam} 已评估完成")
    return pd.DataFrame(rows)


def findLambda(user_num: int, item_num: int, rating_df: pd.DataFrame,
               train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
               test_data_df: pd.DataFrame, user_features_df: pd.DataFrame,
               item_features_df: pd.DataFrame, lambdas=None) -> pd.DataFrame:
    """Reference :50-127 as a function: the LightGCNOpti model (loaded or trained as
    getAllocateMat does), the sweep, and the metrics CSV."""
    from model.SpreadLightGCNOpti.model import getLightGCNOptiModel
    k = cfg.RECOMMEND["k"]
    model = getLightGCNOptiModel(user_num, item_num, rating_df, train_data_df, val_data_df,
                                 test_data_df, user_features_df, item_features_df, k)[0]
    df = sweep_lambdas(model, user_num, item_num, train_data_df, val_data_df, test_data_df,
                       k, lambdas)
    out = cfg.EVALUATION["save_path"] + "lambda_evaluation_" + str(k) + ".csv"
    os.makedirs(os.path.dirname(out), exist_ok=True)
    df.to_csv(out, index=False)
    return df


if __name__ == "__main__":
    p = cfg.PREPROCESSING["save_path"]
    rating_df = pd.read_csv(p + "filter_rating.csv")
    findLambda(len(rating_df["user_id"].unique()), len(rating_df["item_id"].unique()), rating_df,
               pd.read_csv(p + "train_data.csv"), pd.read_csv(p + "val_data.csv"),
               pd.read_csv(p + "test_data.csv"),
               pd.read_csv(p + "user_features.csv", sep="\t"),
               pd.read_csv(p + "item_features.csv", sep="\t"))
