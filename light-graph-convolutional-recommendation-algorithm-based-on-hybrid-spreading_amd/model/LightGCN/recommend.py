"""LightGCN recommendation with the reference's interface
(reference model/LightGCN/recommend.py:22-159).

recommendForAllUser scores with the layer-0 embeddings, masks train and val positives with
-1024 and takes the top-k — in one HIP kernel (lg_score_topk_screened_f32: a bf16 MFMA
screen, the exact fp32 chain of lg_score_topk_f32 on the tiles it cannot rule out, the same
lists bit for bit) that never holds the U x I score matrix; ties are ordered (score desc,
item asc).
"""
import numpy as np
import pandas as pd
import torch

from const import cfg
from lgcnhs import ops
from lgcnhs.recs import exclusion_from_coo, gpu_device, save_recs, topk_to_dict
from utils.graph import convertEdgeIndexToAdjMatrix
from utils.log import logger
from utils.wrapper import calTimes


def _edge_index(df: pd.DataFrame) -> torch.Tensor:
    return torch.stack([torch.tensor(df["user_id"].values, dtype=torch.long),
                        torch.tensor(df["item_id"].values, dtype=torch.long)])


@calTimes(logger, "LightGCN图建立完成")
def buildGraph(user_num: int, item_num: int, rating_df: pd.DataFrame,
               train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
               test_data_df: pd.DataFrame) -> tuple:
    """-> (edge_index of all ratings [2, E], train/val/test symmetric COO adjacencies)
    (reference :22-66)."""
    edge_index = _edge_index(rating_df)
    return (edge_index,
            convertEdgeIndexToAdjMatrix(user_num, item_num, _edge_index(train_data_df)),
            convertEdgeIndexToAdjMatrix(user_num, item_num, _edge_index(val_data_df)),
            convertEdgeIndexToAdjMatrix(user_num, item_num, _edge_index(test_data_df)))


def topk_for_all_users(model, user_num: int, item_num: int, train_edge_index,
                       val_edge_index, k: int):
    """Device result of recommendForAllUser: (scores [U,k] fp32, items [U,k] int64)."""
    w_u = model.users_emb.weight.detach()
    dev = gpu_device(w_u)
    eu = w_u.to(dev, torch.float32).contiguous()
    ei = model.items_emb.weight.detach().to(dev, torch.float32).contiguous()
    excl = exclusion_from_coo(user_num, item_num, train_edge_index, val_edge_index, device=dev)
    return ops.score_topk(eu, ei, k, excl, mask_value=float(-(1 << 10)))


def recommendForAllUser(model, user_num: int, item_num: int,
                        train_edge_index: torch.Tensor, val_edge_index: torch.Tensor,
                        test_edge_index: torch.Tensor, k: int) -> dict:
    """{uid: top-k items} (reference :68-125)."""
    _, idx = topk_for_all_users(model, user_num, item_num, train_edge_index, val_edge_index, k)
    recs = topk_to_dict(idx)
    save_recs(recs, cfg.RECOMMEND["save_path"] + "all_user_recommend_dict_" + cfg.MODEL["name"]
              + "_" + str(cfg.RECOMMEND["k"]) + ".npy")
    return recs


def recommendLightGCN(user_num: int, item_num: int, rating_df: pd.DataFrame,
                      train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                      test_data_df: pd.DataFrame) -> dict:
    """Reference :127-159. A cached model is a state_dict loaded with weights_only=True
    (the reference's whole-model pickle cannot load on torch>=2.6)."""
    from model.LightGCN.model import LightGCN
    from model.LightGCN.train import trainLightGCN

    k = cfg.RECOMMEND["k"]
    edge_index, train_ei, val_ei, test_ei = buildGraph(user_num, item_num, rating_df,
                                                       train_data_df, val_data_df, test_data_df)
    path = cfg.MODEL["save_path"] + str(k) + "_LightGCN.pth"
    try:
        hp = cfg.MODEL["HyperParameter"]
        model = LightGCN(user_num, item_num, hp["embedding_dim"], hp["layers"])
        model.load_state_dict(torch.load(path, weights_only=True))
        model = model.to(gpu_device())
        logger.info("模型加载完毕")
    except Exception:
        logger.info("模型加载失败，正在重新训练模型")
        model = trainLightGCN(user_num, item_num, edge_index, train_ei, val_ei)
    return recommendForAllUser(model, user_num, item_num, train_ei, val_ei, test_ei, k)
