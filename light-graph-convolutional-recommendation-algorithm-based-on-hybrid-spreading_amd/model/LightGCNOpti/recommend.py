"""LightGCNOpti recommendation with the reference's interface
(reference model/LightGCNOpti/recommend.py:22-177); scoring as model.LightGCN.recommend."""
import pandas as pd
import torch

from const import cfg
from lgcnhs.features import features_tensor
from lgcnhs.recs import gpu_device, save_recs, topk_to_dict
from model.LightGCN.recommend import buildGraph, topk_for_all_users  # noqa: F401
from utils.log import logger


def recommendForAllUser(model, user_num: int, item_num: int, train_edge_index,
                        val_edge_index, test_edge_index, k: int) -> dict:
    """Reference :68-125 (its save name has no '_' before k: :122)."""
    _, idx = topk_for_all_users(model, user_num, item_num, train_edge_index, val_edge_index, k)
    recs = topk_to_dict(idx)
    save_recs(recs, cfg.RECOMMEND["save_path"] + "all_user_recommend_dict_" + cfg.MODEL["name"]
              + str(cfg.RECOMMEND["k"]) + ".npy")
    return recs


def load_or_train_opti(user_num, item_num, edge_index, train_ei, val_ei, user_features,
                       item_features, k):
    from model.LightGCNOpti.model import LightGCNOpti
    from model.LightGCNOpti.train import trainLightGCNOpti
    try:
        hp = cfg.MODEL["HyperParameter"]
        model = LightGCNOpti(user_num, item_num, hp["embedding_dim"], hp["layers"],
                             user_features, item_features)
        model.load_state_dict(torch.load(cfg.MODEL["save_path"] + str(k) + "_LightGCNOpti.pth",
                                         weights_only=True))
        model = model.to(gpu_device())
        logger.info("LightGCNOpti模型加载完毕")
    except Exception:
        logger.info("LightGCNOpti模型加载失败，正在重新训练模型")
        model = trainLightGCNOpti(user_num, item_num, edge_index, train_ei, val_ei,
                                  user_features, item_features)
    return model


def recommendLightGCNOpti(user_num: int, item_num: int, rating_df: pd.DataFrame,
                          train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                          test_data_df: pd.DataFrame, user_features_df: pd.DataFrame,
                          item_features_df: pd.DataFrame) -> dict:
    """Reference :127-177."""
    k = cfg.RECOMMEND["k"]
    edge_index, train_ei, val_ei, test_ei = buildGraph(user_num, item_num, rating_df,
                                                       train_data_df, val_data_df, test_data_df)
    uf = features_tensor(user_features_df, "user_id", "user_features")
    itf = features_tensor(item_features_df, "item_id", "item_features")
    model = load_or_train_opti(user_num, item_num, edge_index, train_ei, val_ei, uf, itf, k)
    return recommendForAllUser(model, user_num, item_num, train_ei, val_ei, test_ei, k)
