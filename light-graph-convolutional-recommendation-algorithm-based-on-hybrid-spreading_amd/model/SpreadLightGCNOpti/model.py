"""LGCNHS (LightGCNOpti e0 scores x hybrid spreading) with the reference's interface
(reference model/SpreadLightGCNOpti/model.py:25-243)."""
import numpy as np
import pandas as pd

from const import cfg
from lgcnhs.features import features_tensor
from model.LightGCN.recommend import buildGraph
from model.LightGCNOpti.recommend import load_or_train_opti
from model.SpreadLightGCN.model import allocate_from_model, getHybridSResourceMat  # noqa: F401
from model.SpreadMethod.model import getSpreadingGeneralMat
from utils.log import logger
from utils.trans import getInteractionMatrixByDataframe
from utils.wrapper import calTimes


def getLightGCNOptiModel(user_num: int, item_num: int, rating_df: pd.DataFrame,
                         train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                         test_data_df: pd.DataFrame, user_features_df: pd.DataFrame,
                         item_features_df: pd.DataFrame, k: int) -> tuple:
    """Reference :25-94."""
    edge_index, train_ei, val_ei, test_ei = buildGraph(user_num, item_num, rating_df,
                                                       train_data_df, val_data_df, test_data_df)
    uf = features_tensor(user_features_df, "user_id", "user_features")
    itf = features_tensor(item_features_df, "item_id", "item_features")
    model = load_or_train_opti(user_num, item_num, edge_index, train_ei, val_ei, uf, itf, k)
    return model, edge_index, train_ei, val_ei, test_ei


@calTimes(logger, "分配权重矩阵计算完成")
def getAllocateMat(user_num: int, item_num: int, rating_df: pd.DataFrame,
                   train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                   test_data_df: pd.DataFrame, user_features_df: pd.DataFrame,
                   item_features_df: pd.DataFrame, k: int) -> np.ndarray:
    """Reference :97-169."""
    model, _, train_ei, val_ei, _ = getLightGCNOptiModel(
        user_num, item_num, rating_df, train_data_df, val_data_df, test_data_df,
        user_features_df, item_features_df, k)
    return allocate_from_model(model, user_num, item_num, train_ei, val_ei).cpu().numpy()


def getResourceMat(user_num: int, item_num: int, rating_df: pd.DataFrame,
                   train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                   test_data_df: pd.DataFrame, user_features_df: pd.DataFrame,
                   item_features_df: pd.DataFrame) -> np.ndarray:
    """F_new = G * F (reference :191-243)."""
    k = cfg.RECOMMEND["k"]
    G = getAllocateMat(user_num, item_num, rating_df, train_data_df, val_data_df,
                       test_data_df, user_features_df, item_features_df, k)
    A = getInteractionMatrixByDataframe(user_num, item_num,
                                        pd.concat([train_data_df, val_data_df]))
    F = getHybridSResourceMat(A, getSpreadingGeneralMat(A), cfg.MODEL["HyperParameter"]["lambda"])
    return G * F
