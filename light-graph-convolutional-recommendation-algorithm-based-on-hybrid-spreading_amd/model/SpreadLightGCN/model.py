"""LGCNHS-e (LightGCN e0 scores x hybrid spreading) with the reference's interface
(reference model/SpreadLightGCN/model.py:24-153).

getAllocateMat / getHybridSResourceMat / getResourceMat keep their dense numpy returns
(findLambda.py calls them directly); G comes from lg_score_dense_f32, F from the sparse
spreading kernels. The fused end-to-end path (never materialising G, W-rows of F or F on
the host) is model.SpreadLightGCN.recommend.spread_lightgcn_topk.
"""
import numpy as np
import pandas as pd
import torch

from const import cfg
from lgcnhs import ops
from lgcnhs.recs import exclusion_from_coo, gpu_device
from model.LightGCN.recommend import buildGraph
from model.SpreadMethod.model import getResource, getSpreadingGeneralMat, HybridS
from utils.log import logger
from utils.trans import getInteractionMatrixByDataframe
from utils.wrapper import calTimes


def getLightGCNModel(user_num: int, item_num: int, rating_df: pd.DataFrame,
                     train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                     test_data_df: pd.DataFrame, k: int) -> tuple:
    """-> (model, edge_index, train/val/test adjacencies) (reference :24-53)."""
    from model.LightGCN.model import LightGCN
    from model.LightGCN.train import trainLightGCN

    edge_index, train_ei, val_ei, test_ei = buildGraph(user_num, item_num, rating_df,
                                                       train_data_df, val_data_df, test_data_df)
    try:
        hp = cfg.MODEL["HyperParameter"]
        model = LightGCN(user_num, item_num, hp["embedding_dim"], hp["layers"])
        model.load_state_dict(torch.load(cfg.MODEL["save_path"] + str(k) + "_LightGCN.pth",
                                         weights_only=True))
        model = model.to(gpu_device())
        logger.info("LightGCN模型加载完毕")
    except Exception:
        logger.info("LightGCN模型加载失败，正在重新训练模型")
        model = trainLightGCN(user_num, item_num, edge_index, train_ei, val_ei)
    return model, edge_index, train_ei, val_ei, test_ei


def allocate_from_model(model, user_num: int, item_num: int, train_edge_index,
                        val_edge_index) -> torch.Tensor:
    """G on the device: e0 scores with train|val positives set to -1024."""
    dev = gpu_device(model.users_emb.weight)
    eu = model.users_emb.weight.detach().to(dev, torch.float32).contiguous()
    ei = model.items_emb.weight.detach().to(dev, torch.float32).contiguous()
    excl = exclusion_from_coo(user_num, item_num, train_edge_index, val_edge_index, device=dev)
    return ops.score_dense(eu, ei, excl, float(-(1 << 10)))


@calTimes(logger, "分配权重矩阵计算完成")
def getAllocateMat(user_num: int, item_num: int, rating_df: pd.DataFrame,
                   train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                   test_data_df: pd.DataFrame, k: int) -> np.ndarray:
    """Masked e0 score matrix G, fp32 numpy [U, I] (reference :55-104)."""
    model, _, train_ei, val_ei, _ = getLightGCNModel(user_num, item_num, rating_df,
                                                     train_data_df, val_data_df,
                                                     test_data_df, k)
    return allocate_from_model(model, user_num, item_num, train_ei, val_ei).cpu().numpy()


@calTimes(logger, "资源扩散矩阵计算完成")
def getHybridSResourceMat(A: np.ndarray, general_W: np.ndarray, lambad_val: float) -> np.ndarray:
    """F = A @ HybridS(A, general_W, lambda) (reference :106-120)."""
    return getResource(A, HybridS(A, general_W, lambad_val))


def getResourceMat(user_num: int, item_num: int, rating_df: pd.DataFrame,
                   train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                   test_data_df: pd.DataFrame) -> np.ndarray:
    """F_new = G * F, fp64 [U, I] (reference :122-153)."""
    k = cfg.RECOMMEND["k"]
    lambda_val = cfg.MODEL["HyperParameter"]["lambda"]
    G = getAllocateMat(user_num, item_num, rating_df, train_data_df, val_data_df,
                       test_data_df, k)
    A = getInteractionMatrixByDataframe(user_num, item_num,
                                        pd.concat([train_data_df, val_data_df]))
    general_W = getSpreadingGeneralMat(A)
    F = getHybridSResourceMat(A, general_W, lambda_val)
    return G * F
