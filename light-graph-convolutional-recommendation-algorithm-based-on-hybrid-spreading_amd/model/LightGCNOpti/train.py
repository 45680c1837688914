"""LightGCNOpti training (reference model/LightGCNOpti/train.py:62-230)."""
import torch

from const import cfg
from model.LightGCN.train import getEmbeddingForBPR, train_model  # noqa: F401
from utils.log import logger
from utils.wrapper import calTimes


@calTimes(logger, "模型训练完成")
def trainLightGCNOpti(user_num: int, item_num: int, edge_index, train_edge_index,
                      val_edge_index, user_features, item_features):
    from model.LightGCNOpti.model import LightGCNOpti
    hp = cfg.MODEL["HyperParameter"]
    torch.manual_seed(hp["seed"])
    model = LightGCNOpti(user_num, item_num, hp["embedding_dim"], hp["layers"],
                         user_features, item_features)
    return train_model(model, user_num, item_num, train_edge_index, val_edge_index,
                       "LightGCNOpti")
