"""LightGCN training with the reference's interface (reference model/LightGCN/train.py:
26-223): Adam + ExponentialLR, BPR on mini-batches of structured negative samples, the
forward/backward through the HIP propagation. Plots and metric CSVs are not produced;
the model is saved as a state_dict (loadable with weights_only=True)."""
import os

import torch

from const import cfg
from lgcnhs.recs import gpu_device
from model.LightGCN.loss import BPRLoss, sampleMiniBatch
from utils.graph import convertAdjMatrixToEdgeIndex
from utils.log import logger
from utils.wrapper import calTimes


def getEmbeddingForBPR(model, user_num: int, item_num: int, train_edge_index,
                       batch_size: int, device, r_edge_index=None) -> tuple:
    """Reference :26-59."""
    users_final, users_0, items_final, items_0 = model.forward(train_edge_index)
    if r_edge_index is None:
        r_edge_index = convertAdjMatrixToEdgeIndex(user_num, item_num, train_edge_index)
    u, p, n = sampleMiniBatch(batch_size, r_edge_index.to(device), item_num)
    return (users_final[u], users_0[u], items_final[p], items_0[p], items_final[n], items_0[n])


def train_model(model, user_num: int, item_num: int, train_edge_index, val_edge_index,
                name: str):
    hp = cfg.MODEL["HyperParameter"]
    device = gpu_device()
    model = model.to(device)
    train_edge_index = train_edge_index.to(device)
    r_train = convertAdjMatrixToEdgeIndex(user_num, item_num, train_edge_index).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=hp["lr"])
    sched = torch.optim.lr_scheduler.ExponentialLR(opt, gamma=hp["gamma"])
    model.train()
    for epoch in range(hp["epochs"]):
        batch = getEmbeddingForBPR(model, user_num, item_num, train_edge_index,
                                   hp["batch_size"], device, r_train)
        loss = BPRLoss(*batch, hp["epsilon"])
        opt.zero_grad()
        loss.backward()
        opt.step()
        if epoch % hp["epoch_per_eval"] == 0:
            logger.info(f"[Iteration {epoch}/{hp['epochs']}] train_loss: {round(loss.item(), 5)}")
        if epoch % hp["epoch_per_lr_decay"] == 0 and epoch != 0:
            sched.step()
    path = cfg.MODEL["save_path"] + str(cfg.RECOMMEND["k"]) + f"_{name}.pth"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save(model.state_dict(), path)
    return model


@calTimes(logger, "模型训练完成")
def trainLightGCN(user_num: int, item_num: int, edge_index, train_edge_index,
                  val_edge_index):
    """Reference :61-223."""
    from model.LightGCN.model import LightGCN
    hp = cfg.MODEL["HyperParameter"]
    torch.manual_seed(hp["seed"])
    model = LightGCN(user_num, item_num, hp["embedding_dim"], hp["layers"])
    return train_model(model, user_num, item_num, train_edge_index, val_edge_index, "LightGCN")
