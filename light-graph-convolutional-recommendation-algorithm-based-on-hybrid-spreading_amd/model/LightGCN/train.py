"""LightGCN training with the reference's interface (reference model/LightGCN/train.py:
26-223): Adam + ExponentialLR, BPR on mini-batches of structured negative samples, the
forward/backward through the HIP propagation, and every ``epoch_per_eval`` epochs the
reference's validation block (:147-180): val loss on the val adjacency, train-masked top-k
(model/LightGCN/evaluation.py), P/R/F1/NDCG against the val positives and H/I diversity.
The per-eval metrics are written to the reference's ``<k>_val_metrics.csv`` and drawn as its
curves (:205-221, utils.picture.plotMetric); the model is saved as a state_dict (loadable with
weights_only=True)."""
import os

import pandas as pd
import torch

from const import cfg
from lgcnhs.graph import RowSets
from lgcnhs.recs import gpu_device
from metrics.accurate import getAccurateMetrics
from metrics.diversity import getDiversityMetrics
from model.LightGCN.evaluation import calValLoss, getValRecommendations
from model.LightGCN.loss import BPRLoss, sampleMiniBatch
from utils.graph import convertAdjMatrixToEdgeIndex
from utils.log import logger
from utils.trans import getItemDegreeByUserPosItemDict, getUserItemsDictByEdgeIndex
from utils.wrapper import calTimes


def getEmbeddingForBPR(model, user_num: int, item_num: int, train_edge_index,
                       batch_size: int, device, r_edge_index=None) -> tuple:
    """Reference :26-59: the mini-batch's final and initial embeddings. The reference runs
    the full forward and then gathers the batch's rows; here the batch is drawn first (the
    forward draws no random numbers, so the triples are the same) and a model with
    ``forward_rows`` computes each layer only where those rows depend on it (layer L at the
    <= 3 x batch rows, layer L-1 there and at their neighbours, ...), bitwise the same rows."""
    if r_edge_index is None:
        r_edge_index = convertAdjMatrixToEdgeIndex(user_num, item_num, train_edge_index)
    u, p, n = sampleMiniBatch(batch_size, r_edge_index.to(device), item_num)
    rows = getattr(model, "forward_rows", None)
    if rows is None:
        users_final, users_0, items_final, items_0 = model.forward(train_edge_index)
        return (users_final[u], users_0[u], items_final[p], items_0[p], items_final[n],
                items_0[n])
    u, p, n = u.long(), p.long(), n.long()
    f = rows(train_edge_index, torch.cat([u, user_num + p, user_num + n]))
    fu, fp, fn = torch.split(f, [u.numel(), p.numel(), n.numel()])
    users_0, items_0 = model.users_emb.weight, model.items_emb.weight
    return (fu, users_0[u], fp, items_0[p], fn, items_0[n])


class ValidationState:
    """What the reference's eval block reads, built once per training run (reference
    :115-122): the val user -> items dict, train item degrees and the train interactions
    (a device RowSets instead of the dense U x I matrix; calInternalSimilarity takes
    either)."""

    def __init__(self, user_num: int, item_num: int, r_train: torch.Tensor, val_edge_index,
                 device):
        r_val = convertAdjMatrixToEdgeIndex(user_num, item_num, val_edge_index)
        self.val_pos = getUserItemsDictByEdgeIndex(r_val)
        self.train_deg = getItemDegreeByUserPosItemDict(getUserItemsDictByEdgeIndex(r_train))
        self.train_mat = RowSets.from_pairs(r_train[0], r_train[1], user_num, item_num, device)
        self.rows = []


def evaluate_epoch(model, user_num: int, item_num: int, train_edge_index, val_edge_index,
                   state: ValidationState, epoch: int, train_loss: float, k: int,
                   epsilon: float, generator=None) -> dict:
    """One pass of the reference's eval block (:147-180): val loss, train-masked top-k,
    accuracy against the val positives, diversity over the train interactions."""
    model.eval()
    with torch.no_grad():
        val_loss = calValLoss(model, user_num, item_num, val_edge_index, epsilon, generator)
        recs = getValRecommendations(model, user_num, item_num, train_edge_index,
                                     val_edge_index, k)
        P, R, F1, NDCG = getAccurateMetrics(state.val_pos, recs, k)
        H, I = getDiversityMetrics(recs, state.train_deg, state.train_mat, k)
    model.train()
    row = {"iters": epoch, "train_loss": round(train_loss, 5), "val_loss": val_loss,
           "val_precision": P, "val_recall": R, "val_f1": F1, "val_ndcg": NDCG,
           "val_H": H, "val_I": I}
    state.rows.append(row)
    logger.info(f"[Iteration {epoch}] train_loss: {row['train_loss']}, val_loss: {val_loss}, "
                f"val_precision@{k}: {P}, val_recall@{k}: {R}, val_f1@{k}: {F1}, "
                f"val_NDCG@{k}: {NDCG}, val_H@{k}: {H}, val_I@{k}: {I}")
    return row


def train_model(model, user_num: int, item_num: int, train_edge_index, val_edge_index,
                name: str, evaluate: bool = True):
    hp = cfg.MODEL["HyperParameter"]
    k = cfg.RECOMMEND["k"]
    device = gpu_device()
    model = model.to(device)
    train_edge_index = train_edge_index.to(device)
    r_train = convertAdjMatrixToEdgeIndex(user_num, item_num, train_edge_index).to(device)
    state = None
    if evaluate and val_edge_index is not None:
        val_edge_index = val_edge_index.to(device)
        state = ValidationState(user_num, item_num, r_train, val_edge_index, device)
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
            if state is not None:
                evaluate_epoch(model, user_num, item_num, train_edge_index, val_edge_index,
                               state, epoch, loss.item(), k, hp["epsilon"])
            else:
                logger.info(f"[Iteration {epoch}/{hp['epochs']}] train_loss: "
                            f"{round(loss.item(), 5)}")
        if epoch % hp["epoch_per_lr_decay"] == 0 and epoch != 0:
            sched.step()
    path = cfg.MODEL["save_path"] + str(k) + f"_{name}.pth"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save(model.state_dict(), path)
    if state is not None and state.rows and getattr(cfg, "PICTURES", None):
        # reference :188-203 (iters = eval index * epoch_per_eval, as the reference writes)
        out = cfg.PICTURES["save_path"] + f"{name}_{k}_val_metrics.csv"
        os.makedirs(os.path.dirname(out), exist_ok=True)
        df = pd.DataFrame(state.rows)
        df["iters"] = [i * hp["epoch_per_eval"] for i in range(len(df))]
        df.to_csv(out, index=False)
        plot_curves(df, cfg.PICTURES["save_path"] + f"{name}_{k}")
    model.val_metrics = None if state is None else list(state.rows)
    return model


def plot_curves(df: pd.DataFrame, save_path: str) -> None:
    """The reference's training curves (:205-221): train / validation loss, then one plot per
    validation metric, as <save_path>_<metric>.png."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    from utils.picture import plotMetric
    it = df["iters"].tolist()
    fig = plt.figure()
    plt.plot(it, df["train_loss"].tolist(), label="train")
    plt.plot(it, df["val_loss"].tolist(), label="validation")
    plt.xlabel("iteration")
    plt.ylabel("loss")
    plt.title("training and validation loss curves")
    plt.legend()
    plt.savefig(save_path + "_loss_curves.png")
    plt.close(fig)
    for col, label, suffix in (("val_precision", "precision", "precision"),
                               ("val_recall", "recall", "recall"),
                               ("val_f1", "F1-score", "F1-score"),
                               ("val_ndcg", "NDCG", "NDCG"), ("val_H", "H", "H"),
                               ("val_I", "I", "I")):
        plotMetric(it, df[col].tolist(), "iteration", label, f"{label} curves",
                   save_path + f"_{suffix}.png")


@calTimes(logger, "模型训练完成")
def trainLightGCN(user_num: int, item_num: int, edge_index, train_edge_index,
                  val_edge_index):
    """Reference :61-223."""
    from model.LightGCN.model import LightGCN
    hp = cfg.MODEL["HyperParameter"]
    torch.manual_seed(hp["seed"])
    model = LightGCN(user_num, item_num, hp["embedding_dim"], hp["layers"])
    return train_model(model, user_num, item_num, train_edge_index, val_edge_index, "LightGCN")
