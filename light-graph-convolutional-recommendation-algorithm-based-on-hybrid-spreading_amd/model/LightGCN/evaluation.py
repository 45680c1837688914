"""LightGCN validation with the reference's interface (reference
model/LightGCN/evaluation.py:17-86), called from the periodic-eval block of the training
loop (reference model/LightGCN/train.py:147-180, here model/LightGCN/train.py).

getValRecommendations scores with the layer-0 embeddings, masks the TRAIN positives only
with -1024 and takes the top-k (reference :30-52) in one HIP kernel
(lg_score_topk_screened_f32, lists bit for bit lg_score_topk_f32's; ties ordered by (score
desc, item asc)); the val adjacency is accepted and unused, as in
the reference (it converts it at :38 and never reads it). calValLoss runs the forward on the
val adjacency (HIP propagation), draws one negative per val edge (structured negative
sampling, on the device) and returns the BPR loss of those triples rounded to 5 decimals
(reference :56-86)."""
import torch

from lgcnhs import ops
from lgcnhs.recs import exclusion_from_coo, gpu_device
from model.LightGCN.loss import BPRLoss, structured_negative_sampling
from utils.graph import convertAdjMatrixToEdgeIndex

MASK_VALUE = float(-(1 << 10))  # reference :50


def getValRecommendations(model, user_num: int, item_num: int, train_edge_index,
                          val_edge_index, k: int) -> torch.Tensor:
    """[user_num, k] int64 item ids on the model's device (reference :17-54)."""
    del val_edge_index  # the reference converts it and never reads it (:38)
    w_u = model.users_emb.weight.detach()
    dev = gpu_device(w_u)
    eu = w_u.to(dev, torch.float32).contiguous()
    ei = model.items_emb.weight.detach().to(dev, torch.float32).contiguous()
    excl = exclusion_from_coo(user_num, item_num, train_edge_index, device=dev)
    _, idx = ops.score_topk(eu, ei, k, excl, mask_value=MASK_VALUE)
    return idx


def val_loss_for_triples(model, val_edge_index, users, pos, neg, lambda_val: float) -> float:
    """BPR loss of fixed (user, pos, neg) triples on the forward over the val adjacency
    (reference :67-84 after its sampling step), rounded to 5 decimals (:86)."""
    uf, u0, itf, i0 = model.forward(val_edge_index)
    loss = BPRLoss(uf[users], u0[users], itf[pos], i0[pos], itf[neg], i0[neg], lambda_val)
    return round(loss.item(), 5)


def calValLoss(model, user_num: int, item_num: int, val_edge_index, lambda_val: float,
               generator=None) -> float:
    """Reference :56-86. Negatives are drawn from the item range (PyG draws from
    max(user_num, item_num), which indexes past the item table when U > I)."""
    dev = gpu_device(model.users_emb.weight)
    r = convertAdjMatrixToEdgeIndex(user_num, item_num, val_edge_index).to(dev)
    u, p, n = structured_negative_sampling(r, item_num, generator)
    return val_loss_for_triples(model, val_edge_index, u, p, n, lambda_val)
