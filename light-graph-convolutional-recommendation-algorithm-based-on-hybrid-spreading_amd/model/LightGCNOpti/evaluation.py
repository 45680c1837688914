"""LightGCNOpti validation (reference model/LightGCNOpti/evaluation.py:17-86): the same
functions as LightGCN's (the reference's two files differ only in the model type)."""
from model.LightGCN.evaluation import (calValLoss, getValRecommendations,  # noqa: F401
                                       val_loss_for_triples)
