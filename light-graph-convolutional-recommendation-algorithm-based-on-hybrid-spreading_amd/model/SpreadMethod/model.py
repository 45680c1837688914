"""Mass diffusion / heat conduction / hybrid spreading with the reference's numpy
interface (reference model/SpreadMethod/model.py:13-99): dense fp64 numpy in and out, the
arithmetic on the GPU (lg_spread_general_f64, lg_hybrid_weight_f64,
lg_spread_resource_f64). A is taken sparse from its nonzero pattern (A is 0/1 in every
reference call site: utils/trans.py:13-29), so the two dense GEMMs become sparse row sums
with an ascending, deterministic summation order.

The dense numpy boundary costs PCIe copies of I x I matrices; the recommend paths use
lgcnhs.ops directly and never bring W or F to the host.
"""
import numpy as np
import torch

from lgcnhs import ops
from lgcnhs.recs import gpu_device
from utils.log import logger
from utils.wrapper import calTimes


def _interactions(A: np.ndarray):
    dev = gpu_device()
    return ops.Interactions.from_dense(torch.as_tensor(np.asarray(A)).to(dev)), dev


def _item_degrees(A: np.ndarray, dev) -> torch.Tensor:
    # np.sum(A, axis=0) of a 0/1 matrix: exact integers
    return torch.as_tensor(np.sum(A, axis=0), dtype=torch.float64).to(dev)


@calTimes(logger, "通用扩散矩阵计算完成")
def getSpreadingGeneralMat(A: np.ndarray) -> np.ndarray:
    """general_W = (A.T / k_u) @ A, k_u == 0 -> 1 (reference :14-27)."""
    inter, _ = _interactions(A)
    return ops.spread_general(inter).cpu().numpy()


def _weight(A, general_W, lam, transpose=False):
    dev = gpu_device()
    gW = torch.as_tensor(np.ascontiguousarray(general_W), dtype=torch.float64).to(dev)
    return ops.hybrid_weight(gW, _item_degrees(A, dev), lam, transpose).cpu().numpy()


@calTimes(logger, "扩散资源矩阵计算完成")
def ProbS(A: np.ndarray, general_W: np.ndarray) -> np.ndarray:
    """W = general_W / k_j (k_j == 0 -> 1) (reference :30-43) == HybridS(lambda=1)."""
    return _weight(A, general_W, 1.0)


@calTimes(logger, "扩散资源矩阵计算完成")
def HeatS(A: np.ndarray, general_W: np.ndarray) -> np.ndarray:
    """W = general_W / k_i (k_i == 0 -> 1) (reference :46-60) == HybridS(lambda=0)."""
    return _weight(A, general_W, 0.0)


@calTimes(logger, "扩散资源矩阵计算完成")
def HybridS(A: np.ndarray, general_W: np.ndarray, Lambda: float) -> np.ndarray:
    """W = general_W / (k_i^(1-l) k_j^l), den == 0 -> 1 (reference :63-85)."""
    return _weight(A, general_W, float(Lambda))


@calTimes(logger, "资源矩阵计算完成")
def getResource(A: np.ndarray, W: np.ndarray) -> np.ndarray:
    """F = A @ W (reference :88-99)."""
    inter, dev = _interactions(A)
    Wt = torch.as_tensor(np.ascontiguousarray(W), dtype=torch.float64).to(dev)
    return ops.spread_resource(inter, Wt).cpu().numpy()
