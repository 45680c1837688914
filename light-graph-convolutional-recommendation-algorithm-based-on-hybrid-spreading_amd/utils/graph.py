"""Edge-list <-> symmetric COO conversions with the reference's signatures
(reference utils/graph.py:12-50), computed sparsely: no (U+I)^2 dense matrix, no Python
loop. The COO produced here is identical (values and order) to the reference's
``adj_mat.to_sparse_coo().indices()``: the coalesced, row-major-sorted symmetric index
set with items offset by ``user_num``. The propagation kernels do not consume COO — the
model converts it once into a cached device CSR (lgcnhs.graph.Adjacency).
"""
from __future__ import annotations

import torch


def convertEdgeIndexToAdjMatrix(user_num: int, item_num: int,
                                edge_index: torch.Tensor) -> torch.Tensor:
    """(user, item) edge list [2, E] -> symmetric coalesced COO [2, nnz] int64
    (reference utils/graph.py:12-35)."""
    ei = torch.as_tensor(edge_index).to(torch.int64)
    n = user_num + item_num
    u, i = ei[0], ei[1] + user_num
    keys = torch.unique(torch.cat([u * n + i, i * n + u]))
    return torch.stack([keys // n, keys % n])


def convertAdjMatrixToEdgeIndex(user_num: int, item_num: int,
                                edge_index: torch.Tensor) -> torch.Tensor:
    """Symmetric COO -> the user->item block as a sorted [2, E] edge list
    (reference utils/graph.py:38-50; duplicate entries collapse as the dense round trip's
    nonzero pattern does)."""
    ei = torch.as_tensor(edge_index).to(torch.int64)
    r, c = ei[0], ei[1]
    m = (r < user_num) & (c >= user_num)
    keys = torch.unique(r[m] * item_num + (c[m] - user_num))
    return torch.stack([keys // item_num, keys % item_num])
