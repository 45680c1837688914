"""Restatement of the two third-party libraries the reference's LightGCN modules import
but this image lacks, used ONLY by make_golden.py to run the reference's own LightGCN /
recommend / graph code in this container:

* torch-geometric==2.6.1 (reference environment.yaml:276):
  - torch_geometric.nn.conv.gcn_conv.gcn_norm(edge_index, add_self_loops=False):
      deg = scatter_add(ones, col); dis = deg.pow(-0.5); dis[inf] = 0;
      w = dis[row] * 1 * dis[col]
  - torch_geometric.nn.conv.MessagePassing (aggr='add', flow='source_to_target'):
      propagate(edge_index, x=x, **kw) = scatter_add over col of message(x_j=x[row], **kw)
  - torch_geometric.utils.structured_negative_sampling (imported by loss.py; not called
    on the fixture paths)
* torch-sparse==0.6.17 (environment.yaml:278): SparseTensor(row, col, sparse_sizes)
  .to_dense() with value 1 per entry (duplicates summed), as utils/graph.py:46-47 uses it.

These are restatements of the published algorithms, not copies of the packages.
"""
from __future__ import annotations

import sys
import types

import torch


def gcn_norm(edge_index, edge_weight=None, num_nodes=None, improved=False,
             add_self_loops=True, flow="source_to_target", dtype=None):
    assert not add_self_loops, "the reference calls gcn_norm(add_self_loops=False)"
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1 if edge_index.numel() > 0 else 0
    if edge_weight is None:
        edge_weight = torch.ones(edge_index.size(1), dtype=dtype or torch.float32,
                                 device=edge_index.device)
    row, col = edge_index[0], edge_index[1]
    idx = col if flow == "source_to_target" else row
    deg = torch.zeros(num_nodes, dtype=edge_weight.dtype, device=edge_index.device)
    deg.scatter_add_(0, idx, edge_weight)
    dis = deg.pow_(-0.5)
    dis.masked_fill_(dis == float("inf"), 0)
    return edge_index, dis[row] * edge_weight * dis[col]


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2, **_):
        super().__init__()
        assert aggr == "add" and flow == "source_to_target"

    def propagate(self, edge_index, size=None, **kwargs):
        x = kwargs.pop("x")
        row, col = edge_index[0], edge_index[1]
        msg = self.message(x_j=x.index_select(0, row), **kwargs)
        out = torch.zeros((x.size(0),) + tuple(msg.shape[1:]), dtype=msg.dtype,
                          device=msg.device)
        out.index_add_(0, col, msg)
        return out

    def message(self, x_j, **_):
        return x_j


def structured_negative_sampling(edge_index, num_nodes=None, contains_neg_self_loops=True):
    i, j = edge_index[0], edge_index[1]
    n = int(num_nodes or (int(edge_index.max()) + 1))
    pos = set((i * n + j).tolist())
    k = torch.randint(n, (i.numel(),), dtype=torch.long)
    for t in range(k.numel()):
        while int(i[t]) * n + int(k[t]) in pos:
            k[t] = int(torch.randint(n, (1,)))
    return i, j, k


class SparseTensor:
    def __init__(self, row, col, sparse_sizes, value=None):
        self.row, self.col, self.sizes = row, col, tuple(sparse_sizes)

    def to_dense(self):
        d = torch.zeros(self.sizes, dtype=torch.float32)
        d.index_put_((self.row, self.col), torch.ones(self.row.numel()), accumulate=True)
        return d


def install() -> None:
    """Register the restated modules under the package names the reference imports."""
    tg = types.ModuleType("torch_geometric")
    tg_nn = types.ModuleType("torch_geometric.nn")
    tg_conv = types.ModuleType("torch_geometric.nn.conv")
    tg_gcn = types.ModuleType("torch_geometric.nn.conv.gcn_conv")
    tg_utils = types.ModuleType("torch_geometric.utils")
    tg_conv.MessagePassing = MessagePassing
    tg_gcn.gcn_norm = gcn_norm
    tg_utils.structured_negative_sampling = structured_negative_sampling
    tg.nn, tg_nn.conv, tg_conv.gcn_conv, tg.utils = tg_nn, tg_conv, tg_gcn, tg_utils
    ts = types.ModuleType("torch_sparse")
    ts.SparseTensor = SparseTensor
    sys.modules.update({
        "torch_geometric": tg, "torch_geometric.nn": tg_nn,
        "torch_geometric.nn.conv": tg_conv, "torch_geometric.nn.conv.gcn_conv": tg_gcn,
        "torch_geometric.utils": tg_utils, "torch_sparse": ts,
    })
