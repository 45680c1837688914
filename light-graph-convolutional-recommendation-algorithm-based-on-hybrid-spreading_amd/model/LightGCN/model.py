"""LightGCN with the reference's interface (reference model/LightGCN/model.py:14-84).

``forward(edge_index)`` takes the reference's symmetric COO (or an
``lgcnhs.graph.Adjacency``) and runs the propagation on the HIP kernels: gcn_norm
(lg_gcn_norm_f32, once per graph) and L fused SpMM layers with the layer mean in the
epilogue (lg_spmm_layer_f32). Autograd is supported (backward = the same operator on
A_hat^T), which the reference's training loop needs (model/LightGCN/train.py:142).
"""
import torch
from torch import nn

from lgcnhs import ops
from lgcnhs.graph import as_adjacency


class LightGCN(nn.Module):
    def __init__(self, user_num: int, item_num: int, embedding_dim: int, layers: int) -> None:
        super().__init__()
        self.user_num = user_num
        self.item_num = item_num
        self.embedding_dim = embedding_dim
        self.layers = layers
        # same construction order as the reference, so torch.manual_seed(seed) gives the
        # same e0 (reference :32-38)
        self.users_emb = nn.Embedding(num_embeddings=user_num, embedding_dim=embedding_dim)
        self.items_emb = nn.Embedding(num_embeddings=item_num, embedding_dim=embedding_dim)
        nn.init.normal_(self.users_emb.weight, std=0.1)
        nn.init.normal_(self.items_emb.weight, std=0.1)

    def forward(self, edge_index) -> tuple:
        """-> (e_u^final, e_u^0, e_i^final, e_i^0) (reference :40-74)."""
        w_u, w_i = self.users_emb.weight, self.items_emb.weight
        adj = as_adjacency(edge_index, self.user_num + self.item_num, device=w_u.device)
        emb_0 = torch.cat([w_u, w_i])
        emb_final = ops.propagate(adj, emb_0, self.layers)
        users_final, items_final = torch.split(emb_final, [self.user_num, self.item_num])
        return users_final, w_u, items_final, w_i

    def forward_rows(self, edge_index, nodes: torch.Tensor) -> torch.Tensor:
        """The final embeddings of forward() at node ids ``nodes`` (users 0..U-1, items
        U..U+I-1), computing each layer only at the rows those depend on (the training step,
        whose loss reads the mini-batch's rows only); each row bitwise forward()'s."""
        w_u, w_i = self.users_emb.weight, self.items_emb.weight
        adj = as_adjacency(edge_index, self.user_num + self.item_num, device=w_u.device)
        return ops.propagate_rows(adj, torch.cat([w_u, w_i]), self.layers, nodes)

    def message(self, x_j, norm) -> torch.Tensor:
        """PyG message hook of the reference (:76-84); the fused kernel applies it inline."""
        return norm.view(-1, 1) * x_j
