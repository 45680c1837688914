"""LightGCNOpti with the reference's interface (reference model/LightGCNOpti/model.py:14-96):
e0 comes from Linear(features); propagation is the same HIP path as LightGCN."""
import torch
from torch import nn

from lgcnhs import ops
from lgcnhs.graph import as_adjacency


class LightGCNOpti(nn.Module):
    def __init__(self, user_num: int, item_num: int, embedding_dim: int, layers: int,
                 user_features: torch.Tensor, item_features: torch.Tensor) -> None:
        super().__init__()
        self.user_num = user_num
        self.item_num = item_num
        self.embedding_dim = embedding_dim
        self.layers = layers
        self.user_linear = nn.Linear(user_features.size(1), embedding_dim)
        self.item_linear = nn.Linear(item_features.size(1), embedding_dim)
        user_emb_init = self.user_linear(user_features)
        item_emb_init = self.item_linear(item_features)
        self.users_emb = nn.Embedding(num_embeddings=user_num, embedding_dim=embedding_dim)
        self.users_emb.weight = nn.Parameter(user_emb_init)
        self.items_emb = nn.Embedding(num_embeddings=item_num, embedding_dim=embedding_dim)
        self.items_emb.weight = nn.Parameter(item_emb_init)

    def forward(self, edge_index) -> tuple:
        w_u, w_i = self.users_emb.weight, self.items_emb.weight
        adj = as_adjacency(edge_index, self.user_num + self.item_num, device=w_u.device)
        emb_final = ops.propagate(adj, torch.cat([w_u, w_i]), self.layers)
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
        return norm.view(-1, 1) * x_j
