"""EGNN layer / model restated on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py).

Follows models/layers/egnn_layer.py:7-89 and models/egnn.py:9-87 (module trees and
state_dict keys identical: mlp_msg.{0,1,3,4}, mlp_pos.{0,1,3}, mlp_upd.{0,1,3,4}, emb_in, pred).
PyG conventions: x_j = x[ei[0]], x_i = x[ei[1]], aggregate at ei[1].
"""
import torch
from torch import nn

from .scatter import scatter, global_add_pool, global_mean_pool


def _mlp(dims, act, norm, final_plain=False):
    layers = []
    for k in range(len(dims) - 1):
        layers.append(nn.Linear(dims[k], dims[k + 1]))
        if final_plain and k == len(dims) - 2:
            break
        layers += [norm(dims[k + 1]), act]
    return nn.Sequential(*layers)


class EGNNLayer(nn.Module):
    """egnn_layer.py:7-89. forward(h, pos, edge_index) -> (h_update, pos_update)."""

    def __init__(self, emb_dim, activation="relu", norm="layer", aggr="add"):
        super().__init__()
        self.emb_dim = emb_dim
        self.aggr = aggr
        act = {"swish": nn.SiLU(), "relu": nn.ReLU()}[activation]
        nrm = {"layer": nn.LayerNorm, "batch": nn.BatchNorm1d}[norm]
        d = emb_dim
        self.mlp_msg = _mlp([2 * d + 1, d, d], act, nrm)           # egnn_layer.py:28-35
        self.mlp_pos = _mlp([d, d, 1], act, nrm, final_plain=True)  # egnn_layer.py:37-39
        self.mlp_upd = _mlp([2 * d, d, d], act, nrm)               # egnn_layer.py:41-48

    def forward(self, h, pos, edge_index):
        j, i = edge_index[0], edge_index[1]
        rel = pos[i] - pos[j]                                   # pos_i - pos_j (egnn_layer.py:64)
        dist = rel.norm(dim=-1, keepdim=True)                   # :65
        m = self.mlp_msg(torch.cat([h[i], h[j], dist], dim=-1))  # :66-67 order [h_i, h_j, dist]
        shift = rel * self.mlp_pos(m)                           # :69
        reduce = "sum" if self.aggr in ("add", "sum") else self.aggr
        m_aggr = scatter(m, i, 0, None, reduce)                 # :77 (no dim_size)
        p_aggr = scatter(shift, i, 0, None, "mean")             # :79
        h_new = self.mlp_upd(torch.cat([h, m_aggr], dim=-1))    # :84
        return h_new, pos + p_aggr                              # :85


class EGNNModel(nn.Module):
    """models/egnn.py:9-87."""

    def __init__(self, num_layers=5, emb_dim=128, in_dim=1, out_dim=1, activation="relu",
                 norm="layer", aggr="sum", pool="sum", residual=True, equivariant_pred=False):
        super().__init__()
        self.equivariant_pred = equivariant_pred
        self.residual = residual
        self.emb_in = nn.Embedding(in_dim, emb_dim)
        self.convs = nn.ModuleList(EGNNLayer(emb_dim, activation, norm, aggr)
                                   for _ in range(num_layers))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(emb_dim + 3, out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(emb_dim, emb_dim), nn.ReLU(),
                                      nn.Linear(emb_dim, out_dim))

    def forward(self, batch):
        h = self.emb_in(batch.atoms)
        pos = batch.pos
        for conv in self.convs:
            dh, pos = conv(h, pos, batch.edge_index)
            h = h + dh if self.residual else dh
        feats = torch.cat([h, pos], -1) if self.equivariant_pred else h
        return self.pred(self.pool(feats, batch.batch))
