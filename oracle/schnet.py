"""SchNet (PyG 2.3.1 `torch_geometric.nn.SchNet` internals) restated on CPU
(TEST INFRASTRUCTURE; see oracle/__init__.py).  **Parity unpinned**: PyG is absent from the
container and from /root/reference, so this follows PyG 2.3.1's published algorithm:
  GaussianSmearing(0, cutoff, G): offset = linspace(0, cutoff, G), coeff = -0.5 / (o1 - o0)^2,
    exp(coeff (d - offset)^2);
  ShiftedSoftplus: softplus(x) - log(2);
  CFConv (aggr 'add', flow source_to_target): C = 0.5 (cos(pi d / cutoff) + 1),
    W = nn(edge_attr) * C, x = lin1(x) (no bias), out_i = sum_{e: ei1 = i} x[ei0] * W_e,
    lin2(out);
  InteractionBlock: mlp = Linear(G, F) -> SSP -> Linear(F, F) (shared as conv.nn),
    conv -> SSP -> lin;
  Embedding(100, hidden, padding_idx=0) (the zero-padding row of PyG >= 2.1; with atoms = 0 the
    initial features are zero — recorded in DESIGN.md).
Model wrapper: models/schnet.py:9-80 (SchNetModel: residual interactions, pool, lin1 -> SSP ->
lin2 with lin2 re-created as Linear(hidden // 2, out_dim)).
"""
import math

import torch
from torch import nn
from torch.nn import functional as F

from .scatter import scatter, global_add_pool, global_mean_pool


class ShiftedSoftplus(nn.Module):
    def __init__(self):
        super().__init__()
        self.shift = math.log(2.0)

    def forward(self, x):
        return F.softplus(x) - self.shift


class GaussianSmearing(nn.Module):
    def __init__(self, start=0.0, stop=5.0, num_gaussians=50):
        super().__init__()
        offset = torch.linspace(start, stop, num_gaussians)
        self.coeff = -0.5 / (offset[1] - offset[0]).item() ** 2
        self.register_buffer("offset", offset)

    def forward(self, dist):
        d = dist.view(-1, 1) - self.offset.view(1, -1)
        return torch.exp(self.coeff * d * d)


class CFConv(nn.Module):
    def __init__(self, in_channels, out_channels, num_filters, mlp, cutoff):
        super().__init__()
        self.lin1 = nn.Linear(in_channels, num_filters, bias=False)
        self.lin2 = nn.Linear(num_filters, out_channels)
        self.nn = mlp
        self.cutoff = cutoff

    def forward(self, x, edge_index, edge_weight, edge_attr):
        C = 0.5 * (torch.cos(edge_weight * math.pi / self.cutoff) + 1.0)
        W = self.nn(edge_attr) * C.view(-1, 1)
        x = self.lin1(x)
        msg = x[edge_index[0]] * W
        return self.lin2(scatter(msg, edge_index[1], 0, x.shape[0], "sum"))


class InteractionBlock(nn.Module):
    def __init__(self, hidden_channels, num_gaussians, num_filters, cutoff):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(num_gaussians, num_filters), ShiftedSoftplus(),
                                 nn.Linear(num_filters, num_filters))
        self.conv = CFConv(hidden_channels, hidden_channels, num_filters, self.mlp, cutoff)
        self.act = ShiftedSoftplus()
        self.lin = nn.Linear(hidden_channels, hidden_channels)

    def forward(self, x, edge_index, edge_weight, edge_attr):
        return self.lin(self.act(self.conv(x, edge_index, edge_weight, edge_attr)))


class SchNetModel(nn.Module):
    def __init__(self, hidden_channels=128, in_dim=1, out_dim=1, num_filters=128, num_layers=6,
                 num_gaussians=50, cutoff=10, max_num_neighbors=32, pool="sum"):
        super().__init__()
        self.hidden_channels, self.cutoff = hidden_channels, cutoff
        self.embedding = nn.Embedding(100, hidden_channels, padding_idx=0)
        self.distance_expansion = GaussianSmearing(0.0, cutoff, num_gaussians)
        self.interactions = nn.ModuleList(
            InteractionBlock(hidden_channels, num_gaussians, num_filters, cutoff)
            for _ in range(num_layers))
        self.lin1 = nn.Linear(hidden_channels, hidden_channels // 2)
        self.act = ShiftedSoftplus()
        self.lin2 = nn.Linear(hidden_channels // 2, out_dim)
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool}[pool]

    def forward(self, batch):
        h = self.embedding(batch.atoms)
        row, col = batch.edge_index
        w = (batch.pos[row] - batch.pos[col]).norm(dim=-1)
        attr = self.distance_expansion(w)
        for inter in self.interactions:
            h = h + inter(h, batch.edge_index, w, attr)
        out = self.pool(h, batch.batch)
        return self.lin2(self.act(self.lin1(out)))
