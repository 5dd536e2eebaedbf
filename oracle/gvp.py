"""GVP-GNN restated on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py).

Follows models/layers/gvp_layer.py: _norm_no_nan 66-73, _split/_merge 76-98, GVP 101-170,
_VDropout/Dropout 173-218, LayerNorm 221-243, GVPConv 246-324 (PyG propagate, flow
source_to_target: j = edge_index[0], i = edge_index[1], mean aggregation with dim_size = N),
GVPConvLayer 327-438; and models/gvpgnn.py:10-127 (GVPGNNModel).  Module trees and state_dict
keys are the reference's (dummy_param entries included).  Pinned by tests/golden/gvp_*.pt,
produced by the reference's own code (tests/golden/make_golden.py).
"""
import functools

import torch
from torch import nn
from torch.nn import functional as F

from .radial import RadialEmbeddingBlock
from .scatter import scatter, global_add_pool, global_mean_pool


def norm_no_nan(x, axis=-1, keepdims=False, eps=1e-8, sqrt=True):
    """sqrt(max(sum x^2, eps)) along `axis` (gvp_layer.py:66-73)."""
    sq = torch.clamp(torch.sum(x * x, axis, keepdims), min=eps)
    return torch.sqrt(sq) if sqrt else sq


def split(x, nv):
    return x[..., :-3 * nv], x[..., -3 * nv:].contiguous().view(x.shape[0], nv, 3)


def merge(s, v):
    return torch.cat([s, v.contiguous().view(v.shape[0], v.shape[1] * 3)], -1)


class GVP(nn.Module):
    """gvp_layer.py:101-170: vh = W_h v (over channels, per xyz); s' = W_s [s, |vh|];
    v' = W_v vh, gated by sigmoid(W_sv act_v(s')) (vector_gate); scalar act last."""

    def __init__(self, in_dims, out_dims, h_dim=None, activations=(F.relu, torch.sigmoid),
                 vector_gate=True):
        super().__init__()
        self.si, self.vi = in_dims
        self.so, self.vo = out_dims
        self.vector_gate = vector_gate
        if self.vi:
            self.h_dim = h_dim or max(self.vi, self.vo)
            self.wh = nn.Linear(self.vi, self.h_dim, bias=False)
            self.ws = nn.Linear(self.h_dim + self.si, self.so)
            if self.vo:
                self.wv = nn.Linear(self.h_dim, self.vo, bias=False)
                if self.vector_gate:
                    self.wsv = nn.Linear(self.so, self.vo)
        else:
            self.ws = nn.Linear(self.si, self.so)
        self.scalar_act, self.vector_act = activations
        self.dummy_param = nn.Parameter(torch.empty(0))

    def forward(self, x):
        if self.vi:
            s, v = x
            vh = self.wh(v.transpose(-1, -2))              # (B, 3, h)
            s = self.ws(torch.cat([s, norm_no_nan(vh, axis=-2)], -1))
            if self.vo:
                v = self.wv(vh).transpose(-1, -2)          # (B, vo, 3)
                if self.vector_gate:
                    g = self.wsv(self.vector_act(s) if self.vector_act else s)
                    v = v * torch.sigmoid(g).unsqueeze(-1)
                elif self.vector_act:
                    v = v * self.vector_act(norm_no_nan(v, axis=-1, keepdims=True))
        else:
            s = self.ws(x)
            if self.vo:
                v = torch.zeros(s.shape[0], self.vo, 3, dtype=s.dtype)
        if self.scalar_act:
            s = self.scalar_act(s)
        return (s, v) if self.vo else s


class _VDropout(nn.Module):
    def __init__(self, drop_rate):
        super().__init__()
        self.drop_rate = drop_rate
        self.dummy_param = nn.Parameter(torch.empty(0))

    def forward(self, x):
        if not self.training:
            return x
        mask = torch.bernoulli((1 - self.drop_rate) * torch.ones(x.shape[:-1])).unsqueeze(-1)
        return mask * x / (1 - self.drop_rate)


class Dropout(nn.Module):
    def __init__(self, drop_rate):
        super().__init__()
        self.sdropout = nn.Dropout(drop_rate)
        self.vdropout = _VDropout(drop_rate)

    def forward(self, x):
        if torch.is_tensor(x):
            return self.sdropout(x)
        return self.sdropout(x[0]), self.vdropout(x[1])


class LayerNorm(nn.Module):
    """gvp_layer.py:221-243: scalar LayerNorm; vectors / sqrt(mean_c clamp(|v|^2))."""

    def __init__(self, dims):
        super().__init__()
        self.s, self.v = dims
        self.scalar_norm = nn.LayerNorm(self.s)

    def forward(self, x):
        if not self.v:
            return self.scalar_norm(x)
        s, v = x
        vn = torch.sqrt(torch.mean(norm_no_nan(v, axis=-1, keepdims=True, sqrt=False), dim=-2,
                                   keepdim=True))
        return self.scalar_norm(s), v / vn


class GVPConv(nn.Module):
    """gvp_layer.py:246-324 with propagate restated: message on [s_j, e_s, s_i] / [v_j, e_v, v_i],
    aggregated at edge_index[1] (mean or add) with dim_size = N."""

    def __init__(self, in_dims, out_dims, edge_dims, n_layers=3, module_list=None, aggr="mean",
                 activations=(F.relu, torch.sigmoid), vector_gate=True):
        super().__init__()
        self.aggr = aggr
        self.si, self.vi = in_dims
        self.so, self.vo = out_dims
        self.se, self.ve = edge_dims
        G = functools.partial(GVP, activations=activations, vector_gate=vector_gate)
        mods = list(module_list or [])
        if not mods:
            first_in = (2 * self.si + self.se, 2 * self.vi + self.ve)
            if n_layers == 1:
                mods.append(G(first_in, out_dims, activations=(None, None)))
            else:
                mods.append(G(first_in, out_dims))
                mods.extend(G(out_dims, out_dims) for _ in range(n_layers - 2))
                mods.append(G(out_dims, out_dims, activations=(None, None)))
        self.message_func = nn.Sequential(*mods)

    def forward(self, x, edge_index, edge_attr):
        s, v = x
        j, i = edge_index[0], edge_index[1]
        ms = torch.cat([s[j], edge_attr[0], s[i]], -1)
        mv = torch.cat([v[j], edge_attr[1], v[i]], -2)
        msg = merge(*self.message_func((ms, mv)))
        reduce = "sum" if self.aggr == "add" else self.aggr
        return split(scatter(msg, i, 0, s.shape[0], reduce), self.vo)


class GVPConvLayer(nn.Module):
    """gvp_layer.py:327-438 (non-autoregressive forward; node_mask supported)."""

    def __init__(self, node_dims, edge_dims, n_message=3, n_feedforward=2, drop_rate=0.1,
                 autoregressive=False, activations=(F.relu, torch.sigmoid), vector_gate=True,
                 residual=True):
        super().__init__()
        self.conv = GVPConv(node_dims, node_dims, edge_dims, n_message,
                            aggr="add" if autoregressive else "mean", activations=activations,
                            vector_gate=vector_gate)
        G = functools.partial(GVP, activations=activations, vector_gate=vector_gate)
        self.norm = nn.ModuleList([LayerNorm(node_dims) for _ in range(2)])
        self.dropout = nn.ModuleList([Dropout(drop_rate) for _ in range(2)])
        if n_feedforward == 1:
            ff = [G(node_dims, node_dims, activations=(None, None))]
        else:
            hid = 4 * node_dims[0], 2 * node_dims[1]
            ff = [G(node_dims, hid)] + [G(hid, hid) for _ in range(n_feedforward - 2)] + \
                 [G(hid, node_dims, activations=(None, None))]
        self.ff_func = nn.Sequential(*ff)
        self.residual = residual

    def forward(self, x, edge_index, edge_attr, autoregressive_x=None, node_mask=None):
        if autoregressive_x is not None:
            raise NotImplementedError("autoregressive GVP path is outside the north-star path")
        dh = self.conv(x, edge_index, edge_attr)
        if node_mask is not None:
            x_ = x
            x, dh = (x[0][node_mask], x[1][node_mask]), (dh[0][node_mask], dh[1][node_mask])
        if self.residual:
            d = self.dropout[0](dh)
            x = self.norm[0]((x[0] + d[0], x[1] + d[1]))
        else:
            x = dh
        dh = self.ff_func(x)
        if self.residual:
            d = self.dropout[1](dh)
            x = self.norm[1]((x[0] + d[0], x[1] + d[1]))
        else:
            x = dh
        if node_mask is not None:
            x_[0][node_mask], x_[1][node_mask] = x[0], x[1]
            x = x_
        return x


class GVPGNNModel(nn.Module):
    """models/gvpgnn.py:10-127."""

    def __init__(self, r_max=10.0, num_bessel=8, num_polynomial_cutoff=5, num_layers=5,
                 in_dim=1, out_dim=1, s_dim=128, v_dim=16, s_dim_edge=32, v_dim_edge=1,
                 pool="sum", residual=True, equivariant_pred=False):
        super().__init__()
        self.r_max, self.num_layers = r_max, num_layers
        self.equivariant_pred, self.s_dim, self.v_dim = equivariant_pred, s_dim, v_dim
        acts = (F.relu, None)
        vd, ed = (s_dim, v_dim), (s_dim_edge, v_dim_edge)
        self.emb_in = nn.Embedding(in_dim, s_dim)
        self.W_v = nn.Sequential(LayerNorm((s_dim, 0)),
                                 GVP((s_dim, 0), vd, activations=(None, None), vector_gate=True))
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, num_polynomial_cutoff)
        self.W_e = nn.Sequential(LayerNorm((self.radial_embedding.out_dim, 1)),
                                 GVP((self.radial_embedding.out_dim, 1), ed,
                                     activations=(None, None), vector_gate=True))
        self.layers = nn.ModuleList(GVPConvLayer(vd, ed, activations=acts, vector_gate=True,
                                                 residual=residual)
                                    for _ in range(num_layers))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(s_dim + v_dim * 3, out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(s_dim, s_dim), nn.ReLU(),
                                      nn.Linear(s_dim, out_dim))

    def forward(self, batch):
        vec = batch.pos[batch.edge_index[0]] - batch.pos[batch.edge_index[1]]
        lengths = torch.linalg.norm(vec, dim=-1, keepdim=True)
        h_V = self.emb_in(batch.atoms)
        h_E = (self.radial_embedding(lengths),
               torch.nan_to_num(torch.div(vec, lengths)).unsqueeze(-2))
        h_V = self.W_v(h_V)
        h_E = self.W_e(h_E)
        for layer in self.layers:
            h_V = layer(h_V, batch.edge_index, h_E)
        out = self.pool(merge(*h_V), batch.batch)
        if not self.equivariant_pred:
            out = out[:, :self.s_dim]
        return self.pred(out)
