"""GVP-GNN on the MI355X kernels — drop-in for models/layers/gvp_layer.py:101-438 (GVP,
LayerNorm, Dropout, GVPConv, GVPConvLayer) and models/gvpgnn.py:10-127 (GVPGNNModel), same
module trees / state_dict keys.

GVPConv.forward (gvp_layer.py:304-316) keeps the PyG propagate contract (j = edge_index[0],
i = edge_index[1], mean aggregation with dim_size = N) but evaluates the first message GVP's
scalar Linear on the concatenation [s_j, e_s, s_i, |vh|] as two node projections
(s W_a^T, s W_b^T, N-row GEMMs) gathered per edge plus the edge terms — 2·s_in·s_out MACs per
edge fewer than the reference — and its vector Linear W_h likewise on node-level vector rows.
The gathers are the HIP gather kernel, the aggregation the HIP segmented mean on the receiver
CSR (deterministic).  Subclasses with a custom message function or module_list fall back to the
generic propagate path (gather -> message -> segmented reduce).
"""
import functools

import torch
from torch import nn
from torch.nn import functional as F

from . import ops
from .message_passing import MessagePassing
from .scatter import global_add_pool, global_mean_pool


def _norm_no_nan(x, axis=-1, keepdims=False, eps=1e-8, sqrt=True):
    """gvp_layer.py:66-73."""
    out = torch.clamp(torch.sum(torch.square(x), axis, keepdims), min=eps)
    return torch.sqrt(out) if sqrt else out


def _split(x, nv):
    return x[..., :-3 * nv], x[..., -3 * nv:].contiguous().view(x.shape[0], nv, 3)


def _merge(s, v):
    return torch.cat([s, v.contiguous().view(v.shape[0], v.shape[1] * 3)], -1)


def tuple_sum(*args):
    return tuple(map(sum, zip(*args)))


def tuple_cat(*args, dim=-1):
    dim %= len(args[0][0].shape)
    s_args, v_args = list(zip(*args))
    return torch.cat(s_args, dim=dim), torch.cat(v_args, dim=dim)


def tuple_index(x, idx):
    return x[0][idx], x[1][idx]


class GVP(nn.Module):
    """gvp_layer.py:101-170."""

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

    def _tail(self, s, vh):
        """Everything after s' = W_s[...] given the pre-activation s' and vh (B, 3, h)."""
        v = None
        if self.vo:
            v = ops.linear(vh, self.wv.weight).transpose(-1, -2)
            if self.vector_gate:
                gate = ops.linear(self.vector_act(s) if self.vector_act else s,
                                  self.wsv.weight, self.wsv.bias)
                v = v * torch.sigmoid(gate).unsqueeze(-1)
            elif self.vector_act:
                v = v * self.vector_act(_norm_no_nan(v, axis=-1, keepdims=True))
        if self.scalar_act:
            s = self.scalar_act(s)
        return (s, v) if self.vo else s

    def forward(self, x):
        if self.vi:
            s, v = x
            vh = ops.linear(v.transpose(-1, -2), self.wh.weight)
            s = ops.linear(torch.cat([s, _norm_no_nan(vh, axis=-2)], -1), self.ws.weight,
                           self.ws.bias)
            return self._tail(s, vh)
        s = self.ws(x)
        v = torch.zeros(s.shape[0], self.vo, 3, device=s.device, dtype=s.dtype) if self.vo \
            else None
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
        mask = torch.bernoulli((1 - self.drop_rate) * torch.ones(x.shape[:-1], device=x.device))
        return mask.unsqueeze(-1) * x / (1 - self.drop_rate)


class Dropout(nn.Module):
    def __init__(self, drop_rate):
        super().__init__()
        self.sdropout = nn.Dropout(drop_rate)
        self.vdropout = _VDropout(drop_rate)

    def forward(self, x):
        if type(x) is torch.Tensor:
            return self.sdropout(x)
        s, v = x
        return self.sdropout(s), self.vdropout(v)


class LayerNorm(nn.Module):
    """gvp_layer.py:221-243."""

    def __init__(self, dims):
        super().__init__()
        self.s, self.v = dims
        self.scalar_norm = nn.LayerNorm(self.s)

    def forward(self, x):
        if not self.v:
            return self.scalar_norm(x)
        s, v = x
        vn = _norm_no_nan(v, axis=-1, keepdims=True, sqrt=False)
        vn = torch.sqrt(torch.mean(vn, dim=-2, keepdim=True))
        return self.scalar_norm(s), v / vn


class GVPConv(MessagePassing):
    """gvp_layer.py:246-324."""

    def __init__(self, in_dims, out_dims, edge_dims, n_layers=3, module_list=None, aggr="mean",
                 activations=(F.relu, torch.sigmoid), vector_gate=True):
        super().__init__(aggr=aggr)
        self.si, self.vi = in_dims
        self.so, self.vo = out_dims
        self.se, self.ve = edge_dims
        G = functools.partial(GVP, activations=activations, vector_gate=vector_gate)
        self._custom = bool(module_list)
        module_list = module_list or []
        if not module_list:
            if n_layers == 1:
                module_list.append(G((2 * self.si + self.se, 2 * self.vi + self.ve),
                                     (self.so, self.vo), activations=(None, None)))
            else:
                module_list.append(G((2 * self.si + self.se, 2 * self.vi + self.ve), out_dims))
                for _ in range(n_layers - 2):
                    module_list.append(G(out_dims, out_dims))
                module_list.append(G(out_dims, out_dims, activations=(None, None)))
        self.message_func = nn.Sequential(*module_list)

    # --------------------------------------------------------------------------- reference hooks
    def message(self, s_i, v_i, s_j, v_j, edge_attr):
        v_j = v_j.view(v_j.shape[0], v_j.shape[1] // 3, 3)
        v_i = v_i.view(v_i.shape[0], v_i.shape[1] // 3, 3)
        message = tuple_cat((s_j, v_j), edge_attr, (s_i, v_i))
        return _merge(*self.message_func(message))

    def _fast_ok(self, x):
        g0 = self.message_func[0]
        return (not self._custom and self.vi > 0 and g0.vi == 2 * self.vi + self.ve
                and self.aggr in ("mean", "add", "sum") and x[0].is_cuda)

    def forward(self, x, edge_index, edge_attr):
        x_s, x_v = x
        if not self._fast_ok(x):
            msg = self.propagate(edge_index, s=x_s,
                                 v=x_v.contiguous().view(x_v.shape[0], x_v.shape[1] * 3),
                                 edge_attr=edge_attr)
            return _split(msg, self.vo)
        return self._fast_forward(x_s, x_v, edge_index, edge_attr)

    def _fast_forward(self, s, v, edge_index, edge_attr):
        n = s.shape[0]
        j, i = edge_index[0], edge_index[1]
        g0 = self.message_func[0]
        si, se = self.si, self.se
        Ws = g0.ws.weight                          # (so, [s_j | e_s | s_i | vn])
        # node projections: [s W_a^T | s W_b^T]  -> gathered per edge
        P = s.matmul(torch.cat([Ws[:, :si], Ws[:, si + se:2 * si + se]], 0).t())
        Pj = ops.gather(P[:, :g0.so].contiguous(), j, 0)
        Pi = ops.gather(P[:, g0.so:].contiguous(), i, 0)
        # vector channels [v_j | e_v | v_i] mixed by W_h: node-level rows (N, 3, h) gathered
        Wh = g0.wh.weight                          # (h, 2 vi + ve)
        vi, ve = self.vi, self.ve
        vt = v.transpose(-1, -2)                   # (N, 3, vi)
        Q = torch.cat([vt.matmul(Wh[:, :vi].t()), vt.matmul(Wh[:, vi + ve:].t())], -1)
        Q = Q.reshape(n, -1)                       # (N, 3 * 2h)
        h = g0.h_dim
        Qj = ops.gather(Q.view(n, 3, 2 * h)[:, :, :h].reshape(n, 3 * h), j, 0).view(-1, 3, h)
        Qi = ops.gather(Q.view(n, 3, 2 * h)[:, :, h:].reshape(n, 3 * h), i, 0).view(-1, 3, h)
        es, ev = edge_attr
        evt = ev.transpose(-1, -2)                 # (E, 3, ve)
        vh = Qj + Qi + ops.linear(evt, Wh[:, vi:vi + ve])
        vn = _norm_no_nan(vh, axis=-2)
        # edge part of W_s on [e_s | |vh|] as one per-edge Linear (dW by the edge outer sum)
        We = torch.cat([Ws[:, si:si + se], Ws[:, 2 * si + se:]], 1)
        s1 = ops.linear(torch.cat([es, vn], -1), We, g0.ws.bias) + Pj + Pi
        out = g0._tail(s1, vh)
        for mod in list(self.message_func)[1:]:
            out = mod(out)
        msg = _merge(*out) if isinstance(out, tuple) else out
        reduce = "sum" if self.aggr == "add" else self.aggr
        agg = ops.SegmentReduceFn.apply(msg, ops.get_csr(i, n), reduce)
        return _split(agg, self.vo)


class GVPConvLayer(nn.Module):
    """gvp_layer.py:327-438."""

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
            src, dst = edge_index
            mask = src < dst
            dh = tuple_sum(self.conv(x, edge_index[:, mask], tuple_index(edge_attr, mask)),
                           self.conv(autoregressive_x, edge_index[:, ~mask],
                                     tuple_index(edge_attr, ~mask)))
            count = ops.get_csr(dst, dh[0].size(0)).counts().clamp(min=1).unsqueeze(-1)
            count = count.to(dh[0].dtype)
            dh = dh[0] / count, dh[1] / count.unsqueeze(-1)
        else:
            dh = self.conv(x, edge_index, edge_attr)
        if node_mask is not None:
            x_ = x
            x, dh = tuple_index(x, node_mask), tuple_index(dh, node_mask)
        x = self.norm[0](tuple_sum(x, self.dropout[0](dh))) if self.residual else dh
        dh = self.ff_func(x)
        x = self.norm[1](tuple_sum(x, self.dropout[1](dh))) if self.residual else dh
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
        from .equivariant import RadialEmbeddingBlock
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
        ei = batch.edge_index
        vectors = ops.gather(batch.pos, ei[0], 0) - ops.gather(batch.pos, ei[1], 0)
        lengths = torch.linalg.norm(vectors, dim=-1, keepdim=True)
        h_V = ops.gather(self.emb_in.weight, batch.atoms, 0)
        h_E = (self.radial_embedding(lengths),
               torch.nan_to_num(torch.div(vectors, lengths)).unsqueeze_(-2))
        h_V = self.W_v(h_V)
        h_E = self.W_e(h_E)
        for layer in self.layers:
            h_V = layer(h_V, ei, h_E)
        out = self.pool(_merge(*h_V), batch.batch, getattr(batch, "num_graphs", None))
        if not self.equivariant_pred:
            out = out[:, :self.s_dim]
        return self.pred(out)
