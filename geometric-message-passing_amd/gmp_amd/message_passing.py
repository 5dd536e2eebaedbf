"""PyG-compatible `MessagePassing` whose propagate() runs on the MI355X kernels.

API surface kept from torch_geometric 2.3.1 (as used by models/layers/egnn_layer.py:7,59 and
models/layers/gvp_layer.py:246,311): `MessagePassing(aggr, flow, node_dim)`, attributes
`aggr` / `node_dim` / `flow`, `propagate(edge_index, size=None, **kwargs)` with signature-inspected
`message(**)`, `aggregate(inputs, index[, ptr, dim_size])`, `update(aggr_out, **)` hooks and
the `_i` / `_j` suffix routing (flow "source_to_target": x_j = x[edge_index[0]],
x_i = x[edge_index[1]], aggregation at edge_index[1]).

Routing:
  * a subclass may provide `fused_propagate(edge_index, **kwargs)` (+ `fused_supported(**kwargs)`)
    that replaces the whole message->aggregate chain with one fused HIP kernel (EGNN);
  * otherwise the generic path gathers `_i`/`_j` arguments with the HIP gather kernel, runs the
    user's `message` (PyTorch ops on the GPU), and aggregates with the HIP segmented reduce.
"""
import inspect

import torch

from . import ops
from .scatter import scatter


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2):
        super().__init__()
        if flow not in ("source_to_target", "target_to_source"):
            raise ValueError(flow)
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim
        self._msg_params = list(inspect.signature(self.message).parameters)
        self._agg_params = set(inspect.signature(self.aggregate).parameters)
        self._upd_params = list(inspect.signature(self.update).parameters)[1:]

    # -------------------------------------------------------------------------------- hooks
    def message(self, x_j):
        return x_j

    def aggregate(self, inputs, index, ptr=None, dim_size=None):
        return scatter(inputs, index, dim=self.node_dim, dim_size=dim_size, reduce=self.aggr)

    def update(self, inputs):
        return inputs

    # -------------------------------------------------------------------------------- propagate
    def _indices(self, edge_index):
        if self.flow == "source_to_target":
            return edge_index[0], edge_index[1]  # j, i
        return edge_index[1], edge_index[0]

    def _num_nodes(self, size, kwargs):
        if size is not None:
            return size[1] if isinstance(size, (tuple, list)) else int(size)
        for v in kwargs.values():
            if torch.is_tensor(v) and v.dim() > 0:
                return v.size(self.node_dim)
        return None

    def propagate(self, edge_index, size=None, **kwargs):
        fused = getattr(self, "fused_propagate", None)
        if fused is not None and size is None:
            ok = getattr(self, "fused_supported", None)
            if ok is None or ok(**kwargs):
                return fused(edge_index, **kwargs)
        j, i = self._indices(edge_index)
        n = self._num_nodes(size, kwargs)
        msg_kwargs = {}
        for name in self._msg_params:
            if name.endswith("_i") and name[:-2] in kwargs:
                msg_kwargs[name] = ops.gather(kwargs[name[:-2]], i, self.node_dim)
            elif name.endswith("_j") and name[:-2] in kwargs:
                msg_kwargs[name] = ops.gather(kwargs[name[:-2]], j, self.node_dim)
            elif name == "index":
                msg_kwargs[name] = i
            elif name == "edge_index":
                msg_kwargs[name] = edge_index
            elif name in ("size_i", "dim_size"):
                msg_kwargs[name] = n
            else:
                msg_kwargs[name] = kwargs[name]
        out = self.message(**msg_kwargs)
        agg_kwargs = {"index": i}
        if "ptr" in self._agg_params:
            agg_kwargs["ptr"] = None
        if "dim_size" in self._agg_params:
            agg_kwargs["dim_size"] = n
        out = self.aggregate(out, **agg_kwargs)
        return self.update(out, **{k: kwargs[k] for k in self._upd_params if k in kwargs})
