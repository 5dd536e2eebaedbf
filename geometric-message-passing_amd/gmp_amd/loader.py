"""Batching and the host->device input pipeline.

The reference trains with PyG DataLoaders: every step collates a list of graphs on the host
(`Batch.from_data_list`: node concat, edge_index offset by the cumulative node count, `batch`
vector) and copies the batch with a blocking `batch.to(device)`
(experiments/utils/train_utils.py:28,132).  Here:

  * `GraphCollator.stage` packs the per-graph arrays back to back into reusable pinned host
    buffers (one memcpy per field, no per-graph offset arithmetic on the host);
  * `GraphCollator.upload` issues one asynchronous H2D copy per field on a side stream and runs
    K10 (`gmp_batch_collate`) there to offset edge_index and write the `batch` vector;
  * `Prefetcher` keeps `depth` batches in flight, so the copy + collation of step k+1 overlaps
    the compute of step k; the consumer stream waits on an event, never on the host.

Graph objects are anything with tensor attributes `pos` (n, 3), `edge_index` (2, e) with
graph-local indices, and optionally `atoms`, `y`, ... (concatenated along dim 0, like PyG).
The returned `Batch` also carries `ptr` (node prefix sums, on the device) and a host-side
`num_graphs`, so pools need no `.item()` sync.
"""
import ctypes

import numpy as np
import torch

from . import _lib, ops
from .graph import Batch


class _Pinned:
    """Grow-only pinned staging buffer per field."""

    def __init__(self):
        self.buf = {}

    def view(self, name, dtype, shape):
        n = int(np.prod(shape)) if len(shape) else 1
        t = self.buf.get(name)
        if t is None or t.dtype != dtype or t.numel() < n:
            cap = max(n, int(1.5 * (t.numel() if t is not None else 0)), 1)
            t = torch.empty(cap, dtype=dtype, pin_memory=torch.cuda.is_available())
            self.buf[name] = t
        return t[:n].view(shape)


class _Staged:
    __slots__ = ("host", "num_graphs", "num_nodes", "num_edges", "slot")


class GraphCollator:
    """PyG `Batch.from_data_list` for the fields the models read, split into a host packing
    step and a device step (K10).  `fields`: per-graph tensors concatenated along dim 0."""

    def __init__(self, device="cuda", fields=("atoms", "y"), depth=2):
        self.device = torch.device(device)
        self.fields = tuple(fields)
        self.slots = [_Pinned() for _ in range(depth)]
        self.slot_free = [None] * depth  # event: last H2D copy out of the slot has finished
        self.next_slot = 0
        self.stream = None

    def stage(self, graphs):
        """Pack a list of graphs into the next pinned slot (host only)."""
        graphs = list(graphs)
        k = self.next_slot
        self.next_slot = (k + 1) % len(self.slots)
        if self.slot_free[k] is not None:
            self.slot_free[k].synchronize()  # its previous copy has left the buffer
            self.slot_free[k] = None
        pin = self.slots[k]
        B = len(graphs)
        n = np.fromiter((g.pos.shape[0] for g in graphs), np.int64, B)
        e = np.fromiter((g.edge_index.shape[1] for g in graphs), np.int64, B)
        N, E = int(n.sum()), int(e.sum())
        host = {}
        ptrs = pin.view("ptrs", torch.int64, (2, B + 1))
        ptrs[:, 0] = 0
        pn = ptrs.numpy()
        np.cumsum(n, out=pn[0, 1:])
        np.cumsum(e, out=pn[1, 1:])
        host["ptrs"] = ptrs
        pos = pin.view("pos", torch.float32, (N, 3))
        if B:
            torch.cat([g.pos for g in graphs], 0, out=pos)
        host["pos"] = pos
        ei = pin.view("edge_index", torch.int64, (2, E))
        if B:
            torch.cat([g.edge_index for g in graphs], 1, out=ei)
        host["edge_index"] = ei
        for f in self.fields:
            parts = [getattr(g, f, None) for g in graphs]
            if not parts or any(p is None for p in parts):
                continue
            rows = sum(p.shape[0] if p.dim() else 1 for p in parts)
            shape = (rows,) + tuple(parts[0].shape[1:])
            v = pin.view(f, parts[0].dtype, shape)
            torch.cat([p.reshape((-1,) + tuple(parts[0].shape[1:])) for p in parts], 0, out=v)
            host[f] = v
        st = _Staged()
        st.host, st.num_graphs, st.num_nodes, st.num_edges, st.slot = host, B, N, E, k
        return st

    def upload(self, st, consumer=None):
        """Async H2D of a staged batch + K10 on the side stream; the consumer stream (default:
        current) waits on an event.  Returns a device `Batch`."""
        lib = _lib.load()
        dev = self.device
        consumer = consumer or torch.cuda.current_stream(dev)
        if self.stream is None:
            self.stream = torch.cuda.Stream(dev)
        s = self.stream
        s.wait_stream(consumer)  # the previous use of reused allocations is ordered
        with torch.cuda.stream(s):
            d = {k: v.to(dev, non_blocking=True) for k, v in st.host.items()}
            done = torch.cuda.Event()
            done.record(s)
            self.slot_free[st.slot] = done
            ptrs = d.pop("ptrs")
            node_ptr, edge_ptr = ptrs[0], ptrs[1]
            local = d.pop("edge_index")
            ei = torch.empty_like(local)
            batch = torch.empty(st.num_nodes, dtype=torch.int64, device=dev)
            err = torch.zeros(1, dtype=torch.int32, device=dev)
            ops.check(lib.gmp_batch_collate(ops._p(local), st.num_edges, ops._p(node_ptr),
                                            ops._p(edge_ptr), st.num_graphs, st.num_nodes,
                                            ops._p(ei), ops._p(batch), ops._p(err),
                                            ctypes.c_void_p(s.cuda_stream)),
                      "gmp_batch_collate")
        consumer.wait_stream(s)
        outs = [ei, batch, err, node_ptr, local, ptrs] + list(d.values())
        for t in outs:
            t.record_stream(consumer)
        pos = d.pop("pos")
        atoms = d.pop("atoms", None)
        if atoms is None:
            atoms = torch.zeros(st.num_nodes, dtype=torch.int64, device=dev)
        out = Batch(atoms, pos, ei, batch, num_graphs=st.num_graphs, ptr=node_ptr,
                    collate_err=err, **d)
        return out

    def __call__(self, graphs):
        return self.upload(self.stage(graphs))


def check_batch(b):
    """Host-synchronising check of the collation range flag (PyG raises on bad indices)."""
    if int(b.collate_err.item()) != 0:
        raise IndexError("edge_index entry outside its graph's node range")


class Prefetcher:
    """Iterate device batches from an iterable of graph lists with `depth` batches in flight:
    the pinned packing, H2D copy and K10 collation of the next batch run while the caller
    computes on the current one."""

    def __init__(self, batches, device="cuda", fields=("atoms", "y"), depth=2):
        self.it = iter(batches)
        self.col = GraphCollator(device, fields, depth=depth + 1)
        self.depth = depth
        self.queue = []

    def _fill(self):
        while len(self.queue) < self.depth:
            try:
                graphs = next(self.it)
            except StopIteration:
                return
            self.queue.append(self.col.upload(self.col.stage(graphs)))

    def __iter__(self):
        return self

    def __next__(self):
        self._fill()
        if not self.queue:
            raise StopIteration
        b = self.queue.pop(0)
        self._fill()
        return b
