"""Graph inputs: a PyG-`Batch`-like container, PyG collation, and the synthetic benchmark graphs
(SURVEY.md §8(d)): random 3-D radius graphs with ~1M directed edges, and the k-chains pair
(experiments/kchains.ipynb:71, config C1).

The radius-graph builder is host-side input synthesis (scipy cKDTree), not part of the timed
hot path; a device-side builder is SURVEY.md §8(f) row f1.
"""
import math

import numpy as np
import torch


class Batch:
    """Minimal stand-in for torch_geometric.data.Batch: atoms, pos, edge_index, batch."""

    def __init__(self, atoms, pos, edge_index, batch=None, num_graphs=None, **extra):
        self.atoms = atoms
        self.pos = pos
        self.edge_index = edge_index
        self.batch = batch if batch is not None else torch.zeros(pos.shape[0], dtype=torch.long,
                                                                 device=pos.device)
        self.num_graphs = num_graphs
        self.__dict__.update(extra)

    @property
    def num_nodes(self):
        return self.pos.shape[0]

    @property
    def num_edges(self):
        return self.edge_index.shape[1]

    def to(self, device, non_blocking=False):
        kw = {}
        for k, v in self.__dict__.items():
            kw[k] = v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v
        return Batch(**kw)


def collate(graphs):
    """PyG Batch.from_data_list semantics: concat nodes, offset edge_index, batch vector."""
    atoms, pos, ei, bv, off = [], [], [], [], 0
    for b, g in enumerate(graphs):
        n = g.pos.shape[0]
        atoms.append(g.atoms)
        pos.append(g.pos)
        ei.append(g.edge_index + off)
        bv.append(torch.full((n,), b, dtype=torch.long))
        off += n
    return Batch(torch.cat(atoms), torch.cat(pos), torch.cat(ei, 1), torch.cat(bv),
                 num_graphs=len(graphs))


def radius_edges(pos, r):
    """All ordered pairs a != b with |pos_a - pos_b| < r, as (2, E) int64 sorted by (ei[1], ei[0])."""
    from scipy.spatial import cKDTree

    p = np.asarray(pos, dtype=np.float64)
    pairs = cKDTree(p).query_pairs(r, output_type="ndarray")  # a < b, |pa - pb| <= r
    if pairs.size:
        d = np.linalg.norm(p[pairs[:, 0]] - p[pairs[:, 1]], axis=1)
        pairs = pairs[d < r]
    src = np.concatenate([pairs[:, 0], pairs[:, 1]])
    dst = np.concatenate([pairs[:, 1], pairs[:, 0]])
    order = np.lexsort((src, dst))
    return np.stack([src[order], dst[order]]).astype(np.int64)


def _expected_edges(n, box, r):
    # ignoring boundary effects: n(n-1) * (4/3 pi r^3) / box^3
    return n * (n - 1) * (4.0 / 3.0 * math.pi * r ** 3) / box ** 3


def radius_graph(num_nodes=50_000, target_edges=1_000_000, r=5.0, seed=0, tol=0.01,
                 box=None, shuffle=False):
    """Seeded random radius graph: pos ~ U[0, L)^3 fp32, L tuned by bisection
    so that E is within `tol` of `target_edges` (exact E is whatever the graph has).
    Returns a Batch on CPU (atoms = 0, batch = 0)."""
    rng = np.random.default_rng(seed)
    unit = rng.random((num_nodes, 3))
    if box is None:
        lo, hi = None, None
        box = (num_nodes * num_nodes * 4.0 / 3.0 * math.pi * r ** 3 / target_edges) ** (1 / 3)
        for _ in range(40):
            pos = (unit * box).astype(np.float32)
            ei = radius_edges(pos, r)
            e = ei.shape[1]
            if abs(e - target_edges) <= tol * target_edges:
                break
            if e > target_edges:
                lo = box
            else:
                hi = box
            if lo is not None and hi is not None:
                box = 0.5 * (lo + hi)
            else:
                box = box * (e / target_edges) ** (1 / 3)
    else:
        pos = (unit * box).astype(np.float32)
        ei = radius_edges(pos, r)
    if shuffle:
        ei = ei[:, rng.permutation(ei.shape[1])]
    pos_t = torch.from_numpy(pos)
    return Batch(torch.zeros(num_nodes, dtype=torch.long), pos_t,
                 torch.from_numpy(np.ascontiguousarray(ei)), num_graphs=1, box=float(box),
                 radius=float(r), seed=int(seed))


def create_kchains(k=4):
    """experiments/kchains.ipynb:71: two graphs of k+2 nodes differing in one end position."""
    graphs = []
    for sign in (-1.0, 1.0):
        pos = torch.tensor([[4.0 * sign, -3.0, 0.0]] + [[0.0, 5.0 * i, 0.0] for i in range(k)]
                           + [[4.0, 5.0 * (k - 1) + 3.0, 0.0]])
        pos = pos - pos.mean(0)
        a = torch.arange(k + 1)
        ei = torch.cat([torch.stack([a, a + 1]), torch.stack([a + 1, a])], 1)
        ei = ei[:, torch.argsort(ei[0] * (k + 2) + ei[1])]  # to_undirected sorts by (row, col)
        graphs.append(Batch(torch.zeros(k + 2, dtype=torch.long), pos, ei))
    return graphs


def radius_graph_gpu(pos, r, batch=None, max_num_neighbors=32, num_graphs=None):
    """Device radius graph (K9, gmp_radius_*), the builder PyG SchNet constructs
    (models/schnet.py:47: torch_cluster.radius_graph(pos, r, batch, loop=False,
    max_num_neighbors)).  Edge j -> i for j != i of the same graph with
    ((dx*dx + dy*dy) + dz*dz) < r*r in fp32; per target the first max_num_neighbors + 1
    candidates in ascending j (self included) are kept and self is dropped — torch_cluster's
    GPU selection rule; max_num_neighbors=None or <= 0 keeps all.  Returns edge_index (2, E)
    int64 [sources; targets] sorted by (target, source).  pos: (N, 3) fp32 on the GPU.
    Host syncs: the bounding box, num_graphs (if not given) and the edge count."""
    import ctypes
    from . import _lib, ops
    lib = _lib.load()
    pos = ops._f32c(pos)
    ops._need_cuda(pos)
    if pos.dim() != 2 or pos.shape[1] != 3:
        raise ValueError(f"pos must be (N, 3), got {tuple(pos.shape)}")
    if not r > 0:
        raise ValueError("r must be > 0")
    N = pos.shape[0]
    dev = pos.device
    if N == 0:
        return torch.empty((2, 0), dtype=torch.int64, device=dev)
    if batch is not None:
        batch = ops._i64c(batch)
        ops._need_cuda(batch)
        if num_graphs is None:
            num_graphs = int(batch.max().item()) + 1
    num_graphs = 1 if batch is None else int(num_graphs)
    k = 0 if max_num_neighbors is None else max(int(max_num_neighbors), 0)
    lo = pos.min(0).values.cpu().numpy().astype(np.float32)
    hi = pos.max(0).values.cpu().numpy().astype(np.float32)
    r32 = np.float32(r)
    width = float(r32) * (1.0 + 1e-5)  # cell edge > r: rounding in the cell index stays safe
    while True:  # bound the cell table at ~2 cells per node
        inv = float(np.float32(1.0) / np.float32(width))
        if inv > float(np.float32(1.0) / r32):
            width *= 1.0 + 1e-5
            continue
        dims = [max(1, int(np.floor(float(hi[d] - lo[d]) * inv)) + 1) for d in range(3)]
        n_cells = num_graphs * dims[0] * dims[1] * dims[2]
        if n_cells <= 2 * N + 64:
            break
        width *= 1.25
    lo_c = (ctypes.c_float * 3)(*lo.tolist())
    dims_c = (ctypes.c_int * 3)(*dims)
    s = ops._stream()
    cells = torch.empty(N, dtype=torch.int64, device=dev)
    ops.check(lib.gmp_radius_cells_f32(ops._p(pos), ops._p(batch), N, lo_c, inv, dims_c,
                                       ops._p(cells), s), "gmp_radius_cells_f32")
    csr = ops.CSR(cells, n_cells)
    counts = torch.empty(N, dtype=torch.int64, device=dev)
    ops.check(lib.gmp_radius_count_f32(ops._p(pos), ops._p(batch), N, float(r32), k, lo_c, inv,
                                       dims_c, ops._p(cells), ops._p(csr.rowptr),
                                       ops._p(csr.perm), ops._p(counts), s),
              "gmp_radius_count_f32")
    offs = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=offs[1:])
    E = int(offs[-1].item())
    src = torch.empty(E, dtype=torch.int64, device=dev)
    if E == 0:
        return torch.empty((2, 0), dtype=torch.int64, device=dev)
    ops.check(lib.gmp_radius_fill_f32(ops._p(pos), ops._p(batch), N, float(r32), k, lo_c, inv,
                                      dims_c, ops._p(cells), ops._p(csr.rowptr),
                                      ops._p(csr.perm), ops._p(offs), ops._p(src), s),
              "gmp_radius_fill_f32")
    dst = torch.repeat_interleave(torch.arange(N, device=dev), counts, output_size=E)
    return torch.stack([src, dst])
