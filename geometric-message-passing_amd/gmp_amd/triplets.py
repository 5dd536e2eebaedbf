"""Triplet enumeration and angle / torsion featurisation on the device (K11; SURVEY.md §8(f) f3,
the "angles" of the north star's featurisation list).

`xyz_to_dat` mirrors models/layers/spherenet_layer.py:496-564 (same arguments, same returns);
`dimenet_triplets` / `dimenet_angles` mirror the DimeNet forward models/dimenet.py:79-90 (PyG
DimeNet.triplets).  The reference builds the triplets with torch_sparse (a SparseTensor by
target, row-selected by source); here the adjacency by (target, source) comes from two stable
CSR builds (K0), and K11 counts, then fills the triplets with their angles (and SphereNet
torsions) in one pass, in the reference's order.

Like the reference's use of these features (positions are data, not differentiated), there is
no backward: a `pos` that requires grad under autograd raises.
"""
import torch

from . import _lib, ops


def adjacency_by_target(edge_index, num_nodes):
    """Entries of edge_index sorted by (target, source), stable in edge id:
    rowptr (N+1), source per entry, edge id per entry."""
    src, dst = ops._i64c(edge_index[0]), ops._i64c(edge_index[1])
    by_src = ops.CSR(src, num_nodes)
    by_dst = ops.CSR(dst[by_src.perm], num_nodes)
    order = by_src.perm[by_dst.perm]
    return by_dst.rowptr, src[order], order


def _run(pos, edge_index, num_nodes, mode, want_angle, want_torsion, want_dist):
    lib = _lib.load()
    ei = ops._i64c(edge_index)
    ops._need_cuda(ei)
    if pos is not None:
        if pos.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError("triplet features have no backward (positions are data in "
                                      "the reference); detach pos")
        pos = ops._f32c(pos.detach())
        ops._need_cuda(pos)
    dev = ei.device
    E = ei.shape[1]
    N = int(num_nodes)
    rowptr, asrc, aeid = adjacency_by_target(ei, N)
    counts = torch.empty(E, dtype=torch.int64, device=dev)
    dist = torch.empty(E, dtype=torch.float32, device=dev) if want_dist else None
    s = ops._stream()
    ops.check(lib.gmp_triplet_count(ops._p(pos), ops._p(ei), E, N, ops._p(rowptr), ops._p(asrc),
                                    ops._p(counts), ops._p(dist), s), "gmp_triplet_count")
    offs = torch.zeros(E + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=offs[1:])
    T = int(offs[-1].item()) if E else 0
    idx_kj = torch.empty(T, dtype=torch.int64, device=dev)
    idx_ji = torch.empty(T, dtype=torch.int64, device=dev)
    angle = torch.empty(T, dtype=torch.float32, device=dev) if want_angle else None
    torsion = torch.empty(T, dtype=torch.float32, device=dev) if want_torsion else None
    ops.check(lib.gmp_triplet_fill_f32(ops._p(pos), ops._p(ei), E, N, ops._p(rowptr),
                                       ops._p(asrc), ops._p(aeid), ops._p(offs), T, mode,
                                       ops._p(idx_kj), ops._p(idx_ji), ops._p(angle),
                                       ops._p(torsion), s), "gmp_triplet_fill_f32")
    return dist, angle, torsion, idx_kj, idx_ji


def xyz_to_dat(pos, edge_index, num_nodes, use_torsion=False):
    """spherenet_layer.py:496: -> dist, angle, [torsion,] i, j, idx_kj, idx_ji (edge e = j -> i;
    angle in [0, pi] at j; torsion in (0, 2*pi])."""
    dist, angle, torsion, idx_kj, idx_ji = _run(pos, edge_index, num_nodes, 0, True,
                                                use_torsion, True)
    j, i = edge_index
    if use_torsion:
        return dist, angle, torsion, i, j, idx_kj, idx_ji
    return dist, angle, i, j, idx_kj, idx_ji


def dimenet_triplets(edge_index, num_nodes):
    """PyG DimeNet.triplets as called at dimenet.py:79:
    -> col, row, idx_i, idx_j, idx_k, idx_kj, idx_ji."""
    _, _, _, idx_kj, idx_ji = _run(None, edge_index, num_nodes, 1, False, False, False)
    row, col = edge_index
    return col, row, col[idx_ji], row[idx_ji], row[idx_kj], idx_kj, idx_ji


def dimenet_angles(pos, edge_index, num_nodes):
    """dimenet.py:79-90: -> dist (E), angle (T, vertex i), i, j, idx_i, idx_j, idx_k, idx_kj,
    idx_ji."""
    dist, angle, _, idx_kj, idx_ji = _run(pos, edge_index, num_nodes, 1, True, False, True)
    row, col = edge_index
    return (dist, angle, col, row, col[idx_ji], row[idx_ji], row[idx_kj], idx_kj, idx_ji)
