"""Triplet enumeration and angle / torsion featurisation on the device (K11; SURVEY.md §8(f) f3,
the "angles" of the north star's featurisation list).

`xyz_to_dat` mirrors models/layers/spherenet_layer.py:496-564 (same arguments, same returns);
`dimenet_triplets` / `dimenet_angles` mirror the DimeNet forward models/dimenet.py:79-90 (PyG
DimeNet.triplets).  The reference builds the triplets with torch_sparse (a SparseTensor by
target, row-selected by source); here the adjacency by (target, source) comes from two stable
CSR builds (K0), and K11 counts, then fills the triplets with their angles (and SphereNet
torsions) in one pass, in the reference's order.

Distances and angles are differentiable w.r.t. `pos` (PyG DimeNet differentiates its angles,
dimenet.py:79-90, e.g. for forces): the backward kernel gmp_triplet_geom_bwd_f32 writes one
gradient row per (triplet, corner) and per (edge, end), summed per node over a CSR
(deterministic).  The SphereNet torsion (a scatter-min over candidates k_n,
spherenet_layer.py:535-559) is differentiable too: the fill kernel records the winning k_n of
every triplet and gmp_triplet_torsion_bwd_f32 routes the gradient to that candidate only, as
torch_scatter's scatter_min backward does (first index among equal minima).
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


def _run(pos, edge_index, num_nodes, mode, want_angle, want_torsion, want_dist, want_kn=False):
    lib = _lib.load()
    ei = ops._i64c(edge_index)
    ops._need_cuda(ei)
    if pos is not None:
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
    kn = torch.empty(T, dtype=torch.int64, device=dev) if want_kn else None
    ops.check(lib.gmp_triplet_fill_f32(ops._p(pos), ops._p(ei), E, N, ops._p(rowptr),
                                       ops._p(asrc), ops._p(aeid), ops._p(offs), T, mode,
                                       ops._p(idx_kj), ops._p(idx_ji), ops._p(angle),
                                       ops._p(torsion), ops._p(kn), s), "gmp_triplet_fill_f32")
    if want_kn:
        return dist, angle, torsion, idx_kj, idx_ji, kn
    return dist, angle, torsion, idx_kj, idx_ji


class TripletGeomFn(torch.autograd.Function):
    """(dist (E), angle (T), torsion (T, or empty without use_torsion), idx_kj, idx_ji) with the
    backward of dist, angle and torsion w.r.t. pos."""

    @staticmethod
    def forward(ctx, pos, edge_index, num_nodes, mode, use_torsion):
        res = _run(pos, edge_index, num_nodes, mode, True, use_torsion, True, use_torsion)
        dist, angle, torsion, idx_kj, idx_ji = res[:5]
        kn = res[5] if use_torsion else None
        if torsion is None:
            torsion = torch.empty(0, dtype=torch.float32, device=dist.device)
            kn = torch.empty(0, dtype=torch.int64, device=dist.device)
        ctx.save_for_backward(pos, ops._i64c(edge_index), idx_kj, idx_ji, kn)
        ctx.mode, ctx.n, ctx.use_torsion = mode, int(num_nodes), use_torsion
        ctx.mark_non_differentiable(idx_kj, idx_ji)
        return dist, angle, torsion, idx_kj, idx_ji

    @staticmethod
    def backward(ctx, g_dist, g_angle, g_torsion, _g1, _g2):
        pos, ei, idx_kj, idx_ji, kn = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        E, T = ei.shape[1], idx_kj.numel()
        dev = pos.device
        p32 = ops._f32c(pos.detach())
        nt = 4 * T if (ctx.use_torsion and g_torsion is not None) else 0
        rows = torch.empty((3 * T + 2 * E + nt, 3), dtype=torch.float32, device=dev)
        node = torch.empty(3 * T + 2 * E + nt, dtype=torch.int64, device=dev)
        gd = ops._f32c(g_dist) if g_dist is not None else None
        ga = ops._f32c(g_angle) if g_angle is not None else None
        lib = _lib.load()
        s = ops._stream()
        ops.check(lib.gmp_triplet_geom_bwd_f32(ops._p(p32), ops._p(ei), E, ops._p(idx_kj),
                                               ops._p(idx_ji), T, ctx.mode, ops._p(gd),
                                               ops._p(ga), ops._p(rows), ops._p(node), s),
                  "gmp_triplet_geom_bwd_f32")
        if nt:
            m = 3 * T + 2 * E
            ops.check(lib.gmp_triplet_torsion_bwd_f32(ops._p(p32), ops._p(ei), E,
                                                      ops._p(idx_kj), ops._p(idx_ji),
                                                      ops._p(kn), T,
                                                      ops._p(ops._f32c(g_torsion)),
                                                      ops._p(rows[m:]), ops._p(node[m:]), s),
                      "gmp_triplet_torsion_bwd_f32")
        g_pos, _ = ops.segment_reduce(rows, ops.CSR(node, ctx.n), "sum")
        return g_pos.to(pos.dtype), None, None, None, None


def _geom(pos, edge_index, num_nodes, mode, use_torsion=False):
    if pos.requires_grad and torch.is_grad_enabled():
        return TripletGeomFn.apply(pos, edge_index, num_nodes, mode, use_torsion)
    return _run(pos, edge_index, num_nodes, mode, True, use_torsion, True)


def xyz_to_dat(pos, edge_index, num_nodes, use_torsion=False):
    """spherenet_layer.py:496: -> dist, angle, [torsion,] i, j, idx_kj, idx_ji (edge e = j -> i;
    angle in [0, pi] at j; torsion in (0, 2*pi]).  dist, angle and torsion are differentiable
    w.r.t. pos."""
    dist, angle, torsion, idx_kj, idx_ji = _geom(pos, edge_index, num_nodes, 0, use_torsion)
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
    dist, angle, _, idx_kj, idx_ji = _geom(pos, edge_index, num_nodes, 1)
    row, col = edge_index
    return (dist, angle, col, row, col[idx_ji], row[idx_ji], row[idx_kj], idx_kj, idx_ji)
