"""Triplet enumeration + angle / torsion on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py) —
SURVEY.md §8(f) f3.

Restates `xyz_to_dat` (reference models/layers/spherenet_layer.py:496-564) and the triplet /
angle block of the DimeNet forward (models/dimenet.py:79-90, whose `self.triplets` is PyG
2.3.1's DimeNet.triplets: the same torch_sparse construction as spherenet_layer.py:510-523)
with plain torch in place of torch_sparse: the adjacency by target is a (target, source)
lexsort, the triplets of edge e = (j -> i) are the in-edges of j with source != i, in that
order.  The arithmetic is the reference's own torch CPU ops (torch.cross, (x*y).sum(-1),
.norm(-1), atan2, scatter-min), so on the same machine this oracle reproduces the reference's
float behaviour, including the rounding-residual sign that decides the k_n = k torsion
candidate.  Pinned against the reference's own xyz_to_dat run here (tests/golden/triplets.pt,
made by tests/golden/make_golden.py with a torch_sparse stand-in)."""
import math

import torch


def adjacency_by_target(edge_index, num_nodes):
    src, dst = edge_index[0], edge_index[1]
    order = torch.argsort(dst * max(num_nodes, 1) + src, stable=True)
    rowptr = torch.zeros(num_nodes + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(torch.bincount(dst, minlength=num_nodes), 0)
    return rowptr, src[order], order


def triplets(edge_index, num_nodes):
    """-> idx_i, idx_j, idx_k, idx_kj, idx_ji (triplet k -> j -> i), reference order."""
    j, i = edge_index
    rowptr, asrc, aeid = adjacency_by_target(edge_index, num_nodes)
    deg = rowptr[1:] - rowptr[:-1]
    n_t = deg[j]
    idx_ji = torch.repeat_interleave(torch.arange(j.numel()), n_t)
    start = torch.repeat_interleave(rowptr[j], n_t)
    first = torch.repeat_interleave(torch.cumsum(n_t, 0) - n_t, n_t)
    slot = start + torch.arange(idx_ji.numel()) - first
    idx_k, idx_kj = asrc[slot], aeid[slot]
    idx_i, idx_j = i[idx_ji], j[idx_ji]
    mask = idx_i != idx_k
    return idx_i[mask], idx_j[mask], idx_k[mask], idx_kj[mask], idx_ji[mask]


def xyz_to_dat(pos, edge_index, num_nodes, use_torsion=False):
    j, i = edge_index
    dist = (pos[i] - pos[j]).pow(2).sum(dim=-1).sqrt()
    idx_i, idx_j, idx_k, idx_kj, idx_ji = triplets(edge_index, num_nodes)
    pos_ji = pos[idx_i] - pos[idx_j]
    pos_jk = pos[idx_k] - pos[idx_j]
    a = (pos_ji * pos_jk).sum(dim=-1)
    b = torch.cross(pos_ji, pos_jk, dim=-1).norm(dim=-1)
    angle = torch.atan2(b, a)
    if not use_torsion:
        return dist, angle, i, j, idx_kj, idx_ji
    rowptr, asrc, _ = adjacency_by_target(edge_index, num_nodes)
    deg = rowptr[1:] - rowptr[:-1]
    n_c = deg[idx_j]  # candidates k_n: every in-neighbour of j (then != i)
    t_of = torch.repeat_interleave(torch.arange(idx_i.numel()), n_c)
    first = torch.repeat_interleave(torch.cumsum(n_c, 0) - n_c, n_c)
    k_n = asrc[torch.repeat_interleave(rowptr[idx_j], n_c) + torch.arange(t_of.numel()) - first]
    keep = idx_i[t_of] != k_n
    t_of, k_n = t_of[keep], k_n[keep]
    it, jt, kt = idx_i[t_of], idx_j[t_of], idx_k[t_of]
    pos_j0 = pos[kt] - pos[jt]
    pos_ji = pos[it] - pos[jt]
    pos_jk = pos[k_n] - pos[jt]
    dist_ji = pos_ji.pow(2).sum(dim=-1).sqrt()
    plane1 = torch.cross(pos_ji, pos_j0, dim=-1)
    plane2 = torch.cross(pos_ji, pos_jk, dim=-1)
    a = (plane1 * plane2).sum(dim=-1)
    b = (torch.cross(plane1, plane2, dim=-1) * pos_ji).sum(dim=-1) / dist_ji
    torsion1 = torch.atan2(b, a)
    torsion1[torsion1 <= 0] += 2 * math.pi
    # torch_scatter min: rows = max(index) + 1, untouched rows 0, NaN never wins
    n = int(t_of.max()) + 1 if t_of.numel() else 0
    big = torch.finfo(torch.float32).max
    torsion = torch.full((n,), big, dtype=torsion1.dtype).scatter_reduce(0, t_of, torch.nan_to_num(torsion1, nan=big),
                                                   "amin", include_self=True)
    torsion[torsion == big] = 0
    return dist, angle, torsion, i, j, idx_kj, idx_ji


def torsion_with_scatter_min_grad(pos, edge_index, num_nodes):
    """The torsion of xyz_to_dat (spherenet_layer.py:535-559) as a differentiable function of
    pos with torch_scatter's scatter_min backward: the gradient of each triplet reaches only its
    arg candidate (the first k_n among equal minima), untouched triplets get none.  (The
    reference's scatter-min is torch_scatter's; torch's own scatter_reduce("amin") would split
    ties and saves its output, so the in-place `torsion[torsion == big] = 0` above is not
    differentiable through it.)"""
    idx_i, idx_j, idx_k, _, _ = triplets(edge_index, num_nodes)
    rowptr, asrc, _ = adjacency_by_target(edge_index, num_nodes)
    deg = rowptr[1:] - rowptr[:-1]
    n_c = deg[idx_j]
    t_of = torch.repeat_interleave(torch.arange(idx_i.numel()), n_c)
    first = torch.repeat_interleave(torch.cumsum(n_c, 0) - n_c, n_c)
    k_n = asrc[torch.repeat_interleave(rowptr[idx_j], n_c) + torch.arange(t_of.numel()) - first]
    keep = idx_i[t_of] != k_n
    t_of, k_n = t_of[keep], k_n[keep]
    def t1_of(p, t, kn):
        it, jt, kt = idx_i[t], idx_j[t], idx_k[t]
        pos_ji = p[it] - p[jt]
        plane1 = torch.cross(pos_ji, p[kt] - p[jt], dim=-1)
        plane2 = torch.cross(pos_ji, p[kn] - p[jt], dim=-1)
        a = (plane1 * plane2).sum(dim=-1)
        b = ((torch.cross(plane1, plane2, dim=-1) * pos_ji).sum(dim=-1)
             / pos_ji.pow(2).sum(-1).sqrt())
        t1 = torch.atan2(b, a)
        return torch.where(t1 <= 0, t1 + 2 * math.pi, t1)

    # select the winners on detached values, then differentiate the winners only (a losing
    # candidate may sit at atan2(0, 0), whose autograd is NaN even with a zero incoming grad)
    T = idx_i.numel()
    big = torch.finfo(torch.float32).max
    v = torch.nan_to_num(t1_of(pos.detach(), t_of, k_n), nan=big)
    mn = torch.full((T,), big, dtype=v.dtype).scatter_reduce(0, t_of, v, "amin",
                                                             include_self=True)
    m = torch.arange(t_of.numel())
    cand = torch.where(v == mn[t_of], m, torch.full_like(m, t_of.numel()))
    arg = torch.full((T,), t_of.numel()).scatter_reduce(0, t_of, cand, "amin",
                                                        include_self=True)
    has = ((arg < t_of.numel()) & (mn < big)).nonzero()[:, 0]
    # values: the full-batch forward's (torch's CPU cross may round a re-evaluated subset
    # differently); gradient: the winners' atan2 path
    tw = t1_of(pos, t_of[arg[has]], k_n[arg[has]])
    out = torch.zeros(T, dtype=pos.dtype)
    return out.index_put((has,), v[arg[has]] + (tw - tw.detach()))


def dimenet_angles(pos, edge_index, num_nodes):
    """models/dimenet.py:79-90: i, j = PyG triplets' (col, row); angle at vertex i."""
    idx_i, idx_j, idx_k, idx_kj, idx_ji = triplets(edge_index, num_nodes)
    row, col = edge_index
    i, j = col, row
    dist = (pos[i] - pos[j]).pow(2).sum(dim=-1).sqrt()
    pos_i = pos[idx_i]
    pos_ji, pos_ki = pos[idx_j] - pos_i, pos[idx_k] - pos_i
    a = (pos_ji * pos_ki).sum(dim=-1)
    b = torch.cross(pos_ji, pos_ki, dim=-1).norm(dim=-1)
    angle = torch.atan2(b, a)
    return dist, angle, i, j, idx_i, idx_j, idx_k, idx_kj, idx_ji
