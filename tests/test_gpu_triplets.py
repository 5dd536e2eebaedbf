"""GPU triplets + angles / torsions (K11) against the reference's own
xyz_to_dat outputs (tests/golden/triplets.pt) and the oracle (oracle/triplets.py).
Indices bit-exact; dist / angle / torsion within 1e-5 (atan2 / sqrt last-ulp differences)."""
import math
import os

import pytest
import torch

from oracle.triplets import dimenet_angles as o_dimenet, xyz_to_dat as o_xyz

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden", "triplets.pt")
TOL = 1e-5


def _close(a, b, tol=TOL):
    a, b = a.cpu(), b.cpu()
    assert a.shape == b.shape
    na, nb = torch.isnan(a), torch.isnan(b)
    assert torch.equal(na, nb)
    assert (a[~na] - b[~nb]).abs().max().item() <= tol if a.numel() else True


def _check(out, ref, n_float):
    for k, (a, b) in enumerate(zip(out, ref)):
        if k < n_float:
            _close(a, b)
        else:
            assert torch.equal(a.cpu(), b.cpu()), k


def test_xyz_to_dat_golden():
    from gmp_amd.triplets import xyz_to_dat
    g = torch.load(GOLD, weights_only=True)
    names = ["dist", "angle", "torsion", "i", "j", "idx_kj", "idx_ji"]
    for c in range(int(g["n_cases"])):
        pos, ei = g[f"{c}.pos"], g[f"{c}.edge_index"]
        out = xyz_to_dat(pos.to(DEV), ei.to(DEV), pos.shape[0], use_torsion=True)
        _check(out, [g[f"{c}.{n}"] for n in names], 3)
        # the ~0 torsions (k_n = k candidate whose rounding residual is positive) are the same set
        t_ref = g[f"{c}.torsion"]
        assert torch.equal(out[2].cpu() < 1e-6, t_ref < 1e-6)


def _graph(n, box, r, seed, shuffle=True):
    g = torch.Generator().manual_seed(seed)
    pos = torch.rand(n, 3, generator=g) * box
    d = torch.cdist(pos.double(), pos.double())
    ei = torch.nonzero((d < r) & (d > 0)).T.flip(0).contiguous()
    if shuffle:
        ei = ei[:, torch.randperm(ei.shape[1], generator=g)]
    return pos, ei


@pytest.mark.parametrize("n,box,r", [(300, 6.0, 1.5), (2000, 14.0, 1.8)])
def test_xyz_to_dat_vs_oracle(n, box, r):
    from gmp_amd.triplets import xyz_to_dat
    pos, ei = _graph(n, box, r, n)
    out = xyz_to_dat(pos.to(DEV), ei.to(DEV), n, use_torsion=True)
    _check(out, o_xyz(pos, ei, n, use_torsion=True), 3)
    out = xyz_to_dat(pos.to(DEV), ei.to(DEV), n, use_torsion=False)
    _check(out, o_xyz(pos, ei, n, use_torsion=False), 2)


def test_dimenet_vs_oracle():
    from gmp_amd.triplets import dimenet_angles, dimenet_triplets
    pos, ei = _graph(500, 7.0, 1.6, 5)
    out = dimenet_angles(pos.to(DEV), ei.to(DEV), 500)
    ref = o_dimenet(pos, ei, 500)
    _check(out, ref, 2)
    tri = dimenet_triplets(ei.to(DEV), 500)
    for a, b in zip(tri, ref[2:]):
        assert torch.equal(a.cpu(), b)


def test_edge_cases():
    from gmp_amd.triplets import xyz_to_dat
    pos = torch.randn(4, 3)
    # no edges
    out = xyz_to_dat(pos.to(DEV), torch.zeros(2, 0, dtype=torch.long, device=DEV), 4, True)
    assert out[1].numel() == 0 and out[2].numel() == 0
    # one undirected edge: two directed edges, no triplets (k == i always)
    ei = torch.tensor([[0, 1], [1, 0]])
    out = xyz_to_dat(pos.to(DEV), ei.to(DEV), 4, True)
    ref = o_xyz(pos, ei, 4, True)
    _check(out, ref, 3)
    assert out[1].numel() == 0
    # torsion under autograd with no triplets: zero gradient, no launch over empty arrays
    pd = pos.to(DEV).requires_grad_(True)
    out = xyz_to_dat(pd, ei.to(DEV), 4, use_torsion=True)
    (out[0].sum() + out[2].sum()).backward()
    assert pd.grad.shape == (4, 3) and bool(torch.isfinite(pd.grad).all())


@pytest.mark.parametrize("mode", ["spherenet", "dimenet"])
def test_dist_angle_backward_vs_oracle(mode):
    """d pos of sum(g_d dist) + sum(g_a angle) through gmp_triplet_geom_bwd_f32 + the CSR
    segmented sum, against autograd through the oracle's torch ops (dimenet.py:82-89 /
    spherenet_layer.py:509,531-535 restated).  Tolerance 1e-4 of the gradient's scale (atan2
    near-collinear triplets amplify last-ulp differences)."""
    from gmp_amd.triplets import dimenet_angles, xyz_to_dat
    pos, ei = _graph(400, 6.5, 1.6, 11)
    n = pos.shape[0]
    pd = pos.to(DEV).requires_grad_(True)
    pr = pos.clone().requires_grad_(True)
    if mode == "spherenet":
        out, ref = xyz_to_dat(pd, ei.to(DEV), n), o_xyz(pr, ei, n)
    else:
        out, ref = dimenet_angles(pd, ei.to(DEV), n), o_dimenet(pr, ei, n)
    _check(out, [r.detach() for r in ref], 2)
    g = torch.Generator().manual_seed(1)
    gd, ga = (torch.randn(ref[0].shape, generator=g), torch.randn(ref[1].shape, generator=g))
    ((out[0] * gd.to(DEV)).sum() + (out[1] * ga.to(DEV)).sum()).backward()
    ((ref[0] * gd).sum() + (ref[1] * ga).sum()).backward()
    scale = pr.grad.abs().max().item()
    err = (pd.grad.cpu() - pr.grad).abs().max().item()
    assert err <= 1e-4 * scale, (err, scale)
    # deterministic
    g1 = pd.grad.clone()
    pd.grad = None
    out = xyz_to_dat(pd, ei.to(DEV), n) if mode == "spherenet" else dimenet_angles(pd, ei.to(DEV), n)
    ((out[0] * gd.to(DEV)).sum() + (out[1] * ga.to(DEV)).sum()).backward()
    assert torch.equal(g1, pd.grad)


def test_torsion_backward_vs_oracle():
    """d pos of sum(g_d dist) + sum(g_a angle) + sum(g_t torsion) with the torsion's
    scatter-min backward (gmp_triplet_torsion_bwd_f32: the gradient reaches the winning k_n
    only, spherenet_layer.py:535-559), against autograd through the oracle's torch ops with
    torch_scatter's arg routing (oracle.triplets.torsion_with_scatter_min_grad).  The forward
    torsions agree bit-for-bit, so both pick the same winners; tolerance 1e-4 of the gradient's
    scale plus a 1e-3-of-scale bound at the few near-degenerate triplets (|a| + |b| tiny, where
    atan2's derivative amplifies last-ulp differences)."""
    from oracle.triplets import torsion_with_scatter_min_grad
    from gmp_amd.triplets import xyz_to_dat
    pos, ei = _graph(400, 6.5, 1.6, 13)
    n = pos.shape[0]
    pd = pos.to(DEV).requires_grad_(True)
    pr = pos.clone().requires_grad_(True)
    out = xyz_to_dat(pd, ei.to(DEV), n, use_torsion=True)
    ref = o_xyz(pr.detach(), ei, n, True)
    _check(out, ref, 3)
    tr = torsion_with_scatter_min_grad(pr, ei, n)
    assert torch.equal(tr.detach(), ref[2])
    g = torch.Generator().manual_seed(2)
    gd, ga, gt = (torch.randn(ref[k].shape, generator=g) for k in range(3))
    ((out[0] * gd.to(DEV)).sum() + (out[1] * ga.to(DEV)).sum()
     + (out[2] * gt.to(DEV)).sum()).backward()
    d, a = o_xyz(pr, ei, n)[:2]
    ((d * gd).sum() + (a * ga).sum() + (tr * gt).sum()).backward()
    scale = pr.grad.abs().max().item()
    err = (pd.grad.cpu() - pr.grad).abs()
    assert err.max().item() <= 1e-3 * scale, (err.max().item(), scale)
    assert (err > 1e-4 * scale).float().mean().item() < 0.01, err.max().item()
    # only the torsion term: the gradient is non-trivial and deterministic
    pd.grad = None
    out = xyz_to_dat(pd, ei.to(DEV), n, use_torsion=True)
    (out[2] * gt.to(DEV)).sum().backward()
    g1 = pd.grad.clone()
    assert g1.abs().max().item() > 0
    pd.grad = None
    out = xyz_to_dat(pd, ei.to(DEV), n, use_torsion=True)
    (out[2] * gt.to(DEV)).sum().backward()
    assert torch.equal(g1, pd.grad)


def test_benchmark_size_properties():
    """50k nodes / ~1M edges: structural invariants + an fp64 spot check of angles."""
    from gmp_amd.graph import radius_graph
    from gmp_amd.triplets import xyz_to_dat
    gr = radius_graph(num_nodes=50_000, target_edges=1_000_000)
    pos, ei = gr.pos.to(DEV), gr.edge_index.to(DEV)
    dist, angle, torsion, i, j, idx_kj, idx_ji = xyz_to_dat(pos, ei, 50_000, use_torsion=True)
    deg = torch.bincount(ei[1], minlength=50_000)
    assert idx_kj.numel() == int((deg[ei[0]] - 1).sum())  # symmetric simple graph
    assert bool((idx_ji[1:] >= idx_ji[:-1]).all())
    assert torch.equal(ei[1][idx_kj], ei[0][idx_ji])  # kj ends at j
    assert not bool((ei[0][idx_kj] == ei[1][idx_ji]).any())  # k != i
    assert float(angle.min()) >= 0 and float(angle.max()) <= math.pi + 1e-6
    assert float(torsion.min()) >= 0 and float(torsion.max()) <= 2 * math.pi + 1e-6
    sel = torch.randint(0, angle.numel(), (4096,), device=DEV)
    p = pos.double()
    u = p[ei[1][idx_ji[sel]]] - p[ei[0][idx_ji[sel]]]
    v = p[ei[0][idx_kj[sel]]] - p[ei[0][idx_ji[sel]]]
    a64 = torch.atan2(torch.linalg.cross(u, v).norm(dim=-1), (u * v).sum(-1))
    assert (angle[sel].double() - a64).abs().max().item() < 1e-5
