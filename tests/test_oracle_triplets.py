"""The triplet/angle/torsion oracle (oracle/triplets.py) against the golden
vectors made by running the reference's own xyz_to_dat (spherenet_layer.py:496-564,
tests/golden/triplets.pt), plus DimeNet-angle known answers (dimenet.py:79-90)."""
import math
import os

import torch

from oracle.triplets import dimenet_angles, xyz_to_dat

GOLD = os.path.join(os.path.dirname(__file__), "golden", "triplets.pt")
NAMES = ["dist", "angle", "torsion", "i", "j", "idx_kj", "idx_ji"]


def _same(a, b):
    return a.shape == b.shape and torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))


def test_oracle_matches_reference_xyz_to_dat():
    g = torch.load(GOLD, weights_only=True)
    for c in range(int(g["n_cases"])):
        pos, ei = g[f"{c}.pos"], g[f"{c}.edge_index"]
        out = xyz_to_dat(pos, ei, pos.shape[0], use_torsion=True)
        for name, v in zip(NAMES, out):
            assert _same(v, g[f"{c}.{name}"]), (c, name)
        short = xyz_to_dat(pos, ei, pos.shape[0], use_torsion=False)
        for name, v in zip(["dist", "angle", "i", "j", "idx_kj", "idx_ji"], short):
            assert _same(v, g[f"{c}.{name}"]), (c, name)


def test_dimenet_angle_known_answer():
    # 0 -> 1 -> 2 path: triplet k=0 -> j=1 -> i=2 and k=2 -> j=1 -> i=0
    pos = torch.tensor([[1.0, 0, 0], [0, 0, 0], [0, 2.0, 0]])
    ei = torch.tensor([[0, 1, 1, 2], [1, 0, 2, 1]])
    dist, angle, i, j, idx_i, idx_j, idx_k, idx_kj, idx_ji = dimenet_angles(pos, ei, 3)
    assert idx_ji.tolist() == [1, 2] and idx_kj.tolist() == [3, 0]
    assert idx_i.tolist() == [0, 2] and idx_j.tolist() == [1, 1] and idx_k.tolist() == [2, 0]
    # angle at vertex i between (p_j - p_i) and (p_k - p_i)
    want = [math.atan2(2, 1) , math.atan2(1, 2)]  # i=0: j-i=(-1,0,0), k-i=(-1,2,0)
    assert torch.allclose(angle, torch.tensor(want), atol=1e-6)
    assert torch.allclose(dist, torch.tensor([1.0, 1.0, 2.0, 2.0]))


def test_spherenet_angle_right_angle():
    pos = torch.tensor([[1.0, 0, 0], [0, 0, 0], [0, 3.0, 0]])
    ei = torch.tensor([[0, 1, 1, 2], [1, 0, 2, 1]])
    dist, angle, i, j, idx_kj, idx_ji = xyz_to_dat(pos, ei, 3)
    assert torch.allclose(angle, torch.full((2,), math.pi / 2))


def test_oracle_torsion_gradient_matches_finite_differences():
    """The torsion gradient restatement (arg routing of torch_scatter's scatter_min) has the
    same values as xyz_to_dat and, in fp64 on a small graph, its Jacobian equals central finite
    differences wherever the winning candidate does not change under the step (the k_n = k
    candidate's torsion is a rounding residual whose sign flips under any perturbation, so
    entries that jump are not derivatives)."""
    from oracle.triplets import torsion_with_scatter_min_grad
    g = torch.Generator().manual_seed(5)
    pos = (torch.rand(24, 3, generator=g) * 2.5).double()
    d = torch.cdist(pos, pos)
    ei = torch.nonzero((d < 1.3) & (d > 0)).T.flip(0).contiguous()
    t0 = torsion_with_scatter_min_grad(pos, ei, 24)
    assert torch.equal(t0, xyz_to_dat(pos, ei, 24, use_torsion=True)[2])
    J = torch.autograd.functional.jacobian(
        lambda p: torsion_with_scatter_min_grad(p, ei, 24), pos).reshape(t0.numel(), -1)
    h = 1e-6
    n_ok = 0
    for q in range(pos.numel()):
        pp, pm = pos.clone().view(-1), pos.clone().view(-1)
        pp[q] += h
        pm[q] -= h
        tp = torsion_with_scatter_min_grad(pp.view(24, 3), ei, 24)
        tm = torsion_with_scatter_min_grad(pm.view(24, 3), ei, 24)
        ok = ((tp - t0).abs() < 1e-4) & ((tm - t0).abs() < 1e-4) & (t0.abs() > 1e-9)
        fd = (tp - tm) / (2 * h)
        assert torch.allclose(J[ok, q], fd[ok], rtol=1e-4, atol=1e-5), q
        n_ok += int(ok.sum())
    assert n_ok > 0.5 * J.numel() * 0.5  # most entries checked
