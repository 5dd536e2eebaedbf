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
