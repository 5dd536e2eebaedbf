"""GPU radius graph (K9, gmp_radius_*) against the CPU oracle
(oracle/radius.py): edge_index bit-exact, including order."""
import numpy as np
import pytest
import torch

from oracle.radius import radius_graph as oradius, radius_graph_uncapped_kdtree

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gpu(pos, r, batch=None, k=32):
    from gmp_amd.graph import radius_graph_gpu
    b = None if batch is None else torch.as_tensor(batch).to(DEV)
    return radius_graph_gpu(torch.as_tensor(pos).to(DEV), r, b, max_num_neighbors=k).cpu().numpy()


@pytest.mark.parametrize("n,box,r,k", [(1, 1.0, 0.5, 32), (2, 1.0, 5.0, 32), (500, 6.0, 1.5, 0),
                                       (2000, 10.0, 2.0, 32), (2000, 10.0, 2.0, 4),
                                       (3000, 30.0, 1.0, 0)])
def test_radius_random(n, box, r, k):
    rng = np.random.default_rng(n + k)
    pos = (rng.random((n, 3)) * box - box / 3).astype(np.float32)
    assert np.array_equal(_gpu(pos, r, k=k), oradius(pos, r, max_num_neighbors=k))


def test_radius_empty():
    assert _gpu(np.zeros((0, 3), np.float32), 1.0).shape == (2, 0)


@pytest.mark.parametrize("k", [0, 3, 32])
def test_radius_batched_molecules(k):
    # 64 small "molecules" overlapping around the origin, QM9-like sizes and the SchNet cutoff
    rng = np.random.default_rng(7)
    sizes = rng.integers(3, 30, 64)
    pos = np.concatenate([rng.normal(0, 1.5, (s, 3)) for s in sizes]).astype(np.float32)
    batch = np.repeat(np.arange(64), sizes)
    assert np.array_equal(_gpu(pos, 10.0, batch, k), oradius(pos, 10.0, batch, k))


def test_radius_degenerate_inputs():
    rng = np.random.default_rng(1)
    # duplicates (distance 0), a flat sheet, points on exact cell/cutoff boundaries
    pos = np.concatenate([np.zeros((20, 3)), np.repeat(rng.random((5, 3)), 4, 0),
                          np.c_[rng.random((200, 2)) * 5, np.zeros(200)],
                          np.stack(np.meshgrid(*[np.arange(4.0)] * 3), -1).reshape(-1, 3)])
    pos = pos.astype(np.float32)
    for k in (0, 5):
        for r in (1.0, 1.5):
            assert np.array_equal(_gpu(pos, r, k=k), oradius(pos, r, max_num_neighbors=k))


def test_radius_sparse_wide_box():
    # few nodes spread over a huge box: the cell table is capped, cells grow beyond r
    rng = np.random.default_rng(2)
    pos = (rng.random((300, 3)) * 1e4).astype(np.float32)
    pos[150:] = pos[:150] + rng.normal(0, 0.3, (150, 3)).astype(np.float32)
    assert np.array_equal(_gpu(pos, 1.0, k=0), oradius(pos, 1.0, max_num_neighbors=0))


def test_radius_benchmark_size():
    # the synthetic benchmark graph size (50k nodes, ~1M edges), uncapped: exact vs cKDTree+fp32
    from gmp_amd.graph import radius_graph as synth
    g = synth(num_nodes=50_000, target_edges=1_000_000)
    pos = g.pos.numpy()
    got = _gpu(pos, 5.0, k=0)
    want = radius_graph_uncapped_kdtree(pos, 5.0)
    assert got.shape[1] > 900_000
    assert np.array_equal(got, want)
