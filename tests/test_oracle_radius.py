"""Known-answer tests pinning the radius-graph oracle (oracle/radius.py).
torch_cluster is not importable here: these cases fix the rules the oracle restates — strict
`<` cutoff, per-graph neighbourhoods, ascending-source order, torch_cluster's
max_num_neighbors + 1 (self included) cap — and check the brute-force and cKDTree forms agree."""
import numpy as np

from oracle.radius import radius_graph, radius_graph_uncapped_kdtree


def _pairs(ei):
    return sorted(zip(ei[0].tolist(), ei[1].tolist()))


def test_chain_known_answer():
    pos = np.array([[0, 0, 0], [1, 0, 0], [2, 0, 0], [3.5, 0, 0]], np.float32)
    ei = radius_graph(pos, 1.5)
    assert _pairs(ei) == [(0, 1), (1, 0), (1, 2), (2, 1)]
    # sorted by (target, source)
    assert ei[1].tolist() == [0, 1, 1, 2] and ei[0].tolist() == [1, 0, 2, 1]


def test_strict_cutoff():
    pos = np.array([[0, 0, 0], [2, 0, 0]], np.float32)
    assert radius_graph(pos, 2.0).shape == (2, 0)  # |d| == r is not an edge
    assert radius_graph(pos, np.nextafter(np.float32(2), np.float32(3))).shape == (2, 2)


def test_batch_separates_graphs():
    pos = np.zeros((4, 3), np.float32)  # all coincident
    batch = np.array([0, 0, 1, 1])
    assert _pairs(radius_graph(pos, 1.0, batch)) == [(0, 1), (1, 0), (2, 3), (3, 2)]


def test_max_num_neighbors_rule():
    pos = np.zeros((10, 3), np.float32)  # everyone within r of everyone
    ei = radius_graph(pos, 1.0, max_num_neighbors=3)
    for i in range(10):
        srcs = ei[0][ei[1] == i].tolist()
        # first 4 candidates in ascending order, self included, then self dropped
        want = [j for j in range(4) if j != i]
        assert srcs == want, (i, srcs)
    assert (ei[1] == 9).sum() == 4  # target outside the kept prefix keeps k + 1 sources


def test_uncapped_equals_kdtree():
    rng = np.random.default_rng(3)
    pos = (rng.random((600, 3)) * 8).astype(np.float32)
    batch = np.sort(rng.integers(0, 3, 600))
    a = radius_graph(pos, 1.7, batch, max_num_neighbors=0)
    b = radius_graph_uncapped_kdtree(pos, 1.7, batch)
    assert np.array_equal(a, b)
