"""Radius graph on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py) — SURVEY.md §8(f) f1.

Restates torch_cluster.radius_graph(pos, r, batch, loop=False, max_num_neighbors) as PyG
SchNet's RadiusInteractionGraph builds it (reference models/schnet.py:47; torch_cluster is an
external dependency, not in /root/reference and not importable here, so this is parity
UNPINNED against torch_cluster itself and pinned by the known-answer cases in
tests/test_oracle_radius.py).  Selection rule of torch_cluster's GPU kernel (radius_cuda.cu):
target i scans the nodes j of its graph in ascending order, counts j when dist2 < r*r, stops
after max_num_neighbors + 1 hits (loop=False asks radius() for one extra), and the self pair is
dropped afterwards.  dist2 is evaluated in fp32 as ((dx*dx + dy*dy) + dz*dz), dx = p_i - p_j,
every operation rounded (no fused multiply-add) — the definition the device kernel K9 follows.
Output: (2, E) int64 [sources; targets], sorted by (target, source).
"""
import numpy as np


def _dist2_rows(p, i, js):
    d = p[i][None, :] - p[js]  # float32 - float32 -> float32, rounded per element
    sq = d * d
    return (sq[:, 0] + sq[:, 1]) + sq[:, 2]


def radius_graph(pos, r, batch=None, max_num_neighbors=32):
    p = np.ascontiguousarray(np.asarray(pos, dtype=np.float32))
    n = p.shape[0]
    b = np.zeros(n, np.int64) if batch is None else np.asarray(batch, dtype=np.int64)
    r2 = np.float32(np.float32(r) * np.float32(r))
    k = 0 if max_num_neighbors is None else max(int(max_num_neighbors), 0)
    src, dst = [], []
    for i in range(n):
        js = np.nonzero(b == b[i])[0]  # ascending
        hit = js[_dist2_rows(p, i, js) < r2]
        if k > 0:
            hit = hit[:k + 1]
        hit = hit[hit != i]
        src.append(hit)
        dst.append(np.full(hit.shape[0], i, np.int64))
    if n == 0:
        return np.zeros((2, 0), np.int64)
    return np.stack([np.concatenate(src), np.concatenate(dst)]).astype(np.int64)


def radius_graph_uncapped_kdtree(pos, r, batch=None):
    """Same rule with no neighbour cap, for large N: a scipy cKDTree query at a slightly larger
    radius gives a superset of pairs, which the exact fp32 criterion then filters."""
    from scipy.spatial import cKDTree

    p = np.ascontiguousarray(np.asarray(pos, dtype=np.float32))
    n = p.shape[0]
    r2 = np.float32(np.float32(r) * np.float32(r))
    pairs = cKDTree(p.astype(np.float64)).query_pairs(float(r) * (1 + 1e-4),
                                                      output_type="ndarray")
    a, c = pairs[:, 0], pairs[:, 1]
    src = np.concatenate([a, c])
    dst = np.concatenate([c, a])
    d = p[dst] - p[src]
    sq = d * d
    keep = ((sq[:, 0] + sq[:, 1]) + sq[:, 2]) < r2
    if batch is not None:
        bb = np.asarray(batch, dtype=np.int64)
        keep &= bb[src] == bb[dst]
    src, dst = src[keep], dst[keep]
    order = np.lexsort((src, dst))
    return np.stack([src[order], dst[order]]).astype(np.int64)
