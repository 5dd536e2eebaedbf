"""Time the device radius graph (K9) and triplet featurisation (K11) on the benchmark-size graph (50k nodes, ~1M edges) and on a
batch of QM9-sized molecules; the scipy cKDTree builder (host input synthesis) beside it."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "geometric-message-passing_amd"))
from gmp_amd.graph import radius_graph, radius_graph_gpu, radius_edges  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


g = radius_graph(num_nodes=50_000, target_edges=1_000_000)
pos = g.pos.cuda()
ms, ei = timeit(lambda: radius_graph_gpu(pos, 5.0, max_num_neighbors=0))
t = time.perf_counter()
radius_edges(g.pos.numpy(), 5.0)
cpu = (time.perf_counter() - t) * 1e3
print(f"radius 50k nodes / {ei.shape[1]} edges: gpu {ms:.3f} ms (host syncs incl.), "
      f"scipy cKDTree {cpu:.1f} ms")
rng = np.random.default_rng(0)
sizes = rng.integers(9, 29, 1024)
mpos = torch.from_numpy(np.concatenate([rng.normal(0, 1.5, (s, 3)) for s in sizes])
                        .astype(np.float32)).cuda()
mb = torch.from_numpy(np.repeat(np.arange(1024), sizes)).cuda()
ms, ei = timeit(lambda: radius_graph_gpu(mpos, 10.0, mb, 32, num_graphs=1024))
print(f"radius 1024 molecules / {mpos.shape[0]} atoms / {ei.shape[1]} edges, r=10, k=32: "
      f"gpu {ms:.3f} ms")

from gmp_amd.triplets import xyz_to_dat  # noqa: E402

ei = g.edge_index.cuda()
for tors in (False, True):
    ms, out = timeit(lambda: xyz_to_dat(pos, ei, pos.shape[0], use_torsion=tors), reps=10)
    T = out[1].numel()
    print(f"triplets 50k nodes / {ei.shape[1]} edges -> {T} triplets, torsion={tors}: "
          f"gpu {ms:.3f} ms ({T / ms / 1e6:.2f} G triplets/s)")
