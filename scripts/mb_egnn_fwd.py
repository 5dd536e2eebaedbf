"""EGNN C2 inference forward micro-driver for profiling (dev tool): build the bench graph and the
4-layer / 128 model once, run `reps` no_grad forwards (default 5) and print the per-region kernel
times (ops timers) of the last ones.  usage: mb_egnn_fwd.py [reps] [train]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
import gmp_amd  # noqa: E402
from gmp_amd import ops  # noqa: E402
from gmp_amd.graph import radius_graph  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
train = len(sys.argv) > 2 and sys.argv[2] == "train"
g = radius_graph(num_nodes=50_000, target_edges=1_000_000, seed=0)
torch.manual_seed(0)
model = gmp_amd.EGNNModel(num_layers=4, emb_dim=128, in_dim=1, out_dim=1).cuda()
b = g.to("cuda")
with torch.set_grad_enabled(train):
    model(b)
    torch.cuda.synchronize()
    ops.KERNEL_TIMERS = {}
    t0 = time.perf_counter()
    for _ in range(reps):
        out = model(b)
        if train:
            out.sum().backward()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
print({"ms_per_pass": round(dt * 1e3, 3),
       **{k: round(ops.kernel_time_ms(k), 4) for k in ops.KERNEL_TIMERS}})
