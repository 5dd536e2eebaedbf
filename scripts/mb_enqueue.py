"""Host-side launch cost of one bench step: per step, the time the Python thread needs to
enqueue the step (no synchronisation; HIP queues deep enough for one step) against the
synchronised wall time.  Enqueue time close to the wall time means the step is launch-bound.
Usage (GPU box): python scripts/mb_enqueue.py [workload] [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
import bench  # noqa: E402
import gmp_amd  # noqa: E402
from gmp_amd.graph import radius_graph  # noqa: E402
from gmp_amd.step import GraphedStep  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "gvp"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dev = torch.device("cuda", 0)
g = radius_graph(num_nodes=50_000, target_edges=1_000_000, seed=0)
layers = {"egnn": 4, "gvp": 4, "mace": 5, "tfn": 5, "schnet": 4}[w]
emb = {"egnn": 128, "gvp": 128, "mace": 128, "tfn": 64, "schnet": 64}[w]
torch.manual_seed(0)
model = bench.build_model(gmp_amd, w, layers, emb).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True)
batch = g.to(dev)
y = torch.randn(1, device=dev)
step = GraphedStep(model, lambda: torch.nn.functional.l1_loss(model(batch).view(-1), y,
                                                              reduction="sum"),
                   opt, warmup=2, use_graph=False)
for _ in range(3):
    step()
torch.cuda.synchronize()
for _ in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{w}: enqueue {1e3 * (t1 - t0):7.2f} ms  wall {1e3 * (t2 - t0):7.2f} ms", flush=True)
# steady state as in bench.py: no synchronisation between steps
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"{w}: {steps} steps back to back: enqueue {1e3 * (t1 - t0) / steps:7.2f} ms/step  "
      f"wall {1e3 * (t2 - t0) / steps:7.2f} ms/step", flush=True)
# where the step waits: events at the end-of-backward flush on the main stream (before it waits
# for the side stream) and on the side stream, against the step's start and end
from gmp_amd import ops  # noqa: E402

_orig_flush = ops._flush_deferred
marks = []


def _flush_marked():
    if ops._PENDING:
        m = torch.cuda.Event(enable_timing=True)
        m.record(torch.cuda.current_stream())
        s = [torch.cuda.Event(enable_timing=True) for _ in ops._SIDE_STREAMS]
        for e, st in zip(s, ops._SIDE_STREAMS.values()):
            e.record(st)
        marks.append((m, s))
    _orig_flush()


ops._flush_deferred = _flush_marked
for _ in range(steps):
    marks.clear()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    step()
    b.record()
    torch.cuda.synchronize()
    m, s = marks[-1]
    print(f"{w}: main reaches the flush at {a.elapsed_time(m):6.2f} ms, side done at "
          + ", ".join(f"{a.elapsed_time(e):6.2f}" for e in s)
          + f" ms, step end {a.elapsed_time(b):6.2f} ms", flush=True)
