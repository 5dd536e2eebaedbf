"""Dev tool: caching-allocator activity per EGNN training step (device mallocs / frees, retries,
stream syncs) — a step that keeps calling hipMalloc / hipFree synchronises the host."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
import gmp_amd  # noqa: E402
from gmp_amd.graph import radius_graph  # noqa: E402

W = sys.argv[1] if len(sys.argv) > 1 else "egnn"
g = radius_graph(num_nodes=50_000, target_edges=1_000_000, seed=0)
dev = torch.device("cuda")
if W == "egnn":
    model = gmp_amd.EGNNModel(num_layers=4, emb_dim=128, in_dim=1, out_dim=1).to(dev)
else:
    model = gmp_amd.GVPGNNModel(num_layers=4, s_dim=128, v_dim=16, s_dim_edge=32, v_dim_edge=1,
                                in_dim=1, out_dim=1).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True)
batch = g.to(dev)
y = torch.randn(1, device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss = torch.nn.functional.l1_loss(model(batch).view(-1), y, reduction="sum")
    loss.backward()
    opt.step()


keys = ["num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams"]
for _ in range(3):
    step()
torch.cuda.synchronize()
s0 = torch.cuda.memory_stats()
t = time.perf_counter()
host = []
for _ in range(10):
    h = time.perf_counter()
    step()
    host.append((time.perf_counter() - h) * 1e3)
torch.cuda.synchronize()
wall = (time.perf_counter() - t) * 1e3 / 10
s1 = torch.cuda.memory_stats()
print({k: s1.get(k, 0) - s0.get(k, 0) for k in keys})
print(f"host per step (ms): {[round(x, 2) for x in host]}  wall per step {wall:.2f} ms")
print(f"reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB")
