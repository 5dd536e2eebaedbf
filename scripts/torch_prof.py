"""Dev tool: torch.profiler op table (CPU-side aten ops with input shapes) for one training step
of a workload, to attribute small copy / cat / elementwise kernels.  usage: torch_prof.py gvp"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
import gmp_amd  # noqa: E402
from gmp_amd.graph import radius_graph  # noqa: E402

W = sys.argv[1] if len(sys.argv) > 1 else "gvp"
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


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
names = ("aten::mm", "aten::addmm", "aten::addmm_", "aten::copy_", "aten::cat", "aten::contiguous", "aten::clone", "aten::zeros",
         "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::mul", "aten::index_select",
         "aten::constant_pad_nd", "aten::sum", "aten::div", "aten::sub")
tab = prof.key_averages(group_by_input_shape=True)
rows = [e for e in tab if e.key in names]
rows.sort(key=lambda e: -e.count)
for e in rows[:45]:
    dt = getattr(e, "device_time_total", 0.0) or getattr(e, "cuda_time_total", 0.0)
    print(f"{e.count:4d} {dt:9.1f}us {e.key:18s} {str(e.input_shapes)[:100]}")
print("--- top ops by self device time (all ops, grouped by input shape)")
allr = [e for e in tab if (getattr(e, "self_device_time_total", 0.0) or 0.0) > 0]
allr.sort(key=lambda e: -e.self_device_time_total)
for e in allr[:50]:
    print(f"{e.count:4d} {e.self_device_time_total:9.1f}us {e.key[:40]:40s} {str(e.input_shapes)[:90]}")
