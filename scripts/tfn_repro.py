"""Repeatability probe (GPU): TFN at C5 widths on a small graph, forward + backward three times in
one process; prints the max |difference| of every gradient between runs (bitwise expected)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometric-message-passing_amd")]


def main():
    import gmp_amd
    from gmp_amd import ops
    from gmp_amd.graph import radius_graph
    ops.DEFER_WEIGHT_GRADS = os.environ.get("DEFER", "1") == "1"
    dev = torch.device("cuda", 0)
    g = radius_graph(num_nodes=250, target_edges=3000, r=2.5, seed=10, tol=0.2, shuffle=True)
    n = g.num_nodes
    g.edge_index = torch.cat([g.edge_index, torch.tensor([[n - 2, n - 1], [n - 1, n - 2]])], 1)
    b = g.to(dev)
    torch.manual_seed(0)
    model = gmp_amd.TFNModel(num_layers=5, emb_dim=64, mlp_dim=256, r_max=2.5, in_dim=1,
                             out_dim=1).to(dev)
    runs = []
    for _ in range(3):
        model.zero_grad(set_to_none=True)
        y = model(b)
        torch.nn.functional.l1_loss(y.view(-1), torch.tensor([0.25], device=dev),
                                    reduction="sum").backward()
        torch.cuda.synchronize()
        runs.append((y.detach().clone(), {k: p.grad.clone() for k, p in model.named_parameters()
                                          if p.grad is not None}))
    worst = 0.0
    for r in runs[1:]:
        print("y diff", (r[0] - runs[0][0]).abs().max().item())
        for k, v in r[1].items():
            d = (v - runs[0][1][k]).abs().max().item()
            worst = max(worst, d)
            if d > 0:
                print(f"  {k}: {d:.3e} (scale {runs[0][1][k].abs().max().item():.3e})")
    print("worst", worst)


if __name__ == "__main__":
    main()
