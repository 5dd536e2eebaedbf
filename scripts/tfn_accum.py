"""Accumulation probe (GPU): TFN at C5 widths, gradients of two graphs accumulated by two
backward calls vs the sum of the two separately computed gradients (DEFER=1: the weight
gradients deferred to the side stream; DEFER=0 inline)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometric-message-passing_amd")]


def graph(seed):
    from gmp_amd.graph import radius_graph
    g = radius_graph(num_nodes=250, target_edges=3000, r=2.5, seed=seed, tol=0.2, shuffle=True)
    n = g.num_nodes
    g.edge_index = torch.cat([g.edge_index, torch.tensor([[n - 2, n - 1], [n - 1, n - 2]])], 1)
    return g


def main():
    import gmp_amd
    from gmp_amd import ops
    ops.DEFER_WEIGHT_GRADS = os.environ.get("DEFER", "1") == "1"
    kind = os.environ.get("KIND", "tfn_c5")
    dev = torch.device("cuda", 0)
    gs = [graph(10).to(dev), graph(11).to(dev)]
    torch.manual_seed(0)
    if kind == "egnn":
        model = gmp_amd.EGNNModel(num_layers=2, emb_dim=128, in_dim=1, out_dim=1).to(dev)
    else:
        model = gmp_amd.TFNModel(num_layers=5, emb_dim=64, mlp_dim=256, r_max=2.5, in_dim=1,
                                 out_dim=1).to(dev)
    y = torch.tensor([0.25], device=dev)

    def loss(b):
        return torch.nn.functional.l1_loss(model(b).view(-1), y, reduction="sum") / 2

    sep = []
    for b in gs:
        model.zero_grad(set_to_none=True)
        loss(b).backward()
        torch.cuda.synchronize()
        sep.append({k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
    model.zero_grad(set_to_none=True)
    for b in gs:
        loss(b).backward()
    torch.cuda.synchronize()
    worst = 0.0
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        want = sep[0].get(k, 0) + sep[1].get(k, 0)
        d = (p.grad - want).abs().max().item()
        sc = want.abs().max().item()
        worst = max(worst, d / max(sc, 1e-30))
        if d > 1e-6 * sc:
            print(f"  {k}: {d:.3e} (scale {sc:.3e})")
    print("worst relative", worst)


if __name__ == "__main__":
    main()
