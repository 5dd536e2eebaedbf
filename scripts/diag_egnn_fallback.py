"""Diagnostic: errors of the EGNN generic (fallback) path against an fp64 oracle, next to the
same oracle model run in fp32 on the CPU and on the GPU (pure torch), per parameter gradient.
Separates our kernels' contribution from the device's library kernels (GEMM, BatchNorm)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "geometric-message-passing_amd")
from oracle import egnn as oegnn  # noqa: E402


def main():
    import gmp_amd
    from gmp_amd.graph import Batch, collate, radius_graph
    dev = "cuda"
    for kw in (dict(norm="batch", aggr="max", emb_dim=96),
               dict(norm="batch", aggr="mean", emb_dim=128, activation="swish"),
               dict(norm="layer", aggr="max", emb_dim=128, pool="mean"),
               dict(norm="layer", aggr="sum", emb_dim=96)):
        torch.manual_seed(11)
        graphs = []
        for s in (21, 22):
            g = radius_graph(num_nodes=200, target_edges=2500, r=2.0, seed=s, tol=0.2,
                             shuffle=True)
            n = g.num_nodes
            if not bool((g.edge_index[1] == n - 1).any()):
                g.edge_index = torch.cat([g.edge_index,
                                          torch.tensor([[n - 2, n - 1], [n - 1, n - 2]])], 1)
            graphs.append(g)
        for gg in graphs:
            gg.atoms = torch.randint(0, 3, (gg.num_nodes,))
        b = collate(graphs)
        kw = dict(kw, num_layers=3, in_dim=3, out_dim=2)
        ref = oegnn.EGNNModel(**kw).train()
        ref64 = copy.deepcopy(ref).double().train()
        refg = copy.deepcopy(ref).to(dev).train()
        model = gmp_amd.EGNNModel(**kw)
        model.load_state_dict(ref.state_dict())
        model = model.to(dev).train()
        runs = {}
        for name, m, dt, d in (("ours", model, torch.float32, dev), ("cpu32", ref, torch.float32,
                                                                     "cpu"),
                               ("gpu32", refg, torch.float32, dev),
                               ("cpu64", ref64, torch.float64, "cpu")):
            bb = Batch(b.atoms.to(d), b.pos.detach().to(d, dt).clone().requires_grad_(True), b.edge_index.to(d),
                       b.batch.to(d), num_graphs=b.num_graphs)
            y = m(bb)
            y.square().sum().backward()
            runs[name] = (y.detach().cpu().double(),
                          {k: (p.grad.detach().cpu().double() if p.grad is not None else None)
                           for k, p in m.named_parameters()},
                          bb.pos.grad.detach().cpu().double())
        print(kw)
        y64, g64, p64 = runs["cpu64"]
        for name in ("ours", "cpu32", "gpu32"):
            y, g, p = runs[name]
            print(f"  {name:6s} y err {(y - y64).abs().max().item():.3e}  dpos rel "
                  f"{(p - p64).abs().max().item() / p64.abs().max().item():.3e}")
        for k in g64:
            if g64[k] is None:
                continue
            sc = g64[k].abs().max().item()
            errs = []
            for name in ("ours", "cpu32", "gpu32"):
                gg = runs[name][1][k]
                gg = gg if gg is not None else torch.zeros_like(g64[k])
                errs.append((gg - g64[k]).abs().max().item() / max(sc, 1e-30))
            if max(errs) > 1e-5:
                print(f"    {k:28s} scale {sc:.2e}  rel ours {errs[0]:.2e}  cpu32 {errs[1]:.2e}"
                      f"  gpu32 {errs[2]:.2e}")


if __name__ == "__main__":
    main()
