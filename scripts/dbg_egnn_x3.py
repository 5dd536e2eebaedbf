"""Debug (GPU): EGNN layer input gradient with the row GEMMs on x3 vs the library."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometric-message-passing_amd")]


def main():
    import gmp_amd
    from gmp_amd import ops
    from gmp_amd.graph import radius_graph
    dev = torch.device("cuda", 0)
    torch.manual_seed(128)
    g = radius_graph(num_nodes=400, target_edges=6000, r=2.0, seed=128, tol=0.2, shuffle=True)
    lay = gmp_amd.EGNNLayer(128, "relu", "layer", "sum").to(dev)
    h = torch.randn(g.num_nodes, 128, device=dev)
    gh = torch.randn(g.num_nodes, 128, device=dev)
    res = {}
    for mode in ("torch", "x3", "x3"):
        ops.ROW_GEMM = mode
        hd = h.clone().requires_grad_(True)
        pd = g.pos.to(dev).requires_grad_(True)
        ho, po = lay(hd, pd, g.edge_index.to(dev))
        (ho * gh).sum().backward()
        torch.cuda.synchronize()
        if mode in res:
            print("x3 repeat equal:", torch.equal(res[mode][1], hd.grad))
        res[mode] = (ho.detach(), hd.grad.clone())
    for k, name in ((0, "out"), (1, "dh")):
        a, b = res["x3"][k], res["torch"][k]
        d = (a - b).abs()
        print(name, "max", d.max().item(), "scale", b.abs().max().item())
        bad = (d > 1e-5 * b.abs().max()).nonzero()
        print(" bad", bad.shape[0], "rows", bad[:, 0].unique()[:20].tolist(),
              "cols", bad[:, 1].unique()[:20].tolist())
    # the raw GEMM at this shape
    dA = torch.randn(400, 128, device=dev)
    dB = torch.randn(400, 128, device=dev)
    W1 = torch.randn(128, 257, device=dev)
    Wcat = torch.cat([W1[:, :128], W1[:, 128:256]], 0)
    y = ops.linear_x3(dA, dB, Wcat, None, True)
    ref = dA.double() @ W1[:, :128].double() + dB.double() @ W1[:, 128:256].double()
    print("raw gemm err", (y.double() - ref).abs().max().item())


if __name__ == "__main__":
    main()
