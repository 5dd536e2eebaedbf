"""Host-side cost of one EGNN training step (GPU box): cProfile over steps of a tiny graph,
where the step is host-bound; prints the top functions by own time and by cumulative time."""
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometric-message-passing_amd")]


def main():
    import gmp_amd
    from gmp_amd.graph import radius_graph
    from gmp_amd.step import GraphedStep
    dev = torch.device("cuda", 0)
    g = radius_graph(num_nodes=500, target_edges=10000, seed=0).to(dev)
    model = gmp_amd.EGNNModel(num_layers=4, emb_dim=128, in_dim=1, out_dim=1).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    y = torch.zeros(1, device=dev)
    step = GraphedStep(model, lambda: torch.nn.functional.l1_loss(model(g).view(-1), y), opt,
                       warmup=0, use_graph=False)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    n = 50
    pr.enable()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    print(f"host time per step: {st.total_tt / n * 1e3:.2f} ms")
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
