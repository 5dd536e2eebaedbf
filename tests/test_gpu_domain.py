"""Domain decomposition (gmp_amd/domain.py) with the product kernels: the fused
EGNN layers run on each partition's local graph [owned | ghost] (local indices, ghost rows with
no in-edges) and the owned rows are reassembled, layer by layer, for W = 3 emulated ranks in one
process (the exchange itself is covered by tests/test_domain_gloo.py).  Prediction and
parameter gradients must match the whole-graph model; the per-rank weight gradients are
accumulated by the deferred side-stream path (three backward contributions per parameter)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_partitioned_fused_layers_match_whole_graph():
    import gmp_amd
    from gmp_amd.domain import DomainPlan
    from gmp_amd.graph import Batch, radius_graph
    from gmp_amd.scatter import global_add_pool
    torch.manual_seed(3)
    g = radius_graph(num_nodes=3000, target_edges=60_000, r=2.5, seed=11, tol=0.2)
    model = gmp_amd.EGNNModel(num_layers=3, emb_dim=128).to(DEV)
    W = 3
    plans = [DomainPlan(g.pos, g.edge_index, world=W, rank=r).to(DEV) for r in range(W)]
    assert all(p.n_ghost > 0 for p in plans)
    atoms, pos0 = g.atoms.to(DEV), g.pos.to(DEV)

    # whole graph
    y_ref = model(Batch(atoms, pos0, g.edge_index.to(DEV), num_graphs=1))
    y_ref.sum().backward()
    g_ref = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)

    # partitioned: every layer on each rank's local graph, owned rows reassembled
    order = torch.cat([p.owned for p in plans])
    inv = torch.argsort(order)
    h, pos = model.emb_in(atoms), pos0
    for conv in model.convs:
        dhs, ps = [], []
        for p in plans:
            loc = torch.cat([p.owned, p.ghosts])
            dh, pn = conv(h[loc], pos[loc], p.edge_index)
            dhs.append(dh[:p.n_own])
            ps.append(pn[:p.n_own])
        h = h + torch.cat(dhs)[inv]
        pos = torch.cat(ps)[inv]
    batch = torch.zeros(g.num_nodes, dtype=torch.long, device=DEV)
    y = model.pred(global_add_pool(h, batch, 1))
    y.sum().backward()
    torch.testing.assert_close(y, y_ref, atol=1e-4, rtol=1e-5)
    for k, p in model.named_parameters():
        if k not in g_ref:
            continue
        scale = g_ref[k].abs().max().item() + 1e-6
        err = (p.grad - g_ref[k]).abs().max().item()
        assert err <= 1e-4 * scale + 1e-6, f"{k}: {err:.3e} (scale {scale:.3e})"
