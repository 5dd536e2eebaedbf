"""Domain decomposition (gmp_amd/domain.py) with the product kernels.  First:
the fused EGNN layers run on each partition's local graph [owned | ghost] (local indices, ghost rows with
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


# ------------------------------------------------------------------------------------------
# The exchange on device tensors: W gloo ranks spawned on the one GPU, each
# running the product EGNN (K4 message blocks) on its slab of ONE graph through
# gmp_amd.domain.egnn_forward -- halo rows gathered on the device and exchanged every layer, the
# ghost gradients returned along the transposed exchange and summed on the device (segmented
# sum), the readout all-reduced, parameter gradients SUM-reduced -- against the CPU ORACLE EGNN
# on the whole graph (not the HIP whole-graph run).
import os  # noqa: E402
import socket  # noqa: E402
import tempfile  # noqa: E402

import torch.multiprocessing as mp  # noqa: E402

from oracle import egnn as oegnn  # noqa: E402

_G = dict(num_nodes=1500, target_edges=24_000, r=2.2, seed=17, tol=0.2)
_GY = torch.tensor([[0.7, -1.3]])


def _domain_graph():
    from gmp_amd.graph import radius_graph
    g = radius_graph(**_G)
    n = g.num_nodes  # the oracle's aggregate has no dim_size: the last node must receive
    if not bool((g.edge_index[1] == n - 1).any()):
        g.edge_index = torch.cat([g.edge_index, torch.tensor([[n - 2, n - 1], [n - 1, n - 2]])],
                                 1)
    g.atoms = torch.arange(n) % 2
    return g


def _oracle_model(pool):
    torch.manual_seed(0)
    m = oegnn.EGNNModel(num_layers=3, emb_dim=128, in_dim=2, out_dim=2, pool=pool)
    torch.manual_seed(1)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    return m


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _domain_worker(rank, world, port, pool, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    import gmp_amd
    from gmp_amd import dist as gdist
    from gmp_amd import domain
    gdist.init("gloo")
    dev = torch.device("cuda", 0)  # every rank on the one GPU of the box
    torch.cuda.set_device(dev)
    g = _domain_graph()
    model = gmp_amd.EGNNModel(num_layers=3, emb_dim=128, in_dim=2, out_dim=2, pool=pool)
    model.load_state_dict(_oracle_model(pool).state_dict())
    model = model.to(dev)
    plan = domain.DomainPlan(g.pos, g.edge_index).to(dev)
    assert all(c.fused_supported(torch.empty(1, 128, device=dev), torch.empty(1, 3, device=dev))
               for c in model.convs)
    y = domain.egnn_forward(model, g.atoms[plan.owned.cpu()].to(dev),
                            g.pos[plan.owned.cpu()].to(dev), plan)
    (y * _GY.to(dev)).sum().backward()
    domain.allreduce_grads(model.parameters(), replicated=list(model.pred.parameters()))
    torch.cuda.synchronize()
    torch.save({"y": y.detach().cpu(),
                "grads": {k: (p.grad.detach().cpu() if p.grad is not None else None)
                          for k, p in model.named_parameters()},
                "n_own": plan.n_own, "n_ghost": plan.n_ghost},
               os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,pool", [(2, "sum"), (3, "mean")])
def test_domain_decomposition_on_device_vs_oracle(world, pool):
    from gmp_amd.graph import Batch
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_domain_worker, args=(world, _free_port(), pool, d), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True)
               for r in range(world)]
    g = _domain_graph()
    ref = _oracle_model(pool)
    y = ref(Batch(g.atoms, g.pos, g.edge_index))
    (y * _GY).sum().backward()
    assert all(r["n_ghost"] > 0 for r in res)  # the cuts cross edges
    assert sum(r["n_own"] for r in res) == g.num_nodes
    scale_y = y.abs().max().item()
    for r in res:
        err = (r["y"] - y.detach()).abs().max().item()
        assert err <= 1e-5 * max(1.0, scale_y), (err, scale_y)
        for k, p in ref.named_parameters():
            want = p.grad if p.grad is not None else torch.zeros_like(p)
            got = r["grads"][k] if r["grads"][k] is not None else torch.zeros_like(p)
            scale = want.abs().max().item()
            assert (got - want).abs().max().item() <= 1e-4 * scale + 1e-6, k
