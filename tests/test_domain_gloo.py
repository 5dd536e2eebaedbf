"""Spatial domain decomposition with halo exchange (gmp_amd/domain.py) on CPU
with gloo: ONE graph cut into slabs over 2 and 3 ranks, ghost rows exchanged before every layer.
The prediction on every rank and the SUM-reduced parameter gradients must equal the
single-process oracle EGNN on the whole graph.  The model is the CPU oracle (the product kernels
need the MI355X); what is under test is the partition, the exchange and its backward."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from oracle import egnn as oegnn
from oracle.scatter import scatter


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Layer(oegnn.EGNNLayer):
    """oracle EGNNLayer aggregating into one row per input node (dim_size = N): local graphs
    put the ghost nodes (no in-edges) after the owned receivers, and the fused GPU layer
    likewise always returns N rows."""

    def forward(self, h, pos, edge_index):
        j, i = edge_index[0], edge_index[1]
        rel = pos[i] - pos[j]
        m = self.mlp_msg(torch.cat([h[i], h[j], rel.norm(dim=-1, keepdim=True)], dim=-1))
        n = h.shape[0]
        reduce = "sum" if self.aggr in ("add", "sum") else self.aggr
        m_aggr = scatter(m, i, 0, n, reduce)
        p_aggr = scatter(rel * self.mlp_pos(m), i, 0, n, "mean")
        return self.mlp_upd(torch.cat([h, m_aggr], dim=-1)), pos + p_aggr


def _model(pool):
    torch.manual_seed(0)
    m = oegnn.EGNNModel(num_layers=3, emb_dim=16, in_dim=2, out_dim=2, pool=pool)
    m.convs = torch.nn.ModuleList(_Layer(16) for _ in range(3))
    torch.manual_seed(1)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    return m


def _graph():
    from gmp_amd.graph import radius_graph
    g = radius_graph(num_nodes=240, target_edges=4000, r=2.0, seed=7, tol=0.3)
    g.atoms = torch.arange(g.num_nodes) % 2
    return g


def _worker(rank, world, port, pool, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gmp_amd import dist as gdist
    from gmp_amd import domain
    gdist.init("gloo")
    g = _graph()
    model = _model(pool)
    plan = domain.DomainPlan(g.pos, g.edge_index)
    y = domain.egnn_forward(model, g.atoms[plan.owned], g.pos[plan.owned], plan)
    loss = (y * torch.tensor([[0.7, -1.3]])).sum()
    loss.backward()
    domain.allreduce_grads(model.parameters(), replicated=list(model.pred.parameters()))
    torch.save({"y": y.detach(), "grads": {k: p.grad for k, p in model.named_parameters()},
                "n_own": plan.n_own, "n_ghost": plan.n_ghost, "n_edges": plan.edge_index.shape[1]},
               os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_plan_partition_host():
    """Every node owned once, every edge on its receiver's rank, ghost/send lists consistent."""
    from gmp_amd.domain import DomainPlan
    g = _graph()
    W = 3
    plans = [DomainPlan(g.pos, g.edge_index, world=W, rank=r) for r in range(W)]
    owned = torch.cat([p.owned for p in plans])
    assert torch.equal(owned.sort().values, torch.arange(g.num_nodes))
    assert sum(p.edge_index.shape[1] for p in plans) == g.num_edges
    assert torch.equal(torch.cat([p.edge_ids for p in plans]).sort().values,
                       torch.arange(g.num_edges))
    for r, p in enumerate(plans):
        # local edges map back to the global ones
        glob = torch.cat([p.owned, p.ghosts])
        assert torch.equal(glob[p.edge_index], g.edge_index[:, p.edge_ids])
        assert int(p.edge_index[1].max()) < p.n_own  # receivers are owned
        # what q sends to r is exactly r's ghosts owned by q, in r's order
        for q, pq in enumerate(plans):
            if q == r:
                continue
            k0 = sum(pq.send_counts[:r])
            sent = pq.owned[pq.send_idx[k0:k0 + pq.send_counts[r]]]
            r0 = sum(p.recv_counts[:q])
            assert torch.equal(sent, p.ghosts[r0:r0 + p.recv_counts[q]])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,pool", [(2, "sum"), (3, "mean")])
def test_domain_decomposition_matches_single_process(world, pool):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), pool, d), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True)
               for r in range(world)]
    from gmp_amd.graph import Batch
    g = _graph()
    ref = _model(pool)
    y = ref(Batch(g.atoms, g.pos, g.edge_index))
    (y * torch.tensor([[0.7, -1.3]])).sum().backward()
    assert all(r["n_ghost"] > 0 for r in res)  # the cut really crosses edges
    assert sum(r["n_own"] for r in res) == g.num_nodes
    for r in res:
        torch.testing.assert_close(r["y"], y.detach(), atol=1e-5, rtol=1e-5)
        for k, p in ref.named_parameters():
            want = p.grad if p.grad is not None else torch.zeros_like(p)
            torch.testing.assert_close(r["grads"][k], want, atol=1e-5, rtol=1e-4)
