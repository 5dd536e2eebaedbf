"""World-size-2 data-parallel path on CPU (gloo): graph sharding, DDP gradient all-reduce and
the bench's max-over-ranks timing / summed edge counts (gmp_amd/dist.py).  The model is the CPU
oracle EGNN (the product kernels need the MI355X); what is under test is the sharding and
the collective logic, which bench.py shares."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graphs():
    from gmp_amd.graph import radius_graph
    return [radius_graph(num_nodes=60, target_edges=500, r=2.0, seed=s, tol=0.3) for s in range(4)]


def _loss(model, g):
    y = torch.tensor([0.3, -0.2])
    return torch.nn.functional.l1_loss(model(g).view(-1), y, reduction="sum")


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gmp_amd import dist as gdist
    from oracle import egnn as oegnn
    r, w, _ = gdist.init("gloo")
    assert (r, w) == (rank, world)
    torch.manual_seed(0)
    model = gdist.wrap_ddp(oegnn.EGNNModel(num_layers=2, emb_dim=16, out_dim=2))
    graphs = _graphs()
    mine = gdist.shard(len(graphs), rank, world)
    # gradient accumulation over this rank's graphs (DDP syncs on the last backward)
    loss_sum = 0.0
    for k, gi in enumerate(mine):
        if k < len(mine) - 1:
            with model.no_sync():
                loss = _loss(model, graphs[gi]) / len(mine)
                loss.backward()
        else:
            loss = _loss(model, graphs[gi]) / len(mine)
            loss.backward()
        loss_sum += float(loss)
    # a second step: a DDP reducer that waits on unused parameters fails here
    model.zero_grad()
    for gi in mine:
        with model.no_sync():
            (_loss(model, graphs[gi]) * 0.0).backward()
    model.zero_grad()
    for k, gi in enumerate(mine):
        ctx = model.no_sync() if k < len(mine) - 1 else _null()
        with ctx:
            (_loss(model, graphs[gi]) / len(mine)).backward()
    edges = sum(graphs[gi].num_edges for gi in mine)
    t_max = gdist.max_over_ranks(1.0 + rank)
    e_sum = gdist.sum_over_ranks(edges)
    grads = {k: p.grad.clone() for k, p in model.module.named_parameters() if p.grad is not None}
    torch.save({"grads": grads, "t_max": t_max, "e_sum": e_sum, "mine": mine},
               os.path.join(out_dir, f"rank{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_shard_round_robin():
    from gmp_amd.dist import shard
    assert shard(8, 0, 8) == [0] and shard(8, 3, 8) == [3]
    assert shard(8, 1, 2) == [1, 3, 5, 7] and shard(8, 0, 1) == list(range(8))
    assert sorted(sum((shard(10, r, 4) for r in range(4)), [])) == list(range(10))


@pytest.mark.timeout(300)
def test_ddp_gloo_world2_matches_single_process():
    from oracle import egnn as oegnn
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True)
               for r in range(world)]
    graphs = _graphs()
    assert res[0]["mine"] == [0, 2] and res[1]["mine"] == [1, 3]
    assert res[0]["t_max"] == res[1]["t_max"] == 2.0
    assert res[0]["e_sum"] == sum(g.num_edges for g in graphs)
    # single process: mean over all graphs of the per-graph loss gradients
    torch.manual_seed(0)
    ref = oegnn.EGNNModel(num_layers=2, emb_dim=16, out_dim=2)
    for g in graphs:
        (_loss(ref, g) / len(graphs)).backward()
    for k, p in ref.named_parameters():
        if p.grad is None:  # unused by the loss (last layer's position MLP)
            assert all(k not in res[r]["grads"] or res[r]["grads"][k].abs().max() == 0
                       for r in range(world)), k
            continue
        for r in range(world):
            # DDP averages the ranks' (already per-rank averaged) gradients
            torch.testing.assert_close(res[r]["grads"][k], p.grad, atol=1e-6, rtol=1e-5)


def _step_worker(rank, world, port, out_dir):
    """bench.py's step executor (gmp_amd/step.py) in eager mode: parameter broadcast, one flat
    all-reduce of the gradients, Adam step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from gmp_amd import dist as gdist
    from gmp_amd.step import GraphedStep
    from oracle import egnn as oegnn
    gdist.init("gloo")
    torch.manual_seed(rank)  # different init per rank: the executor must broadcast rank 0's
    model = oegnn.EGNNModel(num_layers=2, emb_dim=16, out_dim=2)
    g = _graphs()[rank]
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    step = GraphedStep(model, lambda: _loss(model, g), opt, warmup=0, use_graph=False)
    for _ in range(2):
        step()
    torch.save({k: p.detach().clone() for k, p in model.named_parameters()},
               os.path.join(out_dir, f"step{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
def test_step_executor_gloo_world2_matches_single_process():
    from oracle import egnn as oegnn
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_step_worker, args=(world, _free_port(), d), nprocs=world,
                           start_method="spawn", join=True)
        res = [torch.load(os.path.join(d, f"step{r}.pt"), weights_only=True)
               for r in range(world)]
    # single process: rank 0's init, gradient = mean over the two ranks' graphs, two Adam steps
    torch.manual_seed(0)
    ref = oegnn.EGNNModel(num_layers=2, emb_dim=16, out_dim=2)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-2)
    graphs = _graphs()
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        for r in range(world):
            (_loss(ref, graphs[r]) / world).backward()
        for p in ref.parameters():  # the executor all-reduces zeros for unused parameters
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        opt.step()
    for k, p in ref.named_parameters():
        for r in range(world):
            torch.testing.assert_close(res[r][k], p.detach(), atol=1e-5, rtol=1e-5)
