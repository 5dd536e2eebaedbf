"""The RCCL code path executed on the box: a one-rank "nccl" process group
(`gmp_amd.dist.init`'s device_id branch; RCCL on ROCm) in a spawned child process, running the
bench's collectives on device tensors -- `GraphedStep._allreduce` (parameter broadcast, the flat
gradient all-reduce between the forward/backward graph and the optimizer graph), `max_over_ranks`
and `sum_over_ranks` -- so the first multi-GPU run does not meet this code for the first time.

At world size 1 the all-reduce of the flat gradient buffer and the division by 1 are exact, so
the gradients and parameters after each step must be BITWISE those of the same steps without a
process group (computed in the same child before the group is created).  SURVEY §8(e)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_steps(use_graph, n_steps=2):
    import gmp_amd
    from gmp_amd.graph import Batch, radius_graph
    from gmp_amd.step import GraphedStep
    dev = torch.device("cuda", 0)
    g = radius_graph(num_nodes=300, target_edges=4000, r=2.5, seed=3, tol=0.2, shuffle=True)
    torch.manual_seed(0)
    model = gmp_amd.EGNNModel(num_layers=2, emb_dim=128, in_dim=1, out_dim=1).to(dev)
    b = Batch(g.atoms.to(dev), g.pos.to(dev), g.edge_index.to(dev), g.batch.to(dev),
              num_graphs=1)
    y = torch.tensor([0.25], device=dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=use_graph)

    def loss_fn():
        return torch.nn.functional.l1_loss(model(b).view(-1), y, reduction="sum")

    step = GraphedStep(model, loss_fn, opt, warmup=1, use_graph=use_graph)
    grads = []
    for _ in range(n_steps):
        step()
        torch.cuda.synchronize()
        grads.append([p.grad.detach().clone() if p.grad is not None else None
                      for p in model.parameters()])
    params = [p.detach().clone() for p in model.parameters()]
    return step, grads, params


def _worker(port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from gmp_amd import dist as gdist
    res = {}
    torch.cuda.set_device(0)
    ref = {m: _run_steps(m) for m in (False, True)}  # no process group
    rank, world, local = gdist.init("nccl", force=True)
    assert dist.is_initialized() and dist.get_backend() == "nccl"
    assert (rank, world, local) == (0, 1, 0)
    dev = torch.device("cuda", 0)
    for use_graph in (False, True):
        step, grads, params = _run_steps(use_graph)
        assert step.world == 1
        _, rgrads, rparams = ref[use_graph]
        res[f"grads_equal_{use_graph}"] = all(
            (a is None and b is None) or (a is not None and b is not None and torch.equal(a, b))
            for ga, gb in zip(grads, rgrads) for a, b in zip(ga, gb))
        res[f"params_equal_{use_graph}"] = all(torch.equal(a, b)
                                              for a, b in zip(params, rparams))
    res["max"] = gdist.max_over_ranks(3.25, dev)
    res["sum"] = gdist.sum_over_ranks(999_722, dev)
    t = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    dist.all_reduce(t)
    res["allreduce_identity"] = bool(torch.equal(t, torch.arange(1 << 20, dtype=torch.float32,
                                                                 device=dev)))
    gdist.barrier()
    dist.destroy_process_group()
    torch.save(res, out_path)


def test_rccl_one_rank_collectives_on_device():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.pt")
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=_worker, args=(port, out))
        p.start()
        p.join(240)
        if p.is_alive():
            p.kill()
            pytest.fail("RCCL worker timed out")
        assert p.exitcode == 0, f"RCCL worker exit code {p.exitcode}"
        res = torch.load(out, weights_only=True)
    assert res["max"] == 3.25 and res["sum"] == 999_722
    assert res["allreduce_identity"]
    for k in ("grads_equal_False", "params_equal_False", "grads_equal_True", "params_equal_True"):
        assert res[k], k
