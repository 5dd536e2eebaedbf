"""Multi-process data-parallel path of the PRODUCT models on the GPU: two gloo
ranks share the one MI355X (spawned child processes; the parent pytest process touches no
device tensor), each owning one graph, through

* the bench's executor (gmp_amd/step.py GraphedStep, eager launch): parameter broadcast from
  rank 0, HIP forward/backward with the weight gradients deferred to the side stream, ONE flat
  all-reduce of the gradients, fused Adam;
* DDP (gmp_amd/dist.wrap_ddp: deferral switched off so the reducer's per-parameter hooks see
  every gradient through autograd, find_unused_parameters for the readout slices).

The averaged gradients of BOTH steps (what the collective delivered to the optimizer, read
before Adam uses them) must equal those of a single process that averages the gradients of the
same two graphs (rank 0 computes that reference in its own process after the collective part),
within 1e-5 of each gradient's scale (step 1 measured bitwise equal — the all-reduce sums two
per-rank gradients exactly as the single process accumulates them; scaling by 1/2 is exact;
step 2 against the single process's gradient at the run's own step-1 parameters).  Parameters after one Adam step: 1e-6; after two:
1e-5 for the executor.  (the r04 DDP check compared post-Adam parameters, where
Adam's per-coordinate normalisation amplifies last-bit gradient differences at near-zero
coordinates, with a near-vacuous bound; the gradients are the quantity the data-parallel path
must get right.)
Multi-GPU scaling itself is unmeasured on hardware here (the driver owns 8-GPU runs)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = {
    "egnn": dict(num_layers=2, emb_dim=128, in_dim=1, out_dim=1),
    "tfn": dict(num_layers=2, emb_dim=16, mlp_dim=64, r_max=2.5, in_dim=1, out_dim=1),
    # config C5's per-rank model at its widths (tfn.py:51-60 defaults: 64 channels, radial
    # hidden 256, 5 layers, gated): the K7g path GEMMs and the 307 MB-class gradient all-reduce
    "tfn_c5": dict(num_layers=5, emb_dim=64, mlp_dim=256, r_max=2.5, in_dim=1, out_dim=1),
}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph(rank):
    from gmp_amd.graph import radius_graph
    g = radius_graph(num_nodes=250, target_edges=3000, r=2.5, seed=10 + rank, tol=0.2,
                     shuffle=True)
    n = g.num_nodes  # the reference scatters have no dim_size: the last node must receive
    extra = torch.tensor([[n - 2, n - 1], [n - 1, n - 2]])
    g.edge_index = torch.cat([g.edge_index, extra], 1)
    return g


def _model(kind):
    import gmp_amd
    torch.manual_seed(0)
    cls = {"egnn": gmp_amd.EGNNModel, "tfn": gmp_amd.TFNModel, "tfn_c5": gmp_amd.TFNModel}[kind]
    return cls(**CASES[kind])


def _loss(model, b, y):
    return torch.nn.functional.l1_loss(model(b).view(-1), y, reduction="sum")


def _rank_worker(rank, world, port, out_dir, kind, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from gmp_amd import dist as gdist
    from gmp_amd import ops
    from gmp_amd.step import GraphedStep
    gdist.init("gloo")
    dev = torch.device("cuda", 0)  # both ranks on the one GPU of the box
    torch.cuda.set_device(dev)
    y = torch.tensor([0.25], device=dev)
    if mode == "ddp":
        torch.manual_seed(rank)
        model = _model(kind).to(dev)
        if rank != 0:  # a different init on rank 1: DDP must broadcast rank 0's
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(0.01)
        model = gdist.wrap_ddp(model, local=0)
        assert not ops.DEFER_WEIGHT_GRADS
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        b = _graph(rank).to(dev)
        for it in range(2):
            opt.zero_grad(set_to_none=True)
            _loss(model, b, y).backward()
            gr = {k: p.grad.detach().cpu() for k, p in model.module.named_parameters()
                  if p.grad is not None}
            if it == 0:
                grads = gr
            else:
                grads2 = gr
            opt.step()
            if it == 0:
                params1 = {k: p.detach().cpu() for k, p in model.module.named_parameters()}
        params = {k: p.detach().cpu() for k, p in model.module.named_parameters()}
    else:
        model = _model(kind).to(dev)
        if rank != 0:  # the executor must broadcast rank 0's parameters
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(0.01)
        assert ops.DEFER_WEIGHT_GRADS
        opt = torch.optim.Adam(model.parameters(), lr=1e-2, fused=True)
        b = _graph(rank).to(dev)
        step = GraphedStep(model, lambda: _loss(model, b, y), opt, warmup=0, use_graph=False)
        for it in range(2):
            step()
            torch.cuda.synchronize()
            # p.grad after the step holds the all-reduced gradient Adam consumed
            gr = {k: p.grad.detach().cpu() for k, p in model.named_parameters()
                  if p.grad is not None}
            if it == 0:
                grads = gr
                params1 = {k: p.detach().cpu() for k, p in model.named_parameters()}
            else:
                grads2 = gr
        torch.cuda.synchronize()
        params = {k: p.detach().cpu() for k, p in model.named_parameters()}
    torch.save({"params": params, "params1": params1, "grads": grads, "grads2": grads2},
               os.path.join(out_dir, f"{mode}{rank}.pt"))
    torch.distributed.destroy_process_group()
    if rank == 0:
        own_params1 = params1
        # single-process reference on the same GPU: mean of the two graphs' gradients
        ops.DEFER_WEIGHT_GRADS = mode != "ddp"
        ref = _model(kind).to(dev)
        opt = torch.optim.Adam(ref.parameters(), lr=1e-2, fused=(mode != "ddp"))
        graphs = [_graph(r).to(dev) for r in range(world)]
        for it in range(2):
            opt.zero_grad(set_to_none=True)
            for g in graphs:
                (_loss(ref, g, y) / world).backward()
            for p in ref.parameters():  # the executor all-reduces zeros for unused parameters
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            torch.cuda.synchronize()
            gr = {k: p.grad.detach().cpu() for k, p in ref.named_parameters()}
            if it == 0:
                grads = gr
            else:
                grads2 = gr
            opt.step()
            if it == 0:
                torch.cuda.synchronize()
                params1 = {k: p.detach().cpu() for k, p in ref.named_parameters()}
        torch.cuda.synchronize()
        # step 2's reference gradient at THIS run's parameters after step 1 (rank 0's; the
        # ranks hold the same ones): the collective and the backward path are then checked at
        # 1e-5, independent of how Adam amplified last-bit differences of step 1
        at = _model(kind).to(dev)
        with torch.no_grad():
            for k, p in at.named_parameters():
                p.copy_(own_params1[k])
        for g in graphs:
            (_loss(at, g, y) / world).backward()
        torch.cuda.synchronize()
        grads2_at = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach().cpu()
                     for k, p in at.named_parameters()}
        torch.save({"params": {k: p.detach().cpu() for k, p in ref.named_parameters()},
                    "params1": params1, "grads": grads, "grads2": grads2,
                    "grads2_at": grads2_at},
                   os.path.join(out_dir, f"{mode}_ref.pt"))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("kind", ["egnn", "tfn", "tfn_c5"])
@pytest.mark.parametrize("mode", ["step", "ddp"])
def test_product_world2_gloo_on_gpu_matches_single_process(kind, mode):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank_worker, args=(world, _free_port(), d, kind, mode),
                           nprocs=world, start_method="spawn", join=True)
        res = [torch.load(os.path.join(d, f"{mode}{r}.pt"), weights_only=True)
               for r in range(world)]
        ref = torch.load(os.path.join(d, f"{mode}_ref.pt"), weights_only=True)
    # both steps' averaged gradients (what the collective delivered to the optimizer), 1e-5 of
    # each gradient's scale: step 1 against the single process's, step 2 against the single
    # process's gradient at the run's own step-1 parameters (grads2_at; the two-step reference's
    # second gradient differs from it by up to 3e-5 of scale under DDP, measured r05: step-1
    # parameters agree only to 1e-6 and the EGNN / TFN heads amplify that)
    bad = []
    for step_key, ref_key in (("grads", "grads"), ("grads2", "grads2_at")):
        tol = 1e-5
        for k, g in ref[ref_key].items():
            for r in range(world):
                got = res[r][step_key].get(k, torch.zeros_like(g))
                err, scale = (got - g).abs().max().item(), g.abs().max().item()
                print(f"{step_key} {k} rank {r}: max|d| {err:.3e} scale {scale:.3e}")
                if err > tol * scale + 1e-7:
                    bad.append((step_key, k, r, err, scale))
    assert not bad, bad
    # parameters after ONE optimizer step (equal first-step gradients): 1e-6
    for k, p in ref["params1"].items():
        for r in range(world):
            err = (res[r]["params1"][k] - p).abs().max().item()
            assert err <= 1e-6, ("after one step", k, r, err)
    moved = 0
    for k, p in ref["params"].items():
        if mode != "ddp":  # the executor sums in the single process's order: 1e-5 after two steps
            for r in range(world):
                torch.testing.assert_close(res[r]["params"][k], p, atol=1e-5, rtol=1e-5)
        moved += int(not torch.equal(p, _init_cpu(kind)[k]))
    assert moved > len(ref["params"]) // 2  # the steps really trained (not vacuous)


_INIT = {}


def _init_cpu(kind):
    if kind not in _INIT:
        _INIT[kind] = {k: p.detach().clone() for k, p in _model(kind).named_parameters()}
    return _INIT[kind]
