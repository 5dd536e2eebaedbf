"""Benchmark: edges/s forward+backward (one training step) of the geometric message-passing hot
path on MI355X (BASELINE.json metric).

Workload at N=1: config C2 — EGNN 4 layers, emb_dim 128, one seeded random 3-D radius graph
with 50,000 nodes and ~1M directed edges (r = 5, box tuned), synthetic data, random-init weights.
A step = the reference training step (experiments/utils/train_utils.py:128-139): forward,
L1 loss, backward, Adam step.  Weak scaling: every rank owns its own ~1M-edge graph
(seed = rank) and gradients are all-reduced by DDP (RCCL over xGMI).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel (egnn_edge_bwd, fp32 MFMA
bound), timed with HIP events on the stream it is launched on; `cpu_baseline` times the CPU
oracle (oracle/egnn.py, plain PyTorch on the host cores) on a bounded spatial slab of the same
graph.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "geometric-message-passing_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32 MFMA = f32 vector peak (spec)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--emb", type=int, default=128)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--edges", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def egnn_flops_per_edge(d):
    """Algorithmic fp32 FLOPs per edge of the two fused edge kernels."""
    gemm = 2 * d * d
    return {"egnn_edge_fwd": 2 * gemm, "egnn_edge_bwd": 4 * gemm}


def cpu_baseline(g, args):
    """Time the CPU oracle (fwd + L1 + bwd + Adam) on a spatial slab of the same graph."""
    from oracle import egnn as oegnn
    from gmp_amd.graph import Batch

    threads = min(args.cpu_threads, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    frac = 0.25
    keep = g.pos[:, 0] < g.box * frac
    idx = torch.nonzero(keep).view(-1)
    remap = torch.full((g.num_nodes,), -1, dtype=torch.long)
    remap[idx] = torch.arange(idx.numel())
    ei = g.edge_index
    m = keep[ei[0]] & keep[ei[1]]
    sub = Batch(torch.zeros(idx.numel(), dtype=torch.long), g.pos[idx], remap[ei[:, m]],
                num_graphs=1)
    torch.manual_seed(0)
    model = oegnn.EGNNModel(num_layers=args.layers, emb_dim=args.emb, in_dim=1, out_dim=1)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    y = torch.zeros(1)

    def step():
        opt.zero_grad()
        loss = torch.nn.functional.l1_loss(model(sub).view(-1), y, reduction="sum")
        loss.backward()
        opt.step()

    step()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    return {"value": sub.num_edges / med, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"oracle/egnn.py EGNN {args.layers}x{args.emb} fwd+bwd+Adam on a "
                      f"{frac:.0%} spatial slab of the C2 graph ({sub.num_nodes} nodes, "
                      f"{sub.num_edges} edges), median of 3 steps"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import gmp_amd
    from gmp_amd import ops
    from gmp_amd.graph import radius_graph

    g = radius_graph(num_nodes=args.nodes, target_edges=args.edges, seed=rank)
    torch.manual_seed(0)
    model = gmp_amd.EGNNModel(num_layers=args.layers, emb_dim=args.emb, in_dim=1,
                              out_dim=1).to(dev)
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local],
                                                          bucket_cap_mb=32)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    batch = g.to(dev)
    y = torch.randn(1, device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.l1_loss(model(batch).view(-1), y, reduction="sum")
        loss.backward()
        opt.step()

    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    ops.KERNEL_TIMERS = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
        e = torch.tensor([g.num_edges], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(e)
        total_edges = e.item()
    else:
        total_edges = g.num_edges
    ms_fwd = ops.kernel_time_ms("egnn_edge_fwd")
    ms_bwd = ops.kernel_time_ms("egnn_edge_bwd")
    ops.KERNEL_TIMERS = None

    if rank == 0:
        fl = egnn_flops_per_edge(args.emb)
        achieved = fl["egnn_edge_bwd"] * g.num_edges / (ms_bwd * 1e-3) / 1e12
        rec = {
            "metric": "edges/sec forward+backward, EGNN & MACE L=2, 1M-edge radius graph, "
                      "1/2/4/8 GPU",
            "value": total_edges * args.steps / elapsed,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded random radius graph per rank, random-init weights)",
            "config": {"workload": f"C2 EGNN {args.layers}L/{args.emb} radius graph "
                                   f"{g.num_nodes} nodes / {g.num_edges} edges per GPU "
                                   f"(r={g.radius}, box={g.box:.3f}, seed=rank)",
                       "global_batch": world, "parallelism": f"dp{world}",
                       "step": "fwd + L1 loss + bwd + Adam"},
            "roofline": {"kernel": "egnn_edge_bwd", "bound": "mfma",
                         "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                         "traffic": None, "ms_per_launch": ms_bwd,
                         "flops_per_edge": fl["egnn_edge_bwd"],
                         "fwd_kernel_ms": ms_fwd,
                         "fwd_kernel_tflops": fl["egnn_edge_fwd"] * g.num_edges
                         / (ms_fwd * 1e-3) / 1e12},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(g, args)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
