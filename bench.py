"""Benchmark: edges/s forward+backward (one training step) of the geometric message-passing hot
path on MI355X (BASELINE.json metric).

Workload at N=1 (default, --workload egnn): config C2 — EGNN 4 layers, emb_dim 128, one seeded
random 3-D radius graph with 50,000 nodes and ~1M directed edges (r = 5, box tuned), synthetic
data, random-init weights.  --workload mace: config C4 (MACE L_max=2, correlation 3, 128
channels, 5 layers, same graph); --workload tfn: config C5's per-GPU shard (TFN L_max=2, 64
channels, 5 layers, gated, same graph).
A step = the reference training step (experiments/utils/train_utils.py:128-139): forward,
L1 loss, backward, Adam step (gmp_amd/step.py; weight gradients computed on a side stream and
accumulated at the end of the backward pass).  Weak scaling: every rank owns its own ~1M-edge
graph (seed = rank); gradients are averaged with one flat all-reduce per step (RCCL over
xGMI).  --graph replays the step from a HIP graph instead of launching it eagerly.

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
    ap.add_argument("--workload", choices=("egnn", "gvp", "mace", "tfn", "schnet"),
                    default="egnn")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--emb", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--edges", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--graph", action="store_true",
                    help="replay the step from a HIP graph (measured slower than eager launch "
                         "on ROCm 7 for the EGNN step: off by default)")
    ap.add_argument("--timing-steps", type=int, default=2,
                    help="eager steps after the timed region in which the roofline kernel is "
                         "timed with HIP events (graph mode)")
    return ap.parse_args()


WORKLOADS = {  # name -> (config tag, layers, emb)
    "egnn": ("C2 EGNN", 4, 128),
    "mace": ("C4 MACE L=2 corr=3", 5, 128),
    "tfn": ("C5 TFN L=2 gated (per-GPU shard)", 5, 64),
    "gvp": ("C3 GVP-GNN s=128 v=16 edge=(32,1)", 4, 128),
    # C1's model (SchNet 4L, hidden 64, 128 filters, 50 Gaussians, cutoff 10) on the C2 graph
    "schnet": ("C1-model SchNet hidden=64 filters=128 gaussians=50 cutoff=10", 4, 64),
}


def build_model(mod, args, radius):
    if args.workload == "egnn":
        return mod.EGNNModel(num_layers=args.layers, emb_dim=args.emb, in_dim=1, out_dim=1)
    # r_max = 10 (model default) with radius-5 graphs keeps edges away from the cutoff's fp32
    # cancellation near r_max
    if args.workload == "mace":
        return mod.MACEModel(num_layers=args.layers, emb_dim=args.emb, correlation=3,
                             max_ell=2, in_dim=1, out_dim=1)
    if args.workload == "schnet":
        return mod.SchNetModel(hidden_channels=args.emb, in_dim=1, out_dim=1, num_filters=128,
                               num_layers=args.layers, num_gaussians=50, cutoff=10)
    if args.workload == "gvp":
        return mod.GVPGNNModel(num_layers=args.layers, s_dim=args.emb, v_dim=16, s_dim_edge=32,
                               v_dim_edge=1, in_dim=1, out_dim=1)
    return mod.TFNModel(num_layers=args.layers, emb_dim=args.emb, max_ell=2, in_dim=1,
                        out_dim=1)


def tp_bytes_per_edge(model):
    """Algorithmic HBM bytes per edge per launch of the K7 TP kernels, summed over layers:
    the per-edge weight row (4 * weight_numel) plus the sender row and SH (fwd; bwd also writes
    dW and dx rows)."""
    fwd = bwd = 0
    for conv in model.convs:
        pl = conv.plan
        wn, din = pl.weight_numel, pl.desc.in_dim
        fwd += 4 * (wn + din + 9) + 16
        bwd += 4 * (2 * wn + 2 * din + 18) + 16
    return fwd / len(model.convs), bwd / len(model.convs)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<round>_<workload>_kernels.json, scripts/prof_summary.py: FETCH_SIZE x2 +
    WRITE_SIZE, separate passes), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_kernels.json")))
    for path in reversed(files):
        with open(path) as f:
            rows = json.load(f)["kernels"]
        for r in rows:
            if r["kernel"].startswith(kernel) and r["hbm_read_bytes_per_launch"] is not None \
                    and r["hbm_write_bytes_per_launch"] is not None:
                return (r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"],
                        os.path.basename(path))
    return None


def tp_node_flops(model, n_nodes, n_edges):
    """Algorithmic FLOPs per training step of the receiver-factorised TP convolutions
    (DESIGN.md §K7): per layer, S = sum_e z_e (x) a_e (2 E 257 z_size) and the path GEMMs
    (2 N 257 sum_p (2lo+1) mul1 mul_out); forward 1 x both, backward 3 x S-shaped
    (S recompute, dZ, dA) + 2 x GEMM-shaped (T, dW2)."""
    total = 0
    for conv in model.convs:
        pl = conv.plan
        J = conv.fc[0].out_features + 1
        s_fl = 2 * n_edges * J * pl.desc.z_size
        g_fl = 2 * n_nodes * J * sum((2 * i["lo"] + 1) * i["mul1"] * i["mul_out"]
                                     for i in pl.instructions)
        total += 4 * s_fl + 3 * g_fl
    return total


def egnn_bwd_bytes_per_edge(d, n_nodes, n_edges):
    """Minimum HBM bytes per edge of the fused EGNN edge backward: indices 16,
    pos 24, the forward's saved x_hat1..3 (3 x d x 4) and rstd (12) read, dpre1..3 (3 x d x 4)
    and gdiff (12) written; per-node rows (g_m_aggr + g_pos_aggr read, dA + dpos_recv
    written) once per node, amortised over the edges."""
    per_node = 2 * (d * 4 + 12)
    return 16 + 24 + 3 * d * 4 + 12 + 3 * d * 4 + 12 + per_node * n_nodes / n_edges


def gvp_flops_per_edge(s, v, se, ve):
    """Reference message-function FLOPs per edge per layer, forward (SURVEY §8(d):
    ~186 kFLOP at s=128, v=16, edge (32, 1)): 3 GVPs of the message function."""
    h0, si0, vi0 = max(2 * v + ve, v), 2 * s + se, 2 * v + ve
    g0 = 3 * vi0 * h0 + (h0 + si0) * s + 3 * h0 * v + s * v
    g1 = 3 * v * v + (v + s) * s + 3 * v * v + s * v
    return 2 * (g0 + 2 * g1)


def egnn_flops_per_edge(d):
    """Algorithmic fp32 FLOPs per edge of the two fused edge kernels."""
    gemm = 2 * d * d
    return {"egnn_edge_fwd": 2 * gemm, "egnn_edge_bwd": 2 * gemm}  # bwd: W3^T, W2^T


def _atom_type(args):
    """Synthetic atom type: 0 (in_dim = 1 embeddings), 1 for SchNet, whose Embedding(100) keeps
    row 0 as padding (padding_idx = 0: a zero, gradient-free row)."""
    return 1 if args.workload == "schnet" else 0


def cpu_baseline(g, args):
    """Time the CPU oracle (fwd + L1 + bwd + Adam) on a spatial slab of the same graph."""
    from oracle import egnn as oegnn
    from oracle import mace as omace
    from gmp_amd.graph import Batch

    threads = min(args.cpu_threads, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    if args.workload in ("egnn", "gvp", "schnet"):
        frac = 0.25 if args.workload == "egnn" else 0.1  # slab x < frac * box
        keep = g.pos[:, 0] < g.box * frac
        shape = "spatial slab"
    else:
        # the oracle's TP materialises 4 * weight_numel bytes per edge: a small corner cube
        frac = 0.003
        keep = (g.pos < g.box * frac ** (1.0 / 3.0)).all(dim=1)
        shape = "corner cube"
    idx = torch.nonzero(keep).view(-1)
    remap = torch.full((g.num_nodes,), -1, dtype=torch.long)
    remap[idx] = torch.arange(idx.numel())
    ei = g.edge_index
    m = keep[ei[0]] & keep[ei[1]]
    sub = Batch(torch.full((idx.numel(),), _atom_type(args), dtype=torch.long), g.pos[idx],
                remap[ei[:, m]], num_graphs=1)
    torch.manual_seed(0)
    from oracle import gvp as ogvp
    from oracle import schnet as oschnet
    model = build_model({"egnn": oegnn, "gvp": ogvp, "schnet": oschnet}.get(args.workload, omace),
                        args, g.radius)
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
            "sample": f"oracle {args.workload} {args.layers}x{args.emb} fwd+bwd+Adam on a "
                      f"{frac:.1%}-volume {shape} of the same graph ({sub.num_nodes} nodes, "
                      f"{sub.num_edges} edges), median of 3 steps"}


def main():
    args = parse()
    _, d_layers, d_emb = WORKLOADS[args.workload]
    args.layers = args.layers or d_layers
    args.emb = args.emb or d_emb
    from gmp_amd import dist as gdist
    # GMP_DIST_BACKEND=gloo rehearses the multi-process path with several ranks on one GPU
    backend = os.environ.get("GMP_DIST_BACKEND", "nccl")
    rank, world, local = gdist.init(backend)
    if backend != "nccl":
        local = 0
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)

    import gmp_amd
    from gmp_amd import ops
    from gmp_amd.graph import radius_graph

    g = radius_graph(num_nodes=args.nodes, target_edges=args.edges, seed=rank)
    torch.manual_seed(0)
    model = build_model(gmp_amd, args, g.radius).to(dev)
    core = model
    # Adam (the reference optimizer, train_utils.py): the fused multi-tensor implementation
    # (one launch per step); capturable (step counter on the device) for HIP-graph replay
    opt = (torch.optim.Adam(model.parameters(), lr=1e-4, capturable=True) if args.graph
           else torch.optim.Adam(model.parameters(), lr=1e-4, fused=True))
    batch = g.to(dev)
    if _atom_type(args):
        batch.atoms = torch.full_like(batch.atoms, _atom_type(args))
    y = torch.randn(1, device=dev)

    def loss_fn():
        return torch.nn.functional.l1_loss(model(batch).view(-1), y, reduction="sum")

    # one process per GPU; the step (fwd + L1 + bwd [+ one flat RCCL all-reduce] + Adam) is
    # captured once and replayed (gmp_amd/step.py); --no-graph runs the same sequence eagerly
    from gmp_amd.step import GraphedStep
    step = GraphedStep(model, loss_fn, opt, warmup=args.warmup, use_graph=args.graph)

    barrier = gdist.barrier

    # only the regions the roofline below reads are timed inside the measured steps
    ops.KERNEL_TIMER_NAMES = {"egnn": {"egnn_edge_fwd", "egnn_edge_bwd"}, "gvp": set()}.get(
        args.workload)
    if not args.graph:
        ops.KERNEL_TIMERS = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = gdist.max_over_ranks(elapsed, dev)
    total_edges = gdist.sum_over_ranks(g.num_edges, dev)
    if args.graph:
        # graph replays carry no per-kernel events: time the same kernels in a few eager steps
        ops.KERNEL_TIMERS = {}
        for _ in range(max(1, args.timing_steps)):
            step._eager()
        torch.cuda.synchronize()
    timers = {k: ops.kernel_time_ms(k) for k in list(ops.KERNEL_TIMERS)}
    n_timed_steps = args.steps if not args.graph else max(1, args.timing_steps)
    totals = {k: timers[k] * len(v) for k, v in ops.KERNEL_TIMERS.items()}
    ops.KERNEL_TIMERS = None

    def sum_ms(name):
        return totals.get(name, 0.0)

    if rank == 0:
        if args.workload == "egnn":
            fl = egnn_flops_per_edge(args.emb)
            ms_fwd, ms_bwd = timers["egnn_edge_fwd"], timers["egnn_edge_bwd"]
            tflops = fl["egnn_edge_bwd"] * g.num_edges / (ms_bwd * 1e-3) / 1e12
            bpe = egnn_bwd_bytes_per_edge(args.emb, g.num_nodes, g.num_edges)
            gbs = bpe * g.num_edges / (ms_bwd * 1e-3) / 1e9
            f_mfma, f_hbm = tflops / FP32_MFMA_PEAK_TFLOPS, gbs / HBM_PEAK_GBS
            # both bounds are reported; the primary one is the closer of the two
            if f_mfma >= f_hbm:
                prim = {"bound": "mfma", "achieved": tflops, "peak": FP32_MFMA_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": f_mfma}
            else:
                prim = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": f_hbm}
            roof = {"kernel": "egnn_edge_bwd", **prim,
                    "traffic": None, "ms_per_launch": ms_bwd,
                    "flops_per_edge": fl["egnn_edge_bwd"], "mfma_frac": f_mfma,
                    "bytes_per_edge_min": bpe, "hbm_gbs": gbs, "hbm_frac": f_hbm,
                    "fwd_kernel_ms": ms_fwd,
                    "fwd_kernel_tflops": fl["egnn_edge_fwd"] * g.num_edges
                    / (ms_fwd * 1e-3) / 1e12}
        elif args.workload == "schnet":
            # no single dominant HIP kernel: whole step against the fp32 MFMA peak, counting
            # the CFConv filter network (50 -> F -> F per edge; K6) fwd + 2x bwd per layer
            F = 128
            fl = 3 * 2 * (50 * F + F * F) * args.layers
            achieved = fl * g.num_edges / (elapsed / args.steps) / 1e12
            roof = {"kernel": "whole step (fwd+bwd, all kernels)", "kernel_prefix": "-",
                    "bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                    "traffic": None, "flops_per_edge": fl}
        elif args.workload == "gvp":
            # no single dominant HIP kernel yet (torch GEMMs on gathered rows): whole step
            fl = gvp_flops_per_edge(args.emb, 16, 32, 1) * 3 * args.layers
            achieved = fl * g.num_edges / (elapsed / args.steps) / 1e12
            roof = {"kernel": "whole step (fwd+bwd, all kernels)", "kernel_prefix": "-",
                    "bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                    "traffic": None, "flops_per_edge": fl}
        else:
            # receiver-factorised K7: rocBLAS GEMMs over S / T (timed region "tp_node_gemm"
            # includes the padded gathers) — MFMA-bound; algorithmic flops per step below
            fl = tp_node_flops(core, g.num_nodes, g.num_edges)
            t_gemm = sum(sum_ms(k) for k in ("tp_node_S", "tp_node_W", "tp_node_dW",
                                              "tp_node_dZA")) / n_timed_steps
            achieved = fl / (t_gemm * 1e-3) / 1e12
            roof = {"kernel": "tp_node_gemm", "kernel_prefix": "-", "bound": "mfma",
                    "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": None,
                    "flops_per_step": fl, "tp_node_gemm_ms_per_step": t_gemm,
                    "split_ms_per_step": {k: sum_ms(k) / n_timed_steps for k in
                                          ("tp_node_S", "tp_node_W", "tp_node_dW",
                                           "tp_node_dZA")},
                    "tp_node_prep_ms_per_step": sum_ms("tp_node_prep") / n_timed_steps,
                    "tp_node_edge_bwd_ms_per_step": sum_ms("tp_node_edge_bwd") / n_timed_steps,
                    "symmetric_contraction_ms_per_step":
                        (sum_ms("symmetric_contraction_fwd") +
                         sum_ms("symmetric_contraction_bwd")) / n_timed_steps}
        t = pmc_traffic(args.workload, roof["kernel_prefix"] if "kernel_prefix" in roof
                        else {"egnn_edge_bwd": "egnn_bwd_kernel",
                              "tp_conv_bwd": "tp_bwd_kernel"}[roof["kernel"]])
        if t is not None:
            roof["traffic"], roof["traffic_source"] = t[0], f"profiles/{t[1]}"
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
            "config": {"workload": f"{WORKLOADS[args.workload][0]} {args.layers}L/{args.emb} "
                                   f"radius graph "
                                   f"{g.num_nodes} nodes / {g.num_edges} edges per GPU "
                                   f"(r={g.radius}, box={g.box:.3f}, seed=rank)",
                       "global_batch": world, "parallelism": f"dp{world}",
                       "step": "fwd + L1 loss + bwd + Adam",
                       "launch": "eager" if not args.graph else "hip graph replay"},
            "roofline": roof,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(g, args)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
