"""Benchmark: edges/s forward+backward (one training step) of the geometric message-passing hot
path on MI355X (BASELINE.json metric).

Default (--workload egnn+mace): the two halves of the metric in one run, one JSON line.
`value` is config C2 — EGNN 4 layers, emb_dim 128, one seeded random 3-D radius graph with
50,000 nodes and ~1M directed edges (r = 5, box tuned), synthetic data, random-init weights;
the line's "mace" object is config C4 on the same graph (MACE L_max=2, correlation 3, 128
channels, radial MLP hidden 256, 5 layers) with its own steps, roofline and cpu_baseline.
--workload tfn: config C5's per-GPU shard (TFN L_max=2, 64 channels, 5 layers, gated, same
graph); gvp / schnet: C3 / the C1 model on the C2 graph.
A step = the reference training step (experiments/utils/train_utils.py:128-139): forward,
L1 loss, backward, Adam step (gmp_amd/step.py; weight gradients computed on a side stream and
accumulated at the end of the backward pass).  Weak scaling: every rank owns its own ~1M-edge
graph (seed = rank); gradients are averaged with one flat all-reduce per step (RCCL over
xGMI).  --graph replays the step from a HIP graph instead of launching it eagerly.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (N > 1) without torchrun's environment starts the N rank processes
itself (torch.distributed.run, 127.0.0.1 rendezvous) before this process touches the GPU and exits
with their status; under torchrun, WORLD_SIZE must equal N (else exit status 2).

Rank 0 prints ONE JSON line.  Every `roofline.frac` is ALGORITHMIC work over measured time over
the peak, recomputable from SURVEY §8(d) and the committed profiles/r05_*:
  EGNN  frac = 1,592 B/edge x E / t(egnn_bwd_kernel, HIP events on its stream) / 8 TB/s
  GVP   frac = 2,268 B/edge x 3 (fwd + bwd) x layers x E / t(step) / 8 TB/s
  MACE, TFN  frac = TP-contraction FLOP per step (tp_node_flops) / t(its kernels) / 419.5 TF
                    (the bf16 dense peak / 6: three-plane split products)
and `traffic` = PMC HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, separate passes) of the newest
committed profile, `waste_ratio` = traffic / the algorithmic bytes.  The design's own byte counts
and MFMA fractions are secondary fields.  `cpu_baseline` times the CPU
oracle (oracle/*.py, plain PyTorch on the host cores: the reference's CPU path restated) on a
bounded spatial sample of the same graph, median of the timed steps (CPU_SAMPLE).
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
F16_MFMA_PEAK_TFLOPS = 2516.8   # bf16 / f16 dense MFMA (~2.5 PF, 16x the f32 MFMA)
# f32-equivalent ceilings of the split-operand products: K4's 2-plane f16 form takes 3 MFMA
# products per f32 product, the K7g / wgrad three-plane bf16 form 6
HF2_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 3
X3_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 6
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="egnn+mace+gvp+tfn",
                    help="'+'-joined workloads (egnn, mace, gvp, tfn, schnet); the first is the "
                         "line's value, the others its secondary objects")
    ap.add_argument("--mace-steps", type=int, default=3,
                    help="timed steps of the secondary MACE / TFN workloads")
    ap.add_argument("--mace-warmup", type=int, default=1)
    ap.add_argument("--no-f32-exact", action="store_true",
                    help="skip the egnn_f32_exact leg (EGNN steps with every product on the "
                         "exact f32 MFMA)")
    ap.add_argument("--no-forward", action="store_true",
                    help="skip the forward-only (inference) timing of each workload")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--emb", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--edges", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: OMP_NUM_THREADS = the job's CPU share on "
                         "the GPU box, else the physical cores this process may run on)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step from a HIP graph (measured slower than eager launch "
                         "on ROCm 7 for the EGNN step: off by default)")
    ap.add_argument("--fresh-graph", action="store_true",
                    help="hand the model a new edge_index tensor every step (as a data loader "
                         "would), so the receiver / sender CSRs (K0) are rebuilt inside the "
                         "timed steps instead of coming from the per-graph cache")
    ap.add_argument("--blas", default="default",
                    choices=("default", "hipblaslt", "hipblas"),
                    help="library for the node-level PyTorch GEMMs (torch.backends.cuda."
                         "preferred_blas_library)")
    ap.add_argument("--plumbing", action="store_true",
                    help="launcher / rank / timing path only, on the CPU (gloo) with a small torch "
                         "model in place of the GPU workload (tests/test_bench_launch.py)")
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


def build_model(mod, workload, layers, emb):
    if workload == "egnn":
        return mod.EGNNModel(num_layers=layers, emb_dim=emb, in_dim=1, out_dim=1)
    # r_max = 10 (model default) with radius-5 graphs keeps edges away from the cutoff's fp32
    # cancellation near r_max
    if workload == "mace":
        return mod.MACEModel(num_layers=layers, emb_dim=emb, correlation=3, max_ell=2,
                             mlp_dim=256, in_dim=1, out_dim=1)
    if workload == "schnet":
        return mod.SchNetModel(hidden_channels=emb, in_dim=1, out_dim=1, num_filters=128,
                               num_layers=layers, num_gaussians=50, cutoff=10)
    if workload == "gvp":
        return mod.GVPGNNModel(num_layers=layers, s_dim=emb, v_dim=16, s_dim_edge=32,
                               v_dim_edge=1, in_dim=1, out_dim=1)
    return mod.TFNModel(num_layers=layers, emb_dim=emb, max_ell=2, mlp_dim=256, in_dim=1,
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


def step_traffic(workload):
    """HBM bytes per training step (all kernels) from the newest committed PMC summary
    (profiles/<round>_<workload>_kernels.json with steps_in_trace), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_kernels.json")))
    for path in reversed(files):
        with open(path) as f:
            d = json.load(f)
        steps = d.get("steps_in_trace")
        rows = d["kernels"]
        if not steps or any(r["hbm_read_bytes_per_launch"] is None or
                            r["hbm_write_bytes_per_launch"] is None for r in rows):
            continue
        return (sum(r["calls"] * (r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"])
                    for r in rows) / steps, os.path.basename(path))
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


def egnn_xhat_planes():
    """LayerNorm outputs the EGNN forward saves and the backward reads (ops.EGNN_XHAT_PLANES:
    2 = x_hat1, x_hat2 with x_hat3 recomputed (default), 3 = x_hat1..3)."""
    from gmp_amd import ops
    return ops.EGNN_XHAT_PLANES


def egnn_bwd_bytes_per_edge(d, n_nodes, n_edges, planes=3):
    """HBM bytes per edge the fused EGNN edge backward must move in this design:
    indices 16, pos 24, the forward's saved LayerNorm outputs (`planes` x d x 4; x_hat3 is
    recomputed in the default mode) and rstd (12) read, dpre1..3 (3 x d x 4) and gdiff (12)
    written; per-node rows (g_m_aggr + g_pos_aggr read, dA + dpos_recv written) once per node,
    amortised over the edges.  (Modes 0 / 3 also write the rebuilt x_hat1 (, x_hat2) for the
    weight sums: 2 - planes rows of d x 4.)"""
    per_node = 2 * (d * 4 + 12)
    rebuilt = (2 - planes) * d * 4 if planes < 2 else 0
    return (16 + 24 + planes * d * 4 + 12 + 3 * d * 4 + 12 + rebuilt
            + per_node * n_nodes / n_edges)


# SURVEY §8(d) algorithmic bytes per edge and layer of the EGNN forward (fused minimum: idx 16 +
# pos 24 + h_i, h_j 1,024 + message scatter 512 + pos 12 + count 4)
EGNN_SURVEY_BYTES_PER_EDGE = 1592
# ... and of a GVP layer (2,268 B/edge)
GVP_SURVEY_BYTES_PER_EDGE = 2268


def tp_forward_flops(model, n_nodes, n_edges):
    """Algorithmic FLOPs of the TP convolutions' forward (tp_node_flops' forward share: per layer
    S = 2 E J z_size plus the path GEMMs 2 N J sum_p (2lo+1) mul1 mul_out)."""
    total = 0
    for conv in model.convs:
        pl = conv.plan
        J = conv.fc[0].out_features + 1
        total += 2 * n_edges * J * pl.desc.z_size
        total += 2 * n_nodes * J * sum((2 * i["lo"] + 1) * i["mul1"] * i["mul_out"]
                                       for i in pl.instructions)
    return total


def time_forward(model, batch, reps):
    """Inference forward (no autograd; the kernels save nothing for a backward): average wall
    seconds per pass over `reps` passes after one warm-up pass, synchronised on both sides, with
    the per-kernel timers OFF (their event records sit between the kernels); then `reps` more
    passes with the timers on for the per-region kernel times (ops timers)."""
    from gmp_amd import ops
    with torch.no_grad():
        model(batch)
        torch.cuda.synchronize()
        ops.KERNEL_TIMERS = None
        t0 = time.perf_counter()
        for _ in range(reps):
            model(batch)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        ops.KERNEL_TIMERS = {}
        for _ in range(reps):
            model(batch)
        torch.cuda.synchronize()
    timers = {k: ops.kernel_time_ms(k) * len(v) / reps for k, v in ops.KERNEL_TIMERS.items()}
    ops.KERNEL_TIMERS = None
    return dt, timers


def forward_roofline(workload, model, g, layers, dt, timers):
    """north_star's forward target (>= 50 % of the HBM roofline on EGNN + MACE forward): the
    inference forward's rate and its fraction of 8 TB/s for SURVEY §8(d)'s algorithmic bytes (and,
    for the TP models, of the three-plane MFMA ceiling for the contraction's FLOPs)."""
    E = g.num_edges
    out = {"edges_per_s": E / dt, "ms": dt * 1e3, "mode": "inference (torch.no_grad)"}
    if workload == "egnn":
        algo = EGNN_SURVEY_BYTES_PER_EDGE * E * layers
        k4 = timers.get("egnn_edge_fwd")
        out.update({"survey_bytes_per_edge_layer": EGNN_SURVEY_BYTES_PER_EDGE,
                    "hbm_frac_model": algo / dt / 1e9 / HBM_PEAK_GBS,
                    "k4_fwd_ms_per_layer": None if k4 is None else k4 / layers,
                    "hbm_frac_k4": None if not k4 else
                    EGNN_SURVEY_BYTES_PER_EDGE * E / (k4 / layers * 1e-3) / 1e9 / HBM_PEAK_GBS})
    elif workload in ("mace", "tfn"):
        algo = tp_algorithmic_bytes(model, E) / 3  # the forward's third
        fl = tp_forward_flops(model, g.num_nodes, E)
        t_tp = sum(timers.get(k, 0.0) for k in ("tp_node_S", "tp_node_W"))
        out.update({"survey_bytes": algo, "hbm_frac_model": algo / dt / 1e9 / HBM_PEAK_GBS,
                    "tp_flops": fl, "tp_ms": t_tp,
                    "tp_mfma_frac": (fl / (t_tp * 1e-3) / 1e12 / X3_PEAK_TFLOPS) if t_tp else None,
                    "bound_note": "the TP contraction is MFMA-bound (arithmetic intensity far "
                                  "above the ridge): its MFMA fraction is the binding one"})
    return out


def gvp_flops_per_edge(s, v, se, ve):
    """Reference message-function FLOPs per edge per layer, forward (SURVEY §8(d):
    ~186 kFLOP at s=128, v=16, edge (32, 1)): 3 GVPs of the message function."""
    h0, si0, vi0 = max(2 * v + ve, v), 2 * s + se, 2 * v + ve
    g0 = 3 * vi0 * h0 + (h0 + si0) * s + 3 * h0 * v + s * v
    g1 = 3 * v * v + (v + s) * s + 3 * v * v + s * v
    return 2 * (g0 + 2 * g1)


def egnn_flops_per_edge(d, planes=3):
    """fp32 FLOPs per edge of the two fused edge kernels: the backward's W3^T,
    W2^T products plus the recomputation products of what the forward did not save (W3 for
    x_hat3; W2 as well in mode 0)."""
    gemm = 2 * d * d
    return {"egnn_edge_fwd": 2 * gemm,
            "egnn_edge_bwd": (2 + {3: 0, 2: 1, 1: 1, 0: 2}[planes]) * gemm}


def _atom_type(workload):
    """Synthetic atom type: 0 (in_dim = 1 embeddings), 1 for SchNet, whose Embedding(100) keeps
    row 0 as padding (padding_idx = 0: a zero, gradient-free row)."""
    return 1 if workload == "schnet" else 0


def cpu_info():
    """Host CPU model and the physical cores this process may run on (lscpu-equivalent)."""
    model, cores = None, set()
    try:
        allowed = os.sched_getaffinity(0)
    except AttributeError:  # pragma: no cover
        allowed = set(range(os.cpu_count() or 1))
    try:
        cpu = phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f.read().splitlines() + [""]:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    cpu = int(v)
                elif k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not line.strip() and cpu is not None:
                    if cpu in allowed:
                        cores.add((phys, core, cpu if core is None else None))
                    cpu = phys = core = None
    except OSError:  # pragma: no cover
        pass
    return model, (len(cores) or len(allowed)), len(allowed)


def cpu_threads(args):
    """Threads of the CPU baseline: --cpu-threads, else the job's CPU share (OMP_NUM_THREADS: the
    GPU pool grants a 1-GPU job 16 of the host's cores, which serve all eight GPUs' jobs), else
    every physical core this process may run on."""
    if args.cpu_threads:
        return args.cpu_threads
    env = os.environ.get("OMP_NUM_THREADS")
    _, phys, _ = cpu_info()
    return min(int(env), phys) if env and env.isdigit() and int(env) > 0 else phys


# CPU-baseline samples of the bench graph (bounded: ~10-30 s of CPU work per workload) and the
# timed steps (median): EGNN / GVP / SchNet a slab x < frac * box; MACE / TFN a corner cube of
# frac of the volume.  The reference's TP materialises the per-edge weights (721 KB per edge and
# layer for MACE-128: ~28 TFLOP per step at 20k edges, minutes per step on the CPU), so its sample
# is small; its timing is overhead-light from ~1k edges on (r03 probe: 27 edges/s at 662 edges,
# 64 at 7.3k on 8 threads here).
CPU_SAMPLE = {"egnn": ("slab", 0.2, 5), "gvp": ("slab", 0.1, 5), "schnet": ("slab", 0.1, 5),
              "mace": ("cube", 0.003, 3), "tfn": ("cube", 0.003, 3)}


def cpu_baseline(g, args, workload):
    """Time the CPU oracle (fwd + L1 + bwd + Adam; plain PyTorch on the host cores, the
    reference's torch_scatter / PyG / e3nn CPU path restated) on a bounded spatial sample of
    the bench graph: one warm-up step, then the median of the timed steps (CPU_SAMPLE)."""
    from oracle import egnn as oegnn
    from oracle import gvp as ogvp
    from oracle import mace as omace
    from oracle import schnet as oschnet
    from gmp_amd.graph import Batch

    threads = cpu_threads(args)
    torch.set_num_threads(threads)
    layers, emb = args.layers_of[workload], args.emb_of[workload]
    kind, frac, timed = CPU_SAMPLE[workload]
    if kind == "slab":
        keep = g.pos[:, 0] < g.box * frac
        shape = f"{frac:.0%}-volume spatial slab"
    else:
        keep = (g.pos < g.box * frac ** (1.0 / 3.0)).all(dim=1)
        shape = f"{frac:.1%}-volume corner cube"
    idx = torch.nonzero(keep).view(-1)
    remap = torch.full((g.num_nodes,), -1, dtype=torch.long)
    remap[idx] = torch.arange(idx.numel())
    ei = g.edge_index
    m = keep[ei[0]] & keep[ei[1]]
    sub = Batch(torch.full((idx.numel(),), _atom_type(workload), dtype=torch.long),
                g.pos[idx], remap[ei[:, m]], num_graphs=1)
    torch.manual_seed(0)
    mod = {"egnn": oegnn, "gvp": ogvp, "schnet": oschnet}.get(workload, omace)
    model = build_model(mod, workload, layers, emb)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    y = torch.zeros(1)

    def step():
        opt.zero_grad()
        loss = torch.nn.functional.l1_loss(model(sub).view(-1), y, reduction="sum")
        loss.backward()
        opt.step()

    step()  # warm-up (allocator, thread pool)
    ts = []
    for _ in range(timed):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    cpu_model, phys, logical = cpu_info()
    return {"value": sub.num_edges / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "cpu": cpu_model, "host_cores_visible": {"physical": phys, "logical": logical},
            "step_s": ts,
            "sample": f"oracle/{mod.__name__.split('.')[-1]}.py {workload} {layers}L/{emb} "
                      f"fwd+L1+bwd+Adam (torch {torch.__version__} CPU, {threads} threads = "
                      f"this job's CPU share of the host's {phys} physical cores) on the "
                      f"{shape} of the bench graph ({sub.num_nodes} nodes, {sub.num_edges} "
                      f"edges): 1 warm-up + median of {timed} timed steps, {t:.2f} s/step"}


def tp_node_s_bytes(model, n_nodes, n_edges):
    """HBM bytes the S-build launches (gmp_tp_node_outer_f32) move per training
    step: one launch per (layer, path, receiver chunk), forward and backward recompute; each reads
    its z rows (E w) and hidden radial rows a (E H) once and writes S (N w H) and Sb (N w), fp32.
    S is an intermediate of this design, not algorithmic work: reported beside the roofline."""
    total = 0
    for conv in model.convs:
        H = conv.fc[0].out_features
        for _, w in conv.plan.z_regions:
            total += 2 * 4 * (n_edges * (w + H) + n_nodes * w * (H + 1))
    return total


def tp_algorithmic_bytes(model, n_edges):
    """SURVEY §8(d) minimum HBM bytes of the TP convolutions per training step: per layer and
    edge 16 (indices) + 4 in_dim (sender row) + 36 (Y) + 32 (radial) + 4 out_dim (receiver row),
    9,300 B at a MACE-128 hidden layer; x 3 for forward + backward."""
    return sum(3 * n_edges * (16 + 4 * c.plan.desc.in_dim + 36 + 32 + 4 * c.plan.desc.out_dim)
               for c in model.convs)


# kernels of the node-form TP contraction (the roofline's kernel set; prefixes as rocprofv3
# names them in profiles/<round>_<workload>_kernels.json)
TP_KERNELS = ("tp_node_outer_kernel", "tp_gemm_x3_kernel", "tp_gemm_x3_widen_kernel",
              "outer_sum_x3_kernel", "outer_cols_x3g_kernel", "split_g_kernel",
              "sum_partials_cols", "tp_node_apply", "tp_split_w2_kernel")


def pmc_step(workload):
    """(kernel ms per step of the TP kernel set, HBM bytes per step over every kernel, profile
    file) from the newest committed rocprofv3 summary that records its step count, or None."""
    import glob
    for path in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles",
                                                       f"r*_{workload}_kernels.json")))):
        with open(path) as f:
            d = json.load(f)
        n = d.get("steps_in_trace")
        if not n:
            continue
        rows = d["kernels"]
        tp_ms = sum(r["total_ms"] for r in rows if r["kernel"].startswith(TP_KERNELS)) / n
        if any(r["hbm_read_bytes_per_launch"] is None for r in rows):
            return tp_ms, None, os.path.basename(path)
        hbm = sum(r["calls"] * (r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"])
                  for r in rows) / n
        return tp_ms, hbm, os.path.basename(path)
    return None


def mace_roofline(model, n_nodes, n_edges, timers, counts, n_steps, workload="mace"):
    """Roofline of the MACE / TFN step's dominant work, the receiver-factorised TP contraction
    (S build, K7g path GEMMs, dW2p, apply; ~90 % of the step), against the ceiling
    of the arithmetic it runs: bf16 MFMA dense peak / 6 (three-plane split products) = 419 TF
    f32-equivalent.  achieved = algorithmic FLOP per step (tp_node_flops) / the contraction's
    device time per step, measured with HIP events around its launches inside the timed steps.
    traffic = HBM bytes per step of the whole step from the committed PMC summary
    (FETCH_SIZE x2 + WRITE_SIZE), against SURVEY §8(d)'s algorithmic bytes of the TP
    convolutions (~9.3 KB per edge and hidden layer, x 3 for fwd + bwd): waste_ratio says how
    much of it the S / T intermediates add."""
    fl = tp_node_flops(model, n_nodes, n_edges)
    keys = ("tp_node_S", "tp_node_W", "tp_node_dW", "tp_node_dZA")
    t_tp = sum(timers.get(k, 0.0) for k in keys) / n_steps
    tflops = fl / (t_tp * 1e-3) / 1e12 if t_tp > 0 else 0.0
    algo = tp_algorithmic_bytes(model, n_edges)
    s_bytes = tp_node_s_bytes(model, n_nodes, n_edges)
    s_ms = timers.get("tp_node_S", 0.0) / n_steps
    roof = {"kernel": "TP contraction (K7 S build + K7g path GEMMs + dW2p + apply)",
            "kernel_prefix": list(TP_KERNELS), "bound": "mfma", "achieved": tflops,
            "peak": X3_PEAK_TFLOPS, "unit": "TFLOP/s (f32-equivalent)",
            "frac": tflops / X3_PEAK_TFLOPS,
            "peak_note": "bf16 MFMA dense peak / 6 (three-plane split products)",
            "flops_per_step": fl,
            "flops_formula": "per layer 4 x 2 E J z_size + 3 x 2 N J sum_p (2lo+1) mul1 mul_out "
                             "(J = radial hidden + 1; DESIGN.md §4)",
            "tp_ms_per_step": t_tp,
            "traffic": None, "traffic_unit": "HBM bytes per step (all kernels)",
            "algorithmic_bytes_per_step": algo, "waste_ratio": None,
            "split_ms_per_step": {k: timers.get(k, 0.0) / n_steps for k in keys},
            "s_build": {"hbm_bytes_per_step": s_bytes, "ms_per_step": s_ms,
                        "gbs": s_bytes / (s_ms * 1e-3) / 1e9 if s_ms > 0 else None},
            "tp_node_prep_ms_per_step": timers.get("tp_node_prep", 0.0) / n_steps,
            "tp_node_edge_bwd_ms_per_step": timers.get("tp_node_edge_bwd", 0.0) / n_steps,
            "symmetric_contraction_ms_per_step":
                (timers.get("symmetric_contraction_fwd", 0.0) +
                 timers.get("symmetric_contraction_bwd", 0.0)) / n_steps}
    p = pmc_step(workload)
    if p is not None:
        tp_ms, hbm, src = p
        roof["profile"] = {"source": f"profiles/{src}", "tp_kernel_ms_per_step": tp_ms,
                           "frac_from_profile": fl / (tp_ms * 1e-3) / 1e12 / X3_PEAK_TFLOPS}
        if hbm is not None:
            roof["traffic"], roof["waste_ratio"] = hbm, hbm / algo
    return roof


TIMER_NAMES = {"egnn": {"egnn_edge_fwd", "egnn_edge_bwd"}, "gvp": set(), "schnet": set()}


def run_workload(workload, args, g, rank, world, dev, steps, warmup, exact=False):
    """Build the model, warm up, time `steps` steps (barrier + synchronize on both sides, max
    over ranks); returns the bench record fields of this workload (rank 0) or None."""
    import gmp_amd
    from gmp_amd import dist as gdist
    from gmp_amd import ops
    from gmp_amd.step import GraphedStep

    layers, emb = args.layers_of[workload], args.emb_of[workload]
    if exact:  # every product on the exact f32 MFMA (K4 and the weight-gradient outer sums)
        from gmp_amd import _lib
        prev = (_lib.load().gmp_egnn_set_f32_mfma(1), _lib.load().gmp_wgrad_set_f32_mfma(1))
    torch.manual_seed(0)
    model = build_model(gmp_amd, workload, layers, emb).to(dev)
    # Adam (the reference optimizer, train_utils.py): the fused multi-tensor implementation
    # (one launch per step); capturable (step counter on the device) for HIP-graph replay
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True, capturable=args.graph)
    batch = g.to(dev)
    if _atom_type(workload):
        batch.atoms = torch.full_like(batch.atoms, _atom_type(workload))
    y = torch.randn(1, device=dev)

    def loss_fn():
        if args.fresh_graph:  # a new tensor object: the CSR caches miss, K0 runs every step
            batch.edge_index = batch.edge_index.clone()
        return torch.nn.functional.l1_loss(model(batch).view(-1), y, reduction="sum")

    step = GraphedStep(model, loss_fn, opt, warmup=warmup, use_graph=args.graph)
    # only the regions the roofline reads are timed inside the measured steps
    ops.KERNEL_TIMER_NAMES = TIMER_NAMES.get(workload)
    if not args.graph:
        ops.KERNEL_TIMERS = {}
    gdist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    gdist.barrier()
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
    n_timed = steps if not args.graph else max(1, args.timing_steps)
    totals = {k: timers[k] * len(v) for k, v in ops.KERNEL_TIMERS.items()}
    counts = {k: len(v) for k, v in ops.KERNEL_TIMERS.items()}
    ops.KERNEL_TIMERS = None
    if exact:
        _lib.load().gmp_egnn_set_f32_mfma(prev[0])
        _lib.load().gmp_wgrad_set_f32_mfma(prev[1])
        rec = None
        if rank == 0:
            rec = {"value": total_edges * steps / elapsed, "unit": "edges/s", "steps": steps,
                   "warmup": warmup, "ms_per_step": elapsed / steps * 1e3,
                   "products": "exact f32 MFMA everywhere (gmp_egnn_set_f32_mfma(1), "
                               "gmp_wgrad_set_f32_mfma(1)): the A/B rate of the line's "
                               "split-operand products"}
        del step, opt, model, batch
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        return rec
    fwd = None
    if not args.no_forward:
        ops.KERNEL_TIMER_NAMES = None
        dt, ftimers = time_forward(model, batch, 1 if workload in ("mace", "tfn") else 5)
        fwd = forward_roofline(workload, model, g, layers, dt, ftimers)
    rec = None
    if rank == 0:
        if workload == "egnn":
            planes = egnn_xhat_planes()
            fl = egnn_flops_per_edge(emb, planes)
            ms_fwd, ms_bwd = timers["egnn_edge_fwd"], timers["egnn_edge_bwd"]
            tflops = fl["egnn_edge_bwd"] * g.num_edges / (ms_bwd * 1e-3) / 1e12
            bpe = egnn_bwd_bytes_per_edge(emb, g.num_nodes, g.num_edges, planes)
            gbs = bpe * g.num_edges / (ms_bwd * 1e-3) / 1e9
            from gmp_amd import _lib
            lib = _lib.load()
            f32_mode = lib.gmp_egnn_set_f32_mfma(0)
            lib.gmp_egnn_set_f32_mfma(f32_mode)
            # the f32-equivalent MFMA ceiling of the arithmetic K4 runs: the 2-plane f16 products
            # (default) or the exact f32 MFMA
            peak = FP32_MFMA_PEAK_TFLOPS if f32_mode else HF2_PEAK_TFLOPS
            f_mfma, f_hbm = tflops / peak, gbs / HBM_PEAK_GBS
            # primary: SURVEY §8(d)'s algorithmic bytes, 1,592 B per edge and
            # layer, over this kernel's time at 8 TB/s.  The bytes this design's backward moves
            # (saved x_hat planes, the dpre rows of the weight sums) and its MFMA ceiling are
            # secondary fields; waste_ratio = PMC bytes per launch / the algorithmic bytes.
            algo = EGNN_SURVEY_BYTES_PER_EDGE * g.num_edges
            frac_survey = algo / (ms_bwd * 1e-3) / 1e9 / HBM_PEAK_GBS
            roof = {"kernel": "egnn_edge_bwd", "kernel_prefix": "egnn_bwd_kernel",
                    "bound": "hbm", "achieved": algo / (ms_bwd * 1e-3) / 1e9,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": frac_survey,
                    "algorithmic_bytes_per_launch": algo,
                    "frac_note": "SURVEY §8(d) 1,592 B/edge per layer x E / kernel time / 8 TB/s",
                    "traffic": None, "ms_per_launch": ms_bwd,
                    "design_bytes_per_edge": bpe, "design_gbs": gbs, "design_frac": f_hbm,
                    "flops_per_edge": fl["egnn_edge_bwd"], "mfma_achieved": tflops,
                    "mfma_frac": f_mfma, "mfma_peak": peak, "products": "f32 MFMA" if f32_mode
                    else "f16 MFMA, 2-plane split operands (3 products per f32 product)",
                    "xhat_planes_saved": planes,
                    "fwd_kernel_ms": ms_fwd,
                    "fwd_kernel_tflops": fl["egnn_edge_fwd"] * g.num_edges
                    / (ms_fwd * 1e-3) / 1e12}
        elif workload in ("schnet", "gvp"):
            # no single dominant HIP kernel: whole step against the fp32 MFMA peak
            if workload == "schnet":  # CFConv filter network (50 -> F -> F per edge; K6)
                F = 128
                fl = 3 * 2 * (50 * F + F * F) * layers
            else:
                fl = gvp_flops_per_edge(emb, 16, 32, 1) * 3 * layers
            achieved = fl * g.num_edges / (elapsed / steps) / 1e12
            roof = {"kernel": "whole step (fwd+bwd, all kernels)", "kernel_prefix": "-",
                    "bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                    "traffic": None, "flops_per_edge": fl}
            st = step_traffic(workload)
            if workload == "gvp":
                # primary: SURVEY §8(d)'s algorithmic bytes (2,268 B per edge and
                # layer, x 3 for forward + backward) over the step time at 8 TB/s; the committed
                # PMC bytes per step are `traffic`, waste_ratio = traffic / algorithmic
                algo = GVP_SURVEY_BYTES_PER_EDGE * 3 * layers * g.num_edges
                gbs = algo / (elapsed / steps) / 1e9
                roof = {"kernel": "whole step (fwd+bwd, all kernels)", "kernel_prefix": "-",
                        "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_step": algo,
                        "frac_note": "SURVEY §8(d) 2,268 B/edge per layer x 3 (fwd + bwd) x "
                                     "layers x E / step time / 8 TB/s",
                        "traffic": None, "mfma_achieved": achieved,
                        "mfma_peak": FP32_MFMA_PEAK_TFLOPS,
                        "mfma_frac": achieved / FP32_MFMA_PEAK_TFLOPS, "flops_per_edge": fl}
                if st is not None:
                    roof.update({"traffic": st[0], "waste_ratio": st[0] / algo,
                                 "traffic_note": "PMC HBM bytes per training step (FETCH_SIZE "
                                                 "x2 + WRITE_SIZE) of the committed profile",
                                 "traffic_source": f"profiles/{st[1]}",
                                 "traffic_gbs": st[0] / (elapsed / steps) / 1e9})
        else:
            roof = mace_roofline(model, g.num_nodes, g.num_edges, totals, counts, n_timed,
                                 workload)
        t = None if workload in ("mace", "tfn", "gvp") else pmc_traffic(workload,
                                                                         roof["kernel_prefix"])
        if t is not None:
            roof["traffic"], roof["traffic_source"] = t[0], f"profiles/{t[1]}"
            if "algorithmic_bytes_per_launch" in roof:
                roof["waste_ratio"] = t[0] / roof["algorithmic_bytes_per_launch"]
        rec = {"value": total_edges * steps / elapsed, "unit": "edges/s", "steps": steps,
               "warmup": warmup, "ms_per_step": elapsed / steps * 1e3,
               "workload": f"{WORKLOADS[workload][0]} {layers}L/{emb} radius graph "
                           f"{g.num_nodes} nodes / {g.num_edges} edges per GPU "
                           f"(r={g.radius}, box={g.box:.3f}, seed=rank)",
               "roofline": roof, "forward": fwd, "cpu_baseline": None}
    del step, opt, model, batch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return rec


def launch_ranks(args):
    """--gpus N: under torchrun (WORLD_SIZE set) the world must be N; without it and N > 1, start
    N rank processes as children (torch.distributed.run, one per GPU, 127.0.0.1 rendezvous) —
    before anything here touches the GPU — and exit with their status."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} ranks were launched",
                  file=sys.stderr, flush=True)
            sys.exit(2)
        return
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.gpus == 1:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def run_plumbing(args):
    """--plumbing: this script's launcher / rank / barrier / max-over-ranks / JSON path on the
    CPU (gloo), with a small torch model stepped by the same executor (GraphedStep, flat
    all-reduce) in place of the GPU workload."""
    from gmp_amd import dist as gdist
    from gmp_amd.step import GraphedStep
    rank, world, _ = gdist.init("gloo")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1))
    x = torch.randn(64, 16, generator=torch.Generator().manual_seed(rank))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    step = GraphedStep(model, lambda: model(x).abs().sum(), opt, warmup=args.warmup,
                       use_graph=False)
    gdist.barrier(cuda=False)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    gdist.barrier(cuda=False)
    elapsed = gdist.max_over_ranks(time.perf_counter() - t0)
    rows = gdist.sum_over_ranks(x.shape[0])
    if rank == 0:
        print(json.dumps({"metric": "plumbing rows/s (CPU, gloo)", "value": rows * args.steps /
                          elapsed, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "config": {"workload": "plumbing", "parallelism": f"dp{world}"}}),
              flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    launch_ranks(args)
    if args.plumbing:
        run_plumbing(args)
        return
    names = args.workload.split("+")
    for w in names:
        if w not in WORKLOADS:
            raise SystemExit(f"bench.py: unknown workload {w!r} (choices: {', '.join(WORKLOADS)})")
    args.layers_of = {w: args.layers or WORKLOADS[w][1] for w in names}
    args.emb_of = {w: args.emb or WORKLOADS[w][2] for w in names}
    from gmp_amd import dist as gdist
    # GMP_DIST_BACKEND=gloo rehearses the multi-process path with several ranks on one GPU
    backend = os.environ.get("GMP_DIST_BACKEND", "nccl")
    rank, world, local = gdist.init(backend)
    if backend != "nccl":
        local = 0
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)
    if args.blas != "default":
        torch.backends.cuda.preferred_blas_library(args.blas)
    from gmp_amd.graph import radius_graph

    g = radius_graph(num_nodes=args.nodes, target_edges=args.edges, seed=rank)
    recs = {}
    for k, w in enumerate(names):
        if k == 0:
            steps, warmup = args.steps, args.warmup
        elif w in ("mace", "tfn"):
            steps = min(args.steps, args.mace_steps)
            warmup = max(1, min(args.warmup, args.mace_warmup))
        else:
            steps, warmup = min(args.steps, 10), max(1, min(args.warmup, 2))
        recs[w] = run_workload(w, args, g, rank, world, dev, steps, warmup)
    exact = None
    if names[0] == "egnn" and not args.no_f32_exact:
        exact = run_workload("egnn", args, g, rank, world, dev, min(args.steps, 5),
                             max(1, min(args.warmup, 2)), exact=True)
    if rank == 0:
        main_rec = recs[names[0]]
        rec = {
            "metric": "edges/sec forward+backward, EGNN & MACE L=2, 1M-edge radius graph, "
                      "1/2/4/8 GPU",
            "value": main_rec["value"],
            "unit": "edges/s",
            "n_gpus": world,
            "steps": main_rec["steps"],
            "warmup": main_rec["warmup"],
            "ms_per_step": main_rec["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "precision": "f32 storage and f32 accumulation throughout; products on split-operand "
                         "MFMA: EGNN K4 and its dW2/dW3 sums 2-plane f16 (22-bit operands), "
                         "the TP GEMMs, the GVP layer GVPs' 128 x 128 products and other "
                         "weight sums 3-plane bf16 (24-bit); "
                         "egnn_f32_exact is the EGNN rate with every product on the exact f32 "
                         "MFMA",
            "data": "synthetic (seeded random radius graph per rank, random-init weights)",
            "config": {"fresh_graph": bool(args.fresh_graph), "workload": main_rec["workload"], "value_is": names[0],
                       "global_batch": world, "parallelism": f"dp{world}",
                       "step": "fwd + L1 loss + bwd + Adam",
                       "launch": "eager" if not args.graph else "hip graph replay",
                       "blas": str(torch.backends.cuda.preferred_blas_library())},
            "roofline": main_rec["roofline"],
            "cpu_baseline": None,
        }
        if exact is not None:
            rec["egnn_f32_exact"] = exact
        rec["forward"] = main_rec.get("forward")
        for w in names[1:]:
            rec[w] = {k: v for k, v in recs[w].items()}
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(g, args, names[0])
            for w in names[1:]:
                rec[w]["cpu_baseline"] = cpu_baseline(g, args, w)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
