"""Microbenchmark of the MACE-128 forward path contraction at the lo = 2 (and lo = 1) shapes
(50k receivers, ~1M edges, mul1 = mul_out = 128, H = 256): the unfused pair (S kernel + K7g
forward GEMM) against K7s (gmp_tp_node_fwd_fused_f32, S built in-kernel), HIP-event timing,
f32-equivalent TFLOP/s of the contraction (S build + GEMM FLOPs) and the max relative
difference of the two outputs.  Usage (GPU box): python scripts/mb_tpfwd.py [reps] [d3 ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402
from gmp_amd.ops import _p, _stream  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d3s = [int(x) for x in sys.argv[2:]] or [5, 3]
lib = _lib.load()
dev = "cuda"
torch.manual_seed(0)
N, E, m1, mo, H = 50_000, 1_000_000, 128, 128, 256
K1 = m1 * H
DLO, DHI = (int(x) for x in os.environ.get("MB_DEG", "12,28").split(","))
deg = torch.randint(DLO, DHI + 1, (N,))  # default ~20 +- 5 (the radius graph's in-degrees)
if DLO != DHI:
    deg = (deg * (E / deg.sum())).round().long().clamp(min=0)
E = int(deg.sum())
eoff = torch.zeros(N + 1, dtype=torch.int64, device=dev)
eoff[1:] = torch.cumsum(deg, 0).to(dev)
A = torch.relu(torch.randn(E, H, device=dev))
W2 = torch.randn(m1 * mo, H, device=dev) * 0.05
b2 = torch.randn(m1 * mo, device=dev) * 0.05
Bf = torch.empty(3 * mo * (K1 + m1), dtype=torch.int16, device=dev)
lib.gmp_tp_split_w2_f32(m1, mo, H, _p(W2), _p(b2), _p(Bf), None, _stream())


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for d3 in d3s:
    w = m1 * d3
    Z = torch.randn(E + 1, w, device=dev)
    fl = 2 * E * w * H + 2 * N * d3 * (K1 + m1) * mo
    out_u = torch.zeros(N, mo * d3, device=dev)
    out_f = torch.zeros(N, mo * d3, device=dev)
    S = torch.empty(N, w, H, device=dev)
    Sb = torch.empty(N, w, device=dev)

    def unfused():
        lib.gmp_tp_node_outer_f32(N, w, H, _p(eoff), _p(Z), _p(A), _p(S), _p(Sb), _stream())
        lib.gmp_tp_gemm_x3_f32(N * d3, mo, K1, _p(S), K1, m1, _p(Sb), m1, _p(Bf), K1 + m1,
                               mo * (K1 + m1), _p(out_u), d3, mo * d3, 1, d3, 1, _stream())

    U = 16 // d3
    Zf = torch.empty(lib.gmp_tp_z_fused_layout_floats(E + 1, d3, m1), device=dev)
    lib.gmp_tp_z_fused_layout_f32(_p(Z), E + 1, d3, m1, _p(Zf), _stream())

    def fused():
        lib.gmp_tp_node_fwd_fused_f32(N, d3, m1, H, mo, _p(eoff), _p(Zf), E + 1, _p(A), _p(Bf),
                                      _p(out_f), mo * d3, _stream())

    tu = timeit(unfused)
    del S, Sb
    tf = timeit(fused)
    rel = ((out_f - out_u).abs().max() / out_u.abs().max()).item()
    print(f"d3={d3}: unfused {tu:8.3f} ms ({fl / tu / 1e9:6.1f} TF)   fused {tf:8.3f} ms "
          f"({fl / tf / 1e9:6.1f} TF)   max rel diff {rel:.2e}", flush=True)
    tl = timeit(lambda: lib.gmp_tp_z_fused_layout_f32(_p(Z), E + 1, d3, m1, _p(Zf), _stream()))
    print(f"d3={d3}: z layout conversion {tl:8.3f} ms", flush=True)
    del Z, Zf, out_u, out_f
    torch.cuda.empty_cache()
