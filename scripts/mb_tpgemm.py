"""Microbenchmark of the K7 node-form kernels at the MACE-128 lo = 2 path shape (50k receivers,
~1M edges, mul1 = mul_out = 128, H = 256): S = outer, forward path GEMM (gemm_x3), T GEMM
(gemm_x3_widen), dW2p (outer_sum_cols), apply.  HIP-event timing, TFLOP/s (f32-equivalent) and
GB/s per kernel.  Usage (GPU box): python scripts/mb_tpgemm.py [reps] [only]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402
from gmp_amd.ops import _p, _stream  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
only = sys.argv[2] if len(sys.argv) > 2 else ""
lib = _lib.load()
dev = "cuda"
torch.manual_seed(0)
N, E, m1, mo, H, d3 = 50_000, 1_000_000, 128, 128, 256, 5
w = m1 * d3
K1 = m1 * H
deg = torch.full((N,), E // N, dtype=torch.int64)
eoff = torch.zeros(N + 1, dtype=torch.int64, device=dev)
eoff[1:] = torch.cumsum(deg, 0).to(dev)
Z = torch.randn(E + 1, w, device=dev)
A = torch.relu(torch.randn(E, H, device=dev))
W2 = torch.randn(m1 * mo, H, device=dev) * 0.05
b2 = torch.randn(m1 * mo, device=dev) * 0.05


def timeit(name, fn, flops, bytes_):
    if only and only not in name:
        return
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{name:14s} {ms:8.3f} ms  {flops / ms / 1e9:8.1f} TFLOP/s  {bytes_ / ms / 1e6:8.1f} GB/s",
          flush=True)


S = torch.empty(N, w, H, device=dev)
if only and only not in "outer":  # the S kernel is skipped: time the GEMMs on real values
    S.normal_()
Sb = torch.empty(N, w, device=dev)
timeit("outer", lambda: lib.gmp_tp_node_outer_f32(N, w, H, _p(eoff), _p(Z), _p(A), _p(S), _p(Sb),
                                                   _stream()),
       2 * E * w * H, 4 * (N * w * H + E * (w + H)))
Bf = torch.empty(3 * mo * (K1 + m1), dtype=torch.int16, device=dev)
Bt = torch.empty(3 * K1 * mo, dtype=torch.int16, device=dev)
lib.gmp_tp_split_w2_f32(m1, mo, H, _p(W2), _p(b2), _p(Bf), _p(Bt), _stream())
out = torch.zeros(N, 1152, device=dev)
timeit("fwd_gemm", lambda: lib.gmp_tp_gemm_x3_f32(N * d3, mo, K1, _p(S), K1, m1, _p(Sb), m1,
                                                  _p(Bf), K1 + m1, mo * (K1 + m1), _p(out[:, 512:]),
                                                  d3, 1152, 1, d3, 1, _stream()),
       2 * N * d3 * (K1 + m1) * mo, 4 * N * w * H)
G = torch.randn(N * d3, mo, device=dev)
del S
T = torch.empty(N * d3, K1, device=dev)
timeit("T_gemm", lambda: lib.gmp_tp_gemm_x3_widen_f32(N * d3, K1, mo, _p(G), mo, _p(Bt), mo,
                                                      K1 * mo, _p(T), K1, _stream()),
       2 * N * d3 * K1 * mo, 4 * N * w * H)
dZ = torch.empty(E + 1, w, device=dev)
dA = torch.zeros(E, H, device=dev)
Tb = torch.randn(N, w, device=dev)
timeit("apply", lambda: lib.gmp_tp_node_apply_f32(N, w, H, _p(eoff), _p(Z), _p(A), _p(T), _p(Tb),
                                                  _p(dZ), _p(dA), _stream()),
       4 * E * w * H, 4 * (N * w * H + 2 * E * w + 2 * E * H))
S = T  # same shape: dW2p reads it as S
dW = torch.empty(K1, mo, device=dev)
ws_b = lib.gmp_outer_sum_cols_workspace_size(N * d3, K1, mo)
ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
timeit("dW_cols", lambda: lib.gmp_outer_sum_cols_f32(N * d3, K1, mo, _p(S), K1, _p(G), mo,
                                                     _p(dW), mo, _p(ws), ws_b, _stream()),
       2 * N * d3 * K1 * mo, 4 * N * w * H)
