"""Micro-benchmark of the edge outer-sum kernels (square K5 vs rectangular K5r) on E x d."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for (E, m, n) in [(1_000_000, 128, 128), (1_000_000, 128, 144), (1_000_000, 16, 128),
                  (3_000_000, 16, 48), (50_000, 128, 128)]:
    A = torch.randn(E, m, device="cuda")
    B = torch.randn(E, n, device="cuda")
    gb = E * (m + n) * 4 / 1e9
    t_rect = timeit(lambda: ops.edge_outer_sum_rect(A, B))
    line = f"E={E} {m}x{n}: rect {t_rect * 1e3:.0f} us ({gb / t_rect * 1e3:.0f} GB/s)"
    if m == n:
        t_sq = timeit(lambda: ops.edge_outer_sum(A, B))
        line += f"  square {t_sq * 1e3:.0f} us ({gb / t_sq * 1e3:.0f} GB/s)"
    t_blas = timeit(lambda: A.t().mm(B))
    line += f"  rocBLAS {t_blas * 1e3:.0f} us"
    print(line, flush=True)

# square outer sum with the activation prologue (EGNN y1 / m from x_hat)
E, d = 1_000_000, 128
A = torch.randn(E, d, device="cuda")
X = torch.randn(E, d, device="cuda")
w = torch.randn(d, device="cuda")
b = torch.randn(d, device="cuda")
t_plain = timeit(lambda: ops.edge_outer_sum(A, X))
t_act = timeit(lambda: ops.edge_outer_sum_act(A, X, w, b, "relu"))
ref = ops.edge_outer_sum(A, torch.relu(X * w + b))[0]
err = (ops.edge_outer_sum_act(A, X, w, b, "relu")[0] - ref).abs().max().item()
print(f"square E={E} d={d}: plain {t_plain * 1e3:.1f} us, act-prologue {t_act * 1e3:.1f} us, "
      f"max|diff| vs materialised {err:.2e}")
