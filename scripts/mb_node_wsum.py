"""Microbenchmark: node-level (K = 50k rows) weight sums A^T B of K17's backward by the gmp outer
sums (ops.edge_outer_sum_rect) and by the library GEMM (torch.mm(A.t(), B))."""
import sys

import torch

sys.path.insert(0, "geometric-message-passing_amd")
from gmp_amd import ops  # noqa: E402

K = 50_000
shapes = [(512, 128), (512, 32), (32, 128), (32, 32), (96, 48), (128, 512), (128, 32), (16, 128),
          (96, 96), (48, 96)]


def timed(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


tot = [0.0, 0.0]
for m, n in shapes:
    A, B = torch.randn(K, m, device="cuda"), torch.randn(K, n, device="cuda")
    t1 = timed(lambda: ops.edge_outer_sum_rect(A, B))
    t2 = timed(lambda: (torch.mm(A.t(), B), A.sum(0)))
    tot[0] += t1
    tot[1] += t2
    print(f"{m:4d} x {n:4d}: outer sum {t1:7.1f} us, library {t2:7.1f} us")
print(f"total: outer sums {tot[0]:.1f} us, library {tot[1]:.1f} us")
