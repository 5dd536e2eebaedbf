"""K8 symmetric contraction timing at the C4 shape (50k nodes, 128 channels, 0e+1o+2e,
correlation 3) and the widened shapes: forward and backward (dx + dA partials), HIP events.
Usage (GPU box): python scripts/mb_sc.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402

ops = _lib.torch_ops()


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


torch.manual_seed(0)
N, C = 50_000, 128
for D, corr in [(9, 3), (9, 2), (9, 4), (16, 3), (4, 4)]:
    x = torch.randn(N, C, D, device="cuda")
    A = [torch.randn(C, D, sum(1 for _ in range(1)) * 0 + __import__("math").comb(D + nu - 1, nu),
                     device="cuda") * 0.1 for nu in range(1, corr + 1)]
    Ao = A + [None] * (4 - len(A))
    g = torch.randn(N, D * C, device="cuda")
    tf = timeit(lambda: ops.symmetric_contraction_fwd(x, corr, *Ao))
    tb = timeit(lambda: ops.symmetric_contraction_bwd(x, corr, *Ao, g))
    print(f"D={D:2d} corr={corr}: fwd {tf:7.3f} ms  bwd {tb:7.3f} ms", flush=True)
