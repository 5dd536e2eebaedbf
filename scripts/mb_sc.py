"""K8 symmetric contraction timing (sparse term plan, gmp_sc.hip): forward and backward (dx +
dcoef partials) at the C4 shape (50k nodes, 128 channels, 0e+1o+2e, correlation 3) and the
widened shapes (both parities, max_ell 3 / 5, correlation 4), HIP events.
Usage (GPU box): python scripts/mb_sc.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402
from gmp_amd import equivariant as eq  # noqa: E402

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
N = 50_000
CASES = [("128x0e+128x1o+128x2e", 3), ("128x0e+128x1o+128x2e", 2),
                  ("128x0e+128x1o+128x2e", 4), ("128x0e+128x1o+128x2e+128x3o", 3),
                  ("32x0e+32x0o+32x1e+32x1o+32x2e+32x2o", 3),
                  ("64x0e+64x1o+64x2e+64x3o+64x4e+64x5o", 2),
                  ("32x0e+32x1o+32x2e+32x3o", 4)]
for irr, corr in CASES[:int(sys.argv[1])] if len(sys.argv) > 1 else CASES:
    sc = eq.SymmetricContraction(irr, irr, corr).cuda()
    C = int(irr.split("x")[0])
    D = sum(2 * int(t.split("x")[1][:-1]) + 1 for t in irr.split("+"))
    x = torch.randn(N, C, D, device="cuda")
    coef = sc.k8_coefficients().detach().contiguous()
    plan, M = sc._k8_plan, sc._k8_rows
    g = torch.randn(N, M * C, device="cuda")
    tf = timeit(lambda: ops.symmetric_contraction_fwd(x, plan, M, coef))
    tb = timeit(lambda: ops.symmetric_contraction_bwd(x, plan, M, coef, g))
    print(f"{irr} corr={corr}: D={D} T={coef.shape[0]} fwd {tf:7.3f} ms  bwd {tb:7.3f} ms",
          flush=True)
