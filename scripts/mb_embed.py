"""K1e edge-embedding kernels (gmp_gvp_edge_embed_{fwd,bwd}_f32) at the C3 edge count, HIP events.
Usage (GPU box): python scripts/mb_embed.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402

ops = _lib.torch_ops()
E, R, so = 999_722, 8, 32
torch.manual_seed(0)
rad = torch.rand(E, R, device="cuda")
unit = torch.nn.functional.normalize(torch.randn(E, 3, device="cuda"), dim=-1)
W = [torch.randn(*sh, device="cuda") * 0.3 for sh in ((R,), (R,), (1, 1), (so, R + 1), (so,),
                                                     (1, 1), (1, so), (1,))]
des, dev = torch.randn(E, so, device="cuda"), torch.randn(E, 1, 3, device="cuda")


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


tf = timeit(lambda: ops.gvp_edge_embed_fwd(rad, unit, W, 1e-5))
tb = timeit(lambda: ops.gvp_edge_embed_bwd(rad, unit, W, 1e-5, des, dev))
print(f"K1e E={E}: fwd {tf:.1f} us ({E * (R + 3 + so + 3) * 4 / tf / 1e3:.0f} GB/s), "
      f"bwd {tb:.1f} us ({E * (R + 3 + so + 3) * 4 / tb / 1e3:.0f} GB/s)", flush=True)
