"""Microbenchmark of K14 (shifted softplus fwd / bwd) on an (E, 128) filter tensor, E = 1M."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402

ops = _lib.torch_ops()
x = torch.randn(1_000_000, 128, device="cuda") * 4
g = torch.randn_like(x)
for name, f in (("ssp_fwd", lambda: ops.ssp_fwd(x, math.log(2.0))),
                ("ssp_bwd", lambda: ops.ssp_bwd(x, g))):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    nbytes = x.numel() * 4 * (2 if name == "ssp_fwd" else 3)
    print(f"{name} {ms * 1e3:.1f} us {nbytes / ms / 1e9:.2f} TB/s", flush=True)
