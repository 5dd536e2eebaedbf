"""Microbenchmark of the K7 apply kernel, f32-MFMA vs x3 (v2) vs v3 forms, over the path widths of C4 MACE
(w = 128, 384, 640) and C5 TFN (w = 64, 192, 320) at H = 256, 50k receivers x 20 edges."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402
from gmp_amd.ops import _p, _stream  # noqa: E402

lib = _lib.load()
N, E, H = 50_000, 1_000_000, 256
eoff = torch.arange(0, E + 1, E // N, dtype=torch.int64, device="cuda")
A = torch.relu(torch.randn(E, H, device="cuda"))
for w in (64, 128, 192, 320, 384, 640):
    Z = torch.randn(E + 1, w, device="cuda")
    T = torch.randn(N, w, H, device="cuda")
    Tb = torch.randn(N, w, device="cuda")
    dZ = torch.empty(E + 1, w, device="cuda")
    dA = torch.zeros(E, H, device="cuda")
    res = []
    for x3 in (0, 1, 2):
        lib.gmp_tp_apply_set_x3(x3)
        f = lambda: lib.gmp_tp_node_apply_f32(N, w, H, _p(eoff), _p(Z), _p(A), _p(T), _p(Tb),
                                              _p(dZ), _p(dA), _stream())
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 5)
    tb = N * w * H * 4 / 1e9
    print(f"w={w:4d} f32 {res[0]:7.3f} ms  x3 {res[1]:7.3f} ms  v3 {res[2]:7.3f} ms "
          f"(T {tb:.1f} GB: {tb / res[2]:.2f} TB/s)", flush=True)
    del Z, T, Tb, dZ, dA
