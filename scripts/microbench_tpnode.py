"""Micro-benchmark of the receiver-factorised TP kernels (gmp_tp_node_outer / _apply) on a
synthetic chunk: c receivers of in-degree deg, path width w, hidden H."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402
from gmp_amd.ops import _p, _stream  # noqa: E402

lib = _lib.load()
c, deg, w, H = (int(os.environ.get("C", 3200)), int(os.environ.get("DEG", 20)),
                int(os.environ.get("W", 640)), 256)
ne = c * deg
dev = "cuda"
eoff = torch.arange(0, ne + 1, deg, device=dev, dtype=torch.int64)
Z = torch.randn(ne + 1, w, device=dev)
A = torch.randn(ne, H, device=dev)
S = torch.empty(c, w, H, device=dev)
Sb = torch.empty(c, w, device=dev)
T = torch.randn(c, w, H, device=dev) if not os.environ.get("OUTER_ONLY") else None
Tb = torch.randn(c, w, device=dev)
dZ = torch.empty(ne + 1, w, device=dev)
dA = torch.zeros(ne, H, device=dev)


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


t_o = timeit(lambda: lib.gmp_tp_node_outer_f32(c, w, H, _p(eoff), _p(Z), _p(A), _p(S), _p(Sb),
                                               _stream()))
if os.environ.get("OUTER_ONLY"):
    print(f"outer: {t_o:.3f} ms  S write {c * w * H * 4 / 1e9 / t_o * 1e3:.0f} GB/s", flush=True)
    sys.exit(0)
t_a = timeit(lambda: lib.gmp_tp_node_apply_f32(c, w, H, _p(eoff), _p(Z), _p(A), _p(T), _p(Tb),
                                               _p(dZ), _p(dA), _stream()))
gb = c * w * H * 4 / 1e9
print(f"outer: {t_o:.3f} ms  S write {gb / t_o * 1e3:.0f} GB/s ; apply: {t_a:.3f} ms  T read "
      f"{gb / t_a * 1e3:.0f} GB/s", flush=True)
