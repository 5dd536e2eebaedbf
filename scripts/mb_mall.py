"""Does a receiver sub-chunk whose S / T fits the 256 MiB Infinity Cache make the K7 pairs
faster?  MACE-128 lo = 2 path shape (50k receivers x 20 edges, w = 640, H = 256).  For each
sub-chunk size R (receivers) the producer writes into ONE reused buffer and the consumer reads
it right after:  backward  T = G W2p^T (widen) -> apply;  forward  S (outer) alone.
Usage (GPU box): python scripts/mb_mall.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib  # noqa: E402
import ctypes  # noqa: E402

from gmp_amd.ops import _p, _stream  # noqa: E402


def _q(t, off):
    return ctypes.c_void_p(t.data_ptr() + off)

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
lib = _lib.load()
dev = "cuda"
torch.manual_seed(0)
N, E, m1, mo, H, d3 = 50_000, 1_000_000, 128, 128, 256, 5
w = m1 * d3
K1 = m1 * H
deg = E // N
eoff = torch.arange(0, E + 1, deg, dtype=torch.int64, device=dev)
Z = torch.randn(E + 1, w, device=dev)
A = torch.relu(torch.randn(E, H, device=dev))
W2 = torch.randn(m1 * mo, H, device=dev) * 0.05
b2 = torch.randn(m1 * mo, device=dev) * 0.05
Bt = torch.empty(3 * K1 * mo, dtype=torch.int16, device=dev)
lib.gmp_tp_split_w2_f32(m1, mo, H, _p(W2), _p(b2), None, _p(Bt), _stream())
G = torch.randn(N * d3, mo, device=dev)
Tb = torch.randn(N, w, device=dev)
dZ = torch.empty(E + 1, w, device=dev)
dA = torch.zeros(E, H, device=dev)
F32 = 4


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


def bwd(R, T):
    def run():
        for r0 in range(0, N, R):
            r = min(R, N - r0)
            lib.gmp_tp_gemm_x3_widen_f32(r * d3, K1, mo, _q(G, r0 * d3 * mo * F32), mo, _p(Bt),
                                         mo, K1 * mo, _p(T), K1, _stream())
            lib.gmp_tp_node_apply_f32(r, w, H, _q(eoff, r0 * 8), _p(Z), _p(A), _p(T),
                                      _q(Tb, r0 * w * F32), _p(dZ), _p(dA), _stream())
    return run


def fwd_s(R, S, Sb):
    def run():
        for r0 in range(0, N, R):
            r = min(R, N - r0)
            lib.gmp_tp_node_outer_f32(r, w, H, _q(eoff, r0 * 8), _p(Z), _p(A), _p(S), _p(Sb),
                                      _stream())
    return run


Tfull = torch.empty(N * d3, K1, device=dev)
t_T = timeit(lambda: lib.gmp_tp_gemm_x3_widen_f32(N * d3, K1, mo, _p(G), mo, _p(Bt), mo, K1 * mo,
                                                  _p(Tfull), K1, _stream()))
t_full = timeit(bwd(N, Tfull))
print(f"full: T gemm {t_T:.3f} ms, T gemm + apply {t_full:.3f} ms", flush=True)
t_S = timeit(fwd_s(N, Tfull.view(N, w, H), Tb))
print(f"full: S {t_S:.3f} ms", flush=True)
del Tfull
torch.cuda.empty_cache()
for R in (64, 128, 192, 256, 384, 512, 1024, 4096):
    T = torch.empty(R * d3, K1, device=dev)
    Sb = torch.empty(R, w, device=dev)
    t_b = timeit(bwd(R, T))
    t_s = timeit(fwd_s(R, T.view(R, w, H), Sb))
    mb = R * d3 * K1 * F32 / 2**20
    print(f"R={R:5d} ({mb:7.1f} MiB): T gemm + apply {t_b:.3f} ms, S {t_s:.3f} ms", flush=True)
    del T, Sb
    torch.cuda.empty_cache()
