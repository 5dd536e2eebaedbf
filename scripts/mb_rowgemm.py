"""Microbenchmark (GPU): row-level Linear GEMMs at the EGNN C2 node shapes, library f32 GEMM
(torch.mm / addmm) vs K7g gemm_x3 (split included), HIP-event timed, median of 20."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometric-message-passing_amd")]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from gmp_amd import ops
    dev = torch.device("cuda", 0)
    for M, N, K1, K2, tr in [(50000, 256, 128, 0, False), (50000, 128, 128, 128, False),
                             (50000, 128, 128, 0, False), (50000, 128, 128, 0, True),
                             (1000000, 128, 128, 0, False), (1000000, 64, 64, 0, False)]:
        a1 = torch.randn(M, K1, device=dev)
        a2 = torch.randn(M, K2, device=dev) if K2 else None
        W = torch.randn((K1 + K2, N) if tr else (N, K1 + K2), device=dev)
        b = torch.randn(N, device=dev)
        A = a1 if a2 is None else torch.cat([a1, a2], 1)
        Bt = W if tr else W.t()
        t_lib = timeit(lambda: torch.addmm(b, A, Bt))
        t_x3 = timeit(lambda: ops.linear_x3(a1, a2, W, b, tr))
        Bp = ops._lib.torch_ops().split_x3(W, tr)
        t_k = timeit(lambda: ops._lib.torch_ops().gemm_x3(a1, a2, Bp, N, b))
        gb = 4 * M * (K1 + K2 + N) / 1e9
        print(f"M={M} N={N} K={K1}+{K2} tr={tr}: library {t_lib:.1f} us, x3 {t_x3:.1f} us "
              f"(kernel {t_k:.1f} us = {gb / t_k * 1e6 / 1e3:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
