"""Standalone timing of the edge outer sums (gmp_wgrad.hip) on both arithmetic paths
(bf16x3 split vs f32 MFMA) for the shapes the models use, K = 1M edges."""
import sys

import torch

sys.path.insert(0, "geometric-message-passing_amd")
from gmp_amd import _lib, ops  # noqa: E402


def main():
    lib = _lib.load()
    dev = "cuda"
    K = 1_000_000
    shapes = [(128, 128, None), (128, 128, "silu"), (128, 144, None), (16, 128, None),
              (128, 16, None), (48, 48, None), (16, 48, None), (128, 48, None)]
    for m, n, act in shapes:
        A = torch.randn(K, m, device=dev)
        B = torch.randn(K, n, device=dev)
        w = torch.randn(n, device=dev)
        b = torch.randn(n, device=dev)
        C = torch.empty(m, n, device=dev)
        cs = torch.empty(m, device=dev)
        res = []
        for mode in (1, 0):
            lib.gmp_wgrad_set_f32_mfma(mode)
            f = lambda: ops.outer_sum_into(A, B, C, cs, act, w if act else None,  # noqa: E731
                                           b if act else None)
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / 20 * 1e3)
        lib.gmp_wgrad_set_f32_mfma(0)
        gb = K * (m + n) * 4 / 1e9
        print(f"{m:4d} x {n:4d} {act or '-':5s} f32mfma {res[0]:7.1f} us   split {res[1]:7.1f} us"
              f"   ({gb / res[1] * 1e6 / 1e3:.2f} TB/s operand read)", flush=True)


if __name__ == "__main__":
    main()
