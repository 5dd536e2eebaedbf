"""Microbenchmark (GPU): the backward dW2p of one TP path at the MACE-128 lo = 2 shape (50k
receivers x 20 edges, d3 = 5, mul1 = 128, H = 256, mul_out = 128) and the TFN-64 lo = 1 shape:
K7f fused (tp_node_dw) vs the unfused S kernel + column-block outer sum; HIP events, median."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "geometric-message-passing_amd")]


def timeit(fn, n=5):
    fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from gmp_amd import _lib
    tops = _lib.torch_ops()
    dev = torch.device("cuda", 0)
    only = sys.argv[1] if len(sys.argv) > 1 else None  # "fused" / "unfused": one shape, 3 runs
    shapes = [(50000, 20, 5, 128, 256, 128), (50000, 20, 3, 64, 256, 64),
              (50000, 20, 1, 128, 256, 128)]
    for (N, deg, d3, mul1, H, mo) in shapes[:1] if only else shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        eoff = torch.arange(N + 1, device=dev, dtype=torch.int64) * deg
        E = N * deg
        w = d3 * mul1
        Z = torch.randn(E + 1, w, device=dev, generator=g)
        A = torch.randn(E, H, device=dev, generator=g)
        G = torch.randn(N * d3, mo, device=dev, generator=g)
        if only == "fused":
            for _ in range(3):
                tops.tp_node_dw(eoff, Z, A, G, d3, mul1)
            torch.cuda.synchronize()
            return
        if only == "unfused":
            S, _ = tops.tp_node_outer(eoff, Z, A, w)
            for _ in range(3):
                tops.outer_sum_cols(S.view(N * d3, mul1 * H), G)
            torch.cuda.synchronize()
            return
        t_f = timeit(lambda: tops.tp_node_dw(eoff, Z, A, G, d3, mul1))

        def unfused():
            S, Sb = tops.tp_node_outer(eoff, Z, A, w)
            return tops.outer_sum_cols(S.view(N * d3, mul1 * H), G)
        t_u = timeit(unfused)
        S, _ = tops.tp_node_outer(eoff, Z, A, w)
        t_s = timeit(lambda: tops.tp_node_outer(eoff, Z, A, w))
        t_o = timeit(lambda: tops.outer_sum_cols(S.view(N * d3, mul1 * H), G))
        del S
        tf = 2 * N * d3 * mul1 * H * mo / 1e12
        print(f"N={N} deg={deg} d3={d3} mul1={mul1} H={H} mo={mo}: fused {t_f:.2f} ms "
              f"({tf / t_f * 1e3:.0f} TF-eq of dW), unfused {t_u:.2f} ms (S {t_s:.2f} + "
              f"outer sum {t_o:.2f})", flush=True)
        del Z, A, G


if __name__ == "__main__":
    main()
