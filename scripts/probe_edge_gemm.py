"""Probe: library GEMM forms for the SchNet filter-network edge Linears (E x 50 -> 128,
E x 128 -> 128, fp32) on MI355X.  Prints us per call for each form / BLAS backend."""
import torch

E = 999_722
dev = "cuda"


def bench(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for lib in ("hipblaslt", "rocblas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as ex:  # noqa: BLE001
        print(lib, "unavailable", ex)
        continue
    for K in (50, 64, 128):
        x = torch.randn(E, K, device=dev)
        W = torch.randn(128, K, device=dev)
        b = torch.randn(128, device=dev)
        Wt = W.t().contiguous()
        g = torch.randn(E, 128, device=dev)
        forms = {
            "addmm(b,x,W.t())": lambda: torch.addmm(b, x, W.t()),
            "x.mm(W.t())": lambda: x.mm(W.t()),
            "x.mm(Wt)": lambda: x.mm(Wt),
            "addmm(b,x,Wt)": lambda: torch.addmm(b, x, Wt),
            "g.mm(W) (dx)": lambda: g.mm(W),
            "g.mm(Wt.t()) (dx)": lambda: g.mm(Wt.t()),
            "W@x.t() (yT)": lambda: W.mm(x.t()),
        }
        for name, fn in forms.items():
            print(f"{lib:10s} K={K:3d} {name:22s} {bench(fn):9.1f} us", flush=True)
