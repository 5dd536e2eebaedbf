"""Micro-benchmark: f32 GEMM (rocBLAS f32 MFMA) vs f32 emulated by a 3-way bf16 split with the
six significant partial products (bf16 MFMA, f32 accumulate), on the MACE path-GEMM shapes
(M = nodes * (2l+1), K = mul1 * H = 32768, N = mul_out = 128).  Prints time and max error vs
fp64 on sampled rows for both."""
import sys
import time

import torch


def split3(x):
    x0 = x.to(torch.bfloat16)
    r = x - x0.float()
    x1 = r.to(torch.bfloat16)
    x2 = (r - x1.float()).to(torch.bfloat16)
    return x0, x1, x2


def emu_mm(A3, K, B0s, B1s, B2):
    """A3 = [A0|A1|A2] (M, 3K) bf16; B0s = [B0;B0;B0] (3K, N), B1s = [B1;B1] (2K, N)."""
    C = torch.mm(A3, B0s, out_dtype=torch.float32)
    C = torch.addmm(C, A3[:, :2 * K], B1s, out_dtype=torch.float32)
    return torch.addmm(C, A3[:, :K], B2, out_dtype=torch.float32)


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = "cuda"
    torch.manual_seed(0)
    for M, K, N in [(50000, 32768, 128), (150000, 32768, 128), (250000, 8192, 128),
                    (50000, 8192, 128)]:
        A = torch.randn(M, K, device=dev) * torch.rand(M, 1, device=dev)
        B = torch.randn(K, N, device=dev) / K ** 0.5
        t32 = timeit(lambda: torch.mm(A, B))
        C32 = torch.mm(A, B)
        A0, A1, A2 = split3(A)
        A3 = torch.cat([A0, A1, A2], 1)
        del A0, A1, A2
        B0, B1, B2 = split3(B)
        B0s, B1s = torch.cat([B0, B0, B0], 0), torch.cat([B1, B1], 0)
        temu = timeit(lambda: emu_mm(A3, K, B0s, B1s, B2))
        tsplit = timeit(lambda: split3(A))
        Ce = emu_mm(A3, K, B0s, B1s, B2)
        rows = torch.randint(0, M, (256,), device=dev)
        ref = A[rows].double().mm(B.double())
        scale = (A[rows].double().abs().mm(B.double().abs()))
        e32 = ((C32[rows].double() - ref).abs() / scale).max().item()
        eem = ((Ce[rows].double() - ref).abs() / scale).max().item()
        fl = 2 * M * K * N
        print(f"M={M} K={K} N={N}: f32 {t32*1e3:.2f} ms ({fl/t32/1e12:.0f} TF)  emu "
              f"{temu*1e3:.2f} ms ({fl/temu/1e12:.0f} TF-equiv)  split {tsplit*1e3:.2f} ms  "
              f"rel.err f32 {e32:.2e} emu {eem:.2e}", flush=True)
        del A, A3, C32, Ce


if __name__ == "__main__":
    sys.exit(main())
