"""HBM ceilings on this box: write (fill_), read (sum), copy for a 32 GB f32 buffer (the S / T
intermediate size of a C4 lo = 2 path).  HIP-event timing."""
import torch

n = 8 * 1024 ** 3  # 32 GiB of f32
x = torch.empty(n, device="cuda")
y = torch.empty(n // 4, device="cuda")


def t(name, fn, nbytes, reps=3):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{name:10s} {ms:8.3f} ms {nbytes / ms / 1e9:8.1f} TB/s", flush=True)


t("fill", lambda: x.fill_(1.0), 4 * n)
t("sum", lambda: x.sum(), 4 * n)
t("copy8G", lambda: y.copy_(x[: n // 4]), 2 * 4 * n // 4)
