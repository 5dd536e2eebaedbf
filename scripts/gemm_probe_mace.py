"""Dev tool: layout forms of the MACE path GEMMs (M = receivers x (2l+1), K = mul1 * H = 32768,
N = mul_out = 128) on hipBLASLt: op = S W2p (NN vs NT), dW2p = S^T G (TN vs (G^T S)^T)."""
import torch

dev = "cuda"
M, K, N = 150_000, 32_768, 128


def t(f, n=5):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


S = torch.randn(M, K, device=dev)
W = torch.randn(K, N, device=dev)
Wt = W.t().contiguous()
G = torch.randn(M, N, device=dev)
print(f"op NN  S @ W        {t(lambda: S.mm(W)):.2f} ms")
print(f"op NT  S @ Wt.t()   {t(lambda: S.mm(Wt.t())):.2f} ms")
print(f"dW TN  S.t() @ G    {t(lambda: S.t().mm(G)):.2f} ms")
print(f"dW^T   G.t() @ S    {t(lambda: G.t().mm(S)):.2f} ms")
print(f"T  NT  G @ W.t()    {t(lambda: G.mm(W.t())):.2f} ms")
print(f"T  NN  G @ Wt       {t(lambda: G.mm(Wt)):.2f} ms")
