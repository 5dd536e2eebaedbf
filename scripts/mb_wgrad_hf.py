"""Microbenchmark: EGNN weight-gradient outer sum (K = 1M edges, d = 128, silu prologue) in the
split-plane x3 form and the HF form (gmp_edge_outer_sum_act{,_hf}_f32).  GPU box."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import ops  # noqa: E402

K, d = 1_000_000, 128
A = torch.randn(K, d, device="cuda")
X = torch.randn(K, d, device="cuda")
X = (X - X.mean(1, keepdim=True)) / X.std(1, unbiased=False, keepdim=True)
w, b = torch.randn(d, device="cuda"), torch.randn(d, device="cuda")
amax = torch.zeros(1, dtype=torch.int32, device="cuda")
amax[0] = A.abs().max().view(1).view(torch.int32)[0]
for name, am in (("x3", None), ("hf", amax)):
    for _ in range(3):
        ops.edge_outer_sum_act(A, X, w, b, "silu", am)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.edge_outer_sum_act(A, X, w, b, "silu", am)
    e1.record()
    torch.cuda.synchronize()
    print(name, round(e0.elapsed_time(e1) / 20 * 1e3, 1), "us", flush=True)
