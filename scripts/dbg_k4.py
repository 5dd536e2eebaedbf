"""K4 forward debug (dev tool): the fused edge op against an fp64 torch restatement of the EGNN
message (egnn_layer.py:62-80) on a small graph; HF and f32 products, inference and training
(saved x_hat / rstd checked too).  Prints max errors."""
import sys
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
from gmp_amd import _lib, ops  # noqa: E402
from gmp_amd.graph import radius_graph  # noqa: E402

torch.manual_seed(0)
d = 128
g = radius_graph(num_nodes=400, target_edges=6000, r=2.5, seed=1, tol=0.3)
dev = "cuda"
N, ei = g.num_nodes, g.edge_index
h = torch.randn(N, d, dtype=torch.float64)
pos = g.pos.double()
W1 = torch.randn(d, 2 * d + 1, dtype=torch.float64) / (2 * d) ** 0.5
P = {k: torch.randn(d, dtype=torch.float64) * 0.3 for k in ("b1", "b2", "b3")}
P.update({k: 1 + 0.2 * torch.randn(d, dtype=torch.float64) for k in ("l1w", "l2w", "l3w")})
P.update({k: 0.2 * torch.randn(d, dtype=torch.float64) for k in ("l1b", "l2b", "l3b")})
W2 = torch.randn(d, d, dtype=torch.float64) / d ** 0.5 + 0.05
W3 = torch.randn(d, d, dtype=torch.float64) / d ** 0.5 - 0.03
w4 = torch.randn(1, d, dtype=torch.float64) / d ** 0.5
b4 = torch.randn(1, dtype=torch.float64)


def ln(x, w, b):
    mu = x.mean(-1, keepdim=True)
    xc = x - mu
    r = 1 / torch.sqrt((xc * xc).mean(-1, keepdim=True) + 1e-5)
    return xc * r, r


src, dst = ei[0], ei[1]
pd = pos[dst] - pos[src]
dist = pd.norm(dim=-1, keepdim=True)
pre1 = torch.cat([h[dst], h[src], dist], -1) @ W1.T + P["b1"]
x1, r1 = ln(pre1, None, None)
y1 = torch.relu(x1 * P["l1w"] + P["l1b"])
x2, r2 = ln(y1 @ W2.T + P["b2"], None, None)
m = torch.relu(x2 * P["l2w"] + P["l2b"])
x3, r3 = ln(m @ W3.T + P["b3"], None, None)
s = torch.relu(x3 * P["l3w"] + P["l3b"]) @ w4.T + b4
m_ref = torch.zeros(N, d, dtype=torch.float64).index_add_(0, dst, m)
p_ref = torch.zeros(N, 3, dtype=torch.float64).index_add_(0, dst, pd * s)
cnt = torch.zeros(N, dtype=torch.float64).index_add_(0, dst, torch.ones_like(dist[:, 0]))
p_ref = p_ref / cnt.clamp(min=1)[:, None]

graph = ops.egnn_graph(ei.to(dev), N)
f = lambda t: t.float().to(dev).contiguous()
AB = f(torch.cat([h @ W1[:, :d].T, h @ W1[:, d:2 * d].T], 1))
params = [f(W1[:, 2 * d]), f(P["b1"]), f(P["l1w"]), f(P["l1b"]), f(W2), f(P["b2"]), f(P["l2w"]),
          f(P["l2b"]), f(W3), f(P["b3"]), f(P["l3w"]), f(P["l3b"]), f(w4), f(b4)]
perm = graph.recv_csr.perm if hasattr(graph.recv_csr, "perm") else None
lib = _lib.load()
for f32 in (0, 1):
    lib.gmp_egnn_set_f32_mfma(f32)
    for train in (False, True):
        mo, po, xh, rs = _lib.torch_ops().egnn_edge_fwd(AB, f(pos), graph.rowptr, graph.recv,
                                                        graph.send, params, 0, False, 1e-5,
                                                        train, 2)
        torch.cuda.synchronize()
        em = (mo.double().cpu() - m_ref).abs().max().item() / m_ref.abs().max().item()
        ep = (po.double().cpu() - p_ref).abs().max().item() / p_ref.abs().max().item()
        line = f"f32={f32} train={train}: m_aggr rel {em:.2e}  pos_aggr rel {ep:.2e}"
        if train and perm is not None:
            pm = perm.cpu()
            for name, ref, got in (("x1", x1[pm], xh[0]), ("x2", x2[pm], xh[1])):
                line += f"  {name} {(got.double().cpu() - ref).abs().max().item():.2e}"
            rr = torch.cat([r1, r2, r3], 1)[pm]
            line += f"  rstd {((rs.double().cpu() - rr).abs() / rr).max().item():.2e}"
        print(line, flush=True)
lib.gmp_egnn_set_f32_mfma(0)
