"""Microbenchmark: K17 (gmp_gvp_ff fwd / bwd) alone at the C3 node count, HIP-event timed, next to
the module chain it replaces (forward + backward of the two GVPs)."""
import sys

import torch

sys.path.insert(0, "geometric-message-passing_amd")
import gmp_amd.gvp as g  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
R = torch.nn.functional.relu
lay = torch.nn.Sequential(g.GVP((128, 16), (512, 32), activations=(R, None)),
                          g.GVP((512, 32), (128, 16), activations=(None, None))).cuda()
s = torch.randn(N, 128, device="cuda", requires_grad=True)
v = torch.randn(N, 16, 3, device="cuda", requires_grad=True)
gs, gv = torch.randn(N, 128, device="cuda"), torch.randn(N, 16, 3, device="cuda")
W = [lay[0].wh.weight, lay[0].ws.weight, lay[0].ws.bias, lay[0].wv.weight, lay[0].wsv.weight,
     lay[0].wsv.bias, lay[1].wh.weight, lay[1].ws.weight, lay[1].ws.bias, lay[1].wv.weight,
     lay[1].wsv.weight, lay[1].wsv.bias]
ops = g._lib.torch_ops()
Wd = [w.detach() for w in W]


def timed(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


out = ops.gvp_ff_fwd(s.detach(), v.detach(), Wd)
t_f = timed(lambda: ops.gvp_ff_fwd(s.detach(), v.detach(), Wd))
t_b = timed(lambda: ops.gvp_ff_bwd(v.detach(), Wd, out[2], out[4], out[0], gs, gv))


def step(fused):
    g.GVP_FF_FUSED = fused
    so, vo = g.gvp_ff(lay, (s, v))
    ((so * gs).sum() + (vo * gv).sum()).backward()


t_fused = timed(lambda: step(True))
t_chain = timed(lambda: step(False))
print(f"N={N}: K17 fwd {t_f:.1f} us, bwd {t_b:.1f} us; fwd+bwd incl. weight sums: "
      f"fused {t_fused:.1f} us, chain {t_chain:.1f} us")
