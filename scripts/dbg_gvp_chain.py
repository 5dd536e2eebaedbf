"""Diagnostic: the GVP node feed-forward's module chain (library GEMMs through ops.linear,
XyzNormFn, torch gating) at 50k nodes -- run-to-run determinism and per-op gradients against
torch references, to locate a wrong gradient row."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "geometric-message-passing_amd")
sys.path.insert(0, "tests")
import test_gpu_gvp as T  # noqa: E402
import gmp_amd.gvp as g  # noqa: E402
from gmp_amd import ops  # noqa: E402

ref = T._ff_pair(5)
lay = torch.nn.Sequential(g.GVP((128, 16), (512, 32), activations=(T.RELU, None)),
                          g.GVP((512, 32), (128, 16), activations=(None, None)))
lay.load_state_dict(ref.state_dict())
lay = lay.cuda()
s, v = T._ff_inputs(50_000, 3)
gs, gv = torch.randn(50_000, 128, device="cuda"), torch.randn(50_000, 16, 3, device="cuda")
g.GVP_FF_FUSED = False


def run(defer=True, sync=False):
    ops.DEFER_WEIGHT_GRADS = defer
    lay.zero_grad(set_to_none=True)
    sd, vd = s.cuda().requires_grad_(True), v.cuda().requires_grad_(True)
    so, vo = g.gvp_ff(lay, (sd, vd))
    if sync:
        torch.cuda.synchronize()
    ((so * gs).sum() + (vo * gv).sum()).backward()
    torch.cuda.synchronize()
    return sd.grad.clone(), vd.grad.clone()


a, b, c = run(), run(), run(defer=False)
for nm, x in (("b", b), ("nodefer", c)):
    d = (a[0] - x[0]).abs().amax(1)
    print(nm, "ds rows differing:", torch.nonzero(d > 1e-3).view(-1)[:10].tolist())
# per-op: ops.linear dx at 150k rows vs torch
x = torch.randn(150_000, 16, device="cuda", requires_grad=True)
W = torch.randn(32, 16, device="cuda", requires_grad=True)
y = ops.linear(x, W)
gy = torch.randn_like(y)
(y * gy).sum().backward()
x64, W64 = x.detach().double().requires_grad_(True), W.detach().double().requires_grad_(True)
((x64 @ W64.t()) * gy.double()).sum().backward()
e = (x.grad.double() - x64.grad).abs().amax(1)
print("linear dx 150k: max", e.max().item(), "rows", torch.nonzero(e > 1e-3).view(-1)[:10].tolist())
print("linear dW 150k: max", (W.grad.double() - W64.grad).abs().max().item())

# the oracle modules in fp32 on the device (pure torch) and the row in question
import copy  # noqa: E402
refg = copy.deepcopy(ref).cuda()
sd, vd = s.cuda().requires_grad_(True), v.cuda().requires_grad_(True)
so, vo = refg((sd, vd))
((so * gs).sum() + (vo * gv).sum()).backward()
ref64 = copy.deepcopy(ref).double()
s64, v64 = s.double().requires_grad_(True), v.double().requires_grad_(True)
so64, vo64 = ref64((s64, v64))
((so64 * gs.cpu().double()).sum() + (vo64 * gv.cpu().double()).sum()).backward()
e_torch = (sd.grad.cpu().double() - s64.grad).abs().amax(1)
e_chain = (a[0].cpu().double() - s64.grad).abs().amax(1)
print("torch-on-device ds bad rows", torch.nonzero(e_torch > 1e-3).view(-1)[:10].tolist(),
      "chain bad rows", torch.nonzero(e_chain > 1e-3).view(-1)[:10].tolist())
r = int(torch.argmax(e_chain))
# intermediates at that row
with torch.no_grad():
    g1 = ref64[0]
    vt = v64[r:r + 1].transpose(-1, -2)
    vh = g1.wh(vt)
    vn = torch.sqrt(torch.clamp((vh ** 2).sum(-2), min=1e-8))
    p1 = g1.ws(torch.cat([s64[r:r + 1], vn], -1))
    print("row", r, "min |p1|", p1.abs().min().item(), "min |vh1|^2", (vh ** 2).sum(-2).min().item())
