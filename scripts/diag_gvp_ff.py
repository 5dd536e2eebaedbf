"""Diagnostic: K17 (fused GVP node feed-forward) vs the fp64 oracle and vs the module chain at
a given node count; prints the max error per output and the rows where the error is largest."""
import copy
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "geometric-message-passing_amd")
sys.path.insert(0, "tests")
from oracle import gvp as ogvp  # noqa: E402

RELU = torch.nn.functional.relu


def main(n):
    import gmp_amd.gvp as g
    torch.manual_seed(5)
    ref = torch.nn.Sequential(ogvp.GVP((128, 16), (512, 32), activations=(RELU, None)),
                              ogvp.GVP((512, 32), (128, 16), activations=(None, None)))
    with torch.no_grad():
        for p in ref.parameters():
            p.add_(0.05 * torch.randn_like(p))
    lay = torch.nn.Sequential(g.GVP((128, 16), (512, 32), activations=(RELU, None)),
                              g.GVP((512, 32), (128, 16), activations=(None, None)))
    lay.load_state_dict(ref.state_dict())
    lay = lay.cuda()
    ref64 = copy.deepcopy(ref).double()
    s, v = torch.randn(n, 128), torch.randn(n, 16, 3)
    if len(sys.argv) > 2:  # zero vectors: the clamped norms
        v[3] = 0.0
        v[5, :8] = 0.0
    gs, gv = torch.randn(n, 128), torch.randn(n, 16, 3)
    res = {}
    for name in ("fused", "chain"):
        g.GVP_FF_FUSED = name == "fused"
        lay.zero_grad(set_to_none=True)
        sd, vd = s.cuda().requires_grad_(True), v.cuda().requires_grad_(True)
        so, vo = g.gvp_ff(lay, (sd, vd))
        ((so * gs.cuda()).sum() + (vo * gv.cuda()).sum()).backward()
        res[name] = [so.detach().cpu().double(), vo.detach().cpu().double(), sd.grad.cpu().double(),
                     vd.grad.cpu().double()] + [p.grad.cpu().double() for p in lay.parameters() if p.numel()]
    s64, v64 = s.double().requires_grad_(True), v.double().requires_grad_(True)
    so, vo = ref64((s64, v64))
    ((so * gs.double()).sum() + (vo * gv.double()).sum()).backward()
    r64 = [so.detach(), vo.detach(), s64.grad, v64.grad] + [p.grad for p in ref64.parameters() if p.numel()]
    names = ["s2", "v2", "ds", "dv"] + [k for k, p in lay.named_parameters() if p.numel()]
    for k, a64 in zip(range(len(names)), r64):
        sc = a64.abs().max().item()
        ef = (res["fused"][k] - a64).abs()
        ec = (res["chain"][k] - a64).abs()
        line = f"{names[k]:14s} scale {sc:9.3e} fused {ef.max().item() / sc:9.2e} " \
               f"chain {ec.max().item() / sc:9.2e}"
        if k < 4 and ef.max().item() / sc > 1e-4:
            rows = ef.reshape(n, -1).amax(1)
            bad = torch.nonzero(rows > 1e-4 * sc).view(-1)
            line += f"  bad rows {bad.numel()} first {bad[:8].tolist()}"
        print(line)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50_000)
