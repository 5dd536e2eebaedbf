import copy, sys, torch
sys.path.insert(0, "."); sys.path.insert(0, "geometric-message-passing_amd"); sys.path.insert(0, "tests")
import test_gpu_gvp as T
import gmp_amd.gvp as g
ref = T._ff_pair(5)
lay = torch.nn.Sequential(g.GVP((128, 16), (512, 32), activations=(T.RELU, None)), g.GVP((512, 32), (128, 16), activations=(None, None)))
lay.load_state_dict(ref.state_dict()); lay = lay.cuda()
s, v = T._ff_inputs(50_000, 3)
gs, gv = torch.randn(50_000, 128, device="cuda"), torch.randn(50_000, 16, 3, device="cuda")
def run(fused):
    g.GVP_FF_FUSED = fused
    lay.zero_grad(set_to_none=True)
    sd, vd = s.cuda().requires_grad_(True), v.cuda().requires_grad_(True)
    so, vo = g.gvp_ff(lay, (sd, vd))
    ((so * gs).sum() + (vo * gv).sum()).backward()
    return [so.detach(), vo.detach(), sd.grad, vd.grad]
a = run(True); c = run(False)
ref64 = copy.deepcopy(ref).double()
s64, v64 = s.double().requires_grad_(True), v.double().requires_grad_(True)
so, vo = ref64((s64, v64)); ((so * gs.cpu().double()).sum() + (vo * gv.cpu().double()).sum()).backward()
r = [so.detach(), vo.detach(), s64.grad, v64.grad]
for k in range(4):
    ea = (a[k].cpu().double() - r[k]).abs(); ec = (c[k].cpu().double() - r[k]).abs()
    print(k, r[k].abs().max().item(), ea.max().item(), ec.max().item(), torch.nonzero(ea.reshape(50000,-1).amax(1) > 1e-3).view(-1)[:10].tolist(), torch.nonzero(ec.reshape(50000,-1).amax(1) > 1e-3).view(-1)[:10].tolist())
