"""GPU parity of SchNet / CFConv (gmp_amd/schnet.py) with the CPU restatement of PyG 2.3.1's
SchNet (oracle/schnet.py; parity unpinned against PyG itself, which is absent).  Config C1:
hidden 64, 128 filters, 50 Gaussians, cutoff 10, 4 interactions on the k-chains graphs; plus a
random radius graph.  Tolerance 1e-5 on outputs, 1e-4 of scale on gradients."""
import math

import pytest
import torch

from oracle import schnet as osch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _scaled(a, b, rtol, name):
    a, b = a.detach().cpu(), b.detach().cpu()
    scale = b.abs().max().item() + 1e-6
    err = (a - b).abs().max().item()
    assert err <= rtol * scale + 1e-6, f"{name}: max|d|={err:.3e} scale={scale:.3e}"


def _batches(kind):
    from gmp_amd.graph import collate, create_kchains, radius_graph
    if kind == "kchains":
        return collate(create_kchains(4))
    g = [radius_graph(num_nodes=200, target_edges=3000, r=3.0, seed=s, tol=0.2) for s in (1, 2)]
    for k, gg in enumerate(g):
        gg.atoms = torch.randint(0, 5, (gg.num_nodes,), generator=torch.Generator().manual_seed(k))
    return collate(g)


@pytest.mark.parametrize("kind,edge_path,pos_grad", [
    ("kchains", False, True), ("radius", False, True), ("kchains", True, True),
    ("radius", True, True), ("radius", True, False), ("kchains", False, False)])
def test_schnet_vs_oracle(kind, edge_path, pos_grad, monkeypatch):
    """edge_path: force the filter network's edge Linears onto ops.linear's EdgeLinearFn
    (outer-sum weight gradients, K = 50 zero-padded to 64), which the bench graph takes.
    pos_grad=False (the training-step configuration): the cosine cutoff has no gradient and is
    applied inside K13 (gmp_cfconv_*_scaled_f32) instead of materialising W * C."""
    import gmp_amd
    from gmp_amd import ops
    if edge_path:
        monkeypatch.setattr(ops, "EDGE_LINEAR_MIN_ROWS", 1)
    from gmp_amd.graph import Batch
    torch.manual_seed(3)
    b = _batches(kind)
    ref = osch.SchNetModel(hidden_channels=64, num_filters=128, num_layers=4, num_gaussians=50,
                           cutoff=10, out_dim=2)
    with torch.no_grad():  # atoms = 0 is the padding row: perturb so the test is not trivial
        ref.embedding.weight.normal_()
    model = gmp_amd.SchNetModel(hidden_channels=64, num_filters=128, num_layers=4,
                                num_gaussians=50, cutoff=10, out_dim=2)
    model.load_state_dict(ref.state_dict(), strict=True)
    model = model.to(DEV)
    pd = b.pos.to(DEV).requires_grad_(pos_grad)
    y = model(Batch(b.atoms.to(DEV), pd, b.edge_index.to(DEV), b.batch.to(DEV),
                    num_graphs=b.num_graphs))
    pr = b.pos.clone().requires_grad_(pos_grad)
    yr = ref(Batch(b.atoms, pr, b.edge_index, b.batch, num_graphs=b.num_graphs))
    torch.testing.assert_close(y.detach().cpu(), yr.detach(), atol=1e-5, rtol=1e-5)
    g = torch.randn_like(yr)
    (y * g.to(DEV)).sum().backward()
    (yr * g).sum().backward()
    if pos_grad:
        _scaled(pd.grad, pr.grad, 1e-4, "grad_pos")
    for (k, p), q in zip(model.named_parameters(), ref.parameters()):
        _scaled(p.grad, q.grad, 1e-4, k)


@pytest.mark.parametrize("F,n,E", [(128, 300, 5000), (64, 50, 0), (4, 7, 40), (260, 33, 900)])
def test_cfconv_aggregate_vs_torch(F, n, E):
    """K13 (gmp_cfconv_aggregate_f32 / gmp_cfconv_wgrad_f32) against the plain-PyTorch fp32
    restatement of CFConv's propagate: x[src] * W summed at dst (index_add_), and its
    gradients.  Isolated receivers (n > max dst) come out as zero rows.  Tolerance 1e-5."""
    from gmp_amd import ops
    gen = torch.Generator().manual_seed(F + n + E)
    ei = torch.randint(0, max(n - 3, 1), (2, E), generator=gen)
    x = torch.randn(n, F, generator=gen)
    W = torch.randn(E, F, generator=gen)
    xd, Wd = x.to(DEV).requires_grad_(True), W.to(DEV).requires_grad_(True)
    y = ops.cfconv_propagate(ei.to(DEV), xd, Wd)
    xr, Wr = x.clone().requires_grad_(True), W.clone().requires_grad_(True)
    yr = torch.zeros(n, F).index_add_(0, ei[1], xr[ei[0]] * Wr)
    torch.testing.assert_close(y.detach().cpu(), yr.detach(), atol=1e-5, rtol=1e-5)
    g = torch.randn(n, F, generator=gen)
    (y * g.to(DEV)).sum().backward()
    (yr * g).sum().backward()
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(Wd.grad.cpu(), Wr.grad, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("F,n,E", [(128, 300, 5000), (4, 7, 40)])
def test_cfconv_scaled_vs_torch(F, n, E):
    """K13 scaled forms: x[src] * (W * C) summed at dst with the per-edge factor C applied at
    load time, against torch's (W * C.view(-1, 1)) message and index_add_; gradients of x and
    W (w.r.t. the unscaled W).  Tolerance 1e-5."""
    from gmp_amd import ops
    gen = torch.Generator().manual_seed(F + E)
    ei = torch.randint(0, n, (2, E), generator=gen)
    x, W, C = torch.randn(n, F, generator=gen), torch.randn(E, F, generator=gen), torch.rand(E, generator=gen)
    xd, Wd = x.to(DEV).requires_grad_(True), W.to(DEV).requires_grad_(True)
    y = ops.cfconv_propagate(ei.to(DEV), xd, Wd, C.to(DEV))
    xr, Wr = x.clone().requires_grad_(True), W.clone().requires_grad_(True)
    yr = torch.zeros(n, F).index_add_(0, ei[1], xr[ei[0]] * (Wr * C.view(-1, 1)))
    torch.testing.assert_close(y.detach().cpu(), yr.detach(), atol=1e-5, rtol=1e-5)
    g = torch.randn(n, F, generator=gen)
    (y * g.to(DEV)).sum().backward()
    (yr * g).sum().backward()
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(Wd.grad.cpu(), Wr.grad, atol=1e-5, rtol=1e-5)
    with pytest.raises(ValueError):
        ops.cfconv_propagate(ei.to(DEV), xd, Wd, C.to(DEV).requires_grad_(True))


def test_cfconv_aggregate_out_of_range_raises():
    from gmp_amd import ops
    ei = torch.tensor([[0, 1, 9], [1, 2, 0]], device=DEV)
    x = torch.randn(4, 8, device=DEV)
    W = torch.randn(3, 8, device=DEV)
    with pytest.raises(IndexError):
        ops.cfconv_propagate(ei.flip(0), x, W)  # dst 9 >= N = 4


def test_shifted_softplus_vs_torch():
    """K14 (gmp_ssp_{fwd,bwd}_f32) against torch F.softplus(x) - log 2 on CPU fp32, across the
    threshold (x > 20 is the identity branch) and deep negatives.  Tolerance 1e-6 abs +
    1e-5 rel."""
    import math
    from gmp_amd import ops
    x = torch.cat([torch.randn(4000) * 8, torch.tensor([-100., -20., 0., 19.99, 20., 20.01,
                                                         50., 1e-7])])
    g = torch.randn_like(x)
    xd = x.to(DEV).requires_grad_(True)
    y = ops.shifted_softplus(xd, math.log(2.0))
    y.backward(g.to(DEV))
    xr = x.clone().requires_grad_(True)
    yr = torch.nn.functional.softplus(xr) - math.log(2.0)
    yr.backward(g)
    torch.testing.assert_close(y.detach().cpu(), yr.detach(), atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("E,G,cutoff", [(20000, 50, 10.0), (333, 7, 4.0), (0, 50, 10.0)])
def test_schnet_featurize_vs_oracle(E, G, cutoff):
    """K1 SchNet featurisation (gmp_schnet_featurize_f32 and its backward) against the CPU
    restatement (oracle/schnet.py: |pos[row] - pos[col]|, GaussianSmearing, CFConv's cosine
    cutoff), including a zero-length edge (gradient 0, as torch's norm backward) and edges past
    the cutoff.  Tolerance 1e-5 on the features, 1e-5 of scale on d pos."""
    from gmp_amd import ops
    gen = torch.Generator().manual_seed(E + G)
    n = max(E // 20, 4)
    pos = torch.rand(n, 3, generator=gen) * 1.5 * cutoff
    ei = torch.randint(0, n, (2, E), generator=gen)
    if E:
        ei[:, 0] = 3  # a zero-length edge
    gs = osch.GaussianSmearing(0.0, cutoff, G)
    pd = pos.to(DEV).requires_grad_(True)
    d, rbf, C = ops.SchNetFeaturizeFn.apply(pd, ei.to(DEV), gs.offset.to(DEV), gs.coeff, cutoff)
    pr = pos.clone().requires_grad_(True)
    dr = (pr[ei[0]] - pr[ei[1]]).norm(dim=-1)
    rbfr = gs(dr)
    Cr = 0.5 * (torch.cos(dr * math.pi / cutoff) + 1.0)
    for a, b in ((d, dr), (rbf, rbfr), (C, Cr)):
        torch.testing.assert_close(a.detach().cpu(), b.detach(), atol=1e-5, rtol=1e-5)
    if E == 0:
        return
    g1, g2, g3 = torch.randn_like(dr), torch.randn_like(rbfr), torch.randn_like(Cr)
    ((d * g1.to(DEV)).sum() + (rbf * g2.to(DEV)).sum() + (C * g3.to(DEV)).sum()).backward()
    ((dr * g1).sum() + (rbfr * g2).sum() + (Cr * g3).sum()).backward()
    _scaled(pd.grad, pr.grad, 1e-5, "dpos")


@pytest.mark.parametrize("n,offset", [(4000, 0), (4001, 0), (4008, 1), (4000, 3)])
def test_shifted_softplus_module_gate_and_fallback(n, offset):
    """ShiftedSoftplus through the module: odd numel and misaligned views take the torch path,
    aligned ones K14 (n = 4000, offset 0); the upstream gradient always arrives misaligned (a
    contiguous view at an odd offset), which K14's backward must accept.  Outputs and
    gradients vs torch."""
    import math
    from gmp_amd.schnet import ShiftedSoftplus
    m = ShiftedSoftplus()
    base = torch.randn(n + offset, device=DEV) * 6
    x = base[offset:].detach().requires_grad_(True)
    y = m(x)
    yr = torch.nn.functional.softplus(x.detach().cpu()) - math.log(2.0)
    torch.testing.assert_close(y.detach().cpu(), yr, atol=1e-6, rtol=1e-5)
    g = torch.randn(n + 1, device=DEV)[1:]
    y.backward(g)
    gr = g.cpu() * torch.sigmoid(x.detach().cpu())
    torch.testing.assert_close(x.grad.cpu(), gr, atol=1e-6, rtol=1e-5)
