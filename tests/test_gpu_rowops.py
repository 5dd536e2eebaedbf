"""K12 fused LayerNorm + activation (gmp_ln_act_*) against the PyTorch fp32 reference
(nn.LayerNorm + activation), forward and backward, tolerance 1e-5 (scaled)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("rows,d", [(1, 32), (37, 100), (5000, 128), (50_000, 128), (300, 512),
                                    (200_000, 128), (3000, 64), (7000, 256), (1, 128),
                                    (300_000, 32), (777, 16), (1001, 8), (65, 32)])
@pytest.mark.parametrize("act", ["relu", "silu", None])
def test_ln_act_matches_torch(rows, d, act):
    from gmp_amd import ops
    g = torch.Generator().manual_seed(rows + d)
    x = (torch.randn(rows, d, generator=g) * 3 + 1).to(DEV)
    ln = torch.nn.LayerNorm(d).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(torch.randn(d, generator=g))
        ln.bias.copy_(torch.randn(d, generator=g))
    gy = torch.randn(rows, d, generator=g).to(DEV)
    fn = {"relu": F.relu, "silu": F.silu, None: lambda t: t}[act]

    xa = x.clone().requires_grad_(True)
    y = ops.ln_act(xa, ln, act)
    (y * gy).sum().backward()
    got = (y.detach(), xa.grad, ln.weight.grad.clone(), ln.bias.grad.clone())
    ln.weight.grad = ln.bias.grad = None

    xb = x.clone().requires_grad_(True)
    yr = fn(ln(xb))
    (yr * gy).sum().backward()
    ref = (yr.detach(), xb.grad, ln.weight.grad, ln.bias.grad)
    for a, b in zip(got, ref):
        scale = max(1.0, b.abs().max().item())
        assert (a - b).abs().max().item() <= 1e-5 * scale * (1 + rows ** 0.5 / 10)


@pytest.mark.parametrize("rows,d", [(20_000, 128), (200_000, 32)])
def test_ln_act_deterministic(rows, d):
    from gmp_amd import ops
    x = torch.randn(rows, d, device=DEV)
    ln = torch.nn.LayerNorm(d).to(DEV)
    outs = []
    for _ in range(2):
        xa = x.clone().requires_grad_(True)
        ops.ln_act(xa, ln, "relu").sum().backward()
        outs.append((xa.grad.clone(), ln.weight.grad.clone()))
        ln.weight.grad = ln.bias.grad = None
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_ln_act_bwd_tickets_reset_across_calls():
    """The vectorised backward's two-level last-workgroup sums (tree_finish) leave their ticket
    words zeroed: interleaved launches of different sizes on one stream give the same results
    as each alone."""
    from gmp_amd import ops
    torch.manual_seed(3)
    res = {}
    for rows in (64_000, 900, 64_000, 130_000, 900):
        x = torch.randn(rows, 128, device=DEV, generator=None)
        torch.manual_seed(rows)
        x = torch.randn(rows, 128, device=DEV)
        ln = torch.nn.LayerNorm(128).to(DEV)
        xa = x.clone().requires_grad_(True)
        ops.ln_act(xa, ln, "silu").square().sum().backward()
        got = (xa.grad.clone(), ln.weight.grad.clone(), ln.bias.grad.clone())
        if rows in res:
            assert all(torch.equal(a, b) for a, b in zip(res[rows], got)), rows
        res[rows] = got
