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


def _ln_bwd_c_abi(rows, d, act, with_gb, guard=4096):
    """gmp_ln_act_bwd_f32 through the C ABI.  with_gb=False: the caller-reduces form
    (grad_gamma_beta NULL: the workspace holds gmp_ln_act_bwd_partial_rows(rows) partial rows,
    reduced here by gmp_sum_rows_f32).  The workspace is exactly gmp_ln_act_bwd_workspace_size
    floats followed by a guard band that must stay untouched (the size reported for
    the vectorised form was overrun by the generic fallback below ~16k rows)."""
    import ctypes
    from gmp_amd import _lib, ops
    lib = _lib.load()
    g = torch.Generator().manual_seed(rows * 7 + d)
    x = (torch.randn(rows, d, generator=g) * 2).to(DEV)
    gamma = torch.randn(d, generator=g).to(DEV)
    beta = torch.randn(d, generator=g).to(DEV)
    gy = torch.randn(rows, d, generator=g).to(DEV)
    y, xhat, rstd = _lib.torch_ops().ln_act_fwd(x, gamma, beta, 1e-5, act)
    ws_bytes = lib.gmp_ln_act_bwd_workspace_size(rows, d)
    assert ws_bytes % 4 == 0
    ws = torch.full((ws_bytes // 4 + guard,), 12345.0, device=DEV)
    gx = torch.empty_like(x)
    gb = torch.empty(2 * d, device=DEV) if with_gb else None
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.gmp_ln_act_bwd_f32(rows, d, p(gy), p(xhat), p(rstd), p(gamma), p(beta), act,
                                      p(gx), p(gb), p(ws), ws_bytes, st), "gmp_ln_act_bwd_f32")
    if not with_gb:
        nrows = lib.gmp_ln_act_bwd_partial_rows(rows)
        assert nrows * 2 * d * 4 <= ws_bytes
        gb = torch.empty(2 * d, device=DEV)
        _lib.check(lib.gmp_sum_rows_f32(p(ws), nrows, 2 * d, p(gb), st), "gmp_sum_rows_f32")
    torch.cuda.synchronize()
    assert torch.all(ws[ws_bytes // 4:] == 12345.0), "workspace overrun"
    # torch fp32 reference of the same backward
    xa = x.clone().requires_grad_(True)
    ga = gamma.clone().requires_grad_(True)
    ba = beta.clone().requires_grad_(True)
    fn = {0: F.relu, 1: F.silu, 2: lambda t: t}[act]
    (fn(F.layer_norm(xa, (d,), ga, ba, 1e-5)) * gy).sum().backward()
    for a, b in ((gx, xa.grad), (gb[:d], ga.grad), (gb[d:], ba.grad)):
        scale = max(1.0, b.abs().max().item())
        assert (a - b).abs().max().item() <= 1e-5 * scale * (1 + rows ** 0.5 / 10)


@pytest.mark.parametrize("rows,d", [(1000, 32), (1000, 128), (1000, 100), (17, 64), (20_000, 256)])
@pytest.mark.parametrize("act", [0, 1])
def test_ln_act_bwd_caller_reduces(rows, d, act):
    _ln_bwd_c_abi(rows, d, act, with_gb=False)


@pytest.mark.parametrize("rows,d", [(1000, 32), (1000, 128), (1000, 100), (3, 8), (70_000, 128)])
def test_ln_act_bwd_workspace_bound(rows, d):
    _ln_bwd_c_abi(rows, d, 0, with_gb=True)
