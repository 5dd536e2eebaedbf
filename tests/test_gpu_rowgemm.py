"""Row-level Linears on the K7g kernel (gmp_split_x3_f32 + gmp_gemm_x3_f32): [a1 | a2] B^T + b
with B = W or W^T (weight slices included) against an fp64 torch reference of the same op
(three-plane bf16 products: f32-class, bound 2e-6 of the row's |a| |b| scale), and the
EGNN / Linear autograd paths that use it against the library path (GMP_ROW_GEMM=torch
semantics, same module)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ref(a1, a2, B, b):
    a = a1.double() if a2 is None else torch.cat([a1, a2], 1).double()
    y = a @ B.double().t()
    return y + b.double() if b is not None else y


def _bound(a1, a2, B):
    a = a1 if a2 is None else torch.cat([a1, a2], 1)
    return (a.abs().double() @ B.abs().double().t())


@pytest.mark.parametrize("M,N,K1,K2,bias,transpose", [
    (0, 128, 128, 0, True, False), (1, 16, 32, 0, False, False), (1000, 128, 128, 0, True, False),
    (50000, 256, 128, 0, False, False), (50000, 128, 128, 128, True, False),
    (4097, 64, 96, 32, True, False), (3000, 128, 128, 0, False, True),
    (777, 48, 64, 64, True, False), (400, 128, 128, 128, False, True)])
def test_gemm_x3_vs_fp64(M, N, K1, K2, bias, transpose):
    from gmp_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M + N + K1)
    a1 = torch.randn(M, K1, device=DEV, generator=g)
    a2 = torch.randn(M, K2, device=DEV, generator=g) if K2 else None
    W = torch.randn((K1 + K2, N) if transpose else (N, K1 + K2), device=DEV, generator=g) * 0.1
    b = torch.randn(N, device=DEV, generator=g) if bias else None
    y = ops.linear_x3(a1, a2, W, b, transpose)
    B = W.t() if transpose else W
    ref = _ref(a1, a2, B, b)
    assert y.shape == (M, N) and y.dtype == torch.float32
    if M:
        err = (y.double() - ref).abs()
        assert bool((err <= 2e-6 * _bound(a1, a2, B) + 1e-6).all()), err.max().item()


def test_split_x3_strided_slice():
    """A column slice of a weight (SplitLinear's dx operands) splits like its contiguous copy."""
    from gmp_amd import _lib
    tops = _lib.torch_ops()
    W = torch.randn(128, 256, device=DEV)
    for tr in (False, True):
        a = tops.split_x3(W[:, 128:], tr)
        b = tops.split_x3(W[:, 128:].contiguous(), tr)
        assert torch.equal(a, b)


def test_linear_paths_match_library():
    """EdgeLinearFn / SplitLinearFn forward + backward on the x3 GEMMs vs the library path."""
    from gmp_amd import ops
    torch.manual_seed(0)
    x = torch.randn(40000, 128, device=DEV, requires_grad=True)
    xb = torch.randn(40000, 128, device=DEV, requires_grad=True)
    W = (torch.randn(128, 128, device=DEV) * 0.05).requires_grad_(True)
    W2 = (torch.randn(128, 256, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(128, device=DEV, requires_grad=True)
    gy = torch.randn(40000, 128, device=DEV)
    outs = {}
    prev = ops.ROW_GEMM
    for mode in ("x3", "torch"):
        ops.ROW_GEMM = mode
        try:
            for t in (x, xb, W, W2, b):
                t.grad = None
            y = ops.linear(x, W, b) + ops.split_linear(x, xb, W2, b)
            (y * gy).sum().backward()
            torch.cuda.synchronize()
            outs[mode] = [y.detach()] + [t.grad.clone() for t in (x, xb, W, W2, b)]
        finally:
            ops.ROW_GEMM = prev
    for a, r in zip(outs["x3"], outs["torch"]):
        scale = r.abs().max().item()
        assert (a - r).abs().max().item() <= 1e-5 * scale + 1e-6
