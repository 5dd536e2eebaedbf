"""Receiver-factorised TP kernels (gmp_tpnode.hip) at the C ABI against an fp64 torch evaluation,
with in-degrees on both sides of the one-stage fast path of the S kernel (0, 1, 31, 32 edges:
Z prefetched per k step; 33, 64, 100: multi-stage path) and path widths that are not a multiple
of the 64-row workgroup block."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(degs, w, H, seed):
    g = torch.Generator().manual_seed(seed)
    degs = torch.tensor(degs, dtype=torch.int64)
    eoff = torch.zeros(len(degs) + 1, dtype=torch.int64)
    eoff[1:] = torch.cumsum(degs, 0)
    ne = int(eoff[-1])
    Z = torch.randn(ne + 1, w, generator=g)
    A = torch.randn(ne, H, generator=g)
    return eoff, Z, A, ne


@pytest.mark.parametrize("w,H", [(40, 48), (640, 256), (96, 16)])
def test_node_outer_matches_fp64(w, H):
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    degs = [0, 1, 31, 32, 33, 64, 100, 20, 7, 0, 45]
    eoff, Z, A, ne = _setup(degs, w, H, seed=w + H)
    c = len(degs)
    S = torch.empty(c, w, H, device=DEV)
    Sb = torch.empty(c, w, device=DEV)
    eo_d, Z_d, A_d = eoff.to(DEV), Z.to(DEV), A.to(DEV)  # held: raw pointers go to the ABI
    rc = lib.gmp_tp_node_outer_f32(c, w, H, _p(eo_d), _p(Z_d), _p(A_d), _p(S), _p(Sb), _stream())
    assert rc == 0
    torch.cuda.synchronize()
    for n in range(c):
        e0, e1 = int(eoff[n]), int(eoff[n + 1])
        ref = Z[e0:e1].double().t() @ A[e0:e1].double()
        refb = Z[e0:e1].double().sum(0)
        scale = Z[e0:e1].double().abs().t() @ A[e0:e1].double().abs()
        if e1 > e0:
            err = ((S[n].cpu().double() - ref).abs() / scale.clamp_min(1e-30)).max().item()
        else:
            err = S[n].abs().max().item()
        assert err < 1e-6, (n, degs[n], err)
        torch.testing.assert_close(Sb[n].cpu().double(), refb, atol=1e-5, rtol=1e-5)


def test_node_apply_matches_fp64():
    """dZ[e, r] = sum_j T[n, r, j] A[e, j] + Tb[n, r];  dA[e, j] += sum_r Z[e, r] T[n, r, j]"""
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    degs = [0, 1, 31, 32, 33, 64, 5]
    w, H = 72, 48
    eoff, Z, A, ne = _setup(degs, w, H, seed=3)
    c = len(degs)
    g = torch.Generator().manual_seed(4)
    T = torch.randn(c, w, H, generator=g)
    Tb = torch.randn(c, w, generator=g)
    dZ = torch.zeros(ne + 1, w, device=DEV)
    dA = torch.zeros(ne, H, device=DEV)
    eo_d, Z_d, A_d, T_d, Tb_d = (t.to(DEV) for t in (eoff, Z, A, T, Tb))
    rc = lib.gmp_tp_node_apply_f32(c, w, H, _p(eo_d), _p(Z_d), _p(A_d), _p(T_d), _p(Tb_d),
                                   _p(dZ), _p(dA), _stream())
    assert rc == 0
    torch.cuda.synchronize()
    for n in range(c):
        e0, e1 = int(eoff[n]), int(eoff[n + 1])
        if e1 == e0:
            continue
        rz = A[e0:e1].double() @ T[n].double().t() + Tb[n].double()
        ra = Z[e0:e1].double() @ T[n].double()
        torch.testing.assert_close(dZ[e0:e1].cpu().double(), rz, atol=1e-4, rtol=1e-5)
        torch.testing.assert_close(dA[e0:e1].cpu().double(), ra, atol=1e-4, rtol=1e-5)
