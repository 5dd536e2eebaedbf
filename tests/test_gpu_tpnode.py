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


def _planes_to_f64(planes, shape):
    """Sum of the three bf16 planes (int16 bit patterns) as float64."""
    p = planes.view(torch.bfloat16).view(3, *shape).double()
    return p[0] + p[1] + p[2]


def _frag_order(P):
    """(NP, N, K) row-major planes -> the forward GEMM's MFMA fragment order (gmp.h,
    gmp_tp_gemm_x3_f32): blocks (k step, column tile, plane) of 64 lanes x 8 values, lane
    l = n % 16 + 16 ((k % 32) / 8)."""
    NP, N, K = P.shape
    x = P.reshape(NP, N // 16, 16, K // 32, 4, 8)  # p, ct, li, ks, g, e
    return x.permute(3, 1, 0, 4, 2, 5).contiguous().view(-1)


def _from_frag_order(flat, NP, N, K):
    x = flat.reshape(K // 32, N // 16, NP, 4, 16, 8)  # ks, ct, p, g, li, e
    return x.permute(2, 1, 4, 0, 3, 5).reshape(NP, N, K)


@pytest.mark.parametrize("m1,mo,H", [(128, 128, 256), (64, 64, 256), (32, 128, 64)])
def test_split_w2_planes_exact(m1, mo, H):
    """gmp_tp_split_w2_f32: the three bf16 planes of every W2 / b2 entry sum to it exactly, in
    the forward [w][(u, j) ++ u] (in MFMA fragment order) and backward [(u, j)][w] layouts."""
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    g = torch.Generator().manual_seed(m1 + H)
    W2 = (torch.randn(m1 * mo, H, generator=g) * torch.logspace(-6, 2, H)).to(DEV)
    b2 = torch.randn(m1 * mo, generator=g).to(DEV)
    K1 = m1 * H
    Bf = torch.empty(3 * mo * (K1 + m1), dtype=torch.int16, device=DEV)
    Bt = torch.empty(3 * K1 * mo, dtype=torch.int16, device=DEV)
    assert lib.gmp_tp_split_w2_f32(m1, mo, H, _p(W2), _p(b2), _p(Bf), _p(Bt), _stream()) == 0
    torch.cuda.synchronize()
    W = W2.cpu().double().view(m1, mo, H)                      # [u][w][j]
    f = _planes_to_f64(_from_frag_order(Bf.cpu(), 3, mo, K1 + m1).contiguous(), (mo, K1 + m1))
    assert torch.equal(f[:, :K1], W.permute(1, 0, 2).reshape(mo, K1))
    assert torch.equal(f[:, K1:], b2.cpu().double().view(m1, mo).t())
    t = _planes_to_f64(_from_frag_order(Bt.cpu(), 3, K1, mo).contiguous(), (K1, mo))
    assert torch.equal(t, W.permute(0, 2, 1).reshape(K1, mo))


@pytest.mark.parametrize("M,N,K1,K2,grp", [(1000, 128, 256, 32, 5), (333, 64, 128, 0, 1),
                                           (257, 4096, 128, 0, 1), (130, 128, 4096, 128, 3),
                                           (65, 32, 96, 32, 1), (5003, 64, 1024, 64, 3),
                                           (700, 48, 256, 32, 5)])
def test_tp_gemm_x3_matches_fp64(M, N, K1, K2, grp):
    """gmp_tp_gemm_x3_f32 (bf16 MFMA over three-plane splits) against fp64: error per entry
    <= 1e-6 of sum |a b| (f32-class; f32 unit roundoff 6e-8, a K-term f32 sum ~ sqrt(K) of it),
    ragged M / N tiles, the second A operand, the grouped (r / grp) epilogue addressing with
    accumulation into an existing output; k-step counts that are and are not multiples of the
    8-deep register ring (9, 4 and 132 steps; K <= 256 takes the 2-deep ring); N <= 64 runs the
    256 x 64 tile (C5's 64-channel paths; ragged rows of its 256-row tile)."""
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N)
    A1 = torch.randn(M, K1, generator=g) * torch.logspace(-3, 1, K1)
    A2 = torch.randn(M, max(K2, 1), generator=g)[:, :K2].contiguous()
    B = torch.randn(N, K1 + K2, generator=g)
    # planes of B (RNE splits as the kernel expects; computed here from the fp32 values)
    b0 = B.to(torch.bfloat16)
    r1 = B - b0.float()
    b1 = r1.to(torch.bfloat16)
    b2 = (r1 - b1.float()).to(torch.bfloat16)
    Bp = _frag_order(torch.stack([b0, b1, b2]).contiguous().view(torch.int16)).to(DEV)
    ref = A1.double() @ B[:, :K1].double().t()
    mag = A1.double().abs() @ B[:, :K1].double().abs().t()
    if K2:
        ref += A2.double() @ B[:, K1:].double().t()
        mag += A2.double().abs() @ B[:, K1:].double().abs().t()
    if grp == 1:
        C0 = torch.randn(M, N, generator=g)
        C = C0.clone().to(DEV)
        acc = 1
        args = (1, N, 0, 1)
    else:
        # out[r / grp, (r % grp) + col * grp] of rows (n, k): the forward's mul_ir block
        nr = -(-M // grp)
        C0 = torch.randn(nr, N * grp + 5, generator=g)
        C = C0.clone().to(DEV)
        acc = 1
        args = (grp, N * grp + 5, 1, grp)
    A1d, A2d = A1.to(DEV), A2.to(DEV)
    rc = lib.gmp_tp_gemm_x3_f32(M, N, K1, _p(A1d), K1, K2, _p(A2d) if K2 else None, max(K2, 1),
                                _p(Bp), K1 + K2, N * (K1 + K2), _p(C), *args, acc, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    out = C.cpu().double()
    if grp == 1:
        got = out - C0.double()
    else:
        r = torch.arange(M)
        idx = (r % grp)[:, None] + torch.arange(N)[None, :] * grp
        got = out[(r // grp)[:, None], idx] - C0.double()[(r // grp)[:, None], idx]
        untouched = torch.ones_like(out, dtype=torch.bool)
        untouched[(r // grp)[:, None], idx] = False
        assert torch.equal(out[untouched], C0.double()[untouched])
    err = ((got - ref).abs() / mag.clamp_min(1e-30)).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("K,m_total,n", [(3000, 256, 128), (70000, 1024, 128), (5000, 384, 64),
                                         (4000, 128, 32)])
def test_outer_sum_cols_matches_fp64(K, m_total, n):
    """gmp_outer_sum_cols_f32: C = A^T B over K rows for a wide A (column blocks of 128),
    deterministic, within 1e-6 of sum |a b| per entry."""
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    g = torch.Generator().manual_seed(K + m_total)
    A = torch.randn(K, m_total, generator=g)
    B = torch.randn(K, n, generator=g)
    Ad, Bd = A.to(DEV), B.to(DEV)
    ws_b = lib.gmp_outer_sum_cols_workspace_size(K, m_total, n)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=DEV)
    outs = []
    for _ in range(2):
        C = torch.full((m_total, n), float("nan"), device=DEV)
        assert lib.gmp_outer_sum_cols_f32(K, m_total, n, _p(Ad), m_total, _p(Bd), n, _p(C), n,
                                          _p(ws), ws_b, _stream()) == 0
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = A.double().t() @ B.double()
    mag = A.double().abs().t() @ B.double().abs()
    err = ((outs[0].cpu().double() - ref).abs() / mag).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("M,N,K", [(1000, 8192, 128), (333, 4096 + 64, 64), (130, 1024, 96),
                                   (17, 256, 32), (40, 384, 96)])
def test_tp_gemm_x3_widen_matches_fp64(M, N, K):
    """gmp_tp_gemm_x3_widen_f32 (resident A, swept column tiles): C = A B^T within 1e-6 of
    sum |a b| per entry, ragged M and N, every K / 32 variant."""
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) * torch.logspace(-4, 1, K)
    b0 = B.to(torch.bfloat16)
    r1 = B - b0.float()
    b1 = r1.to(torch.bfloat16)
    b2 = (r1 - b1.float()).to(torch.bfloat16)
    Bp = _frag_order(torch.stack([b0, b1, b2]).contiguous().view(torch.int16)).to(DEV)
    Ad = A.to(DEV)
    C = torch.full((M, N + 3), 7.0, device=DEV)
    assert lib.gmp_tp_gemm_x3_widen_f32(M, N, K, _p(Ad), K, _p(Bp), K, N * K, _p(C), N + 3,
                                        _stream()) == 0
    torch.cuda.synchronize()
    out = C.cpu().double()
    assert torch.equal(out[:, N:], torch.full((M, 3), 7.0, dtype=torch.float64))
    ref = A.double() @ B.double().t()
    mag = A.double().abs() @ B.double().abs().t()
    err = ((out[:, :N] - ref).abs() / mag).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("w,H", [(640, 256), (544, 64), (96, 64), (128, 192), (128, 160),
                                 (192, 256), (32, 256), (96, 256)])
@pytest.mark.parametrize("x3", [2, 1, 0])
def test_node_apply_bf16x3_matches_fp64(w, H, x3):
    """The apply kernels against fp64: x3 = 2 the v3 kernel (per-wave j quarters; H = 256,
    w % 32 == 0), x3 = 1 the v2 bf16x3 kernel (w >= 512, w % 32 == 0, H % 64 == 0), x3 = 0 the
    f32-MFMA kernel; shapes outside a form's range take the next one.  Edge groups of 0, 1, 16,
    17, 31, 32, 33 and 70 edges (one or two 16-edge tiles, several 32-edge groups): dZ
    overwritten (+ Tb), dA accumulated onto existing values; error <= 1e-6 of the sum of |terms|
    per entry."""
    from gmp_amd import _lib
    from gmp_amd.ops import _p, _stream
    lib = _lib.load()
    degs = [0, 1, 31, 32, 33, 70, 20, 5, 16, 17]
    eoff, Z, A, ne = _setup(degs, w, H, seed=w + H)
    c = len(degs)
    g = torch.Generator().manual_seed(9)
    T = torch.randn(c, w, H, generator=g) * torch.logspace(-3, 1, H)
    Tb = torch.randn(c, w, generator=g)
    dA0 = torch.randn(ne, H, generator=g)
    dZ = torch.full((ne + 1, w), 7.0, device=DEV)
    dA = dA0.clone().to(DEV)
    eo_d, Z_d, A_d, T_d, Tb_d = (t.to(DEV) for t in (eoff, Z, A, T, Tb))
    old = lib.gmp_tp_apply_set_x3(x3)
    try:
        rc = lib.gmp_tp_node_apply_f32(c, w, H, _p(eo_d), _p(Z_d), _p(A_d), _p(T_d), _p(Tb_d),
                                       _p(dZ), _p(dA), _stream())
        torch.cuda.synchronize()
    finally:
        lib.gmp_tp_apply_set_x3(old)
    assert rc == 0
    assert torch.equal(dZ[ne].cpu(), torch.full((w,), 7.0))  # padding row untouched
    for n in range(c):
        e0, e1 = int(eoff[n]), int(eoff[n + 1])
        if e1 == e0:
            continue
        rz = A[e0:e1].double() @ T[n].double().t() + Tb[n].double()
        mz = A[e0:e1].double().abs() @ T[n].double().abs().t() + Tb[n].double().abs()
        ra = Z[e0:e1].double() @ T[n].double() + dA0[e0:e1].double()
        ma = Z[e0:e1].double().abs() @ T[n].double().abs() + dA0[e0:e1].double().abs()
        ez = ((dZ[e0:e1].cpu().double() - rz).abs() / mz).max().item()
        ea = ((dA[e0:e1].cpu().double() - ra).abs() / ma).max().item()
        assert ez < 1e-6 and ea < 1e-6, (n, degs[n], ez, ea)
