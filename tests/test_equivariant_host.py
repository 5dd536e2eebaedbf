"""Host-side checks of the TFN / MACE product layers (no GPU): module trees and state_dict keys
match the oracle (hence the reference's), the node-level e3nn pieces (o3.Linear, BatchNorm,
Gate, SymmetricContraction, which run as PyTorch ops on N-row tensors) agree with the oracle,
and the K7 path tables are well formed."""
import os

import pytest
import torch

from oracle import mace as om
from oracle import o3 as oo3


def _eq():
    from gmp_amd import equivariant
    return equivariant


@pytest.mark.parametrize("kind,kw", [("MACEModel", dict(num_layers=3, emb_dim=16, correlation=3)),
                                     ("TFNModel", dict(num_layers=3, emb_dim=16)),
                                     ("MACEModel", dict(num_layers=2, emb_dim=128)),
                                     ("TFNModel", dict(num_layers=2, emb_dim=64, batch_norm=True)),
                                     ("MACEModel", dict(num_layers=2, emb_dim=8, max_ell=3)),
                                     ("MACEModel", dict(num_layers=1, emb_dim=8, correlation=4)),
                                     ("MACEModel", dict(num_layers=1, emb_dim=8, correlation=2,
                                                        hidden_irreps="8x0e+8x0o+8x1e+8x1o+8x2e+8x2o")),
                                     ("TFNModel", dict(num_layers=2, emb_dim=8,
                                                       hidden_irreps="8x0e+8x0o+8x1e+8x1o+8x2e+8x2o"))])
def test_state_dict_keys_and_shapes(kind, kw):
    eq = _eq()
    ours, ref = getattr(eq, kind)(**kw), getattr(om, kind)(**kw)
    a, b = ours.state_dict(), ref.state_dict()
    assert list(a) == list(b)
    for k in b:
        assert a[k].shape == b[k].shape, k
        if "U_matrix" in k or "bessel" in k or k.endswith(("r_max", "prefactor", ".p")):
            torch.testing.assert_close(a[k], b[k], atol=1e-7, rtol=0)
    ours.load_state_dict(b, strict=True)


def test_tp_plan_tables():
    from gmp_amd import _lib, o3
    eq = _eq()
    hid = o3.hidden_irreps(128, 2)
    plan = eq.TPPlan(hid, o3.sh_irreps(2), hid)
    ref = oo3.FullyConnectedTensorProduct("128x0e+128x1o+128x2e", oo3.spherical_harmonics_irreps(2),
                                          "128x0e+128x1o+128x2e")
    assert plan.weight_numel == ref.weight_numel == 180224
    assert plan.desc.n_paths == 11 and plan.layout == 0 and plan.desc.in_dim == 1152
    for k, ins in enumerate(ref.instructions):
        p = plan.paths_host[k]
        assert p.w_off == ins["w_off"] and abs(p.alpha - ins["path_weight"]) < 1e-7
    assert plan.cg_host.numel() == sum(
        (2 * i["l1"] + 1) * (2 * i["l2"] + 1) * (2 * i["lo"] + 1) for i in plan.instructions)
    assert ctypes_size(_lib.TpPath) == 64 and ctypes_size(_lib.TpDesc) == 128
    s, g, v = o3.irreps2gate(o3.hidden_irreps(64, 2))
    gated = s + g + v
    plan_g = eq.TPPlan(o3.parse_irreps("64x0e"), o3.sh_irreps(2), gated)
    assert plan_g.layout == 1 and plan_g.desc.out_dim == 64 + 128 + 192 + 320
    # node form: any block structure with l <= 3 (no per-edge-weight layout)
    p1e = eq.TPPlan(hid, o3.sh_irreps(2), o3.parse_irreps("8x1e"))
    assert p1e.layout is None and p1e.desc.n_blocks == 1
    p3 = eq.TPPlan(o3.parse_irreps("64x0e+64x1o+64x2e+64x3o"), o3.sh_irreps(3),
                   o3.parse_irreps("64x0e+192x0e+64x1o+64x2e+64x3o"))
    assert p3.layout is None and p3.sh_dim == 16 and p3.desc.n_paths == 27
    assert p3.cg_host.numel() == 1959 and p3.z_size == 6592 and len(p3.desc_list) == 32
    assert p3.l_max == 3 and p3.desc_list[-1] == 3
    with pytest.raises(NotImplementedError):
        eq.TPPlan(hid, o3.sh_irreps(2), o3.parse_irreps("8x6e"))  # l <= 5
    with pytest.raises(NotImplementedError):
        eq.TPPlan(hid, o3.sh_irreps(6), hid)
    with pytest.raises(NotImplementedError):
        eq.TPPlan(hid, o3.sh_irreps(2),
                  o3.parse_irreps("8x0e+8x1o+8x0e+8x1o+8x0e+8x1o+8x0e+8x1o+8x2e"))  # 9 blocks
    # both parities / repeated l (the incompleteness configs): node form
    bp = o3.parse_irreps("32x0e+32x0o+32x1e+32x1o+32x2e+32x2o")
    pb = eq.TPPlan(bp, o3.sh_irreps(2), bp)
    assert pb.layout is None and pb.desc.n_paths == 30 and pb.desc.n_blocks == 6


def ctypes_size(t):
    import ctypes
    return ctypes.sizeof(t)


def test_node_ops_vs_oracle():
    eq = _eq()
    torch.manual_seed(0)
    irr = "8x0e+8x1o+8x2e"
    x = torch.randn(37, 72)
    # o3.Linear
    a, b = eq.Linear(irr, irr), oo3.Linear(irr, irr)
    a.load_state_dict(b.state_dict())
    torch.testing.assert_close(a(x), b(x), atol=1e-5, rtol=1e-5)
    # BatchNorm and Gate are HIP kernels (K16): tests/test_gpu_equivariant.py


@pytest.mark.parametrize("corr,irr", [(1, "8x0e+8x1o+8x2e"), (2, "8x0e+8x1o+8x2e"),
                                      (3, "8x0e+8x1o+8x2e"), (4, "4x0e+4x1o+4x2e"),
                                      (4, "4x0e+4x1o"), (3, "4x0e+4x1o+4x2e+4x3o"),
                                      (2, "4x0e+4x0o+4x1e+4x1o+4x2e+4x2o")])
def test_symmetric_contraction_vs_oracle(corr, irr):
    """The per-irrep contraction (the torch path for irreps K8 does not take; K8's own host
    logic, coefficients() and fold_symmetric, is checked through it on the GPU) vs the oracle,
    max_ell 1..3, correlation 4 (natural-parity coupling filter), both parities."""
    eq = _eq()
    torch.manual_seed(corr)
    a, b = eq.SymmetricContraction(irr, irr, corr), om.SymmetricContraction(irr, irr, corr)
    a.load_state_dict(b.state_dict())
    C = int(irr.split("x")[0])
    x = torch.randn(50, C, sum(2 * int(t.split("x")[1][:-1]) + 1 for t in irr.split("+")))
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    eq.Contraction.node_chunk = 16  # exercise node chunking + checkpoint
    try:
        ya, yb = a(xa), b(xb)
        torch.testing.assert_close(ya, yb, atol=1e-5, rtol=1e-5)
        g = torch.randn_like(yb)
        (ya * g).sum().backward()
        (yb * g).sum().backward()
    finally:
        eq.Contraction.node_chunk = 4096
    torch.testing.assert_close(xa.grad, xb.grad, atol=1e-5, rtol=1e-5)
    for (k, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-4, rtol=1e-5, msg=k)


def test_product_basis_block_golden(golden):
    """The reference's own symmetric contraction output (tests/golden, generated by running
    models/mace_modules/symmetric_contraction.py on the restated CG) through the product
    SymmetricContraction."""
    eq = _eq()
    d = golden("mace_symmetric_contraction.pt")
    sc = eq.SymmetricContraction("16x0e+16x1o+16x2e", "16x0e+16x1o+16x2e", 3)
    sc.load_state_dict({k[6:]: v for k, v in d.items() if k.startswith("param.")}, strict=True)
    x = d["x"].clone().requires_grad_(True)
    y = sc(x)
    torch.testing.assert_close(y, d["out"], atol=1e-5, rtol=1e-5)
    (y * d["g_out"]).sum().backward()
    torch.testing.assert_close(x.grad, d["grad_x"], atol=1e-5, rtol=1e-5)


def test_gvp_state_dict_keys():
    from oracle import gvp as ogvp
    import gmp_amd.gvp as g
    for kw in (dict(), dict(num_layers=2, s_dim=32, v_dim=4, s_dim_edge=8)):
        a, b = g.GVPGNNModel(**kw).state_dict(), ogvp.GVPGNNModel(**kw).state_dict()
        assert list(a) == list(b)
        assert all(a[k].shape == b[k].shape for k in b)


def test_schnet_oracle_known_answers():
    """PyG 2.3.1 SchNet internals restated (oracle/schnet.py): closed-form checks."""
    import math
    from oracle import schnet as osch
    gs = osch.GaussianSmearing(0.0, 10.0, 50)
    d = torch.tensor([0.0, 10.0 / 49 * 3])
    e = gs(d)
    assert abs(e[0, 0].item() - 1.0) < 1e-7 and abs(e[1, 3].item() - 1.0) < 1e-6
    assert abs(gs.coeff / (-0.5 / (10.0 / 49) ** 2) - 1) < 1e-6  # fp32 linspace spacing
    assert abs(osch.ShiftedSoftplus()(torch.zeros(1)).item()) < 1e-7
    m = osch.SchNetModel(hidden_channels=16, num_filters=8, num_layers=2)
    assert torch.all(m.embedding.weight[0] == 0)  # padding_idx = 0
    conv = m.interactions[0].conv
    assert conv.nn is m.interactions[0].mlp
    C = 0.5 * (math.cos(math.pi) + 1.0)
    assert abs(C) < 1e-12  # filter vanishes at the cutoff


_WIDENING = [("mace_symmetric_contraction_c4.pt", "4x0e+4x1o+4x2e", 4),
             ("mace_symmetric_contraction_l3.pt", "4x0e+4x1o+4x2e+4x3o", 3),
             ("mace_symmetric_contraction_bp3.pt", "4x0e+4x0o+4x1e+4x1o+4x2e+4x2o", 3),
             ("mace_symmetric_contraction_l5.pt", "4x0e+4x1o+4x2e+4x3o+4x4e+4x5o", 2)]


@pytest.mark.parametrize("name,irr,corr", _WIDENING)
def test_symmetric_contraction_widening_golden(golden, name, irr, corr):
    """The reference's own symmetric contraction at correlation 4 (cg.py's natural-parity
    coupling filter) and at max_ell 3 (tests/golden/make_golden.py mace_widening): the oracle and
    the product module's per-irrep path reproduce outputs and gradients."""
    eq = _eq()
    d = golden(name)
    params = {k[6:]: v for k, v in d.items() if k.startswith("param.")}
    for mod in (eq.SymmetricContraction(irr, irr, corr), om.SymmetricContraction(irr, irr, corr)):
        missing, unexpected = mod.load_state_dict(params, strict=False)
        assert not unexpected and all("U_matrix" in k for k in missing)
        x = d["x"].clone().requires_grad_(True)
        y = mod(x)
        torch.testing.assert_close(y, d["out"], atol=1e-5, rtol=1e-5)
        (y * d["g_out"]).sum().backward()
        torch.testing.assert_close(x.grad, d["grad_x"], atol=1e-5, rtol=1e-5)
        for k, p in mod.named_parameters():
            torch.testing.assert_close(p.grad, d["grad." + k], atol=1e-5, rtol=1e-5, msg=k)


def _eval_plan(sc, x):
    """The K8 term plan evaluated in torch exactly as gmp_sc.hip's forward walks it."""
    plan, M = sc._k8_plan.long(), sc._k8_rows
    C, D = x.shape[1], x.shape[2]
    row_ptr, base, stride = plan[:M + 1], plan[M + 1:2 * M + 1], plan[2 * M + 1:3 * M + 1]
    words = plan[3 * M + 1:] & 0xFFFFFFFF
    coef = sc.k8_coefficients()
    xx = torch.cat([x, torch.ones(x.shape[0], C, 1)], -1)
    out = torch.zeros(x.shape[0], M * C)
    cols = torch.arange(C)
    for m in range(M):
        acc = torch.zeros(x.shape[0], C)
        for t in range(int(row_ptr[m]), int(row_ptr[m + 1])):
            w = int(words[t])
            assert w >> 24 == m
            z = torch.ones(x.shape[0], C)
            for r in range(4):
                z = z * xx[:, :, (w >> (6 * r)) & 63]
            acc = acc + coef[t] * z
        out[:, int(base[m]) + int(stride[m]) * cols] = acc
    return out


@pytest.mark.parametrize("irr,corr", [("3x0e+3x1o+3x2e", 3), ("2x0e+2x0o+2x1e+2x1o+2x2e+2x2o", 3),
                                      ("2x0e+2x1o+2x2e+2x3o+2x4e+2x5o", 2), ("2x0e+2x1o", 4),
                                      ("2x1o+2x0e+2x1e", 2)])
def test_k8_term_plan_matches_contraction(irr, corr):
    """The K8 host logic (k8_plan: the structurally non-zero (row, monomial) pairs, the factor
    words with the 1.0 slot, the output columns; k8_coefficients: fold + gather) evaluated as the
    kernel walks it equals the module's per-irrep contraction (CPU)."""
    eq = _eq()
    torch.manual_seed(corr)
    sc = eq.SymmetricContraction(irr, irr, corr)
    assert sc._k8
    C = int(irr.split("x")[0])
    D = sum(2 * int(t.split("x")[1][:-1]) + 1 for t in irr.split("+"))
    x = torch.randn(6, C, D)
    with torch.no_grad():
        ref = torch.cat([c(x) for c in sc.contractions.values()], dim=-1)
        got = _eval_plan(sc, x)
    torch.testing.assert_close(got, ref, atol=2e-5, rtol=1e-5)


def test_k8_both_parity_correlation4_raises_like_reference():
    """incompleteness.ipynb:530-538's MACE line (correlation 4 on 0e+0o+1e+1o+2e+2o): the
    reference's own SymmetricContraction raises (no path reaches 0o under cg.py's natural-parity
    filter; fixture written by make_golden.py mace_widening); the product module raises too."""
    import json
    from conftest import GOLDEN
    eq = _eq()
    with open(os.path.join(GOLDEN, "mace_symmetric_contraction_bp4_error.json")) as fh:
        rec = json.load(fh)
    assert rec["raised"] == "UnboundLocalError" and rec["correlation"] == 4
    irr = "2x0e+2x0o+2x1e+2x1o+2x2e+2x2o"
    with pytest.raises(ValueError, match="no coupling path"):
        eq.SymmetricContraction(irr, irr, 4)


def test_k8_refuses_correlation_above_four():
    """The K8 term word has four 6-bit factor fields (gmp_sc.hip): correlation >= 5 must not
    select K8 (its fifth factor would be dropped), and k8_plan itself refuses it."""
    from gmp_amd import equivariant as eq
    irr = "2x0e+2x1o"
    sc = eq.SymmetricContraction(irr, irr, 5)
    assert not sc._k8
    with pytest.raises(AssertionError):
        eq.k8_plan(list(sc.contractions.values()), 4, 2, 5)
    assert eq.SymmetricContraction(irr, irr, 4)._k8
