"""CPU-side checks of the C ABI: libgmp.so loads and exports every symbol include/gmp.h
declares, and the ctypes signatures mirror the header (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gmp.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gmp_[a-z0-9_]+)\s*\(", txt)))


def test_header_parses():
    names = _declared()
    assert "gmp_egnn_edge_fwd_f32" in names and "gmp_csr_build" in names
    assert len(names) >= 10


def test_library_exports_all_symbols():
    from gmp_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgmp.so not built")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # every declared entry point has a ctypes signature (and vice versa)
    assert set(_declared()) == set(_lib.SIGNATURES), set(_declared()) ^ set(_lib.SIGNATURES)
    lib2 = _lib.load()
    assert lib2.gmp_abi_version() == _lib.ABI_VERSION == 6
    assert lib2.gmp_error_string(-1) == b"invalid argument"


def test_product_refuses_cpu_tensors():
    import torch
    from gmp_amd import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgmp.so not built")
    with pytest.raises(_lib.GmpError):
        ops.gather_rows(torch.zeros(4, 4), torch.zeros(2, dtype=torch.long))


def test_torch_ops_registered_and_reject_cpu_tensors():
    """TORCH_LIBRARY(gmp) (libgmp_torch.so): every hot-path operator is registered with a Meta
    kernel (shape inference, no device work) and a CPU tensor raises the boundary's error."""
    import torch
    from gmp_amd import _lib
    if not os.path.exists(_lib.TORCH_LIB_PATH):
        pytest.skip("libgmp_torch.so not built")
    tops = _lib.torch_ops()
    for name in ("csr_build", "gather_rows", "segment_reduce", "egnn_edge_fwd", "egnn_edge_bwd",
                 "egnn_node_fwd", "egnn_node_image",
                 "tp_edge_z", "tp_edge_z_bwd", "tp_node_outer", "tp_node_apply", "tp_gemm_x3",
                 "tp_gemm_x3_widen", "outer_sum_cols", "edge_outer_sum_ex",
                 "edge_outer_sum_ex2", "edge_outer_sum_act", "gvp_layer_fwd", "gvp_layer_bwd",
                 "gvp_msg0_fwd", "gvp_msg0_bwd", "tp_conv_fwd", "tp_conv_bwd",
                 "gvp_layer_fwd_agg", "gvp_layer_bwd_agg", "gvp_msg0_bwd_agg",
                 "gvp_edge_embed_fwd", "gvp_edge_embed_bwd", "edge_xyz_dot",
                 "symmetric_contraction_fwd",
                 "symmetric_contraction_bwd"):
        assert hasattr(tops, name), name
    with pytest.raises(RuntimeError, match="HIP device"):
        tops.gather_rows(torch.zeros(4, 4), torch.zeros(2, dtype=torch.long))
    # Meta: shapes only
    s = torch.empty(1000, 128, device="meta")
    v = torch.empty(1000, 16, 3, device="meta")
    W = [torch.empty(*sh, device="meta") for sh in ((128, 144), (128,), (16, 128), (16,),
                                                   (16, 16), (16, 16))]
    out = tops.gvp_layer_bwd(s, v, W, s, v, True)
    assert [tuple(t.shape) for t in out] == [(1000, 128), (1000, 16, 3), (1000, 128),
                                            (1000, 128), (1000, 16), (1000, 16), (1000, 48),
                                            (1000, 48), (1000, 48)]
    # without the optional factor rows (spre, vh), and the aggregation-fused forms (r05)
    out = tops.gvp_layer_bwd(s, v, W, s, v, True, False)
    assert tuple(out[3].shape) == (0, 128) and tuple(out[6].shape) == (0, 48)
    i64 = dict(dtype=torch.long, device="meta")
    sa, va = tops.gvp_layer_fwd_agg(s, v, W, torch.empty(1000, **i64), torch.empty(1000, **i64),
                                    torch.empty(301, **i64), 300, "mean")
    assert tuple(sa.shape) == (300, 128) and tuple(va.shape) == (300, 16, 3)
    # K1e edge embedding: es (E, so), ev (E, 1, 3); packed parameter gradients (2R + 3 + so (R + 3))
    We = [torch.empty(*sh, device="meta") for sh in ((8,), (8,), (1, 1), (32, 9), (32,), (1, 1),
                                                    (1, 32), (1,))]
    rad, unit = torch.empty(700, 8, device="meta"), torch.empty(700, 3, device="meta")
    es, ev = tops.gvp_edge_embed_fwd(rad, unit, We, 1e-5)
    assert tuple(es.shape) == (700, 32) and tuple(ev.shape) == (700, 1, 3)
    assert tuple(tops.gvp_edge_embed_bwd(rad, unit, We, 1e-5, es, ev).shape) == (371,)
    assert tuple(tops.edge_xyz_dot(torch.empty(700, 144, device="meta"), unit).shape) == (48,)
    # K8 on a term plan: out (N, rows C), partials (groups, T, C)
    x = torch.empty(50, 8, 9, device="meta")
    plan = torch.empty(3 * 9 + 1 + 40, dtype=torch.int32, device="meta")
    coef = torch.empty(40, 8, device="meta")
    assert tuple(tops.symmetric_contraction_fwd(x, plan, 9, coef).shape) == (50, 72)
    dx, part = tops.symmetric_contraction_bwd(x, plan, 9, coef, torch.empty(50, 72, device="meta"))
    assert tuple(dx.shape) == (50, 8, 9) and tuple(part.shape)[1:] == (40, 8)
    z = tops.tp_edge_z([11, 1152, 1152, 9, 180224, 4480, 3] + [0] * 18,
                       torch.empty(11 * 64, dtype=torch.uint8, device="meta"),
                       torch.empty(10, device="meta"), torch.empty(50, 1152, device="meta"),
                       torch.empty(700, 9, device="meta"),
                       torch.empty(700, dtype=torch.long, device="meta"),
                       torch.empty(700, dtype=torch.long, device="meta"), 0, 700)
    assert tuple(z.shape) == (701 * 4480,)
