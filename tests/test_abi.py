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
    assert lib2.gmp_abi_version() == 1
    assert lib2.gmp_error_string(-1) == b"invalid argument"


def test_product_refuses_cpu_tensors():
    import torch
    from gmp_amd import _lib, ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgmp.so not built")
    with pytest.raises(_lib.GmpError):
        ops.gather_rows(torch.zeros(4, 4), torch.zeros(2, dtype=torch.long))
