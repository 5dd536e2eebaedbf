"""Dev A/B: bench.py with the r05 pre-xyz-dot first-message sums (ev padded to 16 columns, two
edge outer sums) in place of gmp_edge_xyz_dot_f32.  Usage: python scripts/ab_xyz_dot_off.py
<bench args>"""
import os
import runpy
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "geometric-message-passing_amd"))
import gmp_amd._lib as L  # noqa: E402
import gmp_amd.gvp as g  # noqa: E402


class _Ops:
    def __getattr__(self, n):
        return getattr(L.torch_ops(), n)

    def edge_xyz_dot(self, A, v):
        M, _ = g._osum(torch.nn.functional.pad(v, (0, 13)), A)
        return M[:3].reshape(3, A.shape[1] // 3, 3).diagonal(dim1=0, dim2=2).sum(-1)


class _Lib:
    def __getattr__(self, n):
        return getattr(L, n)

    def torch_ops(self):
        return _Ops()


g._lib = _Lib()
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
