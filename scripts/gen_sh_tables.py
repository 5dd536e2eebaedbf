"""Generate the l = 4, 5 spherical-harmonics recursion tables of the K1 featurise kernel
(gmp_featurize.hip kShRec4 / kShRec5) from the oracle's real-basis wigner_3j:

    Y_l[k] = c_l sum_{i,j} C[i, j, k] Y_{l-1}[i] u_j,  C = wigner_3j(l-1, 1, l),

with c_l fixing |Y_l|^2 = 2l + 1 on the unit sphere (e3nn 'component' normalisation; the same
recursion reproduces the closed-form l = 2, 3 blocks with c_l > 0, tests/test_oracle_o3.py).
Prints the nonzero entries (i, j, k, c_l C[i, j, k]).  Usage: python scripts/gen_sh_tables.py"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import o3  # noqa: E402


def main():
    for l in (4, 5):
        C, c = o3.sh_recursion_table(l)
        ent = [(i, j, k, c * C[i, j, k].item()) for i in range(2 * l - 1) for j in range(3)
               for k in range(2 * l + 1) if abs(C[i, j, k].item()) > 1e-12]
        print(f"// l = {l}: {len(ent)} entries, c_l = {c:.17g}")
        print(f"constexpr ShRec kShRec{l}[{len(ent)}] = {{")
        for i, j, k, v in ent:
            print(f"    {{{i}, {j}, {k}, {v:.9e}f}},")
        print("};")


if __name__ == "__main__":
    main()
