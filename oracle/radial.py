"""Radial basis restated on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py).

models/mace_modules/radial.py:12-52 (BesselBasis), 55-81 (PolynomialCutoff),
models/mace_modules/blocks.py:84-96 (RadialEmbeddingBlock). Buffers/keys identical
(bessel_fn.bessel_weights, bessel_fn.r_max, bessel_fn.prefactor, cutoff_fn.p, cutoff_fn.r_max).
"""
import math

import torch
from torch import nn


class BesselBasis(nn.Module):
    def __init__(self, r_max, num_basis=8, trainable=False):
        super().__init__()
        w = math.pi / r_max * torch.linspace(1.0, num_basis, num_basis)
        if trainable:
            self.bessel_weights = nn.Parameter(w)
        else:
            self.register_buffer("bessel_weights", w)
        self.register_buffer("r_max", torch.tensor(float(r_max)))
        self.register_buffer("prefactor", torch.tensor(math.sqrt(2.0 / r_max)))

    def forward(self, r):  # (..., 1) -> (..., num_basis);  sqrt(2/rmax) sin(n pi r / rmax) / r
        return self.prefactor * (torch.sin(self.bessel_weights * r) / r)


class PolynomialCutoff(nn.Module):
    def __init__(self, r_max, p=6):
        super().__init__()
        self.register_buffer("p", torch.tensor(float(p)))
        self.register_buffer("r_max", torch.tensor(float(r_max)))

    def forward(self, r):
        # same evaluation order as radial.py:71-78 (fp32 cancellation near r_max reproduced)
        p = self.p
        u = r / self.r_max
        env = (1.0 - ((p + 1.0) * (p + 2.0) / 2.0) * torch.pow(u, p)
               + p * (p + 2.0) * torch.pow(u, p + 1) - (p * (p + 1.0) / 2) * torch.pow(u, p + 2))
        return env * (r < self.r_max)


class RadialEmbeddingBlock(nn.Module):
    def __init__(self, r_max, num_bessel, num_polynomial_cutoff):
        super().__init__()
        self.bessel_fn = BesselBasis(r_max=r_max, num_basis=num_bessel)
        self.cutoff_fn = PolynomialCutoff(r_max=r_max, p=num_polynomial_cutoff)
        self.out_dim = num_bessel

    def forward(self, lengths):
        return self.bessel_fn(lengths) * self.cutoff_fn(lengths)
