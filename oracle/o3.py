"""e3nn 0.5.1 semantics restated in plain PyTorch (TEST INFRASTRUCTURE; see oracle/__init__.py).

e3nn is not installed and not vendored in /root/reference, so this restates its published
algorithms (pinned version: e3nn 0.5.1 — the version the reference's notebooks ran,
experiments/rotsym.ipynb:50; README.md:53 pins 0.4.4).  Used by the reference at
models/layers/tfn_layer.py:48-80, models/tfn.py:110-113, models/mace.py:82-85,
models/mace_modules/{blocks,cg,symmetric_contraction,irreps_tools}.py.
**Parity unpinned**: no reference test or fixture pins these numerics; they are checked by
known-answer tests (closed-form SH / CG values) and equivariance tests (tests/test_oracle_o3.py).

Conventions (e3nn): real basis with y as the polar axis; l=1 components are (x, y, z);
wigner_3j = the real-basis SU(2) Clebsch-Gordan tensor normalised to unit Frobenius norm;
"mul_ir" flat layout = for each (mul, ir) block, mul copies of a (2l+1) vector, mul-major.
"""
import math
from fractions import Fraction
from functools import lru_cache

import torch

# ----------------------------------------------------------------------------------- Irreps


class Irreps(tuple):
    """Tuple of (mul, (l, p)).  Parses '128x0e+128x1o+128x2e'."""

    def __new__(cls, spec):
        if isinstance(spec, Irreps):
            return spec
        items = []
        if isinstance(spec, str):
            for tok in spec.replace(" ", "").split("+"):
                if not tok:
                    continue
                mul, ir = tok.split("x") if "x" in tok else ("1", tok)
                l, p = int(ir[:-1]), {"e": 1, "o": -1}[ir[-1]]
                items.append((int(mul), (l, p)))
        else:
            for mul, ir in spec:
                items.append((int(mul), (int(ir[0]), int(ir[1]))))
        return super().__new__(cls, items)

    @property
    def dim(self):
        return sum(m * (2 * l + 1) for m, (l, _) in self)

    def slices(self):
        out, i = [], 0
        for m, (l, _) in self:
            out.append(slice(i, i + m * (2 * l + 1)))
            i += m * (2 * l + 1)
        return out

    def __str__(self):
        return "+".join(f"{m}x{l}{'e' if p == 1 else 'o'}" for m, (l, p) in self)

    def count(self, ir):
        return sum(m for m, i in self if i == tuple(ir))


def spherical_harmonics_irreps(lmax, p=-1):
    return Irreps([(1, (l, p ** l)) for l in range(lmax + 1)])


def ir_mul(ir1, ir2):
    """Irreps of ir1 (x) ir2: l in |l1-l2|..l1+l2, parity p1*p2."""
    (l1, p1), (l2, p2) = ir1, ir2
    return [(l, p1 * p2) for l in range(abs(l1 - l2), l1 + l2 + 1)]


# ----------------------------------------------------------------------------------- SH


def spherical_harmonics_l2(vec, normalize=True):
    """e3nn SphericalHarmonics(lmax=2, normalize, normalization='component') -> (..., 9)."""
    if normalize:
        vec = torch.nn.functional.normalize(vec, dim=-1)
    x, y, z = vec[..., 0], vec[..., 1], vec[..., 2]
    s3, s5, s15 = math.sqrt(3.0), math.sqrt(5.0), math.sqrt(15.0)
    return torch.stack([
        torch.ones_like(x),
        s3 * x, s3 * y, s3 * z,
        s15 * x * z, s15 * x * y, s5 * (y * y - 0.5 * (x * x + z * z)), s15 * y * z,
        s15 / 2.0 * (z * z - x * x),
    ], dim=-1)


@lru_cache(maxsize=None)
def _sh_recursion(l):
    """(C, c_l) of Y_l[k] = c_l sum_ij C[i, j, k] Y_{l-1}[i] u_j with C = wigner_3j(l-1, 1, l)
    and c_l > 0 such that |Y_l|^2 = 2l + 1 on the unit sphere (the contraction's norm there is
    a constant: measured on a fixed set of unit vectors)."""
    C = wigner_3j(l - 1, 1, l)
    g = torch.Generator().manual_seed(l)
    u = torch.nn.functional.normalize(torch.randn(64, 3, generator=g, dtype=torch.float64),
                                      dim=-1)
    Yp = spherical_harmonics(u, l - 1)[:, (l - 1) ** 2:l * l]
    n2 = torch.einsum("ijk,ni,nj->nk", C, Yp, u).pow(2).sum(-1)
    assert float(n2.max() - n2.min()) < 1e-9 * float(n2.max())
    return C, math.sqrt((2 * l + 1) / float(n2.mean()))


def sh_recursion_table(l):
    return _sh_recursion(l)


def spherical_harmonics(vec, lmax, normalize=True):
    """e3nn SphericalHarmonics(range(lmax+1), normalize, 'component') -> (..., (lmax+1)^2),
    lmax <= 5.  e3nn 0.5.1 o3/_spherical_harmonics.py generates each l from l-1 by the CG
    recursion and scales l by sqrt(2l+1); the l = 3 block restated here in closed form, the
    l = 4, 5 blocks by that recursion (Y_l = c_l wigner_3j(l-1, 1, l) . (Y_{l-1} (x) u), which
    reproduces the closed-form l = 2, 3 blocks: tests/test_oracle_o3.py; unit-vector norm 2l+1
    and equivariance checked there too)."""
    assert 0 <= lmax <= 5
    Y = spherical_harmonics_l2(vec, normalize)[..., :(lmax + 1) ** 2]
    if lmax < 3:
        return Y
    if normalize:
        vec = torch.nn.functional.normalize(vec, dim=-1)
    x, y, z = vec[..., 0], vec[..., 1], vec[..., 2]
    s20 = math.sqrt(3.0) * x * z                 # e3nn's un-normalised sh_2_0 / sh_2_4
    s24 = math.sqrt(3.0) / 2.0 * (z * z - x * x)
    q = 4.0 * y * y - x * x - z * z
    s7 = math.sqrt(7.0)
    l3 = torch.stack([
        math.sqrt(5.0 / 6.0) * (s20 * z + s24 * x),
        math.sqrt(5.0) * s20 * y,
        math.sqrt(3.0 / 8.0) * q * x,
        0.5 * y * (2.0 * y * y - 3.0 * (x * x + z * z)),
        math.sqrt(3.0 / 8.0) * z * q,
        math.sqrt(5.0) * s24 * y,
        math.sqrt(5.0 / 6.0) * (s24 * z - s20 * x),
    ], dim=-1) * s7
    blocks = [Y, l3]
    u = torch.stack([x, y, z], dim=-1)
    for l in range(4, lmax + 1):
        C, c = _sh_recursion(l)
        blocks.append(c * torch.einsum("ijk,...i,...j->...k", C.to(u.dtype), blocks[-1], u))
    return torch.cat(blocks, dim=-1)


# ----------------------------------------------------------------------------------- CG


def _fact(n):
    return math.factorial(int(round(n)))


def _su2_cg_coeff(j1, m1, j2, m2, j3, m3):
    """Racah formula for <j1 m1 j2 m2 | j3 m3> (exact rational arithmetic, then sqrt)."""
    if m3 != m1 + m2:
        return 0.0
    vmin = int(max(-j1 + j2 + m3, -j1 + m1, 0))
    vmax = int(min(j2 + j3 + m1, j3 - j1 + j2, j3 + m3))
    c = Fraction((2 * j3 + 1) * _fact(j3 + j1 - j2) * _fact(j3 - j1 + j2) * _fact(j1 + j2 - j3),
                 _fact(j1 + j2 + j3 + 1))
    c *= Fraction(_fact(j3 + m3) * _fact(j3 - m3), _fact(j1 + m1) * _fact(j1 - m1)
                  * _fact(j2 + m2) * _fact(j2 - m2))
    s = Fraction(0)
    for v in range(vmin, vmax + 1):
        s += (-1) ** int(v + j2 + m2) * Fraction(
            _fact(j2 + j3 + m1 - v) * _fact(j1 - m1 + v),
            _fact(v) * _fact(j3 - j1 + j2 - v) * _fact(j3 + m3 - v) * _fact(v + j1 - j2 - m3))
    return math.sqrt(float(c)) * float(s)


def _su2_cg(l1, l2, l3):
    mat = torch.zeros(2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1, dtype=torch.float64)
    if abs(l1 - l2) <= l3 <= l1 + l2:
        for m1 in range(-l1, l1 + 1):
            for m2 in range(-l2, l2 + 1):
                if abs(m1 + m2) <= l3:
                    mat[l1 + m1, l2 + m2, l3 + m1 + m2] = _su2_cg_coeff(l1, m1, l2, m2, l3, m1 + m2)
    return mat


def change_basis_real_to_complex(l):
    q = torch.zeros(2 * l + 1, 2 * l + 1, dtype=torch.complex128)
    for m in range(-l, 0):
        q[l + m, l + abs(m)] = 1 / math.sqrt(2)
        q[l + m, l - abs(m)] = -1j / math.sqrt(2)
    q[l, l] = 1
    for m in range(1, l + 1):
        q[l + m, l + abs(m)] = (-1) ** m / math.sqrt(2)
        q[l + m, l - abs(m)] = 1j * (-1) ** m / math.sqrt(2)
    return (-1j) ** l * q


@lru_cache(maxsize=None)
def _wigner_3j_cached(l1, l2, l3):
    Q1, Q2, Q3 = (change_basis_real_to_complex(l) for l in (l1, l2, l3))
    C = _su2_cg(l1, l2, l3).to(torch.complex128)
    C = torch.einsum("ij,kl,mn,ikn->jlm", Q1, Q2, torch.conj(Q3.T), C)
    assert torch.all(torch.abs(torch.imag(C)) < 1e-5)
    C = torch.real(C)
    return C / torch.norm(C)


def wigner_3j(l1, l2, l3, dtype=torch.float64):
    assert abs(l2 - l3) <= l1 <= l2 + l3
    return _wigner_3j_cached(l1, l2, l3).to(dtype).clone()


# ----------------------------------------------------------------------------------- Wigner D
def _su2_generators(j):
    m = torch.arange(-j, j, dtype=torch.float64)
    raising = torch.diag(-torch.sqrt(j * (j + 1) - m * (m + 1)), diagonal=-1)
    m = torch.arange(-j + 1, j + 1, dtype=torch.float64)
    lowering = torch.diag(torch.sqrt(j * (j + 1) - m * (m - 1)), diagonal=1)
    m = torch.arange(-j, j + 1, dtype=torch.float64)
    return torch.stack([0.5 * (raising + lowering).to(torch.complex128),
                        torch.diag(1j * m),
                        -0.5j * (raising - lowering).to(torch.complex128)], dim=0)


def so3_generators(l):
    X = _su2_generators(l)
    Q = change_basis_real_to_complex(l)
    X = torch.conj(Q.T) @ X @ Q
    assert torch.all(torch.abs(torch.imag(X)) < 1e-5)
    return torch.real(X)


def wigner_D(l, alpha, beta, gamma):
    X = so3_generators(l)
    return (torch.matrix_exp(alpha * X[1]) @ torch.matrix_exp(beta * X[0])
            @ torch.matrix_exp(gamma * X[1]))


def D_from_matrix_l1(R):
    """For the l=1 basis (x, y, z), D^1(R) = R (used by the equivariance tests)."""
    return R


# ----------------------------------------------------------------------------------- TP
class FullyConnectedTensorProduct(torch.nn.Module):
    """e3nn o3.FullyConnectedTensorProduct(in1, in2, out, shared_weights=False):
    all (i1, i2, o) with ir_o in ir1 (x) ir2, mode 'uvw'; irrep_normalization='component',
    path_normalization='element':  alpha_p = (2 l_o + 1) / sum_{p' -> o} mul1 mul2;
    out_o[w, k] += sqrt(alpha_p) sum_{u,v} W_p[u, v, w] sum_{ij} C_p[i, j, k] x1[u, i] x2[v, j].
    Weights flattened per instruction as (mul1, mul2, mul_out) row-major, concatenated."""

    def __init__(self, irreps_in1, irreps_in2, irreps_out):
        super().__init__()
        self.irreps_in1, self.irreps_in2 = Irreps(irreps_in1), Irreps(irreps_in2)
        self.irreps_out = Irreps(irreps_out)
        ins = []
        for i1, (m1, ir1) in enumerate(self.irreps_in1):
            for i2, (m2, ir2) in enumerate(self.irreps_in2):
                for io, (mo, iro) in enumerate(self.irreps_out):
                    if iro in ir_mul(ir1, ir2):
                        ins.append((i1, i2, io))
        self.instructions = []
        woff = 0
        for (i1, i2, io) in ins:
            m1, m2, mo = self.irreps_in1[i1][0], self.irreps_in2[i2][0], self.irreps_out[io][0]
            lo = self.irreps_out[io][1][0]
            fan = sum(self.irreps_in1[a][0] * self.irreps_in2[b][0] for a, b, c in ins if c == io)
            alpha = (2 * lo + 1) / fan
            self.instructions.append(dict(i1=i1, i2=i2, io=io, w_off=woff, shape=(m1, m2, mo),
                                          path_weight=math.sqrt(alpha)))
            woff += m1 * m2 * mo
        self.weight_numel = woff

    def forward(self, x1, x2, weight):
        s1, s2, so = self.irreps_in1.slices(), self.irreps_in2.slices(), self.irreps_out.slices()
        B = x1.shape[0]
        out = x1.new_zeros(B, self.irreps_out.dim)
        for ins in self.instructions:
            (m1, (l1, _)) = self.irreps_in1[ins["i1"]]
            (m2, (l2, _)) = self.irreps_in2[ins["i2"]]
            (mo, (lo, _)) = self.irreps_out[ins["io"]]
            a = x1[:, s1[ins["i1"]]].reshape(B, m1, 2 * l1 + 1)
            b = x2[:, s2[ins["i2"]]].reshape(B, m2, 2 * l2 + 1)
            W = weight[:, ins["w_off"]:ins["w_off"] + m1 * m2 * mo].reshape(B, m1, m2, mo)
            C = wigner_3j(l1, l2, lo, x1.dtype)
            # contraction order of e3nn's generated code: CG-couple the inputs first, then
            # one batched matmul with the per-edge weights
            zc = torch.einsum("ijk,zui,zvj->zuvk", C, a, b).reshape(B, m1 * m2, 2 * lo + 1)
            r = torch.bmm(W.reshape(B, m1 * m2, mo).transpose(1, 2), zc) * ins["path_weight"]
            sl = so[ins["io"]]
            out[:, sl] = out[:, sl] + r.reshape(B, mo * (2 * lo + 1))
        return out


class Linear(torch.nn.Module):
    """e3nn o3.Linear(irreps_in, irreps_out) (internal, shared weights, no biases):
    out_o[w, m] = sum_{i -> o} sum_u W[u, w] x_i[u, m] / sqrt(sum_{i -> o} mul_i);
    weight = flat concatenation of the (mul_in, mul_out) blocks, init N(0, 1)."""

    def __init__(self, irreps_in, irreps_out):
        super().__init__()
        self.irreps_in, self.irreps_out = Irreps(irreps_in), Irreps(irreps_out)
        self.instructions = [(i, o) for i, (_, iri) in enumerate(self.irreps_in)
                             for o, (_, iro) in enumerate(self.irreps_out) if iri == iro]
        n = sum(self.irreps_in[i][0] * self.irreps_out[o][0] for i, o in self.instructions)
        self.weight = torch.nn.Parameter(torch.randn(n))

    def forward(self, x):
        si, so = self.irreps_in.slices(), self.irreps_out.slices()
        B = x.shape[0]
        out = x.new_zeros(B, self.irreps_out.dim)
        off = 0
        for i, o in self.instructions:
            mi, (l, _) = self.irreps_in[i]
            mo = self.irreps_out[o][0]
            fan = sum(self.irreps_in[a][0] for a, b in self.instructions if b == o)
            W = self.weight[off:off + mi * mo].reshape(mi, mo)
            off += mi * mo
            xi = x[:, si[i]].reshape(B, mi, 2 * l + 1)
            r = torch.einsum("uw,zum->zwm", W, xi) / math.sqrt(fan)
            out[:, so[o]] = out[:, so[o]] + r.reshape(B, -1)
        return out


class BatchNorm(torch.nn.Module):
    """e3nn nn.BatchNorm(irreps) with defaults eps=1e-5, momentum=0.1, affine=True,
    reduce='mean', normalization='component', instance=False."""

    def __init__(self, irreps, eps=1e-5, momentum=0.1):
        super().__init__()
        self.irreps = Irreps(irreps)
        self.eps, self.momentum = eps, momentum
        ns = sum(m for m, (l, p) in self.irreps if l == 0 and p == 1)
        nf = sum(m for m, _ in self.irreps)
        self.register_buffer("running_mean", torch.zeros(ns))
        self.register_buffer("running_var", torch.ones(nf))
        self.weight = torch.nn.Parameter(torch.ones(nf))
        self.bias = torch.nn.Parameter(torch.zeros(ns))

    def forward(self, x):
        B = x.shape[0]
        fields, new_means, new_vars = [], [], []
        ix = irm = irv = iw = ib = 0
        for mul, (l, p) in self.irreps:
            d = 2 * l + 1
            f = x[:, ix:ix + mul * d].reshape(B, mul, d)
            ix += mul * d
            scalar = (l == 0 and p == 1)
            if scalar:
                if self.training:
                    mean = f.mean(dim=(0, 2))
                    new_means.append((1 - self.momentum) * self.running_mean[irm:irm + mul]
                                     + self.momentum * mean.detach())
                else:
                    mean = self.running_mean[irm:irm + mul]
                irm += mul
                f = f - mean.reshape(1, mul, 1)
            if self.training:
                norm = f.pow(2).mean(2).mean(0)
                new_vars.append((1 - self.momentum) * self.running_var[irv:irv + mul]
                                + self.momentum * norm.detach())
            else:
                norm = self.running_var[irv:irv + mul]
            irv += mul
            scale = (norm + self.eps).pow(-0.5) * self.weight[iw:iw + mul]
            iw += mul
            f = f * scale.reshape(1, mul, 1)
            if scalar:
                f = f + self.bias[ib:ib + mul].reshape(1, mul, 1)
                ib += mul
            fields.append(f.reshape(B, mul * d))
        if self.training:
            with torch.no_grad():
                if new_means:
                    self.running_mean.copy_(torch.cat(new_means))
                self.running_var.copy_(torch.cat(new_vars))
        return torch.cat(fields, dim=1)


# ----------------------------------------------------------------------------------- gates
@lru_cache(maxsize=None)
def normalize2mom_const(name):
    """e3nn normalize2mom: c = E_z[f(z)^2]^(-1/2), z = 1e6 float64 normals drawn from
    torch.Generator().manual_seed(0); treated as 1 if |c - 1| < 1e-4."""
    f = {"silu": torch.nn.functional.silu, "sigmoid": torch.sigmoid}[name]
    z = torch.randn(1_000_000, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    c = f(z).pow(2).mean().pow(-0.5).item()
    return 1.0 if abs(c - 1.0) < 1e-4 else c


class Gate(torch.nn.Module):
    """e3nn nn.Gate(scalars, [silu], gates, [sigmoid], gated) as built by tfn_layer.py:45-63
    via irreps2gate (irreps_tools.py:82-97): input = scalars + gates + gated (unsimplified);
    out = [c_silu silu(scalars), gated_i * c_sig sigmoid(gate_i)]."""

    def __init__(self, irreps_scalars, irreps_gates, irreps_gated):
        super().__init__()
        self.irreps_scalars = Irreps(irreps_scalars)
        self.irreps_gates = Irreps(irreps_gates)
        self.irreps_gated = Irreps(irreps_gated)
        self.irreps_in = Irreps(list(self.irreps_scalars) + list(self.irreps_gates)
                                + list(self.irreps_gated))
        self.irreps_out = Irreps(list(self.irreps_scalars) + list(self.irreps_gated))
        self.c_act = normalize2mom_const("silu")
        self.c_gate = normalize2mom_const("sigmoid")

    def forward(self, x):
        ns, ng = self.irreps_scalars.dim, self.irreps_gates.dim
        s = x[:, :ns]
        g = x[:, ns:ns + ng]
        v = x[:, ns + ng:]
        s = self.c_act * torch.nn.functional.silu(s)
        g = self.c_gate * torch.sigmoid(g)
        outs, gi, vi = [s], 0, 0
        B = x.shape[0]
        for mul, (l, _) in self.irreps_gated:
            d = 2 * l + 1
            blk = v[:, vi:vi + mul * d].reshape(B, mul, d) * g[:, gi:gi + mul].unsqueeze(-1)
            outs.append(blk.reshape(B, mul * d))
            vi += mul * d
            gi += mul
        return torch.cat(outs, dim=1)


def irreps2gate(irreps):
    """models/mace_modules/irreps_tools.py:82-97."""
    irreps = Irreps(irreps)
    scal = [(m, ir) for m, ir in irreps if ir[0] == 0 and ir[1] == 1]
    gated = [(m, ir) for m, ir in irreps if not (ir[0] == 0 and ir[1] == 1)]
    scal, gated = _simplify(scal), _simplify(gated)
    gates = _simplify([(m, (0, 1)) for m, _ in gated]) if gated else []
    return Irreps(scal), Irreps(gates), Irreps(gated)


def _simplify(items):
    out = []
    for m, ir in items:
        if out and out[-1][1] == ir:
            out[-1] = (out[-1][0] + m, ir)
        else:
            out.append((m, ir))
    return out
