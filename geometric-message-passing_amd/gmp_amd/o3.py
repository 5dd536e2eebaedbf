"""Host-side e3nn (0.5.1) conventions for the equivariant layers: irreps algebra, real
Clebsch-Gordan (wigner_3j), FullyConnectedTensorProduct instruction tables, MACE generalised CG
(U) tensors and normalize2mom constants.  Init-time constants only (numpy / float64); the
per-edge and per-node arithmetic runs in the HIP kernels.

Reference call sites: models/layers/tfn_layer.py:48-80, models/mace_modules/cg.py:19-133,
models/mace_modules/irreps_tools.py:63-97, models/mace_modules/symmetric_contraction.py:88-148.
e3nn itself is not available; conventions: real basis with y the polar axis,
l=1 components (x, y, z), CG = real-basis SU(2) Clebsch-Gordan with unit Frobenius norm.
"""
import math
from functools import lru_cache

import numpy as np


# ----------------------------------------------------------------------------------- irreps
def parse_irreps(spec):
    """'128x0e+128x1o' or [(mul, (l, p)), ...] -> tuple of (mul, (l, p))."""
    if isinstance(spec, str):
        out = []
        for tok in spec.replace(" ", "").split("+"):
            if tok:
                mul, ir = tok.split("x") if "x" in tok else ("1", tok)
                out.append((int(mul), (int(ir[:-1]), 1 if ir[-1] == "e" else -1)))
        return tuple(out)
    return tuple((int(m), (int(ir[0]), int(ir[1]))) for m, ir in spec)


def irreps_str(irreps):
    return "+".join(f"{m}x{l}{'e' if p == 1 else 'o'}" for m, (l, p) in irreps)


def irreps_dim(irreps):
    return sum(m * (2 * l + 1) for m, (l, _) in irreps)


def irreps_offsets(irreps):
    offs, o = [], 0
    for m, (l, _) in irreps:
        offs.append(o)
        o += m * (2 * l + 1)
    return offs


def sh_irreps(lmax):
    return tuple((1, (l, (-1) ** l)) for l in range(lmax + 1))


def hidden_irreps(emb_dim, lmax):
    """(sh_irreps * emb_dim).sort().simplify() for lmax <= 5 (models/mace.py:96)."""
    return tuple((emb_dim, (l, (-1) ** l)) for l in range(lmax + 1))


def product_irreps(ir1, ir2):
    (l1, p1), (l2, p2) = ir1, ir2
    return [(l, p1 * p2) for l in range(abs(l1 - l2), l1 + l2 + 1)]


def irreps2gate(irreps):
    """irreps_tools.py:82-97 -> (scalars, gates, gated), each simplified."""
    def simplify(items):
        out = []
        for m, ir in items:
            if out and out[-1][1] == ir:
                out[-1] = (out[-1][0] + m, ir)
            else:
                out.append((m, ir))
        return tuple(out)
    scal = simplify([(m, ir) for m, ir in irreps if ir == (0, 1)])
    gated = simplify([(m, ir) for m, ir in irreps if ir != (0, 1)])
    gates = simplify([(m, (0, 1)) for m, _ in gated])
    return scal, gates, gated


# ----------------------------------------------------------------------------------- CG
def _cg_su2(j1, m1, j2, m2, j3, m3):
    """<j1 m1; j2 m2 | j3 m3> by the Racah formula (exact integer arithmetic)."""
    if m1 + m2 != m3 or abs(m3) > j3:
        return 0.0
    f = math.factorial
    num = (2 * j3 + 1) * f(j3 + j1 - j2) * f(j3 - j1 + j2) * f(j1 + j2 - j3) * \
        f(j3 + m3) * f(j3 - m3)
    den = f(j1 + j2 + j3 + 1) * f(j1 + m1) * f(j1 - m1) * f(j2 + m2) * f(j2 - m2)
    total = 0
    from fractions import Fraction
    for v in range(max(-j1 + j2 + m3, -j1 + m1, 0), min(j2 + j3 + m1, j3 - j1 + j2, j3 + m3) + 1):
        total += Fraction((-1) ** (v + j2 + m2) * f(j2 + j3 + m1 - v) * f(j1 - m1 + v),
                          f(v) * f(j3 - j1 + j2 - v) * f(j3 + m3 - v) * f(v + j1 - j2 - m3))
    return math.sqrt(num / den) * float(total)


def _q_real_to_complex(l):
    """Change of basis with the (-i)^l phase used by e3nn (real CG tensors)."""
    q = np.zeros((2 * l + 1, 2 * l + 1), dtype=np.complex128)
    r2 = 1 / math.sqrt(2)
    for m in range(-l, 0):
        q[l + m, l - m] = r2
        q[l + m, l + m] = -1j * r2
    q[l, l] = 1
    for m in range(1, l + 1):
        q[l + m, l + m] = (-1) ** m * r2
        q[l + m, l - m] = 1j * (-1) ** m * r2
    return (-1j) ** l * q


@lru_cache(maxsize=None)
def wigner_3j(l1, l2, l3):
    """Real-basis CG tensor (2l1+1, 2l2+1, 2l3+1), unit Frobenius norm (e3nn o3.wigner_3j)."""
    assert abs(l1 - l2) <= l3 <= l1 + l2
    su2 = np.zeros((2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1))
    for a in range(2 * l1 + 1):
        for b in range(2 * l2 + 1):
            c = (a - l1) + (b - l2) + l3
            if 0 <= c <= 2 * l3:
                su2[a, b, c] = _cg_su2(l1, a - l1, l2, b - l2, l3, c - l3)
    Q1, Q2, Q3 = _q_real_to_complex(l1), _q_real_to_complex(l2), _q_real_to_complex(l3)
    C = np.einsum("ij,kl,nm,ikn->jlm", Q1, Q2, np.conj(Q3), su2)
    assert np.abs(C.imag).max() < 1e-10
    C = C.real
    C = C / np.linalg.norm(C)
    C.setflags(write=False)
    return C


# ----------------------------------------------------------------------------------- FCTP
def fctp_instructions(irreps_in1, irreps_in2, irreps_out):
    """e3nn FullyConnectedTensorProduct instruction list (mode uvw, component irrep
    normalisation, element path normalisation): dicts with block indices, shapes, weight
    offset and sqrt(alpha)."""
    ins = [(i1, i2, io)
           for i1, (_, ir1) in enumerate(irreps_in1)
           for i2, (_, ir2) in enumerate(irreps_in2)
           for io, (_, iro) in enumerate(irreps_out) if iro in product_irreps(ir1, ir2)]
    out, woff = [], 0
    for i1, i2, io in ins:
        m1, (l1, _) = irreps_in1[i1]
        m2, (l2, _) = irreps_in2[i2]
        mo, (lo, _) = irreps_out[io]
        fan = sum(irreps_in1[a][0] * irreps_in2[b][0] for a, b, c in ins if c == io)
        out.append(dict(i1=i1, i2=i2, io=io, l1=l1, l2=l2, lo=lo, mul1=m1, mul2=m2, mul_out=mo,
                        w_off=woff, alpha=math.sqrt((2 * lo + 1) / fan)))
        woff += m1 * m2 * mo
    return out, woff


# ----------------------------------------------------------------------------------- MACE U
def _cg_chain(irreps_list, filter_ir=None, only=None):
    """Generalised CG of a product of irreps (cg.py:_wigner_nj, component normalisation):
    list of (irrep_out, tensor (2lo+1, d, ..., d)) sorted (stably) by irrep.  filter_ir: the
    irreps allowed at every coupling step (cg.py:_wigner_nj filter_ir_mid).  only: keep just
    this output irrep at the last step (the chain of the left factors is shared, _chain_left)."""
    if len(irreps_list) == 1:
        irreps = irreps_list[0]
        dim = irreps_dim(irreps)
        eye = np.eye(dim)
        out, i = [], 0
        for m, ir in irreps:
            for _ in range(m):
                d = 2 * ir[0] + 1
                out.append((ir, eye[i:i + d]))
                i += d
        return out
    left, right = irreps_list[:-1], irreps_list[-1]
    dims_left = [irreps_dim(x) for x in left]
    dr = irreps_dim(right)
    out = []
    for ir_left, C_left in _chain_left(tuple(left), _fkey(filter_ir)):
        i = 0
        for m, ir in right:
            d = 2 * ir[0] + 1
            for ir_out in product_irreps(ir_left, ir):
                if filter_ir is not None and tuple(ir_out) not in filter_ir:
                    continue
                if only is not None and tuple(ir_out) != tuple(only):
                    continue
                lo = ir_out[0]
                C = wigner_3j(lo, ir_left[0], ir[0]) * math.sqrt(2 * lo + 1)
                # C[i, k, l] = sum_j C_left[j, k] w3j[i, j, l] (BLAS: the einsum's loop form ran
                # ~30 s per output irrep at max_ell 3, correlation 4)
                C = np.tensordot(C, C_left.reshape(C_left.shape[0], -1), axes=([1], [0]))
                C = C.transpose(0, 2, 1).reshape((2 * lo + 1, *dims_left, d))
                for u in range(m):
                    E = np.zeros((2 * lo + 1, *dims_left, dr))
                    E[..., i + u * d:i + (u + 1) * d] = C
                    out.append((ir_out, E))
            i += m * d
    out.sort(key=lambda x: x[0])  # stable: python sort
    return out


def _fkey(filter_ir):
    return None if filter_ir is None else frozenset(filter_ir)


@lru_cache(maxsize=4)
def _chain_left(irreps_list, filter_key):
    """The chain of the left factors, shared by every output irrep of one SymmetricContraction
    (cleared by clear_cg_cache() once the module is built)."""
    return _cg_chain(list(irreps_list), None if filter_key is None else set(filter_key))


def clear_cg_cache():
    _chain_left.cache_clear()


def u_matrix(coupling_irreps, ir_out, nu):
    """cg.py U_matrix_real(coupling, ir_out, nu)[-1]: (2lo+1 [squeezed if 1], d^nu..., K).
    correlation 4 couples through the natural-parity irreps l < 12 only (cg.py:101-115).  An
    output irrep no coupling path reaches raises, as the reference does (cg.py:116-133 leaves
    last_ir unbound: e.g. 0o at correlation 4, where the filter admits natural parity only)."""
    filt = {(l, (-1) ** l) for l in range(12)} if nu == 4 else None
    blocks = [C for ir, C in _cg_chain([tuple(coupling_irreps)] * nu, filt, only=ir_out)
              if ir == tuple(ir_out)]
    if not blocks:
        raise ValueError(f"no coupling path reaches {ir_out} at correlation {nu} (the "
                         "reference's cg.U_matrix_real fails here too)")
    return np.stack([np.squeeze(C) for C in blocks], axis=-1)


# ----------------------------------------------------------------------------------- gates
@lru_cache(maxsize=None)
def normalize2mom(name):
    """e3nn normalize2mom constant for silu / sigmoid (1e6 float64 normals, seed 0)."""
    import torch
    f = {"silu": torch.nn.functional.silu, "sigmoid": torch.sigmoid}[name]
    z = torch.randn(1_000_000, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    c = f(z).pow(2).mean().pow(-0.5).item()
    return 1.0 if abs(c - 1.0) < 1e-4 else c
