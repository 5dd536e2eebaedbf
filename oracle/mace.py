"""TFN / MACE layers and models restated on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py).

Follows models/layers/tfn_layer.py:8-93 (TensorProductConvLayer), models/tfn.py:13-190
(first_node_pooling, TFNModel), models/mace.py:9-190 (MACEModel),
models/mace_modules/blocks.py:99-135 (EquivariantProductBasisBlock),
models/mace_modules/symmetric_contraction.py:20-188 (SymmetricContraction / Contraction, the
element_dependent=False branch used by mace.py:114-124), models/mace_modules/cg.py:19-133
(_wigner_nj, U_matrix_real) and models/mace_modules/irreps_tools.py:63-97.
e3nn primitives come from oracle/o3.py (parity unpinned, see there).
"""
import math

import torch
from torch import nn
from torch.nn import functional as F

from . import o3
from .radial import RadialEmbeddingBlock
from .scatter import scatter, global_add_pool, global_mean_pool


# ----------------------------------------------------------------------------------- cg.py
def _wigner_nj(irrepss, normalization="component", filter_ir_mid=None):
    """cg.py:19-88 (generalised CG of a product of irreps, one entry per output irrep copy)."""
    irrepss = [o3.Irreps(x) for x in irrepss]
    if len(irrepss) == 1:
        (irreps,) = irrepss
        ret, e, i = [], torch.eye(irreps.dim, dtype=torch.float64), 0
        for mul, ir in irreps:
            for _ in range(mul):
                d = 2 * ir[0] + 1
                ret.append((ir, e[i:i + d]))
                i += d
        return ret
    *left, right = irrepss
    ret = []
    dims_left = [x.dim for x in left]
    for ir_left, C_left in _wigner_nj(left, normalization, filter_ir_mid):
        i = 0
        for mul, ir in right:
            for ir_out in o3.ir_mul(ir_left, ir):
                if filter_ir_mid is not None and ir_out not in filter_ir_mid:
                    continue
                C = o3.wigner_3j(ir_out[0], ir_left[0], ir[0])
                if normalization == "component":
                    C = C * (2 * ir_out[0] + 1) ** 0.5
                C = torch.einsum("jk,ijl->ikl", C_left.flatten(1), C)
                C = C.reshape(2 * ir_out[0] + 1, *dims_left, 2 * ir[0] + 1)
                d = 2 * ir[0] + 1
                for u in range(mul):
                    E = torch.zeros(2 * ir_out[0] + 1, *dims_left, right.dim, dtype=torch.float64)
                    E[..., i + u * d:i + (u + 1) * d] = C
                    ret.append((ir_out, E))
            i += mul * (2 * ir[0] + 1)
    return sorted(ret, key=lambda x: x[0])  # stable sort by irrep (l, p)


def U_matrix_real(irreps_in, irreps_out, correlation):
    """cg.py:91-133: stacked generalised CG tensors per output irrep, last dim = path."""
    irreps_out = o3.Irreps(irreps_out)
    wanted = [ir for _, ir in irreps_out]
    filt = None
    if correlation == 4:
        filt = [(l, (-1) ** l) for l in range(12)]
    out, stack, last = [], None, None
    current = None
    for ir, base in _wigner_nj([irreps_in] * correlation, "component", filt):
        b = base.squeeze().unsqueeze(-1)
        if ir in wanted and ir == current:
            stack = torch.cat([stack, b], dim=-1)
            last = current
        elif ir in wanted and ir != current:
            if stack is not None:
                out += [last, stack]
            stack = b
            current, last = ir, ir
        else:
            current = ir
    out += [last, stack]
    return out


# ----------------------------------------------------------------------------------- contraction
class Contraction(nn.Module):
    """symmetric_contraction.py:88-188, element_dependent=False."""

    def __init__(self, irreps_in, irrep_out, correlation):
        super().__init__()
        irreps_in = o3.Irreps(irreps_in)
        self.num_features = irreps_in.count((0, 1))
        coupling = o3.Irreps([(1, ir) for _, ir in irreps_in])
        self.correlation = correlation
        for nu in range(1, correlation + 1):
            U = U_matrix_real(coupling, o3.Irreps([(1, irrep_out)]), nu)[-1]
            self.register_buffer(f"U_matrix_{nu}", U.to(torch.get_default_dtype()))
        self.weights = nn.ParameterDict({
            str(nu): nn.Parameter(torch.randn(self.U(nu).shape[-1], self.num_features)
                                  / self.U(nu).shape[-1]) for nu in range(1, correlation + 1)})

    def U(self, nu):
        return self._buffers[f"U_matrix_{nu}"]

    def forward(self, x):  # x: (B, C, n_irrep_dims)
        out = torch.einsum("...ik,kc,bci->bc...", self.U(self.correlation),
                           self.weights[str(self.correlation)], x)
        for nu in range(self.correlation - 1, 0, -1):
            c = torch.einsum("...k,kc->c...", self.U(nu), self.weights[str(nu)]) + out
            out = torch.einsum("bc...i,bci->bc...", c, x)
        return out.reshape(out.shape[0], -1)


class SymmetricContraction(nn.Module):
    def __init__(self, irreps_in, irreps_out, correlation):
        super().__init__()
        self.irreps_out = o3.Irreps(irreps_out)
        self.contractions = nn.ModuleDict({
            f"{m}x{l}{'e' if p == 1 else 'o'}": Contraction(irreps_in, (l, p), correlation)
            for m, (l, p) in self.irreps_out})

    def forward(self, x):
        return torch.cat([c(x) for c in self.contractions.values()], dim=-1)


def reshape_irreps(irreps, x):
    """irreps_tools.py:63-79: mul_ir (B, sum mul(2l+1)) -> (B, mul, sum(2l+1))."""
    out, ix, B = [], 0, x.shape[0]
    for mul, (l, _) in o3.Irreps(irreps):
        d = 2 * l + 1
        out.append(x[:, ix:ix + mul * d].reshape(B, mul, d))
        ix += mul * d
    return torch.cat(out, dim=-1)


class EquivariantProductBasisBlock(nn.Module):
    """blocks.py:99-135 (element_dependent=False, batch_norm=False)."""

    def __init__(self, node_feats_irreps, target_irreps, correlation, use_sc=True):
        super().__init__()
        self.use_sc = use_sc
        self.symmetric_contractions = SymmetricContraction(node_feats_irreps, target_irreps,
                                                           correlation)
        self.linear = o3.Linear(target_irreps, target_irreps)

    def forward(self, node_feats, sc):
        out = self.linear(self.symmetric_contractions(node_feats))
        return out + sc if self.use_sc else out


# ----------------------------------------------------------------------------------- TP conv
class TensorProductConvLayer(nn.Module):
    """tfn_layer.py:8-93.  forward(node_attr, edge_index, edge_sh, edge_feat): gathers
    node_attr[edge_index[1]] and scatters to edge_index[0] (no dim_size)."""

    def __init__(self, in_irreps, out_irreps, sh_irreps, edge_feats_dim, mlp_dim, aggr="add",
                 batch_norm=False, gate=False):
        super().__init__()
        self.in_irreps = o3.Irreps(in_irreps)
        self.out_irreps = o3.Irreps(out_irreps)
        self.sh_irreps = o3.Irreps(sh_irreps)
        self.aggr = aggr
        if gate:
            s, g, v = o3.irreps2gate(self.out_irreps)
            self.gate = o3.Gate(s, g, v)
            self.out_irreps = self.gate.irreps_in
        else:
            self.gate = None
        self.tp = o3.FullyConnectedTensorProduct(self.in_irreps, self.sh_irreps, self.out_irreps)
        self.fc = nn.Sequential(nn.Linear(edge_feats_dim, mlp_dim), nn.ReLU(),
                                nn.Linear(mlp_dim, self.tp.weight_numel))
        self.batch_norm = o3.BatchNorm(self.out_irreps) if batch_norm else None

    def forward(self, node_attr, edge_index, edge_sh, edge_feat):
        src, dst = edge_index
        tp = self.tp(node_attr[dst], edge_sh, self.fc(edge_feat))
        reduce = "sum" if self.aggr in ("add", "sum") else self.aggr
        out = scatter(tp, src, 0, None, reduce)
        if self.gate is not None:
            out = self.gate(out)
        if self.batch_norm is not None:
            out = self.batch_norm(out)
        return out


def _hidden_irreps(emb_dim, max_ell):
    return o3.Irreps([(emb_dim, (l, (-1) ** l)) for l in range(max_ell + 1)])


def edge_features(pos, edge_index, radial, max_ell=2):
    vectors = pos[edge_index[0]] - pos[edge_index[1]]          # mace.py:170 / tfn.py:171
    lengths = torch.linalg.norm(vectors, dim=-1, keepdim=True)  # mace.py:171
    return o3.spherical_harmonics(vectors, max_ell), radial(lengths)


class MACEModel(nn.Module):
    """models/mace.py:9-190 (max_ell <= 5: the SH restatement is l <= 5; hidden_irreps as
    mace.py:90-93)."""

    def __init__(self, r_max=10.0, num_bessel=8, num_polynomial_cutoff=5, max_ell=2,
                 correlation=3, num_layers=5, emb_dim=64, mlp_dim=256, in_dim=1, out_dim=1,
                 aggr="sum", pool="sum", batch_norm=True, residual=True, equivariant_pred=False,
                 hidden_irreps=None):
        super().__init__()
        assert 1 <= max_ell <= 5
        self.max_ell = max_ell
        self.emb_dim, self.residual, self.equivariant_pred = emb_dim, residual, equivariant_pred
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, num_polynomial_cutoff)
        sh = o3.spherical_harmonics_irreps(max_ell)
        self.emb_in = nn.Embedding(in_dim, emb_dim)
        hidden = o3.Irreps(hidden_irreps) if hidden_irreps else _hidden_irreps(emb_dim, max_ell)
        self.hidden_irreps = hidden
        self.convs, self.prods = nn.ModuleList(), nn.ModuleList()
        for k in range(num_layers):
            inp = o3.Irreps(f"{emb_dim}x0e") if k == 0 else hidden
            self.convs.append(TensorProductConvLayer(inp, hidden, sh, num_bessel, mlp_dim, aggr,
                                                     batch_norm=batch_norm, gate=False))
            self.prods.append(EquivariantProductBasisBlock(hidden, hidden, correlation,
                                                           use_sc=residual))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(hidden.dim, out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(emb_dim, emb_dim), nn.ReLU(),
                                      nn.Linear(emb_dim, out_dim))

    def forward(self, batch):
        h = self.emb_in(batch.atoms)
        edge_sh, edge_feats = edge_features(batch.pos, batch.edge_index, self.radial_embedding,
                                            self.max_ell)
        for conv, prod in zip(self.convs, self.prods):
            hu = conv(h, batch.edge_index, edge_sh, edge_feats)
            sc = F.pad(h, (0, hu.shape[-1] - h.shape[-1]))
            h = prod(reshape_irreps(self.hidden_irreps, hu), sc)
        out = self.pool(h, batch.batch)
        if not self.equivariant_pred:
            out = out[:, :self.emb_dim]
        return self.pred(out)


def first_node_pooling(x, batch, size=None):
    """tfn.py:13-40: the first node of every graph."""
    prev = torch.cat([batch[-1:], batch[:-1]])
    prev[0] = -1
    return x[(batch - prev) == 1]


class TFNModel(nn.Module):
    """models/tfn.py:42-190 (max_ell <= 5)."""

    def __init__(self, r_max=10.0, num_bessel=8, num_polynomial_cutoff=5, max_ell=2,
                 num_layers=5, emb_dim=64, mlp_dim=256, in_dim=1, out_dim=1, aggr="sum",
                 pool="first", gate=True, batch_norm=False, residual=True,
                 equivariant_pred=False, hidden_irreps=None):
        super().__init__()
        assert 1 <= max_ell <= 5
        self.max_ell = max_ell
        self.emb_dim, self.residual, self.equivariant_pred = emb_dim, residual, equivariant_pred
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, num_polynomial_cutoff)
        sh = o3.spherical_harmonics_irreps(max_ell)
        self.emb_in = nn.Embedding(in_dim, emb_dim)
        hidden = o3.Irreps(hidden_irreps) if hidden_irreps else _hidden_irreps(emb_dim, max_ell)
        self.convs = nn.ModuleList()
        for k in range(num_layers):
            inp = o3.Irreps(f"{emb_dim}x0e") if k == 0 else hidden
            self.convs.append(TensorProductConvLayer(inp, hidden, sh, num_bessel, mlp_dim, aggr,
                                                     batch_norm=batch_norm, gate=gate))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool,
                     "first": first_node_pooling}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(hidden.dim, out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(emb_dim, emb_dim), nn.ReLU(),
                                      nn.Linear(emb_dim, out_dim))

    def forward(self, batch):
        h = self.emb_in(batch.atoms)
        edge_sh, edge_feats = edge_features(batch.pos, batch.edge_index, self.radial_embedding,
                                            self.max_ell)
        for conv in self.convs:
            hu = conv(h, batch.edge_index, edge_sh, edge_feats)
            h = hu + F.pad(h, (0, hu.shape[-1] - h.shape[-1])) if self.residual else hu
        out = self.pool(h, batch.batch)
        if not self.equivariant_pred:
            out = out[:, :self.emb_dim]
        return self.pred(out)
