"""TFN / MACE layers and models on the MI355X kernels — drop-ins for
models/layers/tfn_layer.py:8-93 (TensorProductConvLayer), models/tfn.py:13-190 (TFNModel,
first_node_pooling), models/mace.py:9-190 (MACEModel), models/mace_modules/blocks.py:84-135
(RadialEmbeddingBlock, EquivariantProductBasisBlock), symmetric_contraction.py:20-188,
irreps_tools.py:63-97 and the e3nn modules they use (SphericalHarmonics, o3.Linear,
nn.BatchNorm, nn.Gate).

Hot path on HIP: per-edge featurisation (K1: vectors, lengths, SH l<=2, Bessel x cutoff) and
the tensor-product convolution (K7: radial-MLP weights x CG contraction x receiver sum), plus the
gathers / segmented sums of the generic ops.  The radial MLP's wide second Linear
(256 -> weight_numel, e.g. 180,224 for MACE-128) is evaluated chunk by chunk with the library
GEMM so that the per-edge weights (721 KB per edge for MACE-128, 721 GB at 1M edges) never exist
all at once; the HIP TP kernels stream each chunk once.  Node-level pieces (BatchNorm, Gate,
o3.Linear, symmetric contraction) are PyTorch ops on N-row tensors.
"""
import math

import torch
from torch.autograd.function import once_differentiable
from torch import nn
from torch.nn import functional as F

from . import _lib, ops
from . import o3
from .ops import _f32c, _need_cuda, _timed
from .scatter import global_add_pool, global_mean_pool, scatter

CHUNK_BYTES = 6 << 30


# ===================================================================================== radial
class BesselBasis(nn.Module):
    """radial.py:12-52 (same buffers)."""

    def __init__(self, r_max, num_basis=8, trainable=False):
        super().__init__()
        w = math.pi / r_max * torch.linspace(1.0, num_basis, num_basis)
        if trainable:
            self.bessel_weights = nn.Parameter(w)
        else:
            self.register_buffer("bessel_weights", w)
        self.register_buffer("r_max", torch.tensor(float(r_max)))
        self.register_buffer("prefactor", torch.tensor(math.sqrt(2.0 / r_max)))

    def forward(self, x):
        return self.prefactor * (torch.sin(self.bessel_weights * x) / x)


class PolynomialCutoff(nn.Module):
    """radial.py:55-81 (same buffers)."""

    def __init__(self, r_max, p=6):
        super().__init__()
        self.register_buffer("p", torch.tensor(float(p)))
        self.register_buffer("r_max", torch.tensor(float(r_max)))

    def forward(self, x):
        p, u = self.p, x / self.r_max
        env = (1.0 - ((p + 1.0) * (p + 2.0) / 2.0) * torch.pow(u, p)
               + p * (p + 2.0) * torch.pow(u, p + 1) - (p * (p + 1.0) / 2) * torch.pow(u, p + 2))
        return env * (x < self.r_max)


class RadialEmbeddingBlock(nn.Module):
    """blocks.py:84-96."""

    def __init__(self, r_max, num_bessel, num_polynomial_cutoff):
        super().__init__()
        self.bessel_fn = BesselBasis(r_max=r_max, num_basis=num_bessel)
        self.cutoff_fn = PolynomialCutoff(r_max=r_max, p=num_polynomial_cutoff)
        self.out_dim = num_bessel
        # host copies of the constants for the fused featurisation kernel (no device sync)
        self._host = (self.bessel_fn.bessel_weights.detach().cpu().numpy().astype("float32"),
                      float(self.bessel_fn.prefactor), float(r_max), float(num_polynomial_cutoff))

    def forward(self, edge_lengths):
        return self.bessel_fn(edge_lengths) * self.cutoff_fn(edge_lengths)


class EdgeFeaturizeFn(torch.autograd.Function):
    """K1: (pos, edge_index) -> (edge_sh (E, (lmax+1)^2), edge_feats (E,nb)) in one pass over the
    edges (lmax <= 5: the models' max_ell; l = 4, 5 by e3nn's CG recursion)."""

    @staticmethod
    def forward(ctx, pos, edge_index, host_consts, graph, lmax=2):
        w, pref, r_max, p = host_consts
        pos = _f32c(pos)
        ei = edge_index.contiguous()
        _need_cuda(pos, ei)
        with _timed("edge_featurize"):
            sh, rad = _lib.torch_ops().edge_featurize(pos, ei, [float(v) for v in w], pref, r_max,
                                                      p, lmax)
        ctx.save_for_backward(pos, ei)
        ctx.host, ctx.graph, ctx.lmax = host_consts, graph, lmax
        return sh, rad

    @staticmethod
    @once_differentiable
    def backward(ctx, g_sh, g_rad):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        pos, ei = ctx.saved_tensors
        w, pref, r_max, p = ctx.host
        g_vec = _lib.torch_ops().edge_featurize_bwd(
            pos, ei, [float(v) for v in w], pref, r_max, p,
            _f32c(g_sh) if g_sh is not None else None,
            _f32c(g_rad) if g_rad is not None else None, ctx.lmax)
        g = ctx.graph  # vectors = pos[ei0] - pos[ei1]: + into receivers, - into senders
        plus, _ = ops.segment_reduce(g_vec, g.recv_csr, "sum")
        minus, _ = ops.segment_reduce(ops.gather_rows(g_vec, g.perm), g.src_csr, "sum")
        return plus - minus, None, None, None, None


def spherical_harmonics_l2(vec, normalize=True):
    """e3nn SphericalHarmonics(lmax=2, normalize, 'component') on arbitrary vectors (GPU ops)."""
    if normalize:
        vec = F.normalize(vec, dim=-1)
    x, y, z = vec[..., 0], vec[..., 1], vec[..., 2]
    s3, s5, s15 = math.sqrt(3.0), math.sqrt(5.0), math.sqrt(15.0)
    return torch.stack([torch.ones_like(x), s3 * x, s3 * y, s3 * z, s15 * x * z, s15 * x * y,
                        s5 * (y * y - 0.5 * (x * x + z * z)), s15 * y * z,
                        s15 / 2.0 * (z * z - x * x)], dim=-1)


# ===================================================================================== e3nn-like
class Linear(nn.Module):
    """e3nn o3.Linear(irreps_in, irreps_out) with internal shared weights, no biases
    (blocks.py:121-124): out_o[w, m] = sum_{i->o} sum_u W[u, w] x_i[u, m] / sqrt(fan_in_o)."""

    def __init__(self, irreps_in, irreps_out):
        super().__init__()
        self.irreps_in, self.irreps_out = o3.parse_irreps(irreps_in), o3.parse_irreps(irreps_out)
        self.instructions = [(i, j) for i, (_, a) in enumerate(self.irreps_in)
                             for j, (_, b) in enumerate(self.irreps_out) if a == b]
        n = sum(self.irreps_in[i][0] * self.irreps_out[j][0] for i, j in self.instructions)
        self.weight = nn.Parameter(torch.randn(n))

    def forward(self, x):
        B = x.shape[0]
        oi, oo = o3.irreps_offsets(self.irreps_in), o3.irreps_offsets(self.irreps_out)
        outs = [None] * len(self.irreps_out)
        off = 0
        for i, j in self.instructions:
            mi, (l, _) = self.irreps_in[i]
            mo = self.irreps_out[j][0]
            fan = sum(self.irreps_in[a][0] for a, b in self.instructions if b == j)
            W = self.weight[off:off + mi * mo].view(mi, mo)
            off += mi * mo
            d = 2 * l + 1
            xi = x[:, oi[i]:oi[i] + mi * d].reshape(B, mi, d)
            # one (B*d, mi) x (mi, mo) GEMM instead of B batched (mo, mi) x (mi, d) products
            r = xi.transpose(1, 2).reshape(B * d, mi).matmul(W / math.sqrt(fan))
            r = r.reshape(B, d, mo).transpose(1, 2).reshape(B, mo * d)
            outs[j] = r if outs[j] is None else outs[j] + r
        for j, (mo, (l, _)) in enumerate(self.irreps_out):
            if outs[j] is None:
                outs[j] = x.new_zeros(B, mo * (2 * l + 1))
        return torch.cat(outs, dim=1)


def _dev_table(cache, key_fn, device):
    t = cache.get(device)
    if t is None:
        t = tuple(v.to(device) for v in key_fn())
        cache[device] = t
    return t


class IrrepsBatchNormFn(torch.autograd.Function):
    """K16 e3nn BatchNorm (gmp_irreps_bn_{fwd,bwd}_f32): two fixed-order statistics passes and
    one apply pass forward (running stats updated in place when training), one statistics and
    one apply pass backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, tables, running_mean, running_var, training, momentum,
                eps):
        col_chan, chan_col, chan_info = tables
        y, shift, invstd = _lib.torch_ops().irreps_bn_fwd(
            x, col_chan, chan_col, chan_info, weight, bias if bias.numel() else None,
            running_mean, running_var, bool(training), float(momentum), float(eps))
        ctx.save_for_backward(x, weight, shift, invstd)
        ctx.tables, ctx.training, ctx.n_scalar = tables, bool(training), bias.numel()
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        x, weight, shift, invstd = ctx.saved_tensors
        col_chan, chan_col, chan_info = ctx.tables
        gx, gw, gb = _lib.torch_ops().irreps_bn_bwd(x, _f32c(gy), col_chan, chan_col, chan_info,
                                                   weight, shift, invstd, ctx.training,
                                                   ctx.n_scalar)
        return gx, gw, gb, None, None, None, None, None, None


class BatchNorm(nn.Module):
    """e3nn nn.BatchNorm(irreps) (eps 1e-5, momentum 0.1, affine, reduce mean, component) as the
    fused HIP kernels K16 (tfn_layer.py:89-90; e3nn 0.5 nn/_batchnorm.py semantics): scalars
    (0e) centred by the batch mean, every channel scaled by weight (mean f^2 + eps)^-1/2,
    scalars + bias; running_mean / running_var updated with momentum in training."""

    def __init__(self, irreps, eps=1e-5, momentum=0.1):
        super().__init__()
        self.irreps = o3.parse_irreps(irreps)
        self.eps, self.momentum = eps, momentum
        ns = sum(m for m, ir in self.irreps if ir == (0, 1))
        nf = sum(m for m, _ in self.irreps)
        self.register_buffer("running_mean", torch.zeros(ns))
        self.register_buffer("running_var", torch.ones(nf))
        self.weight = nn.Parameter(torch.ones(nf))
        self.bias = nn.Parameter(torch.zeros(ns))
        self._tables = {}

    def _host_tables(self):
        col_chan, chan_col, chan_info = [], [], []
        u = si = col = 0
        for mul, (l, p) in self.irreps:
            d = 2 * l + 1
            scalar = (l == 0 and p == 1)
            for _ in range(mul):
                chan_col.append(col)
                chan_info.append((d, si if scalar else -1))
                col_chan.extend([u] * d)
                si += int(scalar)
                u += 1
                col += d
        i32 = dict(dtype=torch.int32)
        return (torch.tensor(col_chan, **i32), torch.tensor(chan_col, **i32),
                torch.tensor(chan_info, **i32).view(-1, 2))

    def forward(self, x):
        x = _f32c(x)
        _need_cuda(x)
        tables = _dev_table(self._tables, self._host_tables, x.device)
        return IrrepsBatchNormFn.apply(x, self.weight, self.bias, tables, self.running_mean,
                                       self.running_var, self.training, self.momentum, self.eps)


class GateFn(torch.autograd.Function):
    """K16 Gate (gmp_gate_{fwd,bwd}_f32): one pass each way over the node rows."""

    @staticmethod
    def forward(ctx, x, out_map, in_map, c_act, c_gate):
        y = _lib.torch_ops().gate_fwd(x, out_map, c_act, c_gate)
        ctx.save_for_backward(x)
        ctx.in_map, ctx.c = in_map, (c_act, c_gate)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return (_lib.torch_ops().gate_bwd(x, _f32c(gy), ctx.in_map, *ctx.c), None, None, None,
                None)


class Gate(nn.Module):
    """e3nn nn.Gate(scalars, [silu], gates, [sigmoid], gated) (tfn_layer.py:45-63) as the fused
    HIP kernel K16, normalize2mom constants baked in:
    y = [c_act silu(scalars), gated * c_gate sigmoid(gates)]."""

    def __init__(self, irreps_scalars, irreps_gates, irreps_gated):
        super().__init__()
        self.irreps_scalars, self.irreps_gates = irreps_scalars, irreps_gates
        self.irreps_gated = irreps_gated
        self.irreps_in = tuple(irreps_scalars) + tuple(irreps_gates) + tuple(irreps_gated)
        self.irreps_out = tuple(irreps_scalars) + tuple(irreps_gated)
        self.c_act, self.c_gate = o3.normalize2mom("silu"), o3.normalize2mom("sigmoid")
        self._tables = {}

    def _host_tables(self):
        ns, ng = o3.irreps_dim(self.irreps_scalars), o3.irreps_dim(self.irreps_gates)
        n_gated = sum(m for m, _ in self.irreps_gated)
        if ng != n_gated:
            raise ValueError(f"Gate: {ng} gate scalars for {n_gated} gated channels")
        out_map = [(j, -1) for j in range(ns)]
        in_map = [(0, j, 0, 0) for j in range(ns)] + [None] * ng
        gated_in = []
        k = off = 0
        for mul, (l, _) in self.irreps_gated:
            d = 2 * l + 1
            for _ in range(mul):
                in_map[ns + k] = (1, ns + off, ns + ng + off, d)
                for m in range(d):
                    out_map.append((ns + ng + off + m, ns + k))
                    gated_in.append((2, ns + off + m, ns + k, 0))
                k += 1
                off += d
        in_map += gated_in
        i32 = dict(dtype=torch.int32)
        return (torch.tensor(out_map, **i32).view(-1, 2), torch.tensor(in_map, **i32).view(-1, 4))

    def forward(self, x):
        x = _f32c(x)
        _need_cuda(x)
        out_map, in_map = _dev_table(self._tables, self._host_tables, x.device)
        return GateFn.apply(x, out_map, in_map, float(self.c_act), float(self.c_gate))


# ===================================================================================== TP conv
class TPGraph:
    """Receiver (edge_index[0])-sorted CSR for the TP convolution (scatter target ei0,
    gather source ei1: tfn_layer.py:83-87), plus the CSR of the gather source over sorted
    positions for the backward segmented sums.  num_src: rows of the gathered features when they
    differ from the receivers' (the per-edge-message graph of aggr max / min)."""

    def __init__(self, edge_index, num_nodes, num_src=None):
        ei = edge_index.contiguous()
        self.num_nodes, self.num_edges = int(num_nodes), ei.shape[1]
        self.num_src = self.num_nodes if num_src is None else int(num_src)
        self.recv_csr = ops.CSR(ei[0], self.num_nodes, payload=ei[1])
        self.rowptr = self.recv_csr.rowptr
        self.perm = self.recv_csr.perm
        self.src_sorted = self.recv_csr.payload_sorted
        self.recv_sorted = self.recv_csr.sorted
        self.src_csr = ops.CSR(self.src_sorted, self.num_src)
        self._node_form = None

    def node_form(self):
        """Host copy of rowptr (one sync per graph), max in-degree and per-edge slot."""
        if self._node_form is None:
            rp = self.rowptr.cpu()
            deg = rp[1:] - rp[:-1]
            dmax = int(deg.max()) if deg.numel() else 0
            dmax = -(-dmax // 8) * 8  # padded in-degree: 32-byte aligned batched-GEMM operands
            slot = torch.arange(self.num_edges, device=self.rowptr.device) - \
                self.rowptr[self.recv_sorted]
            self._node_form = (rp.tolist(), dmax, slot)
        return self._node_form

    def node_chunks(self, nodes_per_chunk):
        rp, dmax, _ = self.node_form()
        n = self.num_nodes
        for n0 in range(0, n, nodes_per_chunk):
            n1 = min(n, n0 + nodes_per_chunk)
            yield n0, n1, rp[n0], rp[n1]

    def chunk_pad(self, n0, n1, e0, e1):
        """(c * dmax) gather index into the chunk's edge rows (padding -> n_e) and the (n_e,)
        position of every chunk edge in the padded (c, dmax) grid."""
        _, dmax, slot = self.node_form()
        dev = self.rowptr.device
        c, ne = n1 - n0, e1 - e0
        s = torch.arange(dmax, device=dev)
        rp = self.rowptr[n0:n1]
        deg = self.rowptr[n0 + 1:n1 + 1] - rp
        idx = torch.where(s[None, :] < deg[:, None], rp[:, None] - e0 + s[None, :],
                          torch.full((), ne, device=dev, dtype=torch.int64))
        pos = (self.recv_sorted[e0:e1] - n0) * dmax + slot[e0:e1]
        return idx.reshape(-1), pos


_TP_GRAPHS = []


def tp_graph(edge_index, num_nodes, num_src=None):
    if ops.compiling():
        return TPGraph(edge_index, num_nodes, num_src)
    key = (num_nodes, num_src)
    for t, ver, n, g in _TP_GRAPHS:
        if t is edge_index and ver == edge_index._version and n == key:
            return g
    g = TPGraph(edge_index, num_nodes, num_src)
    _TP_GRAPHS.insert(0, (edge_index, edge_index._version, key, g))
    del _TP_GRAPHS[4:]
    return g


_LAYOUTS = {((0, 1), (1, -1), (2, 1)): 0, ((0, 1), (0, 1), (1, -1), (2, 1)): 1}


class TPPlan:
    """Instruction table + CG constants of one FullyConnectedTensorProduct, uploaded once."""

    def __init__(self, irreps_in, irreps_sh, irreps_out):
        self.irreps_in, self.irreps_sh, self.irreps_out = irreps_in, irreps_sh, irreps_out
        self.instructions, self.weight_numel = o3.fctp_instructions(irreps_in, irreps_sh,
                                                                    irreps_out)
        key = tuple(ir for _, ir in irreps_out)
        sh_dim = o3.irreps_dim(irreps_sh)
        # (input irreps with a repeated l -- both parities -- take the dz kernel's grouped form)
        # (l = 4, 5: the runtime-l z / dz kernels, CG table <= 8192 floats; l <= 3 the fixed-l
        # ones, <= 4096)
        lmx = max(ir[0] for _, ir in tuple(irreps_in) + tuple(irreps_out) + tuple(irreps_sh))
        cg_floats = sum((2 * i["l1"] + 1) * (2 * i["l2"] + 1) * (2 * i["lo"] + 1)
                        for i in self.instructions)
        if any(m != 1 for m, _ in irreps_sh) or sh_dim not in (1, 4, 9, 16, 25, 36) or \
                any(m > 128 for m, _ in irreps_in) or len(irreps_out) > 8 or lmx > 5 or \
                len(self.instructions) > 48 or cg_floats > (8192 if lmx > 3 else 4096):
            raise NotImplementedError(f"TP {o3.irreps_str(irreps_in)} x {o3.irreps_str(irreps_sh)}"
                                      f" -> {o3.irreps_str(irreps_out)} not supported by K7")
        # the per-edge-weight kernels (TP_MODE = "edge") take the two l <= 2 layouts; the node
        # form (default) any block structure with l <= 5
        edge_ok = (key in _LAYOUTS and sh_dim == 9 and
                   not any(m > 128 or m % 4 for m, _ in irreps_out))
        self.layout = _LAYOUTS[key] if edge_ok else None
        xo, yo, oo = (o3.irreps_offsets(irreps_in), o3.irreps_offsets(irreps_sh),
                      o3.irreps_offsets(irreps_out))
        paths = (_lib.TpPath * len(self.instructions))()
        cg, z_off = [], 0
        cg_off = 0
        for k, ins in enumerate(self.instructions):
            C = o3.wigner_3j(ins["l1"], ins["l2"], ins["lo"])
            paths[k] = _lib.TpPath(ins["l1"], ins["l2"], ins["lo"], ins["mul1"], ins["mul_out"],
                                   xo[ins["i1"]], yo[ins["i2"]], ins["io"], oo[ins["io"]], z_off,
                                   cg_off, 0, ins["w_off"], ins["alpha"], 0.0)
            cg.append(torch.from_numpy(C.reshape(-1).copy()))
            cg_off += C.size
            z_off += ins["mul1"] * (2 * ins["lo"] + 1)
        self.paths_host = paths
        self.cg_host = torch.cat(cg).float()
        self.desc = _lib.TpDesc()
        self.desc.n_paths = len(self.instructions)
        self.desc.in_dim = o3.irreps_dim(irreps_in)
        self.desc.out_dim = o3.irreps_dim(irreps_out)
        self.desc.sh_dim = sh_dim
        self.sh_dim = sh_dim
        self.desc.weight_numel = self.weight_numel
        self.desc.z_size = z_off
        self.desc.n_blocks = len(irreps_out)
        for b, (m, (l, _)) in enumerate(irreps_out):
            self.desc.blk_off[b], self.desc.blk_mul[b], self.desc.blk_l[b] = oo[b], m, l
        self.blocks = [(oo[b], m) for b, (m, _) in enumerate(irreps_out)]  # (offset, mul)
        # plain-int copies (the autograd Functions read these, never the ctypes descriptor)
        self.in_dim, self.out_dim = self.desc.in_dim, self.desc.out_dim
        self.z_size = self.desc.z_size
        d = self.desc  # the descriptor as torch.ops.gmp.tp_* take it (int[25] + l_max)
        self.l_max = max(max(i["l1"], i["l2"], i["lo"]) for i in self.instructions)
        self.desc_list = ([d.n_paths, d.in_dim, d.out_dim, d.sh_dim, d.weight_numel, d.z_size,
                           d.n_blocks] + list(d.blk_off) + list(d.blk_mul) + list(d.blk_l)
                          + [self.l_max])
        # node form: path p's z rows (mul1 * (2lo+1) floats) at z_off_p * (n_e + 1)
        self.z_regions = [(paths[k].z_off, ins["mul1"] * (2 * ins["lo"] + 1))
                          for k, ins in enumerate(self.instructions)]
        self.max_block_rows = max(w for _, w in self.z_regions)
        self._dev = {}

    def host_tables(self):
        """(path records as uint8 bytes, concatenated CG floats) on the host."""
        return (torch.frombuffer(bytearray(bytes(self.paths_host)), dtype=torch.uint8),
                self.cg_host.clone())

    def device_tables(self, device):
        if device not in self._dev:
            raw, cg = self.host_tables()
            self._dev[device] = (raw.to(device), cg.to(device))
        return self._dev[device]

    def chunk_edges(self):
        e = CHUNK_BYTES // (4 * self.weight_numel)
        return max(256, (e // 256) * 256)


class TPConvFn(torch.autograd.Function):
    """out = scatter_sum_{ei0}( FCTP(x[ei1], sh, fc(radial)) )   (tfn_layer.py:82-87).

    Chunked over receiver-sorted edges: per chunk the radial MLP produces the per-edge weights
    (library GEMM), then the HIP TP kernel contracts them with the CG-coupled features and sums
    into the receiver rows.  Backward recomputes the chunk's weights."""

    @staticmethod
    def forward(ctx, x, sh, rad, W1, b1, W2, b2, plan, graph, paths_dev, cg_dev):
        x, sh, rad = _f32c(x), _f32c(sh), _f32c(rad)
        _need_cuda(x, sh, rad)
        dev = x.device
        N, E = graph.num_nodes, graph.num_edges
        msg = torch.empty((E, plan.out_dim), dtype=torch.float32, device=dev)
        rad_s = ops.gather_rows(rad, graph.perm)  # radial features in receiver-sorted order
        ce = plan.chunk_edges()
        tops = _lib.torch_ops()
        for c0 in range(0, E, ce):
            c1 = min(E, c0 + ce)
            with _timed("radial_gemm"):
                a = torch.relu(torch.addmm(b1, rad_s[c0:c1], W1.t()))
                Wc = torch.addmm(b2, a, W2.t())
            with _timed("tp_conv_fwd"):
                tops.tp_conv_fwd(plan.layout, plan.desc_list, paths_dev, cg_dev, x, sh, Wc,
                                 graph.src_sorted, graph.perm, c0, c1, msg)
            del Wc, a
        # receiver sums over the sorted messages (deterministic, chunk-independent)
        out, _ = ops.segment_reduce(msg, graph.recv_csr, "sum", use_perm=False)
        del msg
        ctx.plan, ctx.graph, ctx.tables = plan, graph, (paths_dev, cg_dev)
        ctx.save_for_backward(x, sh, rad_s, W1, b1, W2, b2)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        x, sh, rad_s, W1, b1, W2, b2 = ctx.saved_tensors
        plan, graph = ctx.plan, ctx.graph
        paths_dev, cg_dev = ctx.tables
        gout = _f32c(gout)
        N, E = graph.num_nodes, graph.num_edges
        f = dict(dtype=torch.float32, device=x.device)
        dx_edge = torch.empty((E, plan.in_dim), **f)
        dY = torch.empty((E, plan.sh_dim), **f)
        drad_s = torch.empty_like(rad_s)
        dW2 = torch.zeros_like(W2)
        db2 = torch.zeros_like(b2)
        dW1 = torch.zeros_like(W1)
        db1 = torch.zeros_like(b1)
        ce = plan.chunk_edges()
        tops = _lib.torch_ops()
        for c0 in range(0, E, ce):
            c1 = min(E, c0 + ce)
            r = rad_s[c0:c1]
            with _timed("radial_gemm"):
                pre = torch.addmm(b1, r, W1.t())
                a = torch.relu(pre)
                Wc = torch.addmm(b2, a, W2.t())
            with _timed("tp_conv_bwd"):
                dWc = tops.tp_conv_bwd(plan.layout, plan.desc_list, paths_dev, cg_dev, x, sh, Wc,
                                       graph.recv_sorted, graph.src_sorted, graph.perm, c0, c1,
                                       gout, dx_edge, dY)
            del Wc
            with _timed("radial_gemm"):
                dW2.addmm_(dWc.t(), a)
                db2.add_(dWc.sum(0))
                da = dWc.mm(W2)
                del dWc
                dpre = da * (pre > 0)
                dW1.addmm_(dpre.t(), r)
                db1.add_(dpre.sum(0))
                drad_s[c0:c1] = dpre.mm(W1)
        dx, _ = ops.segment_reduce(dx_edge, graph.src_csr, "sum")
        dsh = torch.empty_like(sh).index_copy_(0, graph.perm, dY)
        drad = torch.empty((E, rad_s.shape[1]), **f).index_copy_(0, graph.perm, drad_s)
        return dx, dsh, drad, dW1, db1, dW2, db2, None, None, None, None


# Receiver chunk of the node form, in bytes of S (+ T) for the widest path.  Larger chunks give
# the path GEMMs (M = receivers x (2lo+1), N = mul_out = 128, K = mul1 x H) enough row tiles to
# fill the 256 CUs: 2 GiB -> 64 GiB took MACE-128 at 1M edges from 287k to 332k edges/s.  The
# default (None) is a quarter of the device's HBM, capped at 64 GiB (one chunk for a 1M-edge
# graph); tests set a small value to cover the multi-chunk path.
NODE_CHUNK_BYTES = None


_HBM_BYTES = {}


def node_chunk_bytes(device):
    if NODE_CHUNK_BYTES is not None:
        return NODE_CHUNK_BYTES
    if device not in _HBM_BYTES:
        _HBM_BYTES[device] = torch.cuda.get_device_properties(device).total_memory
    return int(min(64 << 30, _HBM_BYTES[device] // 4))
TP_MODE = "node"  # "node" (receiver-factorised) | "edge" (per-edge weights; tests compare)


def _w2_path(W2, b2, P):
    """Path block of W2 as (mul1 * H, mul_out) [row (u, j), column w] and of b2 as
    (mul1, mul_out)."""
    m1, mo, off = P["mul1"], P["mul_out"], P["w_off"]
    H = W2.shape[1]
    return (W2[off:off + m1 * mo].view(m1, mo, H).permute(0, 2, 1).reshape(m1 * H, mo),
            b2[off:off + m1 * mo].view(m1, mo))


def node_form_ok(hidden):
    """The node-form kernels take any radial hidden width H <= 256: a width that is not a
    multiple of 32 runs zero-padded (`_node_radial`)."""
    return 0 < hidden <= 256


def _node_radial(fc):
    """fc's W1, b1, W2, b2 for the node form, the hidden width zero-padded to a multiple of 32
    (the kernels' 16-wide MFMA k steps, and K7g's 32-deep ones): padded units have zero W1 rows
    and bias, so relu(0) = 0 contributes nothing to S, T or the weight sums, and F.pad's
    backward drops their gradient rows (tfn_layer.py:73-77 takes any mlp_dim)."""
    W1, b1, W2, b2 = fc[0].weight, fc[0].bias, fc[2].weight, fc[2].bias
    pad = -W1.shape[0] % 32
    if pad:
        W1, b1, W2 = F.pad(W1, (0, 0, 0, pad)), F.pad(b1, (0, pad)), F.pad(W2, (0, pad))
    return W1, b1, W2, b2


# Path GEMMs of the node form: "x3" = K7g (gmp_tpgemm.hip: bf16 MFMA over exact three-plane f32
# splits; dW2p by the column-block split-plane outer sum), "torch" = the library f32 GEMMs.
def _x3_ok(P, H):
    """Shapes K7g covers: every k range a multiple of the 32-deep MFMA step and mul_out <= 128
    (128 x 128 output tiles; 256 x 64 for the 64-channel paths of config C5)."""
    return (P["mul1"] % 32 == 0 and P["mul_out"] % 32 == 0
            and P["mul_out"] <= 128 and H % 32 == 0)


def _split_w2(W2, b2, P, fwd):
    """Three bf16 planes of path P's W2 / b2 block: forward (B = [W2p | b2p]^T as [w][(u, j) ++ u])
    or backward (B = W2p as [(u, j)][w]) layout (torch.ops.gmp.tp_split_w2)."""
    return _lib.torch_ops().tp_split_w2(W2, b2, P["w_off"], P["mul1"], P["mul_out"], fwd)


class TPConvNodeFn(torch.autograd.Function):
    """out = scatter_sum_{ei0}(FCTP(x[ei1], sh, fc(radial)))  (tfn_layer.py:82-87), evaluated in
    receiver-factorised form: with a_e = relu(W1 r_e + b1) (H) the per-edge weights are
    W_e = W2 a_e + b2, so for receiver n and path p
        out_n[w, k] = sum_{u, j} W2[(u, w), j] S_n[k, u, j] + sum_u b2[u, w] Sb_n[k, u],
        S_n = sum_{e -> n} z_e (x) a_e,   Sb_n = sum_{e -> n} z_e.
    S comes from the per-receiver MFMA kernel (gmp_tp_node_outer_f32, edge index as the MFMA k
    dimension) and the contraction with W2 is one GEMM per path with K = mul1 * H:
    E * H * weight_numel MACs become N * H * sum_p mul1 mul_out (2lo+1) + E * H * z_size
    (N = E / 20 here).  Backward: T = G W2_p^T, Tb = G b2_p^T (GEMMs), then dz = a.T + Tb and
    da = z.T per edge (gmp_tp_node_apply_f32); dW2 = G^T S, db2 = G^T Sb."""

    @staticmethod
    def forward(ctx, x, sh, rad, W1, b1, W2, b2, plan, graph, paths_dev, cg_dev):
        x, sh, rad = _f32c(x), _f32c(sh), _f32c(rad)
        _need_cuda(x, sh, rad)
        dev = x.device
        N, E = graph.num_nodes, graph.num_edges
        H = W1.shape[0]
        tops = _lib.torch_ops()
        out = torch.zeros((N, plan.out_dim), dtype=torch.float32, device=dev)
        rad_s = ops.gather_rows(rad, graph.perm)
        W2c, b2c = W2.contiguous(), b2.contiguous()
        x3 = [_x3_ok(P, H) for P in plan.instructions]
        W2x = [None if ok else _w2_path(W2, b2, P) for P, ok in zip(plan.instructions, x3)]
        Bfs = [None] * len(x3)
        for n0, n1, e0, e1, eoff, a, zbuf, _ in _node_chunks(plan, graph, x, sh, rad_s, W1, b1,
                                                             paths_dev, cg_dev):
            c, ne = n1 - n0, e1 - e0
            for i, (P, (zoff, w)) in enumerate(zip(plan.instructions, plan.z_regions)):
                d3, m1, mo = 2 * P["lo"] + 1, P["mul1"], P["mul_out"]
                Zp = zbuf[zoff * (ne + 1):(zoff + w) * (ne + 1)].view(ne + 1, w)
                blk = plan.blocks[P["io"]]
                S, Sb = _node_outer(eoff, Zp, a, w)
                if x3[i]:
                    # out[n, blk + w' d3 + k] += [S | Sb][(n, k), :] [W2p ; b2p][:, w'] (K7g)
                    if Bfs[i] is None:
                        Bfs[i] = _split_w2(W2c, b2c, P, True)
                    K1 = m1 * H
                    with _timed("tp_node_W"):
                        tops.tp_gemm_x3(S.view(c * d3, K1), K1, Sb.view(c * d3, m1), m1, Bfs[i],
                                        K1 + m1, mo, out, n0 * out.shape[1] + blk[0], d3,
                                        out.shape[1], 1, d3, True)
                else:
                    W2p, b2p = W2x[i]
                    with _timed("tp_node_W"):
                        op = torch.addmm(Sb.view(c * d3, -1).mm(b2p), S.view(c * d3, -1), W2p)
                    out[n0:n1, blk[0]:blk[0] + blk[1] * d3].view(c, blk[1], d3).add_(
                        op.view(c, d3, -1).transpose(1, 2))
                    del op
                del S, Sb
        ctx.plan, ctx.graph, ctx.tables = plan, graph, (paths_dev, cg_dev)
        ctx.save_for_backward(x, sh, rad_s, W1, b1, W2, b2)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        x, sh, rad_s, W1, b1, W2, b2 = ctx.saved_tensors
        plan, graph = ctx.plan, ctx.graph
        paths_dev, cg_dev = ctx.tables
        tops = _lib.torch_ops()
        gout = _f32c(gout)
        N, E = graph.num_nodes, graph.num_edges
        H = W1.shape[0]
        f = dict(dtype=torch.float32, device=x.device)
        dx_edge = torch.empty((E, plan.in_dim), **f)
        dY = torch.empty((E, plan.sh_dim), **f)
        drad_s = torch.empty_like(rad_s)
        dW1, db1 = torch.zeros_like(W1), torch.zeros_like(b1)
        W2c, b2c = W2.contiguous(), b2.contiguous()
        x3 = [_x3_ok(P, H) for P in plan.instructions]
        W2x = [_w2_path(W2, b2, P) for P in plan.instructions]
        dW2x = [(torch.zeros_like(wp), torch.zeros_like(bp)) for wp, bp in W2x]
        Bts = [None] * len(x3)
        first = True
        for n0, n1, e0, e1, eoff, a, zbuf, pre in _node_chunks(plan, graph, x, sh, rad_s, W1,
                                                               b1, paths_dev, cg_dev):
            c, ne = n1 - n0, e1 - e0
            dzbuf = torch.empty_like(zbuf)
            da = torch.zeros((ne, H), **f)
            for i, (P, (W2p, b2p), (dW2p, db2p), (zoff, w)) in enumerate(
                    zip(plan.instructions, W2x, dW2x, plan.z_regions)):
                d3, m1, mo = 2 * P["lo"] + 1, P["mul1"], P["mul_out"]
                blk = plan.blocks[P["io"]]
                Zp = zbuf[zoff * (ne + 1):(zoff + w) * (ne + 1)].view(ne + 1, w)
                G = gout[n0:n1, blk[0]:blk[0] + blk[1] * d3].view(c, mo, d3).transpose(1, 2)
                G = G.reshape(c * d3, mo).contiguous()  # (d3 = 1: reshape alone is a view)
                if x3[i]:
                    K1 = m1 * H
                    S, Sb = _node_outer(eoff, Zp, a, w)  # (timed as tp_node_S)
                    with _timed("tp_node_dW"):
                        # dW2p[(u, j), w] = sum_(n, k) S[(n, k), (u, j)] G[(n, k), w]
                        part = tops.outer_sum_cols(S.view(c * d3, K1), G)
                        del S
                        # db2p[u, w] = sum_(n, k) Sb[(n, k), u] G[(n, k), w]: the deterministic
                        # outer sum (the library's K = 250k reduction GEMM ran 0.4 ms per path)
                        pb, _ = ops.edge_outer_sum_rect(Sb.view(c * d3, m1), G)
                        if first:
                            dW2p.copy_(part)
                            db2p.copy_(pb)
                        else:
                            dW2p.add_(part)
                            db2p.add_(pb)
                    del Sb
                    if Bts[i] is None:
                        Bts[i] = _split_w2(W2c, b2c, P, False)
                    with _timed("tp_node_W"):
                        # T[(n, k), (u, j)] = sum_w G[(n, k), w] W2p[(u, j), w]
                        T = tops.tp_gemm_x3_widen(G, Bts[i], K1)
                        Tb = G.mm(b2p.t())
                else:
                    S, Sb = _node_outer(eoff, Zp, a, w)
                    with _timed("tp_node_dW"):
                        dW2p.addmm_(S.view(c * d3, -1).t(), G)
                        db2p.addmm_(Sb.view(c * d3, -1).t(), G)
                    del S, Sb
                    with _timed("tp_node_W"):
                        T = G.mm(W2p.t())
                        Tb = G.mm(b2p.t())
                dZp = dzbuf[zoff * (ne + 1):(zoff + w) * (ne + 1)].view(ne + 1, w)
                with _timed("tp_node_dZA"):
                    tops.tp_node_apply(eoff, Zp, a, T, Tb.contiguous(), da, dZp)
                del T, Tb
            first = False
            with _timed("tp_node_edge_bwd"):
                dxc, dYc = tops.tp_edge_z_bwd(plan.desc_list, paths_dev, cg_dev, x, sh,
                                              graph.src_sorted, graph.perm, e0, e1, dzbuf)
                dx_edge[e0:e1] = dxc
                dY[e0:e1] = dYc
            dpre = da * (pre > 0)
            r = rad_s[e0:e1]
            # dW1 = dpre^T r, db1 = colsum(dpre): one deterministic edge outer sum over E rows
            gw1, gb1 = ops.edge_outer_sum_rect(dpre, r)
            dW1.add_(gw1)
            db1.add_(gb1)
            drad_s[e0:e1] = dpre.mm(W1)
        dW2, db2 = torch.empty_like(W2), torch.empty_like(b2)
        for P, (gw, gb) in zip(plan.instructions, dW2x):
            m1, mo, off = P["mul1"], P["mul_out"], P["w_off"]
            dW2[off:off + m1 * mo] = gw.view(m1, H, mo).permute(0, 2, 1).reshape(m1 * mo, H)
            db2[off:off + m1 * mo] = gb.reshape(-1)
        dx, _ = ops.segment_reduce(dx_edge, graph.src_csr, "sum")
        dsh = torch.empty_like(sh).index_copy_(0, graph.perm, dY)
        drad = torch.empty((E, rad_s.shape[1]), **f).index_copy_(0, graph.perm, drad_s)
        return dx, dsh, drad, dW1, db1, dW2, db2, None, None, None, None


def _node_outer(eoff, Zp, a, w):
    with _timed("tp_node_S"):
        return _lib.torch_ops().tp_node_outer(eoff, Zp, a, w)


def _node_chunks(plan, graph, x, sh, rad_s, W1, b1, paths_dev, cg_dev):
    """Receiver chunks with their chunk-local edge offsets, hidden radial rows a and z rows
    (recomputed per pass).  One chunk (the 1M-edge configs) needs no host copy of rowptr."""
    if graph.num_edges == 0:
        return
    H = W1.shape[0]
    per_node = plan.max_block_rows * H * 4 * 2  # S (+ T) of the widest path
    npc = max(1, min(65535, node_chunk_bytes(x.device) // per_node))
    chunks = ([(0, graph.num_nodes, 0, graph.num_edges)] if npc >= graph.num_nodes
              else graph.node_chunks(npc))
    for n0, n1, e0, e1 in chunks:
        if e1 == e0:
            continue
        eoff = graph.rowptr[n0:n1 + 1] - e0
        with _timed("tp_node_prep"):
            pre = torch.addmm(b1, rad_s[e0:e1], W1.t())
            a = torch.relu(pre)
            zbuf = _lib.torch_ops().tp_edge_z(plan.desc_list, paths_dev, cg_dev, x, sh,
                                              graph.src_sorted, graph.perm, e0, e1)
        yield n0, n1, e0, e1, eoff, a, zbuf, pre


class TensorProductConvLayer(nn.Module):
    """tfn_layer.py:8-93 (same arguments; module tree fc.{0,2}, batch_norm, gate)."""

    def __init__(self, in_irreps, out_irreps, sh_irreps, edge_feats_dim, mlp_dim, aggr="add",
                 batch_norm=False, gate=False):
        super().__init__()
        self.in_irreps = o3.parse_irreps(in_irreps)
        self.out_irreps = o3.parse_irreps(out_irreps)
        self.sh_irreps = o3.parse_irreps(sh_irreps)
        self.edge_feats_dim = edge_feats_dim
        self.aggr = aggr
        if gate:
            s, g, v = o3.irreps2gate(self.out_irreps)
            self.gate = Gate(s, g, v)
            self.out_irreps = self.gate.irreps_in
        else:
            self.gate = None
        self.plan = TPPlan(self.in_irreps, self.sh_irreps, self.out_irreps)
        # the plan's constant tables as (non-persistent) buffers: they follow the module's
        # .to(device), and torch.compile sees them as module state
        paths, cg = self.plan.host_tables()
        self.register_buffer("_tp_paths", paths, persistent=False)
        self.register_buffer("_tp_cg", cg, persistent=False)
        self.fc = nn.Sequential(nn.Linear(edge_feats_dim, mlp_dim), nn.ReLU(),
                                nn.Linear(mlp_dim, self.plan.weight_numel))
        self.batch_norm = BatchNorm(self.out_irreps) if batch_norm else None

    def forward(self, node_attr, edge_index, edge_sh, edge_feat):
        if self.aggr in ("max", "min"):
            return self._forward_extremum(node_attr, edge_index, edge_sh, edge_feat)
        graph = tp_graph(edge_index, node_attr.shape[0])
        node = TP_MODE == "node" and node_form_ok(self.fc[0].out_features)
        fn = TPConvNodeFn if node else TPConvFn
        # (a plain bool: torch.compile cannot trace `is` between autograd Function classes)
        if not node and self.plan.layout is None:
            raise NotImplementedError("the per-edge-weight TP kernels take l <= 2 layouts only; "
                                      "use the node form (TP_MODE = \"node\", mlp_dim <= 256)")
        paths, cg = self._tp_paths, self._tp_cg
        if paths.device != node_attr.device or cg.dtype != torch.float32:
            paths, cg = self.plan.device_tables(node_attr.device)
        fcw = (_node_radial(self.fc) if node else
               (self.fc[0].weight, self.fc[0].bias, self.fc[2].weight, self.fc[2].bias))
        out = fn.apply(node_attr, edge_sh, edge_feat, *fcw, self.plan, graph, paths, cg)
        if self.aggr == "mean":
            out = out / graph.recv_csr.counts().clamp(min=1).unsqueeze(1).to(out.dtype)
        elif self.aggr not in ("add", "sum"):
            raise NotImplementedError(f"aggr={self.aggr}")
        return self._epilogue(out)

    def _epilogue(self, out):
        if self.gate is not None:
            out = self.gate(out)
        if self.batch_norm is not None:
            out = self.batch_norm(out)
        return out

    def _forward_extremum(self, node_attr, edge_index, edge_sh, edge_feat):
        """aggr = max / min (tfn_layer.py:87 passes aggr to torch_scatter's scatter): the per-edge
        messages through the node-form kernels on a graph where every edge is its own receiver
        (edge e -> receiver e, sender edge_index[1][e]), then the deterministic segmented max /
        min (K3) over edge_index[0] with torch_scatter's arg routing of the gradient.  The
        receiver sum of the node form is what makes it cheap; per-edge messages cost ~ the
        in-degree times more (not a benchmark path)."""
        if not node_form_ok(self.fc[0].out_features):
            raise NotImplementedError(f"aggr={self.aggr}: the node-form kernels need "
                                      "mlp_dim <= 256")
        E = edge_index.shape[1]
        ar = torch.arange(E, device=edge_index.device, dtype=edge_index.dtype)
        ei_e = torch.stack([ar, edge_index[1]])
        graph = tp_graph(ei_e, E, num_src=node_attr.shape[0])
        paths, cg = self._tp_paths, self._tp_cg
        if paths.device != node_attr.device or cg.dtype != torch.float32:
            paths, cg = self.plan.device_tables(node_attr.device)
        msg = TPConvNodeFn.apply(node_attr, edge_sh, edge_feat, *_node_radial(self.fc),
                                 self.plan, graph, paths, cg)
        out = scatter(msg, edge_index[0], dim=0, dim_size=node_attr.shape[0], reduce=self.aggr)
        return self._epilogue(out)


# ===================================================================================== MACE node
def reshape_irreps(irreps, x):
    """irreps_tools.py:63-79."""
    B, out, ix = x.shape[0], [], 0
    for mul, (l, _) in irreps:
        d = 2 * l + 1
        out.append(x[:, ix:ix + mul * d].reshape(B, mul, d))
        ix += mul * d
    return torch.cat(out, dim=-1)


class Contraction(nn.Module):
    """symmetric_contraction.py:88-188 (element_dependent=False): same buffers
    U_matrix_{nu} and weights.{nu} (K_nu, C).  Evaluated as a per-channel polynomial in x with
    coefficient tensors A_nu[c] = sum_k U_nu[..., k] W_nu[k, c] (identical algebra to the
    reference's einsum chain, no (N, C, d, 9, 9) HBM intermediates held for backward)."""

    node_chunk = 4096

    def __init__(self, irreps_in, irrep_out, correlation):
        super().__init__()
        irreps_in = o3.parse_irreps(irreps_in)
        self.irrep_out = tuple(irrep_out)
        self.num_features = sum(m for m, ir in irreps_in if ir == (0, 1))
        coupling = tuple((1, ir) for _, ir in irreps_in)
        self.correlation = correlation
        for nu in range(1, correlation + 1):
            U = torch.from_numpy(o3.u_matrix(coupling, irrep_out, nu).copy())
            self.register_buffer(f"U_matrix_{nu}", U.to(torch.get_default_dtype()))
        self.weights = nn.ParameterDict({
            str(nu): nn.Parameter(torch.randn(self.U(nu).shape[-1], self.num_features)
                                  / self.U(nu).shape[-1]) for nu in range(1, correlation + 1)})

    def U(self, nu):
        return self._buffers[f"U_matrix_{nu}"]

    def _chunk(self, x, *A):
        out = torch.einsum("c...i,bci->bc...", A[-1], x)
        for nu in range(self.correlation - 1, 0, -1):
            out = torch.einsum("bc...i,bci->bc...", A[nu - 1].unsqueeze(0) + out, x)
        return out.reshape(out.shape[0], -1)

    def forward(self, x):
        A = [torch.einsum("...k,kc->c...", self.U(nu), self.weights[str(nu)])
             for nu in range(1, self.correlation + 1)]
        outs = []
        for b0 in range(0, x.shape[0], self.node_chunk):
            xb = x[b0:b0 + self.node_chunk]
            if torch.is_grad_enabled():
                outs.append(torch.utils.checkpoint.checkpoint(self._chunk, xb, *A,
                                                              use_reentrant=False))
            else:
                outs.append(self._chunk(xb, *A))
        return torch.cat(outs, dim=0)


class SymmetricContractionFn(torch.autograd.Function):
    """K8 (torch.ops.gmp.symmetric_contraction_{fwd,bwd}): out (N, M C) from x (N, C, D) and the
    coefficients coef (T, C) of the module's sparse term plan (gmp_sc.hip)."""

    @staticmethod
    def forward(ctx, x, coef, plan, rows):
        x, coef = _f32c(x), _f32c(coef)
        _need_cuda(x, coef, plan)
        with _timed("symmetric_contraction_fwd"):
            out = _lib.torch_ops().symmetric_contraction_fwd(x, plan, rows, coef)
        ctx.rows = rows
        ctx.save_for_backward(x, coef, plan)
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        x, coef, plan = ctx.saved_tensors
        with _timed("symmetric_contraction_bwd"):
            dx, part = _lib.torch_ops().symmetric_contraction_bwd(x, plan, ctx.rows, coef,
                                                                  _f32c(g))
        dcoef = part.sum(0) if ctx.needs_input_grad[1] else None  # fixed-order group sum
        return (dx if ctx.needs_input_grad[0] else None, dcoef, None, None)


_SYM_IDX = {}


def _sym_index(nu, device, D=9):
    """(n_q, n_perm) flat indices into the D^nu axis of every distinct permutation of each
    sorted monomial (i <= j <= k, lexicographic), padded with D^nu (an appended zero column)."""
    key = (nu, D, device)
    if key not in _SYM_IDX:
        import itertools
        rows = []
        for t in itertools.combinations_with_replacement(range(D), nu):
            perms = sorted(set(itertools.permutations(t)))
            rows.append([sum(p * D ** (nu - 1 - r) for r, p in enumerate(pm)) for pm in perms])
        width = max(len(r) for r in rows)
        idx = torch.tensor([r + [D ** nu] * (width - len(r)) for r in rows], dtype=torch.int64)
        _SYM_IDX[key] = idx.to(device)
    return _SYM_IDX[key]


def fold_symmetric(A, nu):
    """A (..., D^nu) -> A~ (..., C(D - 1 + nu, nu)): every permutation's coefficient summed
    into the sorted monomial (differentiable; the adjoint spreads dA~ back to each permutation)."""
    if nu == 1:
        return A
    D = round(A.shape[-1] ** (1.0 / nu))
    idx = _sym_index(nu, A.device, D)
    Ap = torch.cat([A, A.new_zeros(A.shape[:-1] + (1,))], dim=-1)
    return Ap[..., idx].sum(-1)


_K8_MAX_DIM, _K8_MAX_ROWS, _K8_MAX_CORR = 63, 255, 4


def k8_plan(contractions, D, C, correlation):
    """The K8 term plan of a SymmetricContraction (gmp.h gmp_symmetric_contraction_fwd_f32):
    the (row m, monomial) pairs whose folded coefficient can be non-zero for some weights --
    the fold of some U_nu[m, ..., k] over the monomial's permutations is (structurally) non-zero
    -- in row order, monomials ascending within a row.  Returns (plan int32, gather int64): coef
    (T, C) = the rows `gather` of cat_nu(A~_nu) (C, M, NQ) flattened over (m, q) and transposed."""
    import itertools
    # the term word holds four 6-bit factor fields (gmp_sc.hip): degree <= 4
    assert 1 <= correlation <= _K8_MAX_CORR, "K8 term words hold at most 4 factors"
    masks, nq = [], []
    for nu in range(1, correlation + 1):
        rows = []
        for con in contractions:
            U = con.U(nu).double()
            if U.dim() == nu + 1:  # scalar output: the m axis was squeezed
                U = U.unsqueeze(0)
            K = U.shape[-1]
            F = fold_symmetric(U.reshape(U.shape[0], -1, K).permute(2, 0, 1), nu)  # (K, Mk, NQ)
            tol = 1e-6 * float(U.abs().max())
            rows.append((F.abs() > tol).any(0))
        masks.append(torch.cat(rows, 0))
        nq.append(masks[-1].shape[1])
    M = masks[0].shape[0]
    factors = [list(itertools.combinations_with_replacement(range(D), nu))
               for nu in range(1, correlation + 1)]
    row_ptr, terms, gather = [0], [], []
    nq_total, q_off = sum(nq), [sum(nq[:i]) for i in range(len(nq))]
    for m in range(M):
        for nu in range(1, correlation + 1):
            for q in torch.nonzero(masks[nu - 1][m]).view(-1).tolist():
                f = list(factors[nu - 1][q]) + [D] * (4 - nu)
                terms.append(f[0] | f[1] << 6 | f[2] << 12 | f[3] << 18 | m << 24)
                gather.append(m * nq_total + q_off[nu - 1] + q)
        row_ptr.append(len(terms))
    base, stride, m0 = [], [], 0
    for con in contractions:
        d = 2 * con.irrep_out[0] + 1
        for mm in range(d):
            base.append(C * m0 + mm)
            stride.append(d)
        m0 += d
    assert m0 == M
    words = torch.tensor(terms, dtype=torch.int64)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words)  # int32 bit patterns
    plan = torch.cat([torch.tensor(row_ptr + base + stride, dtype=torch.int64), words])
    return plan.to(torch.int32), torch.tensor(gather, dtype=torch.int64)


class SymmetricContraction(nn.Module):
    def __init__(self, irreps_in, irreps_out, correlation):
        super().__init__()
        self.irreps_out = o3.parse_irreps(irreps_out)
        self.correlation = correlation
        irreps_in = o3.parse_irreps(irreps_in)
        C = irreps_in[0][0]
        D = sum(2 * l + 1 for _, (l, _) in irreps_in)
        self.contractions = nn.ModuleDict({
            f"{m}x{l}{'e' if p == 1 else 'o'}": Contraction(irreps_in, (l, p), correlation)
            for m, (l, p) in self.irreps_out})
        o3.clear_cg_cache()
        M = sum(2 * l + 1 for _, (l, _) in self.irreps_out)
        # K8 takes any irreps with C channels each (x (N, C, D) is reshape_irreps' layout; the
        # reference's Contraction needs the same, symmetric_contraction.py:102), D <= 63, M <= 255,
        # correlation 1..4 (four factor fields per term word); higher correlations run the
        # per-irrep torch contraction
        self._k8 = (all(m == C for m, _ in irreps_in) and all(m == C for m, _ in self.irreps_out)
                    and D <= _K8_MAX_DIM and M <= _K8_MAX_ROWS
                    and 1 <= correlation <= _K8_MAX_CORR)
        if self._k8:
            plan, gather = k8_plan(list(self.contractions.values()), D, C, correlation)
            self.register_buffer("_k8_plan", plan, persistent=False)
            self.register_buffer("_k8_gather", gather, persistent=False)
            self._k8_rows = M

    def coefficients(self):
        """A_nu (C, M, D^nu): per-channel coefficient tensors, output rows in irreps_out order."""
        out = []
        for nu in range(1, self.correlation + 1):
            rows = []
            for con in self.contractions.values():
                U = con.U(nu)
                if U.dim() == nu + 1:  # scalar output: the m axis was squeezed
                    U = U.unsqueeze(0)
                A = torch.einsum("m...k,kc->cm...", U, con.weights[str(nu)])
                rows.append(A.reshape(A.shape[0], A.shape[1], -1))
            out.append(torch.cat(rows, dim=1))
        return out

    def k8_coefficients(self):
        """coef (T, C): the folded coefficients at the plan's terms, term-major
        (differentiable)."""
        A = torch.cat([fold_symmetric(a, nu + 1) for nu, a in enumerate(self.coefficients())],
                      dim=-1)
        return A.reshape(A.shape[0], -1).t().index_select(0, self._k8_gather)

    def forward(self, x, y=None):
        if self._k8 and x.is_cuda:
            return SymmetricContractionFn.apply(x, self.k8_coefficients(), self._k8_plan,
                                                self._k8_rows)
        return torch.cat([c(x) for c in self.contractions.values()], dim=-1)


class EquivariantProductBasisBlock(nn.Module):
    """blocks.py:99-135 (element_dependent=False, batch_norm=False)."""

    def __init__(self, node_feats_irreps, target_irreps, correlation, element_dependent=False,
                 use_sc=True, batch_norm=False, num_elements=None):
        super().__init__()
        self.use_sc = use_sc
        self.symmetric_contractions = SymmetricContraction(node_feats_irreps, target_irreps,
                                                           correlation)
        self.linear = Linear(target_irreps, target_irreps)
        self.batch_norm = BatchNorm(target_irreps) if batch_norm else None

    def forward(self, node_feats, sc, node_attrs=None):
        out = self.linear(self.symmetric_contractions(node_feats, node_attrs))
        if self.batch_norm is not None:
            out = self.batch_norm(out)
        return out + sc if self.use_sc else out


# ===================================================================================== models
def _edge_features(model, batch):
    graph = tp_graph(batch.edge_index, batch.pos.shape[0])
    return EdgeFeaturizeFn.apply(batch.pos, batch.edge_index, model.radial_embedding._host, graph,
                                 model.max_ell)


class MACEModel(nn.Module):
    """models/mace.py:9-190 (same kwargs/defaults; max_ell 1..5: K1 / K7 node form take l <= 5,
    K8 the 0e+1o[+2e[+3o]] hidden irreps, other hidden irreps the per-irrep contraction)."""

    def __init__(self, r_max=10.0, num_bessel=8, num_polynomial_cutoff=5, max_ell=2,
                 correlation=3, num_layers=5, emb_dim=64, hidden_irreps=None, mlp_dim=256,
                 in_dim=1, out_dim=1, aggr="sum", pool="sum", batch_norm=True, residual=True,
                 equivariant_pred=False):
        super().__init__()
        if max_ell not in (1, 2, 3, 4, 5):
            raise NotImplementedError("K1 / K7 take max_ell <= 5")
        self.r_max, self.max_ell, self.num_layers = r_max, max_ell, num_layers
        self.emb_dim, self.mlp_dim, self.residual = emb_dim, mlp_dim, residual
        self.batch_norm, self.equivariant_pred = batch_norm, equivariant_pred
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, num_polynomial_cutoff)
        sh = o3.sh_irreps(max_ell)
        self.emb_in = nn.Embedding(in_dim, emb_dim)
        hidden = o3.parse_irreps(hidden_irreps) if hidden_irreps else o3.hidden_irreps(emb_dim,
                                                                                       max_ell)
        self.hidden_irreps = hidden
        self.convs, self.prods = nn.ModuleList(), nn.ModuleList()
        for k in range(num_layers):
            inp = ((emb_dim, (0, 1)),) if k == 0 else hidden
            self.convs.append(TensorProductConvLayer(inp, hidden, sh,
                                                     self.radial_embedding.out_dim, mlp_dim, aggr,
                                                     batch_norm=batch_norm, gate=False))
            self.prods.append(EquivariantProductBasisBlock(hidden, hidden, correlation,
                                                           element_dependent=False,
                                                           use_sc=residual, num_elements=in_dim))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(o3.irreps_dim(hidden), out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(emb_dim, emb_dim), nn.ReLU(),
                                      nn.Linear(emb_dim, out_dim))

    def forward(self, batch):
        h = ops.gather(self.emb_in.weight, batch.atoms)
        edge_sh, edge_feats = _edge_features(self, batch)
        for conv, prod in zip(self.convs, self.prods):
            hu = conv(h, batch.edge_index, edge_sh, edge_feats)
            sc = F.pad(h, (0, hu.shape[-1] - h.shape[-1]))
            h = prod(reshape_irreps(self.hidden_irreps, hu), sc, None)
        out = self.pool(h, batch.batch, getattr(batch, "num_graphs", None))
        if not self.equivariant_pred:
            out = out[:, :self.emb_dim]
        return self.pred(out)


def first_node_pooling(x, batch, size=None):
    """tfn.py:13-40: first node of each graph (batch vector sorted)."""
    prev = torch.cat([batch[-1:], batch[:-1]])
    prev[0] = -1
    return x[(batch - prev) == 1]


class TFNModel(nn.Module):
    """models/tfn.py:42-190 (same kwargs/defaults; max_ell 1..5, l = 4, 5 on the runtime-l z / dz
    kernels: experiments/rotsym.ipynb's max_ell = 5 at one layer)."""

    def __init__(self, r_max=10.0, num_bessel=8, num_polynomial_cutoff=5, max_ell=2,
                 num_layers=5, emb_dim=64, hidden_irreps=None, mlp_dim=256, in_dim=1, out_dim=1,
                 aggr="sum", pool="first", gate=True, batch_norm=False, residual=True,
                 equivariant_pred=False):
        super().__init__()
        if max_ell not in (1, 2, 3, 4, 5):
            raise NotImplementedError("K1 / K7 take max_ell <= 5")
        self.max_ell = max_ell
        self.emb_dim, self.residual, self.equivariant_pred = emb_dim, residual, equivariant_pred
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, num_polynomial_cutoff)
        sh = o3.sh_irreps(max_ell)
        self.emb_in = nn.Embedding(in_dim, emb_dim)
        hidden = o3.parse_irreps(hidden_irreps) if hidden_irreps else o3.hidden_irreps(emb_dim,
                                                                                       max_ell)
        self.convs = nn.ModuleList()
        for k in range(num_layers):
            inp = ((emb_dim, (0, 1)),) if k == 0 else hidden
            self.convs.append(TensorProductConvLayer(inp, hidden, sh,
                                                     self.radial_embedding.out_dim, mlp_dim, aggr,
                                                     batch_norm=batch_norm, gate=gate))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool,
                     "first": first_node_pooling}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(o3.irreps_dim(hidden), out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(emb_dim, emb_dim), nn.ReLU(),
                                      nn.Linear(emb_dim, out_dim))

    def forward(self, batch):
        h = ops.gather(self.emb_in.weight, batch.atoms)
        edge_sh, edge_feats = _edge_features(self, batch)
        for conv in self.convs:
            hu = conv(h, batch.edge_index, edge_sh, edge_feats)
            h = hu + F.pad(h, (0, hu.shape[-1] - h.shape[-1])) if self.residual else hu
        if self.pool is first_node_pooling:
            out = first_node_pooling(h, batch.batch)
        else:
            out = self.pool(h, batch.batch, getattr(batch, "num_graphs", None))
        if not self.equivariant_pred:
            out = out[:, :self.emb_dim]
        return self.pred(out)
