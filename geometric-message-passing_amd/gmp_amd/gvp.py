"""GVP-GNN on the MI355X kernels — drop-in for models/layers/gvp_layer.py:101-438 (GVP,
LayerNorm, Dropout, GVPConv, GVPConvLayer) and models/gvpgnn.py:10-127 (GVPGNNModel), same
module trees / state_dict keys.

GVPConv.forward (gvp_layer.py:304-316) keeps the PyG propagate contract (j = edge_index[0],
i = edge_index[1], mean aggregation with dim_size = N) but evaluates the first message GVP's
scalar Linear on the concatenation [s_j, e_s, s_i, |vh|] as two node projections
(s W_a^T, s W_b^T, N-row GEMMs) gathered per edge plus the edge terms — 2·s_in·s_out MACs per
edge fewer than the reference — and its vector Linear W_h likewise on node-level vector rows.
The gathers are the HIP gather kernel, the aggregation the HIP segmented mean on the receiver
CSR (deterministic).  Subclasses with a custom message function or module_list fall back to the
generic propagate path (gather -> message -> segmented reduce).
"""
import functools

import torch
from torch.autograd.function import once_differentiable
from torch import nn
from torch.nn import functional as F

from . import _lib, ops
from .message_passing import MessagePassing
from .scatter import global_add_pool, global_mean_pool


def _norm_no_nan(x, axis=-1, keepdims=False, eps=1e-8, sqrt=True):
    """gvp_layer.py:66-73."""
    out = torch.clamp(torch.sum(torch.square(x), axis, keepdims), min=eps)
    return torch.sqrt(out) if sqrt else out


def _split(x, nv):
    return x[..., :-3 * nv], x[..., -3 * nv:].contiguous().view(x.shape[0], nv, 3)


def _merge(s, v):
    return torch.cat([s, v.contiguous().view(v.shape[0], v.shape[1] * 3)], -1)


def tuple_sum(*args):
    # (the reference's map(sum, ...) starts from 0: one extra full-size add per component)
    return tuple(functools.reduce(lambda a, b: a + b, xs) for xs in zip(*args))


def tuple_cat(*args, dim=-1):
    dim %= len(args[0][0].shape)
    s_args, v_args = list(zip(*args))
    return torch.cat(s_args, dim=dim), torch.cat(v_args, dim=dim)


def tuple_index(x, idx):
    return x[0][idx], x[1][idx]


class GVP(nn.Module):
    """gvp_layer.py:101-170."""

    def __init__(self, in_dims, out_dims, h_dim=None, activations=(F.relu, torch.sigmoid),
                 vector_gate=True):
        super().__init__()
        self.si, self.vi = in_dims
        self.so, self.vo = out_dims
        self.vector_gate = vector_gate
        if self.vi:
            self.h_dim = h_dim or max(self.vi, self.vo)
            self.wh = nn.Linear(self.vi, self.h_dim, bias=False)
            self.ws = nn.Linear(self.h_dim + self.si, self.so)
            if self.vo:
                self.wv = nn.Linear(self.h_dim, self.vo, bias=False)
                if self.vector_gate:
                    self.wsv = nn.Linear(self.so, self.vo)
        else:
            self.ws = nn.Linear(self.si, self.so)
        self.scalar_act, self.vector_act = activations
        self.dummy_param = nn.Parameter(torch.empty(0))

    def _tail(self, s, vh):
        """Everything after s' = W_s[...] given the pre-activation s' and vh (B, 3, h)."""
        v = None
        if self.vo:
            v = ops.linear(vh, self.wv.weight).transpose(-1, -2)
            if self.vector_gate:
                gate = ops.linear(self.vector_act(s) if self.vector_act else s,
                                  self.wsv.weight, self.wsv.bias)
                v = v * torch.sigmoid(gate).unsqueeze(-1)
            elif self.vector_act:
                v = v * self.vector_act(_norm_no_nan(v, axis=-1, keepdims=True))
        if self.scalar_act:
            s = self.scalar_act(s)
        return (s, v) if self.vo else s

    def forward(self, x):
        if self.vi:
            s, v = x
            vh = ops.linear(v.transpose(-1, -2), self.wh.weight)
            s = ops.linear(torch.cat([s, _xyz_norm(vh)], -1), self.ws.weight, self.ws.bias)
            return self._tail(s, vh)
        s = self.ws(x)
        v = torch.zeros(s.shape[0], self.vo, 3, device=s.device, dtype=s.dtype) if self.vo \
            else None
        if self.scalar_act:
            s = self.scalar_act(s)
        return (s, v) if self.vo else s


class _VDropout(nn.Module):
    def __init__(self, drop_rate):
        super().__init__()
        self.drop_rate = drop_rate
        self.dummy_param = nn.Parameter(torch.empty(0))

    def forward(self, x):
        if not self.training:
            return x
        mask = torch.bernoulli((1 - self.drop_rate) * torch.ones(x.shape[:-1], device=x.device))
        return mask.unsqueeze(-1) * x / (1 - self.drop_rate)


class Dropout(nn.Module):
    def __init__(self, drop_rate):
        super().__init__()
        self.sdropout = nn.Dropout(drop_rate)
        self.vdropout = _VDropout(drop_rate)

    def forward(self, x):
        if type(x) is torch.Tensor:
            return self.sdropout(x)
        s, v = x
        return self.sdropout(s), self.vdropout(v)


# False: the vector LayerNorm as the reference's torch chain (tests compare the two)
VEC_NORM_FUSED = True


class VecNormFn(torch.autograd.Function):
    """v / sqrt(mean_c clamp(|v_c|^2, 1e-8)) over (rows, C, 3): the vector half of the GVP
    LayerNorm (gvp_layer.py:232-243) in one HIP pass each way (gmp_vec_norm_{fwd,bwd}_f32) instead
    of the square / sum / clamp / mean / sqrt / divide chain and its autograd graph."""

    @staticmethod
    def forward(ctx, v):
        v = ops._f32c(v)
        ops._need_cuda(v)
        ctx.save_for_backward(v)
        return _lib.torch_ops().vec_norm_fwd(v)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (v,) = ctx.saved_tensors
        return _lib.torch_ops().vec_norm_bwd(v, ops._f32c(g))


class XyzNormFn(torch.autograd.Function):
    """_norm_no_nan(vh, axis=-2) of GVP.forward (gvp_layer.py:66-73, :101-170) for vh (rows, 3, h):
    one HIP pass each way (gmp_xyz_norm_{fwd,bwd}_f32) instead of square / sum / clamp / sqrt."""

    @staticmethod
    def forward(ctx, vh):
        vh = ops._f32c(vh)
        ops._need_cuda(vh)
        ctx.save_for_backward(vh)
        return _lib.torch_ops().xyz_norm_fwd(vh)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (vh,) = ctx.saved_tensors
        return _lib.torch_ops().xyz_norm_bwd(vh, ops._f32c(g))


def _xyz_norm(vh):
    if VEC_NORM_FUSED and vh.is_cuda and vh.dtype == torch.float32 and vh.dim() == 3 \
            and vh.shape[1] == 3:
        return XyzNormFn.apply(vh)
    return _norm_no_nan(vh, axis=-2)


class LayerNorm(nn.Module):
    """gvp_layer.py:221-243."""

    def __init__(self, dims):
        super().__init__()
        self.s, self.v = dims
        self.scalar_norm = nn.LayerNorm(self.s)

    def forward(self, x):
        if not self.v:
            return ops.ln_act(x, self.scalar_norm)  # K12 (act = identity)
        s, v = x
        if (VEC_NORM_FUSED and v.is_cuda and v.dtype == torch.float32 and v.dim() >= 2
                and v.shape[-1] == 3 and 1 <= v.shape[-2] <= 64):
            # (..., C, 3) inputs as (rows, C, 3) for the kernel (a batched input
            # used to reach the op's 3-D check and raise)
            vv = VecNormFn.apply(v.reshape(-1, v.shape[-2], 3)).view(v.shape)
            return ops.ln_act(s, self.scalar_norm), vv
        vn = _norm_no_nan(v, axis=-1, keepdims=True, sqrt=False)
        vn = torch.sqrt(torch.mean(vn, dim=-2, keepdim=True))
        return ops.ln_act(s, self.scalar_norm), v / vn


# ------------------------------------------------------------------------------------ K5g
# False: the reference-shaped per-edge chain (tests compare the two)
GVP_FUSED = True


def _diag3(M, a, b):
    """sum_x M[3o + x, 3c + x] for M (3a, 3b) -> (a, b): weight gradient of a per-xyz Linear
    from the outer sum of (channel, xyz)-flattened rows."""
    return M.reshape(a, 3, b, 3).diagonal(dim1=1, dim2=3).sum(-1)


def _osum(A, B):
    return ops.edge_outer_sum_rect(A, B)


class GvpLayerFn(torch.autograd.Function):
    """One GVP (128, 16) -> (128, 16) over edge rows (gmp_gvp_layer_{fwd,bwd}_f32)."""

    @staticmethod
    def forward(ctx, s, v, Ws, bs, Wsv, bsv, Wh, Wv, relu):
        s, v = ops._f32c(s), ops._f32c(v)
        ops._need_cuda(s, v)
        W = [ops._f32c(t) for t in (Ws, bs, Wsv, bsv, Wh, Wv)]
        with ops._timed("gvp_layer_fwd"):
            s_out, v_out = _lib.torch_ops().gvp_layer_fwd(s, v, W, bool(relu))
        ctx.relu = relu
        ctx.save_for_backward(s, v, *W)
        return s_out, v_out

    @staticmethod
    @once_differentiable
    def backward(ctx, ds, dv):
        s, v, *W = ctx.saved_tensors
        ds = ops._f32c(ds) if ds is not None else torch.zeros_like(s)
        dv = ops._f32c(dv) if dv is not None else torch.zeros_like(v)
        with ops._timed("gvp_layer_bwd"):
            ds_in, dv_in, dspre, _, dgate, vn, vh, dvpre, dvh = _lib.torch_ops().gvp_layer_bwd(
                s, v, W, ds, dv, bool(ctx.relu), False)
        return (ds_in, dv_in) + _layer_wgrads(ctx.needs_input_grad, 2, s, v, W, dspre, dgate, vn,
                                              vh, dvpre, dvh) + (None,)


def _layer_wgrads(needs_input_grad, first, s, v, W, dspre, dgate, vn, vh, dvpre, dvh):
    """Weight gradients of one GVP layer (edge outer sums) on the side stream, deferred to the
    end of the backward pass; needs_input_grad[first + i] belongs to W[i]."""
    E = s.shape[0]
    f = dict(dtype=torch.float32, device=s.device)
    with ops.side_work(dspre, s, vn, dgate, dvh, v, dvpre) as sw:
        # dWs = dspre^T [s | vn]: one pass over dspre where the split-plane kernel applies
        dWs, dbs = torch.empty((128, 144), **f), torch.empty(128, **f)
        ops.outer_sum_into2(dspre, s.view(E, 128), vn, dWs, dbs)
        # dWsv = sum_e dgate (x) spre with spre = Ws [s | vn] + bs, without the (E, 128) spre
        # rows: (sum_e dgate (x) [s | vn]) Ws^T + (sum_e dgate) (x) bs
        Gx, dbsv = torch.empty((16, 144), **f), torch.empty(16, **f)
        ops.outer_sum_into2(dgate, s.view(E, 128), vn, Gx, dbsv)
        dWsv = torch.addmm(torch.outer(dbsv, W[1]), Gx, W[0].t())
        dWh = _diag3(_osum(dvh, v.reshape(E, 48))[0], 16, 16)
        # dWv = sum_(e,x) dvpre[e, o, x] vh[e, h, x] with vh = Wh v: (sum dvpre (x) v) Wh^T, so
        # the kernel does not write the (E, 48) vh rows (gmp.h gmp_gvp_layer_bwd_f32).  (r05: the
        # two products as one x3 pass v^T [dvh | dvpre] measured 331 us against 2 x ~130 us)
        dWv = _diag3(_osum(dvpre, v.reshape(E, 48))[0], 16, 16).mm(W[4].t())
    grads = (dWs, dbs, dWsv, dbsv, dWh, dWv)
    return sw.deliver(needs_input_grad, first, W, grads)


class GvpLayerAggFn(torch.autograd.Function):
    """The last message GVP (no scalar activation) followed by the receivers' sum / mean
    aggregation (GVPConv.forward, gvp_layer.py:319-324), neither direction materialising the
    (E, 176) per-edge rows: forward = gmp_gvp_layer_fwd_agg_f32 (the layer over the
    receiver-sorted edges with an in-wave segmented sum per receiver), backward =
    gmp_gvp_layer_bwd_agg_f32 (the aggregation's node gradient gathered per edge in the layer
    kernel's loads)."""

    @staticmethod
    def forward(ctx, s, v, Ws, bs, Wsv, bsv, Wh, Wv, csr, reduce):
        s, v = ops._f32c(s), ops._f32c(v)
        ops._need_cuda(s, v)
        W = [ops._f32c(t) for t in (Ws, bs, Wsv, bsv, Wh, Wv)]
        with ops._timed("gvp_layer_fwd"):
            agg_s, agg_v = _lib.torch_ops().gvp_layer_fwd_agg(s, v, W, csr.perm, csr.sorted,
                                                               csr.rowptr, csr.n_seg, reduce)
        ctx.csr, ctx.reduce = csr, reduce
        ctx.save_for_backward(s, v, *W)
        return agg_s, agg_v

    @staticmethod
    @once_differentiable
    def backward(ctx, gs, gv):
        s, v, *W = ctx.saved_tensors
        csr = ctx.csr
        n = csr.n_seg
        gs = ops._f32c(gs) if gs is not None else torch.zeros((n, 128), device=s.device)
        gv = ops._f32c(gv) if gv is not None else torch.zeros((n, 16, 3), device=s.device)
        with ops._timed("gvp_layer_bwd"):
            ds_in, dv_in, dspre, _, dgate, vn, vh, dvpre, dvh = \
                _lib.torch_ops().gvp_layer_bwd_agg(s, v, W, gs, gv, csr.index, csr.rowptr,
                                                   ctx.reduce, False, False)
        return (ds_in, dv_in) + _layer_wgrads(ctx.needs_input_grad, 2, s, v, W, dspre, dgate, vn,
                                              vh, dvpre, dvh) + (None, None)


class GvpMsg0Fn(torch.autograd.Function):
    """First message GVP (gmp_gvp_msg0_{fwd,bwd}_f32) from node projections P, Q.  Takes the
    leaf parameters (Ws0 = ws.weight, bias, Wv = wv.weight, wsv.*, Wh0 = wh.weight) and slices /
    pads the per-edge blocks itself, so their weight gradients are leaf gradients: computed on
    the side stream and accumulated at the end of the backward pass (ops.side_work)."""

    @staticmethod
    def forward(ctx, P, Q, es, ev, Ws0, b, Wv, Wsv, bsv, Wh0, send_csr, recv_csr, ei):
        P, Q, es, ev = (ops._f32c(t) for t in (P, Q, es, ev))
        pad = torch.nn.functional.pad
        vi = Wv.shape[1]  # 2 vi + ve = 33
        W = [ops._f32c(t) for t in (Ws0[:, 128:160], pad(Ws0[:, 288:288 + vi], (0, 48 - vi)),
                                    b, pad(Wv, (0, 48 - vi)), Wsv, bsv,
                                    pad(Wh0[:, 16], (0, 48 - Wh0.shape[0])))]
        send, recv = ei[0].contiguous(), ei[1].contiguous()
        with ops._timed("gvp_msg0_fwd"):
            s_out, v_out = _lib.torch_ops().gvp_msg0_fwd(send, recv, P, Q, es, ev, W)
        ctx.csrs = (send_csr, recv_csr)
        ctx.leaves = (Ws0, b, Wv, Wsv, bsv, Wh0)
        ctx.save_for_backward(P, Q, es, ev, send, recv, *W)
        return s_out, v_out

    @staticmethod
    @once_differentiable
    def backward(ctx, ds, dv):
        P, Q, es, ev, send, recv, *W = ctx.saved_tensors
        send_csr, recv_csr = ctx.csrs
        Ws0, b, Wv, Wsv, bsv, Wh0 = ctx.leaves
        E = es.shape[0]
        ds = ops._f32c(ds) if ds is not None else torch.zeros((E, 128), device=P.device)
        dv = ops._f32c(dv) if dv is not None else torch.zeros((E, 16, 3), device=P.device)
        f = dict(dtype=torch.float32, device=P.device)
        n = P.shape[0]
        with ops._timed("gvp_msg0_bwd"):
            # receiver-sorted walk; the receiver-side sums (dPb, dQb and the weight sums' S_i
            # dgate, S_i dvpre) come out of the kernel's segmented scan
            (dspre, _, dgate, vn, _, dvpre, dvh, des, dev, dPb, dQb, sg_i,
             sv_i) = _lib.torch_ops().gvp_msg0_bwd_agg(send, recv, P, Q, es, ev, W, ds, dv,
                                                       recv_csr.perm, recv_csr.rowptr, n, False)
        # weight gradients (edge outer sums) on the side stream, as full-size leaf gradients.
        # The pre-activation rows spre and the mixed vectors vh are not written by the kernel
        # (gmp.h gmp_gvp_msg0_bwd_f32): both are sums of per-edge terms and the gathered node
        # projections, so their sums split into edge sums and node-level products of the
        # sender / receiver segment sums of dgate / dvpre.
        with ops.side_work(dspre, es, vn, dgate, dvpre, ev, dvh, P, Q, sg_i, sv_i) as sw:
            vi = Wv.shape[1]
            # [dWe | dWn] = dspre^T [es | vn]: one pass over dspre when the split path applies
            Cen, db = torch.empty((128, 80), **f), torch.empty(128, **f)
            ops.outer_sum_into2(dspre, es, vn, Cen, db)
            dWe, dWn = Cen[:, :32], Cen[:, 32:]
            # dWsv = dgate^T spre, spre = [es | vn] [We | Wn]^T + Pa[j] + Pb[i] + b
            Gx, dbsv = torch.empty((16, 80), **f), torch.empty(16, **f)
            ops.outer_sum_into2(dgate, es, vn, Gx, dbsv)
            Sg = torch.cat([ops.segment_reduce(dgate, send_csr, "sum")[0], sg_i], 0)  # (2N, 16)
            Pab = P.view(n, 2, 128).transpose(0, 1).reshape(2 * n, 128)      # [Pa ; Pb]
            dWsv = _osum(Sg, Pab)[0].addmm_(Gx[:, :32], W[0].t()).addmm_(Gx[:, 32:], W[1].t())
            dWsv.add_(torch.outer(dbsv, W[2]))
            # dWv = sum_(e,x) dvpre[e, o, x] vh[e, h, x], vh = Qa[j] + Qb[i] + wev (x) ev
            Sv = torch.cat([ops.segment_reduce(dvpre, send_csr, "sum")[0], sv_i], 0)  # (2N, 48)
            Qab = Q.view(n, 2, 144).transpose(0, 1).reshape(2 * n, 144)      # [Qa ; Qb]
            dWv = _diag3(_osum(Sv, Qab)[0], 16, 48)
            # u[o] = sum_(e,x) dvpre[e, o, x] ev[e, x], dwev[h] = sum_(e,x) dvh[e, h, x] ev[e, x]:
            # one pass over each (gmp_edge_xyz_dot_f32)
            xdot = _lib.torch_ops().edge_xyz_dot
            u = xdot(dvpre, ev)                                              # (16,)
            dWv.add_(torch.outer(u, W[6]))
            dwev = xdot(dvh, ev)                                             # (48,)
            gWs0 = torch.zeros_like(Ws0)
            gWs0[:, 128:160] = dWe
            gWs0[:, 288:288 + vi] = dWn[:, :vi]
            gWh0 = torch.zeros_like(Wh0)
            gWh0[:, 16] = dwev[:Wh0.shape[0]]
            grads = (gWs0, db, dWv[:, :vi].contiguous(), dWsv, dbsv, gWh0)
        # node-projection gradients: deterministic segmented sums at the senders (the receivers'
        # came out of the kernel)
        dPa, _ = ops.segment_reduce(dspre, send_csr, "sum")
        dQa, _ = ops.segment_reduce(dvh, send_csr, "sum")
        return ((torch.cat([dPa, dPb], 1), torch.cat([dQa, dQb], 1).view(-1, 288), des, dev)
                + sw.deliver(ctx.needs_input_grad, 4, ctx.leaves, grads) + (None, None, None))


# False: the edge embedding W_e as the module chain (tests compare the two)
EDGE_EMBED_FUSED = True


class GvpEdgeEmbedFn(torch.autograd.Function):
    """K1e: the edge embedding W_e = LayerNorm((R, 1)) + GVP((R, 1), (so, 1)) (gvpgnn.py:73-77,
    applied at :116) over the edge rows in one HIP pass each way (gmp_gvp_edge_embed_{fwd,bwd}_f32):
    the module chain's 1M-row library GEMMs with K or N = 1 and its elementwise passes (~0.6 ms
    forward, ~1.5 ms of the backward's tail per C3 step) become two kernels.  The backward
    returns only the parameters' gradients (radial / unit come from positions without
    requires_grad; the caller checks)."""

    @staticmethod
    def forward(ctx, radial, unit, eps, ln_w, ln_b, wh, ws, bs, wv, wsv, bsv):
        radial, unit = ops._f32c(radial), ops._f32c(unit)
        ops._need_cuda(radial, unit)
        W = [ops._f32c(t) for t in (ln_w, ln_b, wh, ws, bs, wv, wsv, bsv)]
        es, ev = _lib.torch_ops().gvp_edge_embed_fwd(radial, unit, W, float(eps))
        ctx.eps = float(eps)
        ctx.shapes = [t.shape for t in (ln_w, ln_b, wh, ws, bs, wv, wsv, bsv)]
        ctx.save_for_backward(radial, unit, *W)
        return es, ev

    @staticmethod
    @once_differentiable
    def backward(ctx, des, dev):
        radial, unit, *W = ctx.saved_tensors
        E, so = radial.shape[0], W[3].shape[0]
        des = ops._f32c(des) if des is not None else radial.new_zeros((E, so))
        dev = ops._f32c(dev) if dev is not None else radial.new_zeros((E, 1, 3))
        g = _lib.torch_ops().gvp_edge_embed_bwd(radial, unit, W, ctx.eps, des, dev)
        grads, o = [], 0
        for shp in ctx.shapes:
            n = int(torch.Size(shp).numel())
            grads.append(g[o:o + n].view(shp))
            o += n
        return (None, None, None) + tuple(grads)


def _edge_embed_ok(W_e, rad, unit):
    if not (EDGE_EMBED_FUSED and len(W_e) == 2 and rad.is_cuda and rad.dtype == torch.float32
            and unit.dtype == torch.float32 and rad.dim() == 2 and rad.shape[1] == 8):
        return False
    ln, g = W_e
    if torch.is_grad_enabled() and (rad.requires_grad or unit.requires_grad):
        return False  # the fused backward gives the edge rows no gradient
    return (type(ln) is LayerNorm and type(g) is GVP and (ln.s, ln.v) == (8, 1)
            and ln.scalar_norm.elementwise_affine and ln.scalar_norm.bias is not None
            and (g.si, g.vi, g.vo) == (8, 1, 1) and 1 <= g.so <= 32 and g.h_dim == 1
            and g.vector_gate and g.scalar_act is None and g.vector_act is None)


def edge_embed(W_e, rad, unit):
    """W_e((rad, unit[:, None])) -> (es (E, so), ev (E, 1, 3)): K1e when the module is the
    reference's shape, else the module chain."""
    if _edge_embed_ok(W_e, rad, unit):
        ln, g = W_e
        return GvpEdgeEmbedFn.apply(rad, unit, ln.scalar_norm.eps, ln.scalar_norm.weight,
                                    ln.scalar_norm.bias, g.wh.weight, g.ws.weight, g.ws.bias,
                                    g.wv.weight, g.wsv.weight, g.wsv.bias)
    return W_e((rad, unit.unsqueeze(-2)))


class NodeProjFn(torch.autograd.Function):
    """P = s [Ws0[:, :si] ; Ws0[:, si + se : 2 si + se]]^T (N, 2 so): the sender / receiver
    scalar blocks of the first message GVP's Linear applied once per node.  dWs0 (a K = N
    reduction) on the side stream by the outer-sum kernel, deferred like the edge weights."""

    @staticmethod
    def forward(ctx, s, Ws0, si, se):
        Wcat = torch.cat([Ws0[:, :si], Ws0[:, si + se:2 * si + se]], 0)
        ctx.save_for_backward(s, Wcat)
        ctx.Ws0, ctx.si, ctx.se = Ws0, si, se
        return s.matmul(Wcat.t())

    @staticmethod
    @once_differentiable
    def backward(ctx, dP):
        s, Wcat = ctx.saved_tensors
        Ws0, si, se = ctx.Ws0, ctx.si, ctx.se
        dP = dP.contiguous()
        ds = ops._mm_wt(dP, Wcat.t().contiguous()) if ctx.needs_input_grad[0] else None
        if not ctx.needs_input_grad[1]:
            return ds, None, None, None
        so = Ws0.shape[0]
        with ops.side_work(dP, s) as sw:
            dWcat, _ = _osum(dP, s)
            g = torch.zeros_like(Ws0)
            g[:, :si] = dWcat[:so]
            g[:, si + se:2 * si + se] = dWcat[so:]
        return (ds,) + sw.deliver(ctx.needs_input_grad, 1, (Ws0,), (g,)) + (None, None)


class NodeVecProjFn(torch.autograd.Function):
    """Q (N, 288) = the sender / receiver vector blocks of the first message GVP's wh applied once
    per node: Q[n, (48 b + o) * 3 + x] = sum_c Wh0[o, 16 b + b + c] v[n, c, x] (b = 0: columns
    0..15, b = 1: 17..32; rows o >= 33 zero padding).  One GEMM over the 3N (node, xyz) rows;
    dWh0 (a K = 3N reduction) on the side stream by the outer-sum kernel, deferred."""

    @staticmethod
    def forward(ctx, v, Wh0, vi):
        n, ho = v.shape[0], Wh0.shape[0]
        Wst = v.new_zeros((96, vi))
        Wst[:ho] = Wh0[:, :vi]
        Wst[48:48 + ho] = Wh0[:, vi + 1:2 * vi + 1]
        vt = v.transpose(1, 2).reshape(3 * n, vi).contiguous()
        Y = vt.mm(Wst.t())                                   # (3N, 96): rows (n, x)
        ctx.save_for_backward(vt, Wst)
        ctx.Wh0, ctx.vi, ctx.n = Wh0, vi, n
        return Y.view(n, 3, 96).transpose(1, 2).reshape(n, 288)

    @staticmethod
    @once_differentiable
    def backward(ctx, dQ):
        vt, Wst = ctx.saved_tensors
        Wh0, vi, n = ctx.Wh0, ctx.vi, ctx.n
        dY = dQ.reshape(n, 96, 3).transpose(1, 2).reshape(3 * n, 96).contiguous()
        dv = None
        if ctx.needs_input_grad[0]:
            dv = ops._mm_wt(dY, Wst.t().contiguous()).view(n, 3, vi).transpose(1, 2)
        if not ctx.needs_input_grad[1]:
            return dv, None, None
        ho = Wh0.shape[0]
        with ops.side_work(dY, vt) as sw:
            dW, _ = _osum(dY, vt)                            # (96, vi)
            g = torch.zeros_like(Wh0)
            g[:, :vi] = dW[:ho]
            g[:, vi + 1:2 * vi + 1] = dW[48:48 + ho]
        return (dv,) + sw.deliver(ctx.needs_input_grad, 1, (Wh0,), (g,)) + (None,)


class GVPConv(MessagePassing):
    """gvp_layer.py:246-324."""

    def __init__(self, in_dims, out_dims, edge_dims, n_layers=3, module_list=None, aggr="mean",
                 activations=(F.relu, torch.sigmoid), vector_gate=True):
        super().__init__(aggr=aggr)
        self.si, self.vi = in_dims
        self.so, self.vo = out_dims
        self.se, self.ve = edge_dims
        G = functools.partial(GVP, activations=activations, vector_gate=vector_gate)
        self._custom = bool(module_list)
        module_list = module_list or []
        if not module_list:
            if n_layers == 1:
                module_list.append(G((2 * self.si + self.se, 2 * self.vi + self.ve),
                                     (self.so, self.vo), activations=(None, None)))
            else:
                module_list.append(G((2 * self.si + self.se, 2 * self.vi + self.ve), out_dims))
                for _ in range(n_layers - 2):
                    module_list.append(G(out_dims, out_dims))
                module_list.append(G(out_dims, out_dims, activations=(None, None)))
        self.message_func = nn.Sequential(*module_list)

    # --------------------------------------------------------------------------- reference hooks
    def message(self, s_i, v_i, s_j, v_j, edge_attr):
        v_j = v_j.view(v_j.shape[0], v_j.shape[1] // 3, 3)
        v_i = v_i.view(v_i.shape[0], v_i.shape[1] // 3, 3)
        message = tuple_cat((s_j, v_j), edge_attr, (s_i, v_i))
        return _merge(*self.message_func(message))

    def _fast_ok(self, x):
        g0 = self.message_func[0]
        return (not self._custom and self.vi > 0 and g0.vi == 2 * self.vi + self.ve
                and self.aggr in ("mean", "add", "sum") and x[0].is_cuda)

    def _fused_ok(self, x, edge_attr):
        mf = self.message_func
        return (GVP_FUSED and len(mf) == 3 and (self.si, self.vi) == (128, 16) and
                (self.so, self.vo) == (128, 16) and (self.se, self.ve) == (32, 1) and
                all(m.vector_gate and m.vector_act is None for m in mf) and
                mf[0].scalar_act is F.relu and mf[1].scalar_act is F.relu and
                mf[2].scalar_act is None and mf[0].h_dim == 33 and
                edge_attr[0].dtype == torch.float32)

    def _fused_forward(self, s, v, edge_index, edge_attr):
        """K5g path: message GVPs 1-3 as fused HIP kernels, mean at the receivers (K3)."""
        n = s.shape[0]
        g0, g1, g2 = self.message_func
        Ws0, Wh0 = g0.ws.weight, g0.wh.weight
        P = NodeProjFn.apply(s, Ws0, 128, 32)                                 # (N, 256)
        Q = NodeVecProjFn.apply(v, Wh0, 16)                                  # (N, 288)
        es, ev = edge_attr
        ei = edge_index
        # range-checked once per graph (one host sync, as index_select / torch_scatter raise):
        # the receiver-sorted kernels visit only in-range edges, so an out-of-range index would
        # leave rows of the per-edge outputs unwritten
        send_csr, recv_csr = ops.checked_csr(ei[0], n), ops.checked_csr(ei[1], n)
        s1, v1 = GvpMsg0Fn.apply(P, Q, es, ev.reshape(-1, 3), Ws0, g0.ws.bias, g0.wv.weight,
                                 g0.wsv.weight, g0.wsv.bias, Wh0, send_csr, recv_csr, ei)
        s2, v2 = GvpLayerFn.apply(s1, v1, g1.ws.weight, g1.ws.bias, g1.wsv.weight, g1.wsv.bias,
                                  g1.wh.weight, g1.wv.weight, True)
        # the last GVP with the receivers' aggregation: scalar and vector channels aggregated
        # separately (no concatenated (E, 176) copy), and its backward gathers the node gradient
        # in the layer kernel's loads (no (E, 176) per-edge gradient rows)
        reduce = "sum" if self.aggr == "add" else self.aggr
        return GvpLayerAggFn.apply(s2, v2, g2.ws.weight, g2.ws.bias, g2.wsv.weight, g2.wsv.bias,
                                   g2.wh.weight, g2.wv.weight, recv_csr, reduce)

    def forward(self, x, edge_index, edge_attr):
        x_s, x_v = x
        if self._fast_ok(x) and self._fused_ok(x, edge_attr):
            return self._fused_forward(x_s, x_v, edge_index, edge_attr)
        if not self._fast_ok(x):
            msg = self.propagate(edge_index, s=x_s,
                                 v=x_v.contiguous().view(x_v.shape[0], x_v.shape[1] * 3),
                                 edge_attr=edge_attr)
            return _split(msg, self.vo)
        return self._fast_forward(x_s, x_v, edge_index, edge_attr)

    def _fast_forward(self, s, v, edge_index, edge_attr):
        n = s.shape[0]
        j, i = edge_index[0], edge_index[1]
        g0 = self.message_func[0]
        si, se = self.si, self.se
        Ws = g0.ws.weight                          # (so, [s_j | e_s | s_i | vn])
        # node projections: [s W_a^T | s W_b^T]  -> gathered per edge
        P = s.matmul(torch.cat([Ws[:, :si], Ws[:, si + se:2 * si + se]], 0).t())
        Pj = ops.gather(P[:, :g0.so].contiguous(), j, 0)
        Pi = ops.gather(P[:, g0.so:].contiguous(), i, 0)
        # vector channels [v_j | e_v | v_i] mixed by W_h: node-level rows (N, 3, h) gathered
        Wh = g0.wh.weight                          # (h, 2 vi + ve)
        vi, ve = self.vi, self.ve
        vt = v.transpose(-1, -2)                   # (N, 3, vi)
        Q = torch.cat([vt.matmul(Wh[:, :vi].t()), vt.matmul(Wh[:, vi + ve:].t())], -1)
        Q = Q.reshape(n, -1)                       # (N, 3 * 2h)
        h = g0.h_dim
        Qj = ops.gather(Q.view(n, 3, 2 * h)[:, :, :h].reshape(n, 3 * h), j, 0).view(-1, 3, h)
        Qi = ops.gather(Q.view(n, 3, 2 * h)[:, :, h:].reshape(n, 3 * h), i, 0).view(-1, 3, h)
        es, ev = edge_attr
        evt = ev.transpose(-1, -2)                 # (E, 3, ve)
        vh = Qj + Qi + ops.linear(evt, Wh[:, vi:vi + ve])
        vn = _xyz_norm(vh)
        # edge part of W_s on [e_s | |vh|] as one per-edge Linear (dW by the edge outer sum)
        We = torch.cat([Ws[:, si:si + se], Ws[:, 2 * si + se:]], 1)
        s1 = ops.linear(torch.cat([es, vn], -1), We, g0.ws.bias) + Pj + Pi
        out = g0._tail(s1, vh)
        for mod in list(self.message_func)[1:]:
            out = mod(out)
        msg = _merge(*out) if isinstance(out, tuple) else out
        reduce = "sum" if self.aggr == "add" else self.aggr
        agg = ops.SegmentReduceFn.apply(msg, ops.get_csr(i, n), reduce)
        return _split(agg, self.vo)


# False: the node feed-forward as the reference's module chain (tests compare the two)
GVP_FF_FUSED = True


def _ff_fusable(ff, x):
    """K17 takes GVPConvLayer's default feed-forward at the GVP-GNN widths (gvp_layer.py:361-366
    with node_dims (128, 16), n_feedforward 2, vector_gate, activations (relu, None))."""
    if not (GVP_FF_FUSED and len(ff) == 2):
        return False
    g1, g2 = ff
    s, v = x
    return ((g1.si, g1.vi, g1.so, g1.vo, g2.si, g2.vi, g2.so, g2.vo) ==
            (128, 16, 512, 32, 512, 32, 128, 16) and g1.h_dim == 32 and g2.h_dim == 32 and
            g1.vector_gate and g2.vector_gate and g1.vector_act is None and
            g2.vector_act is None and g1.scalar_act is F.relu and g2.scalar_act is None and
            s.is_cuda and s.dtype == torch.float32 and v.dtype == torch.float32 and
            s.dim() == 2 and v.dim() == 3 and v.shape[1:] == (16, 3) and
            all(w.data_ptr() % 16 == 0 for w in (g1.ws.weight, g1.wsv.weight, g2.ws.weight)))


class GvpFFFn(torch.autograd.Function):
    """K17 (gmp_gvp_ff_{fwd,bwd}_f32): GVPConvLayer's node feed-forward GVP((128, 16), (512, 32))
    -> GVP((512, 32), (128, 16)) (gvp_layer.py:361-366, :433-434; GVP.forward :140-170) as one
    kernel per direction; the weight gradients are four node outer sums of operands the kernels
    write side by side (gmp.h), on the side stream and deferred to the end of the backward."""

    @staticmethod
    def forward(ctx, s, v, *W):
        s, v = ops._f32c(s), ops._f32c(v)
        ops._need_cuda(s, v)
        Wc = [ops._f32c(w) for w in W]
        with ops._timed("gvp_ff_fwd"):
            s2, v2, gate1, B1, B2, B3, B4 = _lib.torch_ops().gvp_ff_fwd(s, v, Wc)
        ctx.save_for_backward(v, gate1, B1, B2, B3, B4, s2, *Wc)
        return s2, v2

    @staticmethod
    @once_differentiable
    def backward(ctx, ds, dv):
        v, gate1, B1, B2, B3, B4, s2, *W = ctx.saved_tensors
        ds = ops._f32c(ds) if ds is not None else torch.zeros_like(s2)
        dv = ops._f32c(dv) if dv is not None else torch.zeros_like(v)
        with ops._timed("gvp_ff_bwd"):
            ds_in, dv_in, A1, A2, A3, A4 = _lib.torch_ops().gvp_ff_bwd(v, W, gate1, B2, s2, ds, dv)
        return (ds_in, dv_in) + _ff_wgrads(ctx.needs_input_grad, W, (A1, A2, A3, A4),
                                           (B1, B2, B3, B4))


def _ff_wgrads(needs_input_grad, W, As, Bs):
    """K17's weight gradients: C_k = A_k^T B_k (one node outer sum each, the quadrant kernel) and
    their blocks (gmp.h gmp_gvp_ff_bwd_f32), on the side stream, deferred."""
    Wh1, Ws1, b1, _, _, _, Wh2, Ws2, b2, _, _, _ = W
    f = dict(dtype=torch.float32, device=Ws1.device)
    with ops.side_work(*As, *Bs) as sw:
        C, cs = [], []
        for A, B in zip(As, Bs):
            c, k = torch.empty((A.shape[1], B.shape[1]), **f), torch.empty(A.shape[1], **f)
            ops.outer_sum_into(A, B, c, k)
            C.append(c)
            cs.append(k)
        dWs1, db1, dbsv1 = C[0][:512, :160], cs[0][:512], cs[0][512:544]
        dWsv1 = torch.addmm(torch.outer(dbsv1, b1), C[0][512:544, :160], Ws1.t())
        dWs2, db2, dbsv2 = C[1][:128, :544], cs[1][:128], cs[1][128:144]
        dWsv2 = torch.addmm(torch.outer(dbsv2, b2), C[1][128:144, :544], Ws2.t())
        dWh1 = _diag3(C[2][:96, :48], 32, 16)
        dWv1 = _diag3(C[2][96:, :48], 32, 16).mm(Wh1.t())
        dWh2 = _diag3(C[3][:96, :96], 32, 32)
        dWv2 = _diag3(C[3][96:144, :96], 16, 32).mm(Wh2.t())
        grads = [dWh1, dWs1, db1, dWv1, dWsv1, dbsv1, dWh2, dWs2, db2, dWv2, dWsv2, dbsv2]
        grads = [g.contiguous() for g in grads]
    return sw.deliver(needs_input_grad, 2, W, tuple(grads))


def gvp_ff(ff, x):
    """ff_func(x) (gvp_layer.py:433) on K17 where it applies, else the module chain."""
    if _ff_fusable(ff, x):
        g1, g2 = ff
        return GvpFFFn.apply(x[0], x[1], g1.wh.weight, g1.ws.weight, g1.ws.bias, g1.wv.weight,
                             g1.wsv.weight, g1.wsv.bias, g2.wh.weight, g2.ws.weight,
                             g2.ws.bias, g2.wv.weight, g2.wsv.weight, g2.wsv.bias)
    return ff(x)


class GVPConvLayer(nn.Module):
    """gvp_layer.py:327-438."""

    def __init__(self, node_dims, edge_dims, n_message=3, n_feedforward=2, drop_rate=0.1,
                 autoregressive=False, activations=(F.relu, torch.sigmoid), vector_gate=True,
                 residual=True):
        super().__init__()
        self.conv = GVPConv(node_dims, node_dims, edge_dims, n_message,
                            aggr="add" if autoregressive else "mean", activations=activations,
                            vector_gate=vector_gate)
        G = functools.partial(GVP, activations=activations, vector_gate=vector_gate)
        self.norm = nn.ModuleList([LayerNorm(node_dims) for _ in range(2)])
        self.dropout = nn.ModuleList([Dropout(drop_rate) for _ in range(2)])
        if n_feedforward == 1:
            ff = [G(node_dims, node_dims, activations=(None, None))]
        else:
            hid = 4 * node_dims[0], 2 * node_dims[1]
            ff = [G(node_dims, hid)] + [G(hid, hid) for _ in range(n_feedforward - 2)] + \
                 [G(hid, node_dims, activations=(None, None))]
        self.ff_func = nn.Sequential(*ff)
        self.residual = residual

    def forward(self, x, edge_index, edge_attr, autoregressive_x=None, node_mask=None):
        if autoregressive_x is not None:
            src, dst = edge_index
            mask = src < dst
            dh = tuple_sum(self.conv(x, edge_index[:, mask], tuple_index(edge_attr, mask)),
                           self.conv(autoregressive_x, edge_index[:, ~mask],
                                     tuple_index(edge_attr, ~mask)))
            count = ops.get_csr(dst, dh[0].size(0)).counts().clamp(min=1).unsqueeze(-1)
            count = count.to(dh[0].dtype)
            dh = dh[0] / count, dh[1] / count.unsqueeze(-1)
        else:
            dh = self.conv(x, edge_index, edge_attr)
        if node_mask is not None:
            x_ = x
            x, dh = tuple_index(x, node_mask), tuple_index(dh, node_mask)
        x = self.norm[0](tuple_sum(x, self.dropout[0](dh))) if self.residual else dh
        dh = gvp_ff(self.ff_func, x)
        x = self.norm[1](tuple_sum(x, self.dropout[1](dh))) if self.residual else dh
        if node_mask is not None:
            x_[0][node_mask], x_[1][node_mask] = x[0], x[1]
            x = x_
        return x


class GVPGNNModel(nn.Module):
    """models/gvpgnn.py:10-127."""

    def __init__(self, r_max=10.0, num_bessel=8, num_polynomial_cutoff=5, num_layers=5,
                 in_dim=1, out_dim=1, s_dim=128, v_dim=16, s_dim_edge=32, v_dim_edge=1,
                 pool="sum", residual=True, equivariant_pred=False):
        super().__init__()
        from .equivariant import RadialEmbeddingBlock
        self.r_max, self.num_layers = r_max, num_layers
        self.equivariant_pred, self.s_dim, self.v_dim = equivariant_pred, s_dim, v_dim
        acts = (F.relu, None)
        vd, ed = (s_dim, v_dim), (s_dim_edge, v_dim_edge)
        self.emb_in = nn.Embedding(in_dim, s_dim)
        self.W_v = nn.Sequential(LayerNorm((s_dim, 0)),
                                 GVP((s_dim, 0), vd, activations=(None, None), vector_gate=True))
        self.radial_embedding = RadialEmbeddingBlock(r_max, num_bessel, num_polynomial_cutoff)
        self.W_e = nn.Sequential(LayerNorm((self.radial_embedding.out_dim, 1)),
                                 GVP((self.radial_embedding.out_dim, 1), ed,
                                     activations=(None, None), vector_gate=True))
        self.layers = nn.ModuleList(GVPConvLayer(vd, ed, activations=acts, vector_gate=True,
                                                 residual=residual)
                                    for _ in range(num_layers))
        self.pool = {"mean": global_mean_pool, "sum": global_add_pool}[pool]
        if equivariant_pred:
            self.pred = nn.Linear(s_dim + v_dim * 3, out_dim)
        else:
            self.pred = nn.Sequential(nn.Linear(s_dim, s_dim), nn.ReLU(),
                                      nn.Linear(s_dim, out_dim))

    def forward(self, batch):
        ei = batch.edge_index
        # K1: radial embedding of |vec| and nan_to_num(vec / |vec|) in one pass (gvpgnn.py:106-112)
        rad, unit = ops.GvpEdgeFeaturizeFn.apply(batch.pos, ei, self.radial_embedding._host)
        h_V = ops.gather(self.emb_in.weight, batch.atoms, 0)
        h_V = self.W_v(h_V)
        h_E = edge_embed(self.W_e, rad, unit)   # K1e (gvpgnn.py:116)
        for layer in self.layers:
            h_V = layer(h_V, ei, h_E)
        out = self.pool(_merge(*h_V), batch.batch, getattr(batch, "num_graphs", None))
        if not self.equivariant_pred:
            out = out[:, :self.s_dim]
        return self.pred(out)
