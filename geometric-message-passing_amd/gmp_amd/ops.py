"""Thin, checked wrappers over the C ABI (include/gmp.h) + autograd Functions.

Every op launches on the current PyTorch HIP stream, allocates its outputs through the PyTorch
caching allocator and never synchronises.  Inputs must be CUDA (HIP) tensors: there is no CPU
fallback in the product path.
"""
import ctypes

import torch

from . import _lib
from ._lib import check


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# Optional per-kernel timing (bench.py): name -> list of (start, end) HIP events recorded on the
# stream the kernel is launched on (the current stream).  None = disabled (no overhead).
KERNEL_TIMERS = None


class _timed:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if KERNEL_TIMERS is not None:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        return self

    def __exit__(self, *exc):
        if KERNEL_TIMERS is not None:
            self.ev[1].record()
            KERNEL_TIMERS.setdefault(self.name, []).append(self.ev)
        return False


def kernel_time_ms(name):
    """Average device time (ms) per launch of a timed kernel, over the recorded launches."""
    evs = (KERNEL_TIMERS or {}).get(name, [])
    if not evs:
        return None
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / len(evs)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.GmpError("gmp_amd ops run on the MI355X only: got a CPU tensor "
                                "(no CPU fallback in the product path)")


def _f32c(t):
    if t.dtype != torch.float32:
        raise _lib.GmpError(f"expected float32, got {t.dtype}")
    return t.contiguous()


def _i64c(t):
    if t.dtype != torch.int64:
        t = t.long()
    return t.contiguous()


# ----------------------------------------------------------------------------------- CSR
class CSR:
    """Stable CSR of an index array (gmp_csr_build): items sorted by index value.

    perm[k]   : original position of the k-th item in sorted order
    rowptr[s] : first sorted position with index >= s  (len n_seg + 1)
    sorted    : index[perm]; payload_sorted: payload[perm] (if a payload was given)
    """

    __slots__ = ("index", "n_seg", "perm", "rowptr", "sorted", "payload_sorted", "err")

    def __init__(self, index, n_seg, payload=None):
        lib = _lib.load()
        index = _i64c(index)
        _need_cuda(index)
        n = index.numel()
        dev = index.device
        self.index = index
        self.n_seg = int(n_seg)
        self.perm = torch.empty(n, dtype=torch.int64, device=dev)
        self.rowptr = torch.empty(self.n_seg + 1, dtype=torch.int64, device=dev)
        self.sorted = torch.empty(n, dtype=torch.int64, device=dev)
        self.payload_sorted = None
        pl = None
        if payload is not None:
            pl = _i64c(payload)
            self.payload_sorted = torch.empty(n, dtype=torch.int64, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        ws_bytes = lib.gmp_csr_workspace_size(n, self.n_seg)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        check(lib.gmp_csr_build(_p(index), n, self.n_seg, _p(pl), _p(self.perm), _p(self.rowptr),
                                _p(self.sorted), _p(self.payload_sorted), _p(self.err), _p(ws),
                                ws_bytes, _stream()), "gmp_csr_build")

    def counts(self):
        return self.rowptr[1:] - self.rowptr[:-1]

    def check_range(self):
        """Host-synchronising range check (torch_scatter raises on out-of-range indices)."""
        if int(self.err.item()) != 0:
            raise IndexError("index out of range in gmp CSR build")


_CSR_CACHE = []  # [(key, index_tensor, payload_tensor, CSR)] small LRU; holds strong refs


def _tkey(t):
    """Content identity of a (possibly view) tensor while a strong ref is held: storage
    address, geometry and the version counter shared with its base (in-place writes bump it).
    Views such as edge_index[1] taken repeatedly map to the same key."""
    if t is None:
        return None
    return (t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype, t.device, t._version)


def get_csr(index, n_seg, payload=None):
    """Cached CSR for `index` (keyed on storage/geometry/version; holds a strong ref)."""
    key = (_tkey(index), int(n_seg), _tkey(payload))
    for k, (kk, _, _, csr) in enumerate(_CSR_CACHE):
        if kk == key:
            _CSR_CACHE.insert(0, _CSR_CACHE.pop(k))
            return csr
    csr = CSR(index, n_seg, payload)
    _CSR_CACHE.insert(0, (key, index, payload, csr))
    del _CSR_CACHE[16:]
    return csr


def clear_cache():
    _CSR_CACHE.clear()


# ----------------------------------------------------------------------------------- raw ops
def gather_rows(src2d, index):
    lib = _lib.load()
    src2d = _f32c(src2d)
    index = _i64c(index)
    _need_cuda(src2d, index)
    out = torch.empty((index.numel(), src2d.shape[1]), dtype=torch.float32, device=src2d.device)
    check(lib.gmp_gather_rows_f32(_p(src2d), src2d.shape[0], src2d.shape[1], _p(index),
                                  index.numel(), _p(out), None, _stream()), "gmp_gather_rows_f32")
    return out


def segment_reduce(src2d, csr, reduce="sum", use_perm=True):
    lib = _lib.load()
    src2d = _f32c(src2d)
    _need_cuda(src2d)
    F = src2d.shape[1]
    out = torch.empty((csr.n_seg, F), dtype=torch.float32, device=src2d.device)
    argmax = None
    if reduce == "max":
        argmax = torch.empty((csr.n_seg, F), dtype=torch.int64, device=src2d.device)
    red = _lib.REDUCE[reduce]
    ws_bytes = lib.gmp_segment_reduce_workspace_size(src2d.shape[0], csr.n_seg, F, red)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=src2d.device) if ws_bytes else None
    check(lib.gmp_segment_reduce_f32(_p(src2d), src2d.shape[0], F,
                                     _p(csr.perm) if use_perm else None, _p(csr.rowptr),
                                     csr.n_seg, red, _p(out), _p(argmax), _p(ws), ws_bytes,
                                     _stream()), "gmp_segment_reduce_f32")
    return out, argmax


def edge_outer_sum(A, B, with_colsum=True):
    """(A^T B, colsum(A)) over the edge dimension (gmp_edge_outer_sum_f32), deterministic."""
    lib = _lib.load()
    A, B = _f32c(A), _f32c(B)
    _need_cuda(A, B)
    K, d = A.shape
    C = torch.empty((d, d), dtype=torch.float32, device=A.device)
    cs = torch.empty(d, dtype=torch.float32, device=A.device) if with_colsum else None
    ws_bytes = lib.gmp_edge_outer_sum_workspace_size(K, d)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=A.device)
    with _timed("edge_outer_sum"):
        check(lib.gmp_edge_outer_sum_f32(K, d, _p(A), _p(B), _p(C), _p(cs), _p(ws), ws_bytes,
                                         _stream()), "gmp_edge_outer_sum_f32")
    return C, cs


def edge_outer_sum_act(A, X, w, b, act):
    """(A^T act(X * w + b), colsum(A)) with the activation applied at load time
    (gmp_edge_outer_sum_act_f32): the EGNN y1 / m weight-gradient operands from x_hat."""
    lib = _lib.load()
    A, X, w, b = _f32c(A), _f32c(X), _f32c(w), _f32c(b)
    _need_cuda(A, X, w, b)
    K, d = A.shape
    C = torch.empty((d, d), dtype=torch.float32, device=A.device)
    cs = torch.empty(d, dtype=torch.float32, device=A.device)
    ws_bytes = lib.gmp_edge_outer_sum_workspace_size(K, d)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=A.device)
    with _timed("edge_outer_sum"):
        check(lib.gmp_edge_outer_sum_act_f32(K, d, _p(A), _p(X), _p(w), _p(b), _lib.ACT[act],
                                             _p(C), _p(cs), _p(ws), ws_bytes, _stream()),
              "gmp_edge_outer_sum_act_f32")
    return C, cs


def _outer_sum_rect_call(A, B):
    lib = _lib.load()
    K, m, n = A.shape[0], A.shape[1], B.shape[1]
    if m == n and m in (32, 64, 128):  # square tiles: the faster square kernel (K5)
        return edge_outer_sum(A, B)
    mp, np_ = -(-m // 16) * 16, -(-n // 16) * 16
    if mp != m:
        A = torch.nn.functional.pad(A, (0, mp - m))
    if np_ != n:
        B = torch.nn.functional.pad(B, (0, np_ - n))
    C = torch.empty((mp, np_), dtype=torch.float32, device=A.device)
    cs = torch.empty(mp, dtype=torch.float32, device=A.device)
    ws_bytes = lib.gmp_edge_outer_sum_rect_workspace_size(K, mp, np_)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=A.device)
    with _timed("edge_outer_sum"):
        rc = lib.gmp_edge_outer_sum_rect_f32(K, mp, np_, _p(A), _p(B), _p(C), _p(cs), _p(ws),
                                             ws_bytes, _stream())
    if rc == _lib.GMP_ERR_UNSUPPORTED:  # shape outside the kernel's tile buckets
        return None
    check(rc, "gmp_edge_outer_sum_rect_f32")
    return C[:m, :n], cs[:m]


def edge_outer_sum_rect(A, B):
    """(A^T B, colsum(A)) over the rows (edges / nodes) for any widths, deterministic: columns
    zero-padded to multiples of 16 for gmp_edge_outer_sum_rect_f32, wide operands split into
    <= 128 x 144 blocks.  None when a block shape is outside the kernel's buckets."""
    A, B = _f32c(A), _f32c(B)
    _need_cuda(A, B)
    m, n = A.shape[1], B.shape[1]
    if m <= 128 and n <= 144:
        return _outer_sum_rect_call(A, B)
    C = torch.empty((m, n), dtype=torch.float32, device=A.device)
    cs = torch.empty(m, dtype=torch.float32, device=A.device)
    for m0 in range(0, m, 128):
        Am = A[:, m0:m0 + 128].contiguous()
        for n0 in range(0, n, 128):
            r = _outer_sum_rect_call(Am, B[:, n0:n0 + 128].contiguous())
            if r is None:
                return None
            C[m0:m0 + 128, n0:n0 + 128] = r[0]
            if n0 == 0:
                cs[m0:m0 + 128] = r[1]
    return C, cs


class EdgeLinearFn(torch.autograd.Function):
    """y = x W^T (+ b) over many rows (edges): forward and dx with the library GEMM (M = rows),
    dW / db with the deterministic edge outer sum (K = rows), which the library's small-tile
    K-reduction GEMMs run far below the HBM roofline."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return torch.addmm(b, x, W.t()) if b is not None else x.mm(W.t())

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        g = g.contiguous()
        dx = g.mm(W) if ctx.needs_input_grad[0] else None
        dW = db = None
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            r = edge_outer_sum_rect(g, x)
            if r is None:
                dW, db = g.t().mm(x), g.sum(0)
            else:
                dW, db = r
        return dx, dW, (db if ctx.has_b else None)


_LN_ACT = {"relu": 0, "swish": 1, "silu": 1, None: 2, "identity": 2}


class LnActFn(torch.autograd.Function):
    """act(LayerNorm(x)) over the last dim (K12 gmp_ln_act_*): one fused kernel each way,
    deterministic gamma/beta gradients."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, act):
        lib = _lib.load()
        shape = x.shape
        d = shape[-1]
        x2 = _f32c(x).reshape(-1, d)
        gamma, beta = _f32c(gamma), _f32c(beta)
        _need_cuda(x2, gamma, beta)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        xhat = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x2.device)
        a = _LN_ACT[act]
        check(lib.gmp_ln_act_fwd_f32(rows, d, _p(x2), _p(gamma), _p(beta), float(eps), a, _p(y),
                                     _p(xhat), _p(rstd), _stream()), "gmp_ln_act_fwd_f32")
        ctx.save_for_backward(xhat, rstd, gamma, beta)
        ctx.act, ctx.shape = a, shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, gy):
        lib = _lib.load()
        xhat, rstd, gamma, beta = ctx.saved_tensors
        rows, d = xhat.shape
        gy = _f32c(gy).reshape(rows, d)
        gx = torch.empty_like(xhat)
        gb = torch.empty(2 * d, dtype=torch.float32, device=xhat.device)
        ws_bytes = lib.gmp_ln_act_bwd_workspace_size(rows, d)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=xhat.device)
        check(lib.gmp_ln_act_bwd_f32(rows, d, _p(gy), _p(xhat), _p(rstd), _p(gamma), _p(beta),
                                     ctx.act, _p(gx), _p(gb), _p(ws), ws_bytes, _stream()),
              "gmp_ln_act_bwd_f32")
        return gx.view(ctx.shape), gb[:d], gb[d:], None, None


def ln_act(x, ln, act=None):
    """act(ln(x)) for an nn.LayerNorm `ln` (affine) through K12."""
    return LnActFn.apply(x, ln.weight, ln.bias, ln.eps, act)


EDGE_LINEAR_MIN_ROWS = 1 << 15


def linear(x, W, b=None):
    """F.linear for (..., in) inputs; row counts >= EDGE_LINEAR_MIN_ROWS on the GPU take the
    EdgeLinearFn path (deterministic outer-sum weight gradients)."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if x2.is_cuda and x2.shape[0] >= EDGE_LINEAR_MIN_ROWS and x2.dtype == torch.float32:
        y = EdgeLinearFn.apply(x2.contiguous(), W, b)
    else:
        y = torch.nn.functional.linear(x2, W, b)
    return y.reshape(shp[:-1] + (W.shape[0],))


def segment_reduce_bwd(grad_out, csr, reduce, argmax, n_items):
    lib = _lib.load()
    grad_out = _f32c(grad_out)
    F = grad_out.shape[1]
    gsrc = torch.empty((n_items, F), dtype=torch.float32, device=grad_out.device)
    check(lib.gmp_segment_reduce_bwd_f32(_p(grad_out), csr.n_seg, F, _p(csr.index), n_items,
                                         _p(csr.rowptr), _lib.REDUCE[reduce], _p(argmax),
                                         _p(gsrc), _stream()), "gmp_segment_reduce_bwd_f32")
    return gsrc


# ----------------------------------------------------------------------------------- autograd
class SegmentReduceFn(torch.autograd.Function):
    """out[s] = reduce_{e: index[e]==s} src[e]   (torch_scatter.scatter along dim 0)."""

    @staticmethod
    def forward(ctx, src2d, csr, reduce):
        out, argmax = segment_reduce(src2d, csr, reduce)
        ctx.csr, ctx.reduce, ctx.n = csr, reduce, src2d.shape[0]
        ctx.save_for_backward(argmax if argmax is not None else torch.empty(0))
        return out

    @staticmethod
    def backward(ctx, g):
        (argmax,) = ctx.saved_tensors
        gs = segment_reduce_bwd(g.contiguous(), ctx.csr, ctx.reduce,
                                argmax if ctx.reduce == "max" else None, ctx.n)
        return gs, None, None


class GatherRowsFn(torch.autograd.Function):
    """out[e] = src[index[e]]; backward = deterministic segmented sum over the CSR of index."""

    @staticmethod
    def forward(ctx, src2d, index, n_rows):
        ctx.index, ctx.n_rows = index, n_rows
        return gather_rows(src2d, index)

    @staticmethod
    def backward(ctx, g):
        csr = get_csr(ctx.index, ctx.n_rows)
        out, _ = segment_reduce(g.contiguous(), csr, "sum")
        return out, None, None


def gather(src, index, dim=0):
    """index_select(src, dim, index) through the HIP gather kernel (differentiable)."""
    dim = dim % src.dim()
    x = src.movedim(dim, 0)
    shp = x.shape
    x2 = x.reshape(shp[0], -1)
    out = GatherRowsFn.apply(x2, index, shp[0])
    return out.reshape((index.numel(),) + tuple(shp[1:])).movedim(0, dim)


# ----------------------------------------------------------------------------------- EGNN
class EgnnGraph:
    """Receiver-sorted view of an edge_index for the fused EGNN kernels (built on device)."""

    def __init__(self, edge_index, num_nodes):
        ei = _i64c(edge_index)
        _need_cuda(ei)
        self.num_nodes = int(num_nodes)
        self.num_edges = ei.shape[1]
        self.recv_csr = CSR(ei[1], self.num_nodes, payload=ei[0])
        self.recv = self.recv_csr.sorted             # receiver of sorted edge k
        self.send = self.recv_csr.payload_sorted     # sender of sorted edge k
        self.rowptr = self.recv_csr.rowptr
        self.send_csr = CSR(self.send, self.num_nodes)  # sender CSR over sorted positions

    def check_range(self):
        """Host-synchronising check that every edge_index entry is in [0, num_nodes)."""
        self.recv_csr.check_range()
        self.send_csr.check_range()


_EGNN_GRAPHS = []


def egnn_graph(edge_index, num_nodes):
    for k, (t, ver, n, g) in enumerate(_EGNN_GRAPHS):
        if t is edge_index and ver == edge_index._version and n == num_nodes:
            return g
    g = EgnnGraph(edge_index, num_nodes)
    _EGNN_GRAPHS.insert(0, (edge_index, edge_index._version, num_nodes, g))
    del _EGNN_GRAPHS[8:]
    return g


_EGNN_PARAM_NAMES = ("w1d", "b1", "ln1_w", "ln1_b", "W2", "b2", "ln2_w", "ln2_b", "W3", "b3",
                     "ln3_w", "ln3_b", "w4", "b4")


def _egnn_params(tensors):
    return _lib.GmpEgnnParams(*[t.data_ptr() for t in tensors])


class EgnnEdgeFn(torch.autograd.Function):
    """Fused EGNN message + aggregation (egnn_layer.py:62-80) on the receiver-sorted graph.

    Inputs: AB = [h W1a^T | h W1b^T] (N, 2d), pos (N, 3), the 14 message/pos-MLP tensors in
    _EGNN_PARAM_NAMES order.  Returns (m_aggr (N, d), pos_aggr (N, 3)).
    """

    @staticmethod
    def forward(ctx, AB, pos, graph, act, msg_mean, eps, *params):
        lib = _lib.load()
        AB = _f32c(AB)
        pos = _f32c(pos)
        params = tuple(_f32c(t) for t in params)
        _need_cuda(AB, pos, *params)
        N, d = AB.shape[0], AB.shape[1] // 2
        E = graph.num_edges
        m_aggr = torch.empty((N, d), dtype=torch.float32, device=AB.device)
        pos_aggr = torch.empty((N, 3), dtype=torch.float32, device=AB.device)
        train = any(ctx.needs_input_grad)
        xhat = torch.empty((3, E, d), dtype=torch.float32, device=AB.device) if train else None
        rstd = torch.empty((E, 3), dtype=torch.float32, device=AB.device) if train else None
        P = _egnn_params(params)
        with _timed("egnn_edge_fwd"):
            check(lib.gmp_egnn_edge_fwd_f32(N, E, d, _p(AB), _p(pos), _p(graph.rowptr),
                                          _p(graph.recv), _p(graph.send), ctypes.byref(P),
                                          _lib.ACT[act], int(msg_mean), float(eps), _p(m_aggr),
                                          _p(pos_aggr), _p(xhat), _p(rstd), _stream()),
                  "gmp_egnn_edge_fwd_f32")
        ctx.graph, ctx.act, ctx.msg_mean, ctx.eps, ctx.N = graph, act, msg_mean, eps, N
        if train:
            ctx.save_for_backward(pos, xhat, rstd, *params)
        return m_aggr, pos_aggr

    @staticmethod
    def backward(ctx, g_m, g_p):
        lib = _lib.load()
        pos, xhat, rstd, *params = ctx.saved_tensors
        graph = ctx.graph
        N, d = ctx.N, xhat.shape[2]
        E = graph.num_edges
        dev = pos.device
        g_m = torch.zeros((N, d), device=dev) if g_m is None else _f32c(g_m)
        g_p = torch.zeros((N, 3), device=dev) if g_p is None else _f32c(g_p)
        f = dict(dtype=torch.float32, device=dev)
        dA = torch.empty((N, d), **f)
        dpos_recv = torch.empty((N, 3), **f)
        dpre1 = torch.empty((E, d), **f)
        gdiff = torch.empty((E, 3), **f)
        dpre2 = torch.empty((E, d), **f)
        dpre3 = torch.empty((E, d), **f)
        rows = lib.gmp_egnn_edge_bwd_partials_rows(E, d)
        partials = torch.empty((rows, 8 * d + 1), **f)
        P = _egnn_params(params)
        with _timed("egnn_edge_bwd"):
            check(lib.gmp_egnn_edge_bwd_f32(N, E, d, _p(pos), _p(graph.rowptr), _p(graph.recv),
                                          _p(graph.send), ctypes.byref(P), _lib.ACT[ctx.act],
                                          int(ctx.msg_mean), _p(xhat), _p(rstd), _p(g_m),
                                          _p(g_p), _p(dA), _p(dpos_recv), _p(dpre1), _p(gdiff),
                                          _p(dpre2), _p(dpre3), _p(partials), _stream()),
                  "gmp_egnn_edge_bwd_f32")
        # sender-side reductions (deterministic segmented sums over the sender CSR)
        dB, _ = segment_reduce(dpre1, graph.send_csr, "sum")
        dpos_send, _ = segment_reduce(gdiff, graph.send_csr, "sum")
        dAB = torch.cat([dA, dB], dim=1)
        dpos = dpos_recv - dpos_send
        # weight gradients: GEMMs over edges, y1 = act(LN1 affine(x_hat1)) and
        # m = act(LN2 affine(x_hat2)) rebuilt at load time
        pn = dict(zip(_EGNN_PARAM_NAMES, params))
        dW2, db2 = edge_outer_sum_act(dpre2, xhat[0], pn["ln1_w"], pn["ln1_b"], ctx.act)
        dW3, db3 = edge_outer_sum_act(dpre3, xhat[1], pn["ln2_w"], pn["ln2_b"], ctx.act)
        db1 = dA.sum(0)
        v = partials.sum(0)
        dln1w, dln1b, dln2w, dln2b, dln3w, dln3b, dw4, dw1d = v[:8 * d].view(8, d).unbind(0)
        db4 = v[8 * d:8 * d + 1]
        grads = dict(w1d=dw1d, b1=db1, ln1_w=dln1w, ln1_b=dln1b, W2=dW2, b2=db2, ln2_w=dln2w,
                     ln2_b=dln2b, W3=dW3, b3=db3, ln3_w=dln3w, ln3_b=dln3b, w4=dw4.view(1, d),
                     b4=db4)
        pgrads = tuple(grads[n].reshape(t.shape) for n, t in zip(_EGNN_PARAM_NAMES, params))
        return (dAB, dpos, None, None, None, None) + pgrads
