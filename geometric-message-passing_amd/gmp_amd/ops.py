"""Thin, checked wrappers over the C ABI (include/gmp.h) + autograd Functions.

Every op launches on the current PyTorch HIP stream, allocates its outputs through the PyTorch
caching allocator and never synchronises.  Inputs must be CUDA (HIP) tensors: there is no CPU
fallback in the product path.
"""
import ctypes


import torch
from torch.autograd.function import once_differentiable

from . import _lib
from ._lib import check


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# Optional per-kernel timing (bench.py): name -> list of (start, end) HIP events recorded on the
# stream the kernel is launched on (the current stream).  None = disabled (no overhead).
KERNEL_TIMERS = None
KERNEL_TIMER_NAMES = None  # None: every timed region; else only these names (host cost: two
                           # event records per region, on the launch path)


class _timed:
    def __init__(self, name):
        self.name = name
        self.on = KERNEL_TIMERS is not None and (KERNEL_TIMER_NAMES is None
                                                 or name in KERNEL_TIMER_NAMES)

    def __enter__(self):
        if self.on:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        return self

    def __exit__(self, *exc):
        if self.on:
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
        index = _i64c(index)
        _need_cuda(index)
        self.index = index
        self.n_seg = int(n_seg)
        pl = _i64c(payload) if payload is not None else None
        self.perm, self.rowptr, self.sorted, pls, self.err = _lib.torch_ops().csr_build(
            index, self.n_seg, pl)
        self.payload_sorted = pls if pl is not None else None

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
    if compiling():
        return CSR(index, n_seg, payload)
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
    src2d = _f32c(src2d)
    index = _i64c(index)
    _need_cuda(src2d, index)
    return _lib.torch_ops().gather_rows(src2d, index)


def segment_reduce(src2d, csr, reduce="sum", use_perm=True):
    """(out, argmax or None) = torch.ops.gmp.segment_reduce over the CSR's segments."""
    src2d = _f32c(src2d)
    _need_cuda(src2d)
    out, argmax = _lib.torch_ops().segment_reduce(src2d, csr.perm if use_perm else None,
                                                  csr.rowptr, csr.n_seg, reduce)
    return out, (argmax if reduce == "max" else None)


def edge_outer_sum(A, B):
    """(A^T B, colsum(A)) over the edge dimension (torch.ops.gmp.edge_outer_sum), deterministic."""
    A, B = _f32c(A), _f32c(B)
    _need_cuda(A, B)
    with _timed("edge_outer_sum"):
        return _lib.torch_ops().edge_outer_sum(A, B)


def edge_outer_sum_act(A, X, w, b, act, amax=None):
    """(A^T act(X * w + b), colsum(A)) with the activation applied at load time
    (torch.ops.gmp.edge_outer_sum_act): the EGNN y1 / m weight-gradient operands from x_hat.
    With `amax` (device word, max |A| as float bits; X LayerNorm rows) the HF form (scaled fp16
    planes, three products)."""
    A, X, w, b = _f32c(A), _f32c(X), _f32c(w), _f32c(b)
    _need_cuda(A, X, w, b)
    with _timed("edge_outer_sum"):
        return _lib.torch_ops().edge_outer_sum_act(A, X, w, b, _lib.ACT[act], amax)


def outer_sum_into(A, B, C, colsum=None, act=None, w=None, b=None):
    """C[:] = A^T act(B) over the rows (torch.ops.gmp.edge_outer_sum_ex), colsum[:] =
    colsum(A).  A (K, m), B (K, n) and C (m, n) may be strided views (unit column stride; e.g.
    column blocks of a wider tensor or parameter gradient).  Shapes outside the kernels' tile
    buckets run the library GEMM inside the op."""
    _need_cuda(A, B, C)
    a = -1 if act is None else _lib.ACT[act]
    with _timed("edge_outer_sum"):
        _lib.torch_ops().edge_outer_sum_ex(A, B, C, colsum, a, w, b)


def outer_sum_into2(A, B1, B2, C, colsum=None):
    """C[:] = A^T [B1 | B2] (and colsum(A)) in one pass over A where the split-plane kernel
    applies, else as two products inside the op."""
    _need_cuda(A, B1, B2, C)
    with _timed("edge_outer_sum"):
        _lib.torch_ops().edge_outer_sum_ex2(A, B1, B2, C, colsum)


def edge_outer_sum_rect(A, B):
    """(A^T B, colsum(A)) over the rows (edges / nodes) for any widths, deterministic: columns
    zero-padded to multiples of 16 when needed, wide operands processed as <= 128 x 144 column
    blocks read in place (strided) and written into their block of C."""
    A, B = _f32c(A), _f32c(B)
    _need_cuda(A, B)
    m, n = A.shape[1], B.shape[1]
    mp, np_ = -(-m // 16) * 16, -(-n // 16) * 16
    if mp != m:
        A = torch.nn.functional.pad(A, (0, mp - m))
    if np_ != n:
        B = torch.nn.functional.pad(B, (0, np_ - n))
    C = torch.empty((mp, np_), dtype=torch.float32, device=A.device)
    cs = torch.empty(mp, dtype=torch.float32, device=A.device)
    bn = 144 if np_ <= 144 else 128
    for m0 in range(0, mp, 128):
        for n0 in range(0, np_, bn):
            outer_sum_into(A[:, m0:m0 + 128], B[:, n0:n0 + bn], C[m0:m0 + 128, n0:n0 + bn],
                           cs[m0:m0 + 128] if n0 == 0 else None)
    if (mp, np_) != (m, n):
        return C[:m, :n].contiguous(), cs[:m]
    return C, cs


# ----------------------------------------------------------------------------------- deferred
# Weight gradients are leaves of the backward graph: nothing downstream waits for them.  They
# are computed on a side stream (overlapping the critical path's small node-level kernels and
# the host launch gaps between them) and accumulated into param.grad by a callback at the end
# of the backward pass, as DDP does with its reducer.  Disable (DEFER_WEIGHT_GRADS = False)
# when something must see these gradients through autograd (DDP's per-parameter hooks);
# gmp_amd.dist.wrap_ddp does so.  Under torch.autograd.grad (the engine runs no AccumulateGrad)
# they are returned through autograd automatically (_engine_accumulates).
DEFER_WEIGHT_GRADS = True
_SIDE_STREAMS = {}
_PENDING = []   # (param, grad) accumulated at the end of the backward pass
_CB_QUEUED = [False]
# Main-stream tensors read by side-stream work are kept alive here until the main stream has
# waited for the side stream (flush / join), then dropped: their blocks go straight back to the
# main stream's pool, stream-ordered after that wait.  (record_stream instead would hold every
# such block until the allocator sees the side stream's event complete; with the host running a
# step ahead it then allocated fresh HBM every step and synchronised the host doing so.)
_KEEPALIVE = []


def _side_stream(device):
    st = _SIDE_STREAMS.get(device)
    if st is None:
        st = _SIDE_STREAMS[device] = torch.cuda.Stream(device=device)
    return st


def _flush_deferred():
    _CB_QUEUED[0] = False
    if not _PENDING:
        return
    main = torch.cuda.current_stream()
    for st in _SIDE_STREAMS.values():
        main.wait_stream(st)
    _KEEPALIVE.clear()
    for p, g in _PENDING:
        g.record_stream(main)
        if p.grad is None:
            # AccumulateGrad's layout contract: a dense gradient with the parameter's strides
            p.grad = g if g.stride() == p.stride() else g.contiguous()
        else:
            p.grad.add_(g)
    _PENDING.clear()


def deferrable(t):
    return DEFER_WEIGHT_GRADS and t is not None and t.is_leaf and t.requires_grad


def _engine_accumulates(p):
    """True when the running backward pass will execute p's AccumulateGrad (loss.backward());
    False under torch.autograd.grad, which either skips the parameter or captures its gradient
    as an output — then the gradient must travel through autograd, not into p.grad."""
    try:
        with torch.enable_grad():
            acc = p.view_as(p).grad_fn.next_functions[0][0]
        return bool(torch._C._will_engine_execute_node(acc))
    except (RuntimeError, AttributeError, IndexError):
        return False


def compiling():
    """True while torch.compile (dynamo) traces: the ops then run inline on the current stream,
    without the per-graph caches, side streams or end-of-backward callbacks of eager mode."""
    return torch.compiler.is_compiling()


class side_work:
    """with side_work(used_tensors) as sw: ... launches on the side stream after everything
    already queued on the current stream; sw.deliver(...) hands each result to the end-of-
    backward accumulation (deferred leaf gradients) or back through autograd (after joining the
    streams).  Under torch.compile the work runs inline and every gradient goes back through
    autograd."""

    def __init__(self, *used):
        self.used = [t for t in used if t is not None]
        self.inline = compiling()

    def __enter__(self):
        if self.inline:
            return self
        self.main = torch.cuda.current_stream()
        self.side = _side_stream(self.main.device)
        self.side.wait_stream(self.main)
        self.ctx = torch.cuda.stream(self.side)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.inline:
            return False
        self.ctx.__exit__(*exc)
        _KEEPALIVE.extend(self.used)
        return False

    def defer(self, param, grad):
        _PENDING.append((param, grad))
        if not _CB_QUEUED[0]:
            _CB_QUEUED[0] = True
            torch.autograd.Variable._execution_engine.queue_callback(_flush_deferred)

    def join(self, *results):
        """results are needed on the current stream now (returned through autograd)."""
        self.main.wait_stream(self.side)
        _KEEPALIVE.clear()
        for r in results:
            if r is not None:
                r.record_stream(self.main)

    def deliver(self, needs_input_grad, first, targets, grads):
        """Per parameter: defer the gradient (leaf parameter) or hand it back through autograd
        (after joining the streams).  needs_input_grad[first + i] belongs to targets[i]."""
        if self.inline:
            return tuple(gr if needs_input_grad[first + i] else None
                         for i, gr in enumerate(grads))
        out, joined, deferred = [], False, False
        accum = None  # does this backward pass accumulate into .grad (checked once per call)
        for i, (p, gr) in enumerate(zip(targets, grads)):
            if deferrable(p) and needs_input_grad[first + i] and accum is None:
                accum = _engine_accumulates(p)
            if not needs_input_grad[first + i]:
                out.append(None)
            elif deferrable(p) and accum:
                self.defer(p, gr)
                deferred = True
                out.append(None)
            else:
                if not joined:
                    self.join(*[g for g in grads if g is not None])
                    joined = True
                out.append(gr)
        if not (joined or deferred):
            # no parameter gradient wanted (e.g. autograd.grad w.r.t. inputs only): nothing will
            # flush this side work, so join here and release the kept-alive inputs
            self.main.wait_stream(self.side)
            _KEEPALIVE.clear()
        return tuple(out)


def _mm_wt(g, Wt):
    """g @ Wt.t() for a contiguous Wt (n, k): the library GEMM's "NT" form, measured ~1.5x
    faster than the "NN" g @ W for the (50k x 128) x (128 x 128) node GEMMs (22.5 vs 34 us);
    the transposed weight copy is one small kernel."""
    return g.mm(Wt.t())


def _dx(g, W):
    """g @ W for the dx of y = x W^T (W (n_out, n_in))."""
    return _mm_wt(g, W.t().contiguous())


class EdgeLinearFn(torch.autograd.Function):
    """y = x W^T (+ b) over many rows (edges): forward and dx with the library GEMM (M = rows),
    dW / db with the deterministic edge outer sum (K = rows), which the library's small-tile
    K-reduction GEMMs run far below the HBM roofline.  dW / db of leaf parameters are computed
    on the side stream and accumulated at the end of the backward pass (deferred)."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W, b)
        return torch.addmm(b, x, W.t()) if b is not None else x.mm(W.t())

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        x, W, b = ctx.saved_tensors
        g = g.contiguous()
        dx = _dx(g, W) if ctx.needs_input_grad[0] else None
        need_w = ctx.needs_input_grad[1] or (b is not None and ctx.needs_input_grad[2])
        if not need_w:
            return dx, None, None
        with side_work(g, x) as sw:
            dW, db = edge_outer_sum_rect(g, x)
        return (dx,) + sw.deliver(ctx.needs_input_grad, 1, (W, b), (dW, db))


class SplitLinearFn(torch.autograd.Function):
    """y = [xa | xb] W^T + b without materialising the concatenation (egnn_layer.py:37
    mlp_upd[0] over cat([h, m_aggr])): two GEMMs forward, two for dx; dW written block-wise
    into one (out, ina + inb) gradient by the strided outer sum (deferred for leaf params)."""

    @staticmethod
    def forward(ctx, xa, xb, W, b):
        da = xa.shape[1]
        ctx.save_for_backward(xa, xb, W, b)
        y = torch.addmm(b, xa, W[:, :da].t()) if b is not None else xa.mm(W[:, :da].t())
        y.addmm_(xb, W[:, da:].t())
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        xa, xb, W, b = ctx.saved_tensors
        da = xa.shape[1]
        g = g.contiguous()
        dxa = _dx(g, W[:, :da]) if ctx.needs_input_grad[0] else None
        dxb = _dx(g, W[:, da:]) if ctx.needs_input_grad[1] else None
        need_w = ctx.needs_input_grad[2] or (b is not None and ctx.needs_input_grad[3])
        if not need_w:
            return dxa, dxb, None, None
        with side_work(g, xa, xb) as sw:
            dW = torch.empty_like(W)
            db = torch.empty(W.shape[0], dtype=W.dtype, device=W.device)
            outer_sum_into(g, xa, dW[:, :da], db)
            outer_sum_into(g, xb, dW[:, da:], None)
        return (dxa, dxb) + sw.deliver(ctx.needs_input_grad, 2, (W, b), (dW, db))


def split_linear(xa, xb, W, b=None):
    """F.linear(cat([xa, xb], -1), W, b) for 2-D inputs without the concatenation."""
    if (xa.is_cuda and xa.dim() == 2 and xb.dim() == 2 and xa.dtype == torch.float32
            and xa.shape[0] >= EDGE_LINEAR_MIN_ROWS and xa.shape[1] % 4 == 0
            and xb.shape[1] % 4 == 0):
        return SplitLinearFn.apply(xa.contiguous(), xb.contiguous(), W, b)
    return torch.nn.functional.linear(torch.cat([xa, xb], -1), W, b)


_LN_ACT = {"relu": 0, "swish": 1, "silu": 1, None: 2, "identity": 2}


class LnActFn(torch.autograd.Function):
    """act(LayerNorm(x)) over the last dim (K12 gmp_ln_act_*): one fused kernel each way,
    deterministic gamma/beta gradients."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, act):
        shape = x.shape
        d = shape[-1]
        x2 = _f32c(x).reshape(-1, d)
        gamma, beta = _f32c(gamma), _f32c(beta)
        _need_cuda(x2, gamma, beta)
        a = _LN_ACT[act]
        y, xhat, rstd = _lib.torch_ops().ln_act_fwd(x2, gamma, beta, float(eps), a)
        ctx.save_for_backward(xhat, rstd, gamma, beta)
        ctx.act, ctx.shape = a, shape
        return y.view(shape)

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        xhat, rstd, gamma, beta = ctx.saved_tensors
        rows, d = xhat.shape
        gy = _f32c(gy).reshape(rows, d)
        # (deferring the [dgamma | dbeta] reduction to the side stream was measured slower: the
        # extra stream bookkeeping lengthens the host-bound stretch of small node kernels)
        gx, gb = _lib.torch_ops().ln_act_bwd(gy, xhat, rstd, gamma, beta, ctx.act)
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
    return _lib.torch_ops().segment_reduce_bwd(_f32c(grad_out), csr.index, csr.rowptr, reduce,
                                               argmax, n_items)


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
    @once_differentiable
    def backward(ctx, g):
        (argmax,) = ctx.saved_tensors
        gs = segment_reduce_bwd(g.contiguous(), ctx.csr, ctx.reduce,
                                argmax if ctx.reduce == "max" else None, ctx.n)
        return gs, None, None


class SegmentMaxFn(torch.autograd.Function):
    """(out, argmax) of a segmented max (torch_scatter.scatter_max along dim 0): the gradient
    goes to the arg-max item of each (segment, feature); argmax is not differentiable."""

    @staticmethod
    def forward(ctx, src2d, csr):
        out, argmax = segment_reduce(src2d, csr, "max")
        ctx.csr, ctx.n = csr, src2d.shape[0]
        ctx.save_for_backward(argmax)
        ctx.mark_non_differentiable(argmax)
        return out, argmax

    @staticmethod
    @once_differentiable
    def backward(ctx, g, _g_arg):
        (argmax,) = ctx.saved_tensors
        return segment_reduce_bwd(g.contiguous(), ctx.csr, "max", argmax, ctx.n), None


class GatherRowsFn(torch.autograd.Function):
    """out[e] = src[index[e]]; backward = deterministic segmented sum over the CSR of index."""

    @staticmethod
    def forward(ctx, src2d, index, n_rows):
        ctx.index, ctx.n_rows = index, n_rows
        return gather_rows(src2d, index)

    @staticmethod
    @once_differentiable
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


# ----------------------------------------------------------------------------------- CFConv
_CHECKED_CSR = []  # CSRs whose build-time range flag was already read (once per graph)


def checked_csr(index, n):
    """get_csr plus the build's out-of-range flag read once per new graph (one host sync, as
    torch_scatter raises for an index outside the output rows fixed by dim_size / out=)."""
    csr = get_csr(index, n)
    if compiling():
        return csr
    if not any(c is csr for c in _CHECKED_CSR):
        csr.check_range()  # one host sync per new graph, as torch_scatter raises IndexError
        _CHECKED_CSR.insert(0, csr)
        del _CHECKED_CSR[32:]
    return csr


_cfconv_csr = checked_csr


def cfconv_aggregate(x, xidx, w, csr, escale=None):
    """out[s] = sum over CSR segment s of x[xidx[e]] * (w[e] (* escale[e])) (K13
    gmp_cfconv_aggregate_scaled_f32)."""
    return _lib.torch_ops().cfconv_aggregate(x, _i64c(xidx), w, csr.perm, csr.rowptr, csr.n_seg,
                                             escale)


class CFConvAggregateFn(torch.autograd.Function):
    """PyG CFConv propagate (message x_j * W, aggr "add", dim_size = N; schnet.py:72) without
    the (E, F) message: forward and x-gradient by K13 over the receiver / sender CSR, the
    W-gradient as the per-edge product grad[dst] * x[src].  C (optional, no gradient): the
    per-edge cosine cutoff multiplying W (W * C.view(-1, 1) in CFConv.forward), applied at load
    time; the W-gradient is then the gradient w.r.t. the unscaled W."""

    @staticmethod
    def forward(ctx, x, W, src, dst, n, C=None):
        recv = _cfconv_csr(dst, n)
        ctx.save_for_backward(x, W, C)
        ctx.src, ctx.dst, ctx.n = src, dst, n
        return cfconv_aggregate(x, src, W, recv, C)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        x, W, C = ctx.saved_tensors
        g = _f32c(g)
        dx = dW = None
        if ctx.needs_input_grad[0]:
            dx = cfconv_aggregate(g, ctx.dst, W, _cfconv_csr(ctx.src, x.shape[0]), C)
        if ctx.needs_input_grad[1]:
            dW = _lib.torch_ops().cfconv_wgrad(g, _i64c(ctx.dst), x, _i64c(ctx.src), C)
        if ctx.needs_input_grad[5]:
            raise RuntimeError("cfconv_propagate: C must not require grad (use W * C instead)")
        return dx, dW, None, None, None, None


class ShiftedSoftplusFn(torch.autograd.Function):
    """softplus(x) - shift in one pass each way (K14 gmp_ssp_{fwd,bwd}_f32)."""

    @staticmethod
    def forward(ctx, x, shift):
        y = _lib.torch_ops().ssp_fwd(x, float(shift))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = _f32c(g)
        if g.data_ptr() % 16:  # a contiguous view at an odd offset: K14 needs 16-byte rows
            g = g.clone()
        return _lib.torch_ops().ssp_bwd(x, g), None


def shifted_softplus(x, shift):
    """F.softplus(x) - shift through K14 (CUDA fp32, numel % 4 == 0, 16-byte aligned)."""
    x = _f32c(x)
    _need_cuda(x)
    return ShiftedSoftplusFn.apply(x, shift)


def cfconv_propagate(edge_index, x, W, C=None):
    """sum_{e: dst[e] = i} x[src[e]] * W[e] (* C[e]) for edge_index = (src, dst), N =
    x.shape[0]; C (E,) is a per-edge factor without gradient (SchNet's cosine cutoff)."""
    x, W = _f32c(x), _f32c(W)
    _need_cuda(x, W)
    if C is not None:
        if C.requires_grad and torch.is_grad_enabled():
            raise ValueError("cfconv_propagate: C must not require grad")
        C = _f32c(C.detach().reshape(-1))
    ei = _i64c(edge_index)
    return CFConvAggregateFn.apply(x, W, ei[0], ei[1], x.shape[0], C)


# ----------------------------------------------------------------------------------- K1 edges
def edge_vec_to_pos_grad(g_vec, edge_index, n):
    """d pos from d vec for vec = pos[ei0] - pos[ei1]: deterministic segmented sums over the
    cached CSRs of ei0 (+) and ei1 (-)."""
    plus, _ = segment_reduce(g_vec, get_csr(edge_index[0], n), "sum")
    minus, _ = segment_reduce(g_vec, get_csr(edge_index[1], n), "sum")
    return plus - minus


class GvpEdgeFeaturizeFn(torch.autograd.Function):
    """GVP-GNN edge features (gvpgnn.py:106-112) in one pass over the edges (K1,
    gmp_edge_featurize_gvp_f32): (radial (E, nb), unit vectors nan_to_num(vec / |vec|) (E, 3))."""

    @staticmethod
    def forward(ctx, pos, edge_index, host_consts):
        w, pref, r_max, p = host_consts
        pos, ei = _f32c(pos), _i64c(edge_index)
        _need_cuda(pos, ei)
        with _timed("edge_featurize"):
            rad, unit = _lib.torch_ops().edge_featurize_gvp(pos, ei, [float(v) for v in w], pref,
                                                            r_max, p)
        ctx.save_for_backward(pos, ei)
        ctx.host = host_consts
        return rad, unit

    @staticmethod
    @once_differentiable
    def backward(ctx, g_rad, g_unit):
        if not ctx.needs_input_grad[0]:
            return None, None, None
        pos, ei = ctx.saved_tensors
        w, pref, r_max, p = ctx.host
        g_vec = _lib.torch_ops().edge_featurize_gvp_bwd(
            pos, ei, [float(v) for v in w], pref, r_max, p,
            _f32c(g_rad) if g_rad is not None else None,
            _f32c(g_unit) if g_unit is not None else None)
        return edge_vec_to_pos_grad(g_vec, ei, pos.shape[0]), None, None


class SchNetFeaturizeFn(torch.autograd.Function):
    """SchNet edge features (schnet.py:66-68 over PyG SchNet.forward / GaussianSmearing /
    CFConv.forward) in one pass over the edges (gmp_schnet_featurize_f32): edge_weight (E),
    Gaussians (E, G) and the CFConv cosine cutoff C (E)."""

    @staticmethod
    def forward(ctx, pos, edge_index, offsets, coeff, cutoff):
        pos, ei, off = _f32c(pos), _i64c(edge_index), _f32c(offsets)
        _need_cuda(pos, ei, off)
        with _timed("edge_featurize"):
            d, rbf, cut = _lib.torch_ops().schnet_featurize(pos, ei, off, float(coeff),
                                                            float(cutoff))
        ctx.save_for_backward(pos, ei, off)
        ctx.coeff, ctx.cutoff = float(coeff), float(cutoff)
        return d, rbf, cut

    @staticmethod
    @once_differentiable
    def backward(ctx, g_d, g_rbf, g_cut):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        pos, ei, off = ctx.saved_tensors
        opt = [_f32c(t) if t is not None else None for t in (g_d, g_rbf, g_cut)]
        g_vec = _lib.torch_ops().schnet_featurize_bwd(pos, ei, off, ctx.coeff, ctx.cutoff, *opt)
        return edge_vec_to_pos_grad(g_vec, ei, pos.shape[0]), None, None, None, None


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
    if compiling():
        return EgnnGraph(edge_index, num_nodes)
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


# LayerNorm outputs the EGNN forward saves for the backward: 2 = x_hat1, x_hat2 (x_hat3 recomputed
# in the backward, bitwise the forward's), 3 = x_hat1..3 (the r02 form; tests compare the two).
# The backward follows the saved tensor's plane count.
EGNN_XHAT_PLANES = 2


class EgnnMessageFn(torch.autograd.Function):
    """The whole EGNN message block of one layer (egnn_layer.py:62-80 with the MLPs of :28-36):
    the node projections AB = [h W1a^T | h W1b^T] (one GEMM), the fused edge kernel K4 and the
    aggregation; backward = K4 backward, sender-side segmented sums, dh on the critical path,
    and every weight gradient (dW1 assembled in place as [dW1a | dW1b | dw1d], dW2, dW3 via
    the edge outer sums, LayerNorm / vector partials) on the side stream, deferred.

    Parameters in module order: mlp_msg.0.{weight (d, 2d+1), bias}, mlp_msg.1.{weight, bias},
    mlp_msg.3.{weight, bias}, mlp_msg.4.{weight, bias}, mlp_pos.0.{weight, bias},
    mlp_pos.1.{weight, bias}, mlp_pos.3.{weight (1, d), bias}.
    Returns (m_aggr (N, d), pos_aggr (N, 3)).  AB: the node projections precomputed by the
    previous layer's K15 node update (EgnnNodeFn), a constant here: the gradient w.r.t. h still
    comes from this Function's backward (dh = [dA | dB] [W1a ; W1b]).
    """

    @staticmethod
    def forward(ctx, h, pos, graph, act, msg_mean, eps, W1, b1, ln1w, ln1b, W2, b2, ln2w, ln2b,
                W3, b3, ln3w, ln3b, w4, b4, grad_mode=True, AB=None):
        h, pos = _f32c(h), _f32c(pos)
        _need_cuda(h, pos, W1)
        N, d = h.shape
        E = graph.num_edges
        if AB is None:  # [h W1a^T | h W1b^T] (else: K15 produced it with the previous update)
            Wcat = torch.cat([W1[:, :d], W1[:, d:2 * d]], 0)
            AB = h.mm(Wcat.t())
        params = tuple(_f32c(t) for t in (W1[:, 2 * d], b1, ln1w, ln1b, W2, b2, ln2w, ln2b, W3,
                                          b3, ln3w, ln3b, w4, b4))
        # save the LayerNorm outputs only for a backward: grad_mode is the CALLER's
        # torch.is_grad_enabled() (forward() itself always runs with grad disabled, and
        # needs_input_grad follows requires_grad alone: r04's inference forward saved 1 GB of
        # x_hat planes per layer under torch.no_grad)
        train = bool(grad_mode) and any(ctx.needs_input_grad)
        with _timed("egnn_edge_fwd"):
            m_aggr, pos_aggr, xhat, rstd = _lib.torch_ops().egnn_edge_fwd(
                AB, pos, graph.rowptr, graph.recv, graph.send, list(params), _lib.ACT[act],
                bool(msg_mean), float(eps), train, EGNN_XHAT_PLANES)
        ctx.graph, ctx.act, ctx.msg_mean, ctx.N = graph, act, msg_mean, N
        if train:
            ctx.save_for_backward(h, pos, xhat, rstd, W1, *params)
        return m_aggr, pos_aggr

    @staticmethod
    @once_differentiable
    def backward(ctx, g_m, g_p):
        h, pos, xhat, rstd, W1, *params = ctx.saved_tensors
        graph = ctx.graph
        N, d = ctx.N, xhat.shape[2]
        E = graph.num_edges
        dev = pos.device
        g_m = torch.zeros((N, d), device=dev) if g_m is None else _f32c(g_m)
        g_p = torch.zeros((N, 3), device=dev) if g_p is None else _f32c(g_p)
        f = dict(dtype=torch.float32, device=dev)
        # HF weight-gradient outer sums: the backward kernel folds max |dpre2|, |dpre3| into
        # two device words that scale their fp16 planes
        amax = torch.zeros(2, dtype=torch.int32, device=dev)
        with _timed("egnn_edge_bwd"):
            dA, dpos_recv, dpre1, gdiff, dpre2, dpre3, partials = \
                _lib.torch_ops().egnn_edge_bwd(pos, graph.rowptr, graph.recv, graph.send,
                                               list(params), _lib.ACT[ctx.act],
                                               bool(ctx.msg_mean), xhat, rstd, g_m, g_p, amax)
        xh1, xh2 = xhat[0], xhat[1]  # for the dW2 / dW3 sums
        # critical path: sender-side sums (deterministic, sender CSR) and dh
        dB, _ = segment_reduce(dpre1, graph.send_csr, "sum")
        dpos_send, _ = segment_reduce(gdiff, graph.send_csr, "sum")
        W1t = W1[:, :2 * d].t().contiguous()  # [W1a | W1b]^T: NT-form GEMMs for dh
        dh = _mm_wt(dA, W1t[:d])
        dh.addmm_(dB, W1t[d:].t())
        dpos = dpos_recv - dpos_send

        # weight gradients: side stream, accumulated at the end of the backward pass
        (_, b1, ln1w, ln1b, W2, b2, ln2w, ln2b, W3, b3, ln3w, ln3b, w4, b4) = params
        # the edge-level sums (dW2, dW3: ~0.2 ms each) inline on the main stream (r05): on the
        # side stream they took the CUs from the critical path's node-level backward kernels
        # (LayerNorm backward + its column sums 0.33 ms instead of ~0.04 ms per layer, trace);
        # A/B on one box, 20-step runs: 114.4 (113.7-115.0) vs 113.2 (112.9-113.4) M edges/s
        dW2, db2 = edge_outer_sum_act(dpre2, xh1, ln1w, ln1b, ctx.act, amax[0:1])
        dW3, db3 = edge_outer_sum_act(dpre3, xh2, ln2w, ln2b, ctx.act, amax[1:2])
        with side_work(h, dA, dB, partials) as sw:
            dW1 = torch.empty((d, 2 * d + 1), **f)
            db1 = torch.empty(d, **f)
            outer_sum_into(dA, h, dW1[:, :d], db1)
            outer_sum_into(dB, h, dW1[:, d:2 * d])
            v = partials.sum(0)
            dln1w, dln1b, dln2w, dln2b, dln3w, dln3b, dw4, dw1d = v[:8 * d].view(8, d).unbind(0)
            dW1[:, 2 * d].copy_(dw1d)
            grads = (dW1, db1, dln1w, dln1b, dW2, db2, dln2w, dln2b, dW3, db3, dln3w, dln3b,
                     dw4.view(1, d), v[8 * d:8 * d + 1])
        # the caller's parameter tensors (saved tensors unpack to the same objects): W1 itself,
        # then b1 ... b4 (params[0] is the contiguous copy of W1's distance column)
        targets = (W1,) + tuple(params[1:])
        return (dh, dpos, None, None, None, None) + sw.deliver(ctx.needs_input_grad, 6, targets,
                                                               grads) + (None, None)


def egnn_exact_mode():
    """True while the EGNN kernels run their exact-f32 A/B mode (gmp_egnn_set_f32_mfma(1))."""
    lib = _lib.load()
    prev = lib.gmp_egnn_set_f32_mfma(0)
    lib.gmp_egnn_set_f32_mfma(prev)
    return bool(prev)


def egnn_node_images(layers, next_layers):
    """uint8 (L, bytes) K15 weight images (gmp_egnn_node_image_f32, one launch): per EGNN layer
    its mlp_upd.0 / mlp_upd.3 weights and the next layer's mlp_msg.0 weight (None: last layer).
    A constant for autograd (built from the current weights; rebuilt every forward)."""
    with torch.no_grad():
        return _lib.torch_ops().egnn_node_image(
            [_f32c(l.mlp_upd[0].weight) for l in layers], [_f32c(l.mlp_upd[3].weight) for l in layers],
            [None if n is None else n.mlp_msg[0].weight for n in next_layers])


# False: the node update's backward as the composed kernels (K12 LayerNorm backwards + library
# GEMMs; tests compare the two)
EGNN_NODE_BWD_FUSED = True


class EgnnNodeFn(torch.autograd.Function):
    """K15 (gmp_egnn_node_fwd_f32): the EGNN node update of one layer (egnn_layer.py:82-86,
    mlp_upd over [h | m_aggr]), the model's residual (egnn.py:75-76) and the next layer's node
    projections AB' = [h' W1a'^T | h' W1b'^T] in one launch, from the layer's weight image
    (egnn_node_images).  Returns (h', AB' or None) — AB' is a constant for autograd (the next
    EgnnMessageFn differentiates through h').  Backward: the LayerNorm + act backwards (K12) from
    the saved x_hat / 1/std, the dx GEMMs on the critical path, the weight gradients by the
    deterministic outer sums on the side stream (deferred), as the unfused SplitLinearFn /
    LnActFn / EdgeLinearFn chain does."""

    @staticmethod
    def forward(ctx, h, m, W0, b0, ln1w, ln1b, W3, b3, ln2w, ln2b, image, with_ab, act, residual,
                eps, grad_mode):
        h, m = _f32c(h), _f32c(m)
        _need_cuda(h, m, W0)
        vecs = [_f32c(t) for t in (b0, ln1w, ln1b, b3, ln2w, ln2b)]
        train = bool(grad_mode) and any(ctx.needs_input_grad)
        with _timed("egnn_node_fwd"):
            ho, ab, xhat, rstd = _lib.torch_ops().egnn_node_fwd(
                h, m, vecs, image, bool(with_ab), _lib.ACT[act], bool(residual), float(eps), train)
        ctx.act, ctx.residual = act, bool(residual)
        if train:
            ctx.save_for_backward(h, m, xhat, rstd, _f32c(W0), vecs[0], vecs[1], vecs[2],
                                  _f32c(W3), vecs[3], vecs[4], vecs[5])
        ctx.mark_non_differentiable(ab)
        return ho, (ab if with_ab else None)

    @staticmethod
    @once_differentiable
    def backward(ctx, g, _g_ab):
        h, m, xhat, rstd, W0, b0, ln1w, ln1b, W3, b3, ln2w, ln2b = ctx.saved_tensors
        d = h.shape[1]
        g = _f32c(g)
        tops = _lib.torch_ops()
        a = _LN_ACT[ctx.act]
        if EGNN_NODE_BWD_FUSED and a in (0, 1) and d in (32, 64, 128):
            # K15b: both LayerNorm + act backwards, the three dx products and the residual in
            # one launch (gmp_egnn_node_bwd_f32)
            with _timed("egnn_node_bwd"):
                dh, dm, dpre1, dpre2, gb = tops.egnn_node_bwd(g, xhat, rstd, W0, W3,
                                                              [ln1w, ln1b, ln2w, ln2b], a,
                                                              ctx.residual)
            gb1, gb2 = gb[:2 * d], gb[2 * d:]
            dh = dh if ctx.needs_input_grad[0] else None
            dm = dm if ctx.needs_input_grad[1] else None
        else:
            dpre2, gb2 = tops.ln_act_bwd(g, xhat[1], rstd[1], ln2w, ln2b, a)
            dx1 = _dx(dpre2, W3)
            dpre1, gb1 = tops.ln_act_bwd(dx1, xhat[0], rstd[0], ln1w, ln1b, a)
            dh = _dx(dpre1, W0[:, :d]) if ctx.needs_input_grad[0] else None
            if dh is not None and ctx.residual:
                dh += g
            dm = _dx(dpre1, W0[:, d:]) if ctx.needs_input_grad[1] else None
        with side_work(dpre1, dpre2, h, m, xhat) as sw:
            dW0 = torch.empty_like(W0)
            db0 = torch.empty_like(b0)
            outer_sum_into(dpre1, h, dW0[:, :d], db0)
            outer_sum_into(dpre1, m, dW0[:, d:], None)
            dW3 = torch.empty_like(W3)
            db3 = torch.empty_like(b3)
            # x1 = act(x_hat1 ln1w + ln1b), rebuilt at load time
            outer_sum_into(dpre2, xhat[0], dW3, db3, ctx.act, ln1w, ln1b)
        grads = (dW0, db0, gb1[:d], gb1[d:], dW3, db3, gb2[:d], gb2[d:])
        return ((dh, dm) + sw.deliver(ctx.needs_input_grad, 2,
                                      (W0, b0, ln1w, ln1b, W3, b3, ln2w, ln2b), grads)
                + (None, None, None, None, None, None))
