"""The torch.ops.gmp boundary (csrc/torch/gmp_torch.cpp): argument checks raise RuntimeError
instead of reaching a kernel with a bad shape, ops run on their inputs' device, and the
torch_scatter `out=` semantics of gmp_amd.scatter* (reference call sites: PyG aggregate and
models/layers/egnn_layer.py:77,79, tfn_layer.py:87; torch_scatter 2.x restated in
oracle/scatter.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    import gmp_amd  # noqa: F401
    from gmp_amd import _lib
    return _lib.torch_ops()


@pytest.mark.parametrize("reduce", ["sum", "add", "mean", "max", "min"])
def test_scatter_out_semantics(reduce):
    """out= takes part as torch_scatter's does: sum / mean accumulate into it (mean divides by
    the clamped count), max / min include its values, rows that receive nothing keep them."""
    from gmp_amd import scatter, scatter_max, scatter_min
    from oracle.scatter import scatter as oscatter, scatter_arg
    g = torch.Generator().manual_seed(5)
    src = torch.randint(-5, 6, (400, 6), generator=g).float()
    idx = torch.randint(0, 50, (400,), generator=g)
    idx[idx == 7] = 8  # an empty row
    out0 = torch.randint(-5, 6, (60, 6), generator=g).float()
    out = out0.to(DEV)
    r = scatter(src.to(DEV), idx.to(DEV), 0, out=out, reduce=reduce)
    assert r is out
    want = oscatter(src, idx, 0, reduce=reduce, out=out0.clone())
    torch.testing.assert_close(out.cpu(), want, atol=1e-6, rtol=1e-6)
    if reduce in ("max", "min"):
        fn = scatter_max if reduce == "max" else scatter_min
        out = out0.to(DEV)
        val, arg = fn(src.to(DEV), idx.to(DEV), 0, out=out)
        wv, wa = scatter_arg(src, idx, None, reduce, out=out0.clone())
        assert torch.equal(val.cpu(), wv) and torch.equal(arg.cpu(), wa)
        assert torch.equal(out.cpu()[7], out0[7]) and (arg.cpu()[7] == 400).all()


@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
@pytest.mark.parametrize("how", ["out", "dim_size"])
def test_scatter_fixed_rows_range_checked(reduce, how):
    """An index outside the rows fixed by out= or dim_size raises IndexError, as torch_scatter
    raises, instead of dropping the item."""
    from gmp_amd import scatter
    src = torch.randn(40, 3, device=DEV)
    idx = torch.arange(40, device=DEV) % 12  # rows 0..11
    kw = {"out": torch.zeros(10, 3, device=DEV)} if how == "out" else {"dim_size": 10}
    with pytest.raises(IndexError):
        scatter(src, idx, 0, reduce=reduce, **kw)
    kw = {"out": torch.zeros(12, 3, device=DEV)} if how == "out" else {"dim_size": 12}
    scatter(src, idx, 0, reduce=reduce, **kw)  # in range: fine
    torch.cuda.synchronize()


def test_cpu_tensor_raises():
    ops_ = _ops()
    with pytest.raises(RuntimeError, match="HIP device"):
        ops_.gather_rows(torch.zeros(4, 4), torch.zeros(2, dtype=torch.long))


def _bad(fn, *a, match=None):
    with pytest.raises(RuntimeError, match=match):
        fn(*a)
    torch.cuda.synchronize()  # nothing was launched that could fault


def test_shape_checks_index_and_egnn():
    ops_ = _ops()
    f = dict(device=DEV)
    src = torch.randn(10, 4, **f)
    rp = torch.tensor([0, 5, 10], device=DEV)
    _bad(ops_.segment_reduce, src, None, rp, 3, "sum", match="rowptr")
    _bad(ops_.segment_reduce, src, torch.arange(9, device=DEV), rp, 2, "sum", match="perm")
    _bad(ops_.segment_reduce, src.double(), None, rp, 2, "sum", match="dtype")
    _bad(ops_.segment_reduce, src.t(), None, rp, 2, "sum", match="contiguous")
    # EGNN backward: xhat must be (2 or 3, E, d), g_m (N, d)
    N, E, d = 6, 10, 32
    pos = torch.randn(N, 3, **f)
    rowptr = torch.tensor([0, 2, 4, 6, 8, 10, 10], device=DEV)
    recv = torch.arange(E, device=DEV) // 2
    send = (recv + 1) % N
    params = [torch.randn(d, **f) for _ in range(4)] + [torch.randn(d, d, **f)] + \
        [torch.randn(d, **f) for _ in range(3)] + [torch.randn(d, d, **f)] + \
        [torch.randn(d, **f) for _ in range(4)] + [torch.randn(1, **f)]
    xh, rs = torch.randn(3, E, d, **f), torch.randn(E, 3, **f)
    gm, gp = torch.randn(N, d, **f), torch.randn(N, 3, **f)
    _bad(ops_.egnn_edge_bwd, pos, rowptr, recv, send, params, 0, False, xh[:1], rs, gm, gp,
         match="xhat")
    _bad(ops_.egnn_edge_bwd, pos, rowptr, recv, send, params, 0, False, xh, rs[:5], gm, gp,
         match="rstd")
    _bad(ops_.egnn_edge_bwd, pos, rowptr, recv, send, params, 0, False, xh, rs, gm[:, :16], gp,
         match="g_m_aggr")
    _bad(ops_.egnn_edge_fwd, torch.randn(N, 2 * d + 1, **f), pos, rowptr, recv, send, params, 0,
         False, 1e-5, True, match="AB")
    _bad(ops_.egnn_edge_fwd, torch.randn(N, 2 * d, **f), pos, rowptr[:-1], recv, send, params, 0,
         False, 1e-5, True, match="rowptr")


def test_shape_checks_cfconv_featurize_rows():
    ops_ = _ops()
    f = dict(device=DEV)
    x, w = torch.randn(6, 8, **f), torch.randn(10, 8, **f)
    xi = torch.randint(0, 6, (10,), device=DEV)
    perm, rp = torch.arange(10, device=DEV), torch.tensor([0, 5, 10], device=DEV)
    _bad(ops_.cfconv_aggregate, x, xi, w, perm, rp, 2, torch.randn(9, **f), match="escale")
    _bad(ops_.cfconv_aggregate, x, xi[:9], w, perm, rp, 2, None, match="xidx")
    _bad(ops_.cfconv_aggregate, x, xi, w, perm[:9], rp, 2, None, match="perm")
    _bad(ops_.cfconv_wgrad, x, xi, x, xi[:3], None, match="xidx")
    pos = torch.randn(6, 3, **f)
    ei = torch.randint(0, 6, (2, 10), device=DEV)
    _bad(ops_.edge_featurize_bwd, pos, ei, [1.0, 2.0], 1.0, 5.0, 6.0, torch.randn(10, 8, **f),
         None, match="g_sh")
    _bad(ops_.edge_featurize, pos, ei[:1], [1.0], 1.0, 5.0, 6.0, match="edge_index")
    _bad(ops_.ln_act_bwd, torch.randn(5, 8, **f), torch.randn(5, 8, **f), torch.randn(4, **f),
         torch.randn(8, **f), torch.randn(8, **f), 0, match="rstd")
    _bad(ops_.ssp_bwd, torch.randn(16, **f), torch.randn(8, **f), match="grad_y")


def test_shape_checks_irreps_sc_gate():
    ops_ = _ops()
    f = dict(device=DEV)
    i32 = dict(device=DEV, dtype=torch.int32)
    x = torch.randn(7, 9 * 4, **f)
    _bad(ops_.gate_bwd, x, torch.randn(7, 20, **f), torch.zeros(35, 4, **i32), 1.0, 1.0,
         match="in_map")
    _bad(ops_.irreps_bn_fwd, x, torch.zeros(30, **i32), torch.zeros(12, **i32),
         torch.zeros(12, 2, **i32), torch.ones(12, **f), None, torch.zeros(4, **f),
         torch.ones(12, **f), True, 0.1, 1e-5, match="col_chan")
    xs = torch.randn(7, 4, 9, **f)
    plan = torch.zeros(3 * 9 + 1 + 5, **i32)  # 9 rows, 5 terms
    _bad(ops_.symmetric_contraction_fwd, xs, plan, 9, torch.randn(6, 4, **f), match="coef")
    _bad(ops_.symmetric_contraction_fwd, xs, plan.long(), 9, torch.randn(5, 4, **f),
         match="plan")
    _bad(ops_.symmetric_contraction_fwd, xs, plan[:20], 9, torch.randn(5, 4, **f), match="plan")
    _bad(ops_.symmetric_contraction_fwd, torch.randn(7, 4, 64, **f), plan, 9,
         torch.randn(5, 4, **f), match="D must")
    _bad(ops_.symmetric_contraction_bwd, xs, plan, 9, torch.randn(5, 4, **f),
         torch.randn(7, 35, **f), match="gout")


def test_shape_checks_tp_and_outer_sums():
    ops_ = _ops()
    f = dict(device=DEV)
    eoff = torch.tensor([0, 3, 5], device=DEV)
    Z, A = torch.randn(6, 32, **f), torch.randn(5, 16, **f)
    T, Tb = torch.randn(2, 32, 16, **f), torch.randn(2, 32, **f)
    _bad(ops_.tp_node_apply, eoff, Z, A, T[:1], Tb, torch.zeros_like(A), torch.zeros_like(Z),
         match="T")
    _bad(ops_.tp_node_apply, eoff, Z, A, T, Tb, torch.zeros(4, 16, **f), torch.zeros_like(Z),
         match="dA")
    _bad(ops_.tp_node_outer, eoff, Z[:, :16], A, 32, match="Z")
    # path GEMM: the epilogue would reach past the end of C
    A1 = torch.randn(64, 32, **f)
    Bp = torch.zeros(3 * 32 * 32, device=DEV, dtype=torch.int16)
    C = torch.zeros(64 * 32 - 1, **f)
    _bad(ops_.tp_gemm_x3, A1, 32, None, 0, Bp, 32, 32, C, 0, 1, 32, 0, 1, False, match="output")
    _bad(ops_.tp_gemm_x3, A1, 32, None, 0, Bp[:100], 32, 32, torch.zeros(64 * 32, **f), 0, 1, 32,
         0, 1, False, match="B planes")
    _bad(ops_.edge_outer_sum_ex, torch.randn(100, 16, **f), torch.randn(100, 16, **f),
         torch.zeros(16, 8, **f), None, -1, None, None, match="C")
    _bad(ops_.edge_outer_sum_ex, torch.randn(100, 16, **f), torch.randn(99, 16, **f),
         torch.zeros(16, 16, **f), None, -1, None, None, match="A")
    _bad(ops_.edge_outer_sum_act, torch.randn(100, 32, **f), torch.randn(100, 32, **f),
         torch.randn(31, **f), torch.randn(32, **f), 0, None, match="w")


def test_shape_checks_gvp():
    ops_ = _ops()
    f = dict(device=DEV)
    s, v = torch.randn(10, 128, **f), torch.randn(10, 16, 3, **f)
    W = [torch.randn(128, 144, **f), torch.randn(128, **f), torch.randn(16, 128, **f),
         torch.randn(16, **f), torch.randn(16, 16, **f), torch.randn(16, 16, **f)]
    _bad(ops_.gvp_layer_fwd, s, v, W[:5], True, match="weight")
    _bad(ops_.gvp_layer_fwd, s, v, [W[0][:, :140]] + W[1:], True, match="weight")
    _bad(ops_.gvp_layer_fwd, s[:, :64], v, W, True, match="s must")
    _bad(ops_.gvp_layer_bwd, s, v, W, s[:5], v, True, match="ds")


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two HIP devices")
def test_op_runs_on_input_device():
    """An op on cuda:1 tensors while cuda:0 is current launches on cuda:1's stream (device
    guard); mixing devices raises."""
    ops_ = _ops()
    src = torch.randn(1000, 8, device="cuda:1")
    idx = torch.randint(0, 30, (1000,), device="cuda:1")
    with torch.cuda.device(0):
        perm, rowptr, *_ = ops_.csr_build(idx, 30, None)
        out, _ = ops_.segment_reduce(src, perm, rowptr, 30, "sum")
        assert out.device == src.device
        want = torch.zeros(30, 8).index_add_(0, idx.cpu(), src.cpu())
        torch.testing.assert_close(out.cpu(), want, atol=1e-5, rtol=1e-5)
        with pytest.raises(RuntimeError, match="device"):
            ops_.segment_reduce(src, perm.to("cuda:0"), rowptr, 30, "sum")


def _compile_case(module, inputs, loss):
    """Eager vs torch.compile(fullgraph=True, backend="eager") of module(*inputs), forward +
    backward: no graph break, same outputs and gradients (inputs and parameters)."""
    from torch._dynamo.utils import counters
    torch._dynamo.reset()

    def run(fn):
        module.zero_grad(set_to_none=True)
        ins = [t.detach().clone().requires_grad_(t.is_floating_point()) for t in inputs]
        out = fn(*ins)
        loss(out).backward()
        torch.cuda.synchronize()
        grads = [t.grad for t in ins if t.is_floating_point()]
        pgrads = {k: p.grad.clone() for k, p in module.named_parameters() if p.grad is not None}
        outs = out if isinstance(out, (tuple, list)) else (out,)
        flat = []
        for o in outs:
            flat.extend(o if isinstance(o, (tuple, list)) else (o,))
        return [o.detach() for o in flat], grads, pgrads

    ref = run(module)
    counters.clear()
    cf = torch.compile(module, fullgraph=True, backend="eager")
    got = run(cf)
    assert not counters["graph_break"], dict(counters["graph_break"])
    for a, b in zip(got[0], ref[0]):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
    for a, b in zip(got[1], ref[1]):
        torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)
    assert got[2].keys() == ref[2].keys() and got[2]
    for k in ref[2]:
        torch.testing.assert_close(got[2][k], ref[2][k], atol=1e-4, rtol=1e-4, msg=k)


def _small_graph(n, e, seed):
    from gmp_amd.graph import radius_graph
    gr = radius_graph(num_nodes=n, target_edges=e, r=2.5, seed=seed, tol=0.3)
    return gr.edge_index.to(DEV), gr.pos.to(DEV), gr.num_nodes


def test_compile_egnn_layer_fullgraph():
    """One EGNN layer (egnn_layer.py:50-86: fused K4 message block, split Linear, LayerNorm
    rows) under torch.compile(fullgraph=True): the torch.ops.gmp operators are opaque nodes,
    the autograd Functions trace forward and backward, zero graph breaks."""
    import gmp_amd
    torch.manual_seed(0)
    ei, pos, n = _small_graph(400, 6000, 1)
    lay = gmp_amd.EGNNLayer(128, "relu", "layer", "sum").to(DEV)
    h = torch.randn(n, 128, device=DEV)
    _compile_case(lay, [h, pos, ei], lambda o: o[0].square().sum() + (o[1] * 0.1).sum())


def test_compile_gvp_conv_layer_fullgraph():
    """One GVPConvLayer at C3 widths (gvp_layer.py:386-438; K5g message kernels, eval mode)."""
    import gmp_amd
    torch.manual_seed(0)
    ei, pos, n = _small_graph(400, 6000, 2)
    E = ei.shape[1]
    lay = gmp_amd.GVPConvLayer((128, 16), (32, 1), activations=(torch.relu, None),
                               vector_gate=True).to(DEV).eval()

    class Wrap(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lay = lay

        def forward(self, s, v, es, ev, ei):
            return self.lay((s, v), ei, (es, ev))

    m = Wrap()
    ins = [torch.randn(n, 128, device=DEV), torch.randn(n, 16, 3, device=DEV),
           torch.randn(E, 32, device=DEV), torch.randn(E, 1, 3, device=DEV), ei]
    _compile_case(m, ins, lambda o: o[0].square().sum() + o[1].square().sum())


def test_compile_tfn_conv_fullgraph():
    """One TFN tensor-product convolution at C5 widths (tfn_layer.py:82-93: K7 node form,
    K7g path GEMMs, Gate) under torch.compile(fullgraph=True)."""
    import gmp_amd
    from gmp_amd import o3
    torch.manual_seed(0)
    ei, pos, n = _small_graph(300, 5000, 3)
    E = ei.shape[1]
    hidden = o3.hidden_irreps(64, 2)
    conv = gmp_amd.TensorProductConvLayer(hidden, hidden, o3.sh_irreps(2), 8, 256,
                                          gate=True).to(DEV)
    ins = [torch.randn(n, o3.irreps_dim(hidden), device=DEV), ei,
           torch.randn(E, 9, device=DEV), torch.rand(E, 8, device=DEV)]

    class Wrap(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = conv

        def forward(self, x, ei, sh, rad):
            return self.conv(x, ei, sh, rad)

    _compile_case(Wrap(), ins, lambda o: o.square().sum())
