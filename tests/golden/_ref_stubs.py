"""Plumbing-only stand-ins that let the reference's own layer code be *imported and run*
in this container, for generating golden vectors (see make_golden.py).

The reference depends on torch_geometric / torch_scatter / e3nn, none of which is installed
(SURVEY.md §8(c)).  The modules we load from /root/reference (egnn_layer.py, egnn.py,
gvp_layer.py, gvpgnn.py, mace_modules/radial.py, mace_modules/blocks.py's
RadialEmbeddingBlock) do all their arithmetic in plain torch; the third-party pieces they touch
are pure plumbing:

* ``torch_geometric.nn.MessagePassing.propagate`` — the PyG 2.3.1 `_collect` + message →
  aggregate → update dispatch ("PyG propagate").
* ``torch_scatter.scatter`` — out[index[e]] (+)= src[e]; mean = sum / count.clamp(1);
  rows = dim_size or index.max()+1 ("torch_scatter").
* ``global_add_pool`` / ``global_mean_pool`` — scatter over the batch vector.
* ``e3nn.util.jit.compile_mode`` — a no-op decorator; e3nn ``o3``/``nn`` names used only in
  def-time annotations/defaults of blocks.py (never executed by the modules we run).

This file is test infrastructure used only by make_golden.py in the dev container; it never
travels into the product path.
"""
import inspect
import sys
import types

import torch


# ----------------------------------------------------------------------------- torch_scatter
def _broadcast(src, other, dim):
    if dim < 0:
        dim = other.dim() + dim
    if src.dim() == 1:
        for _ in range(0, dim):
            src = src.unsqueeze(0)
    for _ in range(src.dim(), other.dim()):
        src = src.unsqueeze(-1)
    return src.expand(other.size())


def scatter_sum(src, index, dim=-1, out=None, dim_size=None):
    index = _broadcast(index, src, dim)
    if out is None:
        size = list(src.size())
        if dim_size is not None:
            size[dim] = dim_size
        elif index.numel() == 0:
            size[dim] = 0
        else:
            size[dim] = int(index.max()) + 1
        out = torch.zeros(size, dtype=src.dtype, device=src.device)
    return out.scatter_add_(dim, index, src)


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    out = scatter_sum(src, index, dim, out, dim_size)
    dim_size = out.size(dim)
    index_dim = dim
    if index_dim < 0:
        index_dim = index_dim + src.dim()
    if index.dim() <= index_dim:
        index_dim = index.dim() - 1
    ones = torch.ones(index.size(), dtype=src.dtype, device=src.device)
    count = scatter_sum(ones, index, index_dim, None, dim_size)
    count[count < 1] = 1
    count = _broadcast(count, out, dim)
    if out.is_floating_point():
        out = out / count
    else:
        out = torch.div(out, count, rounding_mode="floor")
    return out


def scatter_min(src, index, dim=-1, out=None, dim_size=None):
    """torch_scatter min (1-D use in spherenet_layer.py:561): rows = index.max()+1; each row
    starts at the dtype's max and takes a value only if it compares smaller (so NaN never wins);
    rows still at max become 0."""
    assert src.dim() == 1 and out is None
    n = dim_size if dim_size is not None else (int(index.max()) + 1 if index.numel() else 0)
    big = torch.finfo(src.dtype).max
    res = torch.full((n,), big, dtype=src.dtype).scatter_reduce(
        0, index, torch.nan_to_num(src, nan=big), "amin", include_self=True)
    res[res == big] = 0
    return res


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    if reduce in ("sum", "add"):
        return scatter_sum(src, index, dim, out, dim_size)
    if reduce == "mean":
        return scatter_mean(src, index, dim, out, dim_size)
    if reduce == "min":
        return scatter_min(src, index, dim, out, dim_size)
    raise ValueError(reduce)


# ----------------------------------------------------------------------------- torch_sparse
class _SparseStorage:
    def __init__(self, row, col, value):
        self._row, self._col, self._value = row, col, value

    def row(self):
        return self._row

    def col(self):
        return self._col

    def value(self):
        return self._value


class SparseTensor:
    """The slice of torch_sparse.SparseTensor that spherenet_layer.py:xyz_to_dat uses: COO
    entries kept sorted row-major (by row * n_cols + col), row selection by an index vector
    (the result's row r holds the entries of row index[r]), set_value(None) and sum(dim=1)
    (entries per row)."""

    def __init__(self, row, col, value=None, sparse_sizes=None, _sorted=False):
        self.sizes = tuple(sparse_sizes) if sparse_sizes is not None else (
            int(row.max()) + 1, int(col.max()) + 1)
        if not _sorted:
            perm = torch.argsort(row * self.sizes[1] + col, stable=True)
            row, col = row[perm], col[perm]
            value = value[perm] if value is not None else None
        self.storage = _SparseStorage(row, col, value)

    def set_value(self, value, layout=None):
        s = self.storage
        return SparseTensor(s.row(), s.col(), value, self.sizes, _sorted=True)

    def sum(self, dim):
        assert dim == 1
        s = self.storage
        v = s.value() if s.value() is not None else torch.ones(s.row().numel())
        return torch.zeros(self.sizes[0], dtype=v.dtype).index_add_(0, s.row(), v)

    def __getitem__(self, index):
        s = self.storage
        counts = torch.bincount(s.row(), minlength=self.sizes[0])
        rowptr = torch.zeros(self.sizes[0] + 1, dtype=torch.long)
        rowptr[1:] = torch.cumsum(counts, 0)
        sel = [torch.arange(int(rowptr[r]), int(rowptr[r + 1])) for r in index.tolist()]
        pos = torch.cat(sel) if sel else torch.zeros(0, dtype=torch.long)
        new_row = torch.repeat_interleave(torch.arange(index.numel()), counts[index])
        val = s.value()[pos] if s.value() is not None else None
        return SparseTensor(new_row, s.col()[pos], val, (index.numel(), self.sizes[1]),
                            _sorted=True)


# ----------------------------------------------------------------------------- PyG
class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2):
        super().__init__()
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim

    def _size(self, kwargs):
        for v in kwargs.values():
            if torch.is_tensor(v):
                return v.size(self.node_dim)
        return None

    def propagate(self, edge_index, size=None, **kwargs):
        j_idx, i_idx = (edge_index[0], edge_index[1]) if self.flow == "source_to_target" else (
            edge_index[1], edge_index[0])
        n = self._size(kwargs)
        msg_kwargs = {}
        for name in inspect.signature(self.message).parameters:
            if name.endswith("_i") and name[:-2] in kwargs:
                msg_kwargs[name] = kwargs[name[:-2]].index_select(self.node_dim, i_idx)
            elif name.endswith("_j") and name[:-2] in kwargs:
                msg_kwargs[name] = kwargs[name[:-2]].index_select(self.node_dim, j_idx)
            elif name == "index":
                msg_kwargs[name] = i_idx
            else:
                msg_kwargs[name] = kwargs[name]
        out = self.message(**msg_kwargs)
        agg_params = inspect.signature(self.aggregate).parameters
        agg_kwargs = {"index": i_idx}
        if "ptr" in agg_params:
            agg_kwargs["ptr"] = None
        if "dim_size" in agg_params:
            agg_kwargs["dim_size"] = n
        out = self.aggregate(out, **agg_kwargs)
        upd_params = list(inspect.signature(self.update).parameters)[1:]
        return self.update(out, **{k: kwargs[k] for k in upd_params})

    def aggregate(self, inputs, index, ptr=None, dim_size=None):
        return scatter(inputs, index, dim=self.node_dim, dim_size=dim_size, reduce=self.aggr)

    def update(self, inputs):
        return inputs


def global_add_pool(x, batch, size=None):
    size = int(batch.max()) + 1 if size is None else size
    return scatter(x, batch, dim=-2, dim_size=size, reduce="sum")


def global_mean_pool(x, batch, size=None):
    size = int(batch.max()) + 1 if size is None else size
    return scatter(x, batch, dim=-2, dim_size=size, reduce="mean")


# ----------------------------------------------------------------------------- e3nn (def-time only)
class _Anything:
    """Accepts any construction / attribute access; used only in def-time annotations/defaults."""

    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Anything()

    def __getattr__(self, name):
        return _Anything()

    def __mul__(self, o):
        return _Anything()

    __rmul__ = __add__ = __radd__ = __mul__


def install():
    tg = types.ModuleType("torch_geometric")
    tgnn = types.ModuleType("torch_geometric.nn")
    tgnn.MessagePassing = MessagePassing
    tgnn.global_add_pool = global_add_pool
    tgnn.global_mean_pool = global_mean_pool
    tg.nn = tgnn
    ts = types.ModuleType("torch_scatter")
    ts.scatter = scatter
    ts.scatter_sum = scatter_sum
    ts.scatter_add = scatter_sum
    ts.scatter_mean = scatter_mean
    ts.scatter_min = scatter_min
    tsp = types.ModuleType("torch_sparse")
    tsp.SparseTensor = SparseTensor
    inits = types.ModuleType("torch_geometric.nn.inits")
    inits.glorot_orthogonal = lambda *a, **k: None
    tgnn.inits = inits

    e3 = types.ModuleType("e3nn")
    util = types.ModuleType("e3nn.util")
    jit = types.ModuleType("e3nn.util.jit")
    jit.compile_mode = lambda mode: (lambda cls: cls)
    codegen = types.ModuleType("e3nn.util.codegen")
    codegen.CodeGenMixin = type("CodeGenMixin", (), {})
    o3 = types.ModuleType("e3nn.o3")
    o3.Irreps = _Anything
    o3.Irrep = _Anything
    o3.Linear = _Anything
    o3.TensorProduct = _Anything
    o3.FullyConnectedTensorProduct = _Anything
    o3.wigner_3j = _Anything()
    enn = types.ModuleType("e3nn.nn")
    enn.Activation = _Anything
    enn.Gate = _Anything
    enn.BatchNorm = _Anything
    e3.o3, e3.nn, e3.util = o3, enn, util
    util.jit, util.codegen = jit, codegen
    oe = types.ModuleType("opt_einsum")
    oe.contract = torch.einsum
    for name, mod in {
        "torch_geometric": tg, "torch_geometric.nn": tgnn, "torch_scatter": ts, "e3nn": e3,
        "e3nn.util": util, "e3nn.util.jit": jit, "e3nn.util.codegen": codegen, "e3nn.o3": o3,
        "e3nn.nn": enn, "opt_einsum": oe, "torch_sparse": tsp,
        "torch_geometric.nn.inits": inits,
    }.items():
        sys.modules[name] = mod


def load_reference(ref_root):
    """Load the reference's pure-torch modules by path under an empty `models` package
    (bypasses models/__init__.py, which eagerly imports the e3nn/PyG-only models)."""
    import importlib.util
    import os

    install()
    pkgs = {"models": "models", "models.layers": "models/layers",
            "models.mace_modules": "models/mace_modules"}
    for name, rel in pkgs.items():
        m = types.ModuleType(name)
        m.__path__ = [os.path.join(ref_root, rel)]
        sys.modules[name] = m
    out = {}
    for name, rel in [
        ("models.layers.egnn_layer", "models/layers/egnn_layer.py"),
        ("models.egnn", "models/egnn.py"),
        ("models.mace_modules.radial", "models/mace_modules/radial.py"),
        ("models.layers.gvp_layer", "models/layers/gvp_layer.py"),
        ("models.mace_modules.blocks", "models/mace_modules/blocks.py"),
        ("models.gvpgnn", "models/gvpgnn.py"),
        ("models.layers.spherenet_layer", "models/layers/spherenet_layer.py"),
    ]:
        spec = importlib.util.spec_from_file_location(name, os.path.join(ref_root, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        out[name] = mod
    return out


# ----------------------------------------------------------------------------- e3nn-lite
def install_e3nn_lite():
    """Replace the def-time e3nn.o3 placeholders with a faithful-enough Irreps/Irrep algebra
    and wigner_3j (restated in oracle/o3.py) so that the reference's own
    models/mace_modules/cg.py and symmetric_contraction.py can run.  Parity of wigner_3j itself
    is unpinned (see oracle/o3.py); everything cg.py / symmetric_contraction.py do on top of it
    is the reference's code."""
    import os
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    if root not in _sys.path:
        _sys.path.insert(0, root)
    from oracle import o3 as oo3

    class Irrep(tuple):
        def __new__(cls, l, p=None):
            if isinstance(l, Irrep):
                return l
            if isinstance(l, str):
                return super().__new__(cls, (int(l[:-1]), {"e": 1, "o": -1}[l[-1]]))
            if isinstance(l, tuple):
                l, p = l
            return super().__new__(cls, (int(l), int(p)))

        l = property(lambda self: self[0])
        p = property(lambda self: self[1])
        dim = property(lambda self: 2 * self[0] + 1)

        def is_scalar(self):
            return self == (0, 1)

        def __mul__(self, other):
            other = Irrep(other)
            for l in range(abs(self.l - other.l), self.l + other.l + 1):
                yield Irrep(l, self.p * other.p)

        def __str__(self):
            return f"{self.l}{'e' if self.p == 1 else 'o'}"

        __repr__ = __str__

    class _MulIr(tuple):
        def __new__(cls, mul, ir):
            return super().__new__(cls, (int(mul), Irrep(ir)))

        mul = property(lambda self: self[0])
        ir = property(lambda self: self[1])
        dim = property(lambda self: self[0] * self[1].dim)

        def __str__(self):
            return f"{self.mul}x{self.ir}"

    class Irreps(tuple):
        def __new__(cls, spec=None):
            if isinstance(spec, Irreps):
                return spec
            items = []
            if spec is None:
                pass
            elif isinstance(spec, Irrep):
                items = [_MulIr(1, spec)]
            elif isinstance(spec, str):
                for m, ir in oo3.Irreps(spec):
                    items.append(_MulIr(m, ir))
            else:
                for x in spec:
                    if isinstance(x, Irrep) or isinstance(x, str):
                        items.append(_MulIr(1, Irrep(x)))
                    else:
                        m, ir = x
                        items.append(_MulIr(m, ir))
            return super().__new__(cls, items)

        dim = property(lambda self: sum(mi.dim for mi in self))

        def count(self, ir):
            ir = Irrep(ir)
            return sum(m for m, i in self if i == ir)

        def __contains__(self, ir):
            ir = Irrep(ir)
            return any(i == ir for _, i in self)

        def __str__(self):
            return "+".join(str(mi) for mi in self)

    o3 = sys.modules["e3nn.o3"]
    o3.Irrep = Irrep
    o3.Irreps = Irreps
    o3.wigner_3j = lambda l1, l2, l3, dtype=None, device=None: oo3.wigner_3j(
        l1, l2, l3, dtype or torch.get_default_dtype())


def load_mace_contraction(ref_root):
    """Load the reference's cg.py and symmetric_contraction.py on top of e3nn-lite."""
    import importlib.util
    import os

    install()
    install_e3nn_lite()
    for name in ("models", "models.mace_modules"):
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.__path__ = [os.path.join(ref_root, name.replace(".", "/"))]
            sys.modules[name] = m
    out = {}
    for name, rel in [("models.mace_modules.cg", "models/mace_modules/cg.py"),
                      ("models.mace_modules.symmetric_contraction",
                       "models/mace_modules/symmetric_contraction.py")]:
        spec = importlib.util.spec_from_file_location(name, os.path.join(ref_root, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        out[name] = mod
    return out
