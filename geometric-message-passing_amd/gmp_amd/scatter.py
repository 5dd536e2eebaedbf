"""torch_scatter-compatible scatter on the MI355X (drop-in for the reference's call sites
models/layers/egnn_layer.py:77,79, models/layers/tfn_layer.py:87, gvp_layer.py:415, PyG
aggregate and pools).

Semantics (torch_scatter 2.x): out rows along `dim` = dim_size or index.max()+1 (the latter
costs one host sync, as in torch_scatter); empty rows are 0; mean = sum / count.clamp(1);
scatter(reduce="max"/"min") returns values, scatter_max / scatter_min return (out, arg) with
arg = src.size(dim) for empty rows (torch_scatter's convention).  Reductions are deterministic
segmented sums over a stable receiver-sorted CSR (torch.ops.gmp.csr_build +
torch.ops.gmp.segment_reduce), not atomics; min is -max(-src) (negation is exact).
out= follows torch_scatter too: rows = out.size(dim); sum adds into out, mean divides
(out + sum) by the clamped count, max / min include out's values (rows that receive nothing keep
them, arg = src.size(dim) where out's value wins).
"""
import torch

from . import ops


def _rows(index, dim_size):
    if dim_size is not None:
        return int(dim_size)
    return int(index.max().item()) + 1 if index.numel() else 0


def _csr(index, n, fixed):
    """The segment CSR of `index`; when out= or dim_size fixes the row count, an index outside it
    raises IndexError (checked once per graph), as torch_scatter does — max(index) + 1 rows
    cannot be exceeded."""
    return ops.checked_csr(index, n) if fixed else ops.get_csr(index, n)


def _bcast(v, like, dim):
    """(n,) per-row values broadcast along `dim` of `like`."""
    shp = [1] * like.dim()
    shp[dim] = -1
    return v.view(shp)


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    if reduce not in ("sum", "add", "mean", "max", "min"):
        raise ValueError(f"unsupported reduce {reduce!r}")
    if reduce in ("max", "min"):
        o = _scatter_arg(src, index, dim, dim_size, reduce, out)[0]
        return o
    dim = dim % src.dim()
    if index.dim() != 1:
        # torch_scatter broadcasts index; the reference always passes a 1-D index along dim
        raise NotImplementedError("gmp scatter supports 1-D index along `dim`")
    n = out.shape[dim] if out is not None else _rows(index, dim_size)
    x = src.movedim(dim, 0)
    shp = x.shape
    x2 = x.reshape(shp[0], -1)
    csr = _csr(index, n, out is not None or dim_size is not None)
    red = "sum" if reduce == "add" else reduce
    if out is None:
        return ops.SegmentReduceFn.apply(x2, csr, red).reshape((n,) + tuple(shp[1:])).movedim(0,
                                                                                            dim)
    o = ops.SegmentReduceFn.apply(x2, csr, "sum").reshape((n,) + tuple(shp[1:])).movedim(0, dim)
    out.add_(o)
    if red == "mean":
        out.div_(_bcast(csr.counts().clamp(min=1).to(out.dtype), out, dim))
    return out


def scatter_sum(src, index, dim=-1, out=None, dim_size=None):
    return scatter(src, index, dim, out, dim_size, "sum")


scatter_add = scatter_sum


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    return scatter(src, index, dim, out, dim_size, "mean")


def _scatter_arg(src, index, dim, dim_size, reduce, out=None):
    dim = dim % src.dim()
    if index.dim() != 1:
        raise NotImplementedError("gmp scatter supports 1-D index along `dim`")
    n = out.shape[dim] if out is not None else _rows(index, dim_size)
    x = src.movedim(dim, 0)
    shp = x.shape
    x2 = x.reshape(shp[0], -1)
    csr = _csr(index, n, out is not None or dim_size is not None)
    if reduce == "min":
        o, arg = ops.SegmentMaxFn.apply(-x2, csr)
        o = 0.0 - o  # (+0 for empty rows, not -0)
    else:
        o, arg = ops.SegmentMaxFn.apply(x2, csr)
    o = o.reshape((n,) + tuple(shp[1:])).movedim(0, dim)
    arg = arg.reshape((n,) + tuple(shp[1:])).movedim(0, dim)
    if out is not None:
        # out's values take part in the reduction: a segment value wins where it is >= (max) /
        # <= (min) out's and the segment is not empty; elsewhere out keeps its value
        nonempty = _bcast(csr.counts() > 0, o, dim)
        win = nonempty & ((o >= out) if reduce == "max" else (o <= out))
        arg = torch.where(win, arg, torch.full_like(arg, src.shape[dim]))
        out.copy_(torch.where(win, o, out))
        o = out
    return o, arg


def scatter_max(src, index, dim=-1, out=None, dim_size=None):
    """torch_scatter.scatter_max: (max values, argmax along dim)."""
    return _scatter_arg(src, index, dim, dim_size, "max", out)


def scatter_min(src, index, dim=-1, out=None, dim_size=None):
    """torch_scatter.scatter_min: (min values, argmin along dim)."""
    return _scatter_arg(src, index, dim, dim_size, "min", out)


def global_add_pool(x, batch, size=None):
    """PyG global_add_pool: sum over nodes of each graph (batch vector)."""
    if batch is None:
        return x.sum(dim=-2, keepdim=x.dim() == 1)
    return scatter(x, batch, dim=-2, dim_size=size, reduce="sum")


def global_mean_pool(x, batch, size=None):
    if batch is None:
        return x.mean(dim=-2, keepdim=x.dim() == 1)
    return scatter(x, batch, dim=-2, dim_size=size, reduce="mean")
