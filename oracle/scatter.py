"""torch_scatter.scatter semantics on CPU (TEST INFRASTRUCTURE; see oracle/__init__.py).

Follows the call sites models/layers/egnn_layer.py:77,79, models/layers/tfn_layer.py:87,
models/layers/gvp_layer.py:415 and PyG's default aggregate / global pools:
  out[index[e]] (+)= src[e]; rows = dim_size or index.max()+1; empty rows are 0;
  mean = sum / count.clamp(min=1); max / min: empty rows 0.
scatter_arg: torch_scatter.scatter_max / scatter_min's (values, arg) with arg = src.size(dim)
for empty rows and the first (lowest-index) item among ties, by a plain loop (small inputs).
out= (torch_scatter 2.x, restated: scatter.py / scatter_{max,min} of that package): rows =
out.size(dim); sum adds into out (out.scatter_add_), mean = (out + sum) / count.clamp(1);
max / min include out's values in the reduction (rows that receive nothing keep them; arg =
src.size(dim) where out's value wins).
"""
import torch


def _rows(index, dim_size):
    if dim_size is not None:
        return int(dim_size)
    return int(index.max()) + 1 if index.numel() else 0


def scatter(src, index, dim=0, dim_size=None, reduce="sum", out=None):
    dim = dim % src.dim()
    if out is not None:
        o = out.movedim(dim, 0)
        n = o.shape[0]
        x = src.movedim(dim, 0)
        if reduce in ("sum", "add", "mean"):
            r = o + scatter(src, index, dim, n, "sum").movedim(dim, 0)
            if reduce == "mean":
                cnt = torch.zeros(n, dtype=src.dtype, device=src.device)
                cnt.index_add_(0, index, torch.ones(index.shape[0], dtype=src.dtype, device=src.device))
                r = r / cnt.clamp(min=1).view((n,) + (1,) * (r.dim() - 1))
        else:
            idx = index.view((-1,) + (1,) * (x.dim() - 1)).expand_as(x)
            r = o.scatter_reduce(0, idx, x, reduce="amax" if reduce == "max" else "amin",
                                 include_self=True)
        return r.movedim(0, dim)
    n = _rows(index, dim_size)
    x = src.movedim(dim, 0)
    shape = (n,) + tuple(x.shape[1:])
    if reduce in ("sum", "add", "mean"):
        out = torch.zeros(shape, dtype=src.dtype, device=src.device)
        out.index_add_(0, index, x)
        if reduce == "mean":
            cnt = torch.zeros(n, dtype=src.dtype, device=src.device)
            cnt.index_add_(0, index, torch.ones(index.shape[0], dtype=src.dtype, device=src.device))
            out = out / cnt.clamp(min=1).view((n,) + (1,) * (out.dim() - 1))
    elif reduce == "max":
        out = torch.full(shape, float("-inf"), dtype=src.dtype, device=src.device)
        idx = index.view((-1,) + (1,) * (x.dim() - 1)).expand_as(x)
        out = out.scatter_reduce(0, idx, x, reduce="amax", include_self=True)
        out = torch.where(torch.isinf(out) & (out < 0), torch.zeros_like(out), out)
    elif reduce == "min":
        out = torch.full(shape, float("inf"), dtype=src.dtype, device=src.device)
        idx = index.view((-1,) + (1,) * (x.dim() - 1)).expand_as(x)
        out = out.scatter_reduce(0, idx, x, reduce="amin", include_self=True)
        out = torch.where(torch.isinf(out) & (out > 0), torch.zeros_like(out), out)
    else:
        raise ValueError(reduce)
    return out.movedim(0, dim)


def scatter_arg(src, index, dim_size, reduce, out=None):
    """(values, arg) along dim 0 of a 2-D src for reduce in {max, min}; with `out` its values
    take part (torch_scatter: a src item equal to out's value wins the arg)."""
    n = out.shape[0] if out is not None else _rows(index, dim_size)
    E, F = src.shape
    val = torch.zeros((n, F), dtype=src.dtype) if out is None else out.clone()
    arg = torch.full((n, F), E, dtype=torch.int64)
    seen = torch.zeros((n, F), dtype=torch.bool) if out is None else torch.ones((n, F),
                                                                               dtype=torch.bool)
    for e in range(E):
        s = int(index[e])
        for f in range(F):
            v = src[e, f]
            if out is not None and arg[s, f] == E:
                better = (v >= val[s, f]) if reduce == "max" else (v <= val[s, f])
            else:
                better = (v > val[s, f]) if reduce == "max" else (v < val[s, f])
            if not seen[s, f] or better:
                val[s, f], arg[s, f], seen[s, f] = v, e, True
    return val, arg


def global_add_pool(x, batch, size=None):
    return scatter(x, batch, 0, size if size is not None else int(batch.max()) + 1, "sum")


def global_mean_pool(x, batch, size=None):
    return scatter(x, batch, 0, size if size is not None else int(batch.max()) + 1, "mean")
