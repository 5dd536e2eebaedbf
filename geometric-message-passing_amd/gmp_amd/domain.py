"""Spatial domain decomposition of ONE graph over the ranks, with halo exchange (SURVEY.md §8(f)
row f4 — absent from the reference, whose graphs always fit one device).

A graph too large for one GPU's HBM, or one graph to be processed by several GPUs, is cut into
W slabs along one axis at the node-coordinate quantiles: rank r owns the nodes of slab r and
every edge whose receiver (edge_index[1], the aggregation index of the PyG layers) it owns.  A
message-passing layer then needs, for its owned receivers, the current features of all their
senders; the senders owned by other ranks are this rank's halo ("ghost") nodes.

  forward, before every layer: each owner gathers the rows other ranks hold as ghosts and ONE
      all_to_all (RCCL over xGMI; pairwise send / recv under gloo) delivers them; the rank runs
      the unchanged layer (the fused HIP kernels) on its local graph [owned | ghost] and keeps
      the owned rows of the result (ghost rows receive no messages locally: discarded);
  backward: the gradient arriving at the ghost rows travels back along the transposed exchange
      and is summed into the owners' rows (deterministic segmented sum on the GPU).

Only sender features cross ranks, once per layer: for a radius graph cut into slabs the halo is
the r-thick boundary layer of each cut, so the exchanged bytes are O(surface), the compute
O(volume).  Parameter gradients: every rank holds the contribution of its own receivers to the
SAME loss, so they are SUM-reduced over the ranks (`allreduce_grads`), unlike data parallelism's
average.  Graph-level readout: pooled owned-node sums (and counts, for mean pooling) are
all-reduced (`global_sum`), the gradient flowing back to each rank's own contribution.
"""
import torch
import torch.distributed as dist


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class DomainPlan:
    """Partition of a graph (host-side, built identically on every rank from the global arrays).

    part[v]      : owning rank of node v (slabs along `axis` at the position quantiles)
    owned        : global ids of this rank's nodes (ascending)          -> local 0 .. n_own-1
    ghosts       : global ids of this rank's halo nodes, ordered by (owner rank, id)
                                                                         -> local n_own ..
    edge_index   : this rank's edges (receiver owned) in local ids, original relative order
    edge_ids     : their positions in the global edge list
    send_idx     : local ids of owned rows to send, grouped by destination rank (ascending)
    send_counts / recv_counts : rows per destination / per source rank
    """

    def __init__(self, pos, edge_index, world=None, rank=None, axis=0):
        r0, w0 = _world()
        self.rank = r0 if rank is None else int(rank)
        self.world = w0 if world is None else int(world)
        pos = pos.detach().cpu()
        ei = edge_index.detach().cpu()
        n = pos.shape[0]
        W = self.world
        # slab cut at the quantiles of the coordinate (ties broken by node id: stable sort)
        order = torch.argsort(pos[:, axis], stable=True)
        part = torch.empty(n, dtype=torch.long)
        part[order] = torch.div(torch.arange(n) * W, max(n, 1), rounding_mode="floor")
        self.part = part
        self.num_nodes_global = n
        src, dst = ei[0], ei[1]
        self.owned = torch.nonzero(part == self.rank).view(-1)
        emask = part[dst] == self.rank
        self.edge_ids = torch.nonzero(emask).view(-1)
        lsrc, ldst = src[emask], dst[emask]
        ghost = torch.unique(lsrc[part[lsrc] != self.rank])
        ghost = ghost[torch.argsort(part[ghost] * n + ghost)]  # by owner, then id
        self.ghosts = ghost
        self.n_own, self.n_ghost = self.owned.numel(), ghost.numel()
        loc = torch.full((n,), -1, dtype=torch.long)
        loc[self.owned] = torch.arange(self.n_own)
        loc[ghost] = self.n_own + torch.arange(self.n_ghost)
        self.edge_index = torch.stack([loc[lsrc], loc[ldst]])
        self.recv_counts = [int((part[ghost] == q).sum()) for q in range(W)]
        # what every other rank q needs from me: q's ghosts that I own, in q's (id) order
        send, counts = [], []
        for q in range(W):
            if q == self.rank:
                counts.append(0)
                continue
            qs = src[part[dst] == q]
            need = torch.unique(qs[part[qs] == self.rank])
            send.append(loc[need])
            counts.append(need.numel())
        self.send_idx = torch.cat(send) if send else torch.empty(0, dtype=torch.long)
        self.send_counts = counts

    @property
    def num_local(self):
        return self.n_own + self.n_ghost

    def to(self, device):
        for k in ("owned", "ghosts", "edge_index", "edge_ids", "send_idx"):
            setattr(self, k, getattr(self, k).to(device))
        return self

    def halo_bytes(self, row_bytes):
        """Bytes this rank receives per exchange of rows of `row_bytes`."""
        return self.n_ghost * row_bytes


def _exchange(x, send_counts, recv_counts):
    """Rows of x grouped by destination rank -> rows grouped by source rank (all_to_all)."""
    out = x.new_empty((sum(recv_counts),) + tuple(x.shape[1:]))
    if dist.get_backend() == "gloo":  # gloo has no all_to_all: pairwise send / recv
        rank, W = dist.get_rank(), dist.get_world_size()
        if x.is_cuda:  # the gloo rehearsal of device tensors: pairwise transfers through host
            return _exchange(x.cpu(), send_counts, recv_counts).to(x.device)
        sends = torch.split(x, send_counts)
        recvs = torch.split(out, recv_counts)
        ops = []
        for q in range(W):
            if q != rank and send_counts[q]:
                ops.append(dist.P2POp(dist.isend, sends[q].contiguous(), q))
            if q != rank and recv_counts[q]:
                ops.append(dist.P2POp(dist.irecv, recvs[q], q))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return out
    dist.all_to_all_single(out, x.contiguous(), output_split_sizes=recv_counts,
                           input_split_sizes=send_counts)
    return out


def _scatter_add_rows(dst, index, src):
    """dst[index[k]] += src[k]; deterministic on the GPU (segmented sum over a stable CSR)."""
    if src.shape[0] == 0:
        return dst
    if dst.is_cuda:
        from .scatter import scatter
        s = scatter(src.reshape(src.shape[0], -1), index, dim=0, dim_size=dst.shape[0],
                    reduce="sum")
        return dst + s.view_as(dst)
    return dst.index_add(0, index, src)


class HaloExchangeFn(torch.autograd.Function):
    """x_owned (n_own, ...) -> x_local (n_own + n_ghost, ...) = [x_owned | ghost rows]."""

    @staticmethod
    def forward(ctx, x, plan):
        ctx.plan = plan
        ghost = _exchange(x.index_select(0, plan.send_idx), plan.send_counts, plan.recv_counts)
        return torch.cat([x, ghost], 0)

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        g = g.contiguous()
        back = _exchange(g[plan.n_own:], plan.recv_counts, plan.send_counts)
        return _scatter_add_rows(g[:plan.n_own].clone(), plan.send_idx, back), None


def halo(x, plan):
    """[x_owned | current rows of this rank's ghost nodes] (identity for one rank)."""
    if plan.world == 1:
        return x
    return HaloExchangeFn.apply(x, plan)


class _GlobalSumFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = x.detach().clone()
        dist.all_reduce(y)
        return y

    @staticmethod
    def backward(ctx, g):
        return g  # every rank evaluates the same loss on the same reduced value


def global_sum(x):
    """Sum of x over the ranks; the gradient reaches this rank's own contribution."""
    if _world()[1] == 1:
        return x
    return _GlobalSumFn.apply(x)


def allreduce_grads(params, replicated=()):
    """Reduce the parameter gradients over the ranks (one flat collective): SUM for the
    parameters applied to rank-local rows (each rank holds its receivers' share of the
    gradient), MEAN for the `replicated` ones applied after the global readout (every rank
    evaluates them on the same reduced value, e.g. the EGNN `pred` head)."""
    _, W = _world()
    if W == 1:
        return
    params = [p for p in params if p.requires_grad]
    rep = {id(p) for p in replicated}
    grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    for p, t in zip(params, torch.split(flat, [g.numel() for g in grads])):
        p.grad = t.view_as(p) / W if id(p) in rep else t.view_as(p).clone()


def _add_pool(x, batch, size):
    if x.is_cuda:
        from .scatter import global_add_pool
        return global_add_pool(x, batch, size)
    return torch.zeros((size,) + tuple(x.shape[1:]), dtype=x.dtype).index_add(0, batch, x)


def _pool(model, feats, batch, num_graphs):
    """PyG sum / mean pool of the owned rows, completed over the ranks."""
    s = global_sum(_add_pool(feats, batch, num_graphs))
    if getattr(model.pool, "__name__", "") != "global_mean_pool":
        return s
    ones = torch.ones(feats.shape[0], 1, dtype=feats.dtype, device=feats.device)
    return s / global_sum(_add_pool(ones, batch, num_graphs)).clamp(min=1)


def egnn_forward(model, atoms, pos, plan, batch=None, num_graphs=1):
    """models/egnn.py:66-87 over a DomainPlan.  atoms / pos / batch are this rank's OWNED rows
    (plan.owned order); `model` is an EGNNModel whose convs are called as
    conv(h_local, pos_local, plan.edge_index) and return one row per local node.  Returns the
    prediction (identical on every rank)."""
    h = model.emb_in(atoms)
    n_own = plan.n_own
    for conv in model.convs:
        dh, p_new = conv(halo(h, plan), halo(pos, plan), plan.edge_index)
        h = h + dh[:n_own] if model.residual else dh[:n_own]
        pos = p_new[:n_own]
    feats = torch.cat([h, pos], -1) if model.equivariant_pred else h
    if batch is None:
        batch = torch.zeros(n_own, dtype=torch.long, device=h.device)
    return model.pred(_pool(model, feats, batch, num_graphs))
