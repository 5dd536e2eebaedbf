"""Training-step executor: the reference step (experiments/utils/train_utils.py:128-139: forward,
loss, backward, optimizer step) replayed from a HIP graph.

An EGNN step at 1M edges launches ~400 kernels, most of them a few microseconds long (node-level
LayerNorm / linear / reduction / bookkeeping kernels between the fused edge kernels).  Launched
eagerly from Python, the host cannot keep the GPU fed through those stretches: the rocprofv3
trace of the eager step shows ~1.9 ms of idle gaps per 13 ms step.  With static inputs
(one resident graph per rank) the whole step is captured once into a hipGraph
(`torch.cuda.CUDAGraph`) and replayed: the same kernels in the same order, no host launch
path between them.

Multi-GPU (weak scaling): the graph holds this rank's forward + backward; the
gradients are then averaged with ONE all-reduce over a flat buffer (RCCL over xGMI; the EGNN
gradient is 1.9 MB, so one collective outside the graph costs less than per-bucket overlap
inside it), and the optimizer step replays from a second graph.  Parameters are broadcast from
rank 0 at construction, as DDP does.

Requirements for capture: every op on the step's path launches on the current stream without
host synchronisation (true of gmp_amd's ops once the per-graph CSR caches are built, which the
eager warm-up steps do) and the optimizer is constructed with `capturable=True`.
"""
import torch
import torch.distributed as dist


def _dist_world():
    """World size of the initialised process group, or 0 when there is none (a one-rank group
    still runs the collectives: RCCL's one-rank all-reduce is the same code path)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 0


class GraphedStep:
    """step() == zero_grad(set_to_none) ; loss_fn().backward() ; [all-reduce grads] ; opt.step().

    loss_fn: closure computing the scalar loss from static (resident) inputs.
    use_graph: capture into HIP graphs (CUDA tensors only); False runs the identical sequence
    eagerly (CPU / gloo tests, debugging).
    """

    def __init__(self, model, loss_fn, opt, warmup=3, use_graph=True):
        self.model, self.loss_fn, self.opt = model, loss_fn, opt
        self.world = _dist_world()
        self.use_graph = use_graph
        self.params = [p for p in model.parameters() if p.requires_grad]
        if self.world:
            with torch.no_grad():
                for p in model.parameters():
                    dist.broadcast(p, 0)
        self.graph = self.graph_opt = None
        self.loss = None
        if use_graph:
            self._capture(warmup)
        else:
            for _ in range(warmup):
                self._eager()

    # ------------------------------------------------------------------ eager reference path
    def _fwd_bwd(self):
        self.opt.zero_grad(set_to_none=True)
        loss = self.loss_fn()
        loss.backward()
        return loss

    def _allreduce(self):
        if not self.world:
            return
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        for p, g in zip(self.params, grads):
            p.grad = g
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)
        flat.div_(self.world)
        torch._foreach_copy_(grads, [t.view_as(g) for t, g in
                                     zip(torch.split(flat, [g.numel() for g in grads]), grads)])

    def _eager(self):
        self.loss = self._fwd_bwd()
        self._allreduce()
        self.opt.step()

    # ------------------------------------------------------------------ graph path
    def _capture(self, warmup):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up (builds caches) off the default stream
            for _ in range(max(1, warmup)):
                self._eager()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.opt.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = self.loss_fn()
            self.loss.backward()
            if not self.world:
                self.opt.step()
        if self.world:
            # grads are static tensors now; the all-reduce runs eagerly between the graphs
            for p in self.params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            self.graph_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_opt):
                self.opt.step()

    def __call__(self):
        if not self.use_graph:
            self._eager()
            return self.loss
        self.graph.replay()
        if self.world:
            self._allreduce()
            self.graph_opt.replay()
        return self.loss
