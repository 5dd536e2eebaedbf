"""Data-parallel plumbing for the weak-scaling path: one process per GPU, graphs
sharded by index (rank r owns graphs r, r + W, r + 2W, ...), gradients all-reduced by DDP over
RCCL ("nccl" backend on ROCm; "gloo" in the CPU tests).  No data-path collective."""
import os

import torch
import torch.distributed as dist


def env_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl", force=False):
    """Initialise the default process group from torchrun's env (MASTER_ADDR 127.0.0.1); at
    WORLD_SIZE 1 only when `force` (a one-rank group: the collectives' code path on one GPU)."""
    rank, world, local = env_world()
    if (world > 1 or force) and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard(n_items, rank, world):
    """Round-robin ownership: items r, r + W, ... (balanced to within one item)."""
    return list(range(rank, n_items, world))


def max_over_ranks(x, device=None):
    """Max of a host float over all ranks (the bench's step time)."""
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def sum_over_ranks(x, device=None):
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return t.item()


def barrier(cuda=True):
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    if cuda and torch.cuda.is_available():
        torch.cuda.synchronize()


def wrap_ddp(model, local=None, bucket_cap_mb=32, find_unused_parameters=True):
    """DDP with buckets sized for xGMI ring all-reduce (few, large buckets).
    find_unused_parameters: the reference models leave parameters without gradient (EGNN's last
    position MLP, TFN/MACE readout slices), which a plain DDP reducer would wait for forever."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    # DDP's reducer hooks each parameter's gradient accumulation: weight gradients must reach
    # autograd, not the end-of-backward deferral (ops.DEFER_WEIGHT_GRADS)
    from . import ops
    ops.DEFER_WEIGHT_GRADS = False
    ids = [local] if local is not None else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids,
                                                     bucket_cap_mb=bucket_cap_mb,
                                                     find_unused_parameters=find_unused_parameters)
