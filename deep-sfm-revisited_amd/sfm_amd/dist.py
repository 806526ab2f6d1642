"""One process per GPU: image pairs shard across ranks with no data-path
collective; RCCL (backend "nccl" on ROCm) or gloo is used only to gather
per-pair outputs / validation metrics to rank 0 and to reduce timings.

Replaces the reference's single-process torch.nn.DataParallel (main.py:219),
whose implicit per-forward parameter broadcast / scatter / gather has no
counterpart here: pairs are independent units.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init(backend=None):
    """Initialise the default process group from torchrun's environment (no-op for world 1)."""
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def shard(num_pairs, rank, world):
    """Contiguous block of pair indices for `rank` (sizes differ by at most one)."""
    base, extra = divmod(int(num_pairs), int(world))
    start = rank * base + min(rank, extra)
    stop = start + base + (1 if rank < extra else 0)
    return range(start, stop)


def gather_rows(t, world):
    """All-gather a [n_local, k] tensor whose n_local may differ per rank;
    returns the concatenation in rank order (every rank receives it)."""
    if world == 1 or not dist.is_initialized():
        return t
    n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((m,) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
    pad[: t.shape[0]] = t
    bufs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[: int(s.item())] for b, s in zip(bufs, sizes)], 0)


def reduce_max(value, device=None):
    """Max of a Python float over ranks (timing: the slowest rank defines the step)."""
    if not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_initialized():
        if dist.get_backend() == "nccl" and device is not None:
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
