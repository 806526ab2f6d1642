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
    """Initialise the default process group from torchrun's environment.  A
    plain single process (no WORLD_SIZE / MASTER_PORT) stays without one; a
    torchrun world of 1 gets one, so the RCCL path runs on a one-GPU box too."""
    rank, world, local = env_rank()
    launched = "WORLD_SIZE" in os.environ and "MASTER_PORT" in os.environ
    if (world > 1 or launched) and not dist.is_initialized():
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
    if t.is_cuda and dist.get_backend() == "gloo":      # gloo gathers host tensors only
        return gather_rows(t.cpu(), world).to(t.device)
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
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_initialized():
        if dist.get_backend() == "nccl" and device is not None:
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local(nprocs, argv, env=None):
    """Start ``nprocs`` ranks of ``argv`` (a command line) on this node, one
    process per GPU, with the env torchrun would give them (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT).  The caller must not
    have touched the GPU: the children are fresh processes, never an exec of
    this one.  Returns the first non-zero exit code (0 if all ranks pass); a
    failing rank takes the others down."""
    import subprocess
    import time
    port = free_port()
    procs = []
    for r in range(int(nprocs)):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(argv, env=e))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def device_names(device=None):
    """Per-rank device names, gathered to every rank (rank order)."""
    import torch
    name = torch.cuda.get_device_name(device) if device is not None and device.type == "cuda" else "cpu"
    if not dist.is_initialized():
        return [name]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, name)
    return out
