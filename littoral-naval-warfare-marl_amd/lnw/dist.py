"""One process per GPU. Environments shard by global id (lnw.shard); the step
has no collective. Collectives are used only off the step path: the bench's
max-over-ranks wall time and optional episode-counter sums (RCCL all_reduce
over xGMI on the GPU box, gloo on CPU)."""
import os

import torch
import torch.distributed as dist

from .shard import env_range  # noqa: F401


def world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def launched():
    """True under a launcher (torch.distributed.run sets TORCHELASTIC_RUN_ID)."""
    return "TORCHELASTIC_RUN_ID" in os.environ


def init(backend=None):
    """Initialise the default process group when launched with WORLD_SIZE > 1,
    or under torch.distributed.run with one rank (the RCCL path then runs with
    a world of one). Returns (world_size, rank, local_rank)."""
    ws, rank, local = world()
    if (ws > 1 or launched()) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return ws, rank, local


def backend():
    """The process group's backend ("nccl" = RCCL on ROCm, "gloo"), or None."""
    return dist.get_backend() if dist.is_initialized() else None


def size():
    """The rank count the process group (RCCL / gloo) reports, or None."""
    return dist.get_world_size() if dist.is_initialized() else None


def _dev():
    return torch.device("cuda", torch.cuda.current_device()) if (
        dist.is_initialized() and dist.get_backend() == "nccl") else torch.device("cpu")


def reduce_max(values):
    """Element-wise max over ranks of a list of floats (the slowest rank's time)."""
    t = torch.tensor(values, dtype=torch.float64, device=_dev())
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def reduce_sum(values):
    t = torch.tensor(values, dtype=torch.float64, device=_dev())
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.cpu()]


def barrier():
    if dist.is_initialized():
        dist.barrier()


def finalize():
    if dist.is_initialized():
        dist.destroy_process_group()
