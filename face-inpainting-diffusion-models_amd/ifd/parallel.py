"""Data-parallel image sharding for the sampler: one process per GPU, no per-step communication.

Images are independent through the whole reverse loop (GroupNorm, attention and the sampler
algebra are per sample; t is uniform across the batch), so a batch shards embarrassingly:
rank r samples images [r*B/N, (r+1)*B/N). The only collective is the final gather of the
inpainted images to rank 0 (RCCL all_gather over xGMI on MI355X; gloo on CPU for tests).
"""
from __future__ import annotations

import contextlib
import os
import sys

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment (defaults 0, 1, 0)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_range(global_batch, rank, world_size):
    """Contiguous shard of images for `rank`; sizes differ by at most one."""
    base, extra = divmod(global_batch, world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def device_for(local_rank):
    """The GPU of a local rank. With fewer GPUs than ranks (a rehearsal of the N-rank path on a
    smaller box) ranks share devices round-robin and `init` falls back to gloo, since RCCL needs
    one rank per GPU."""
    n = torch.cuda.device_count()
    return torch.device("cuda", local_rank % n) if n else torch.device("cpu")


@contextlib.contextmanager
def _stdout_to_stderr():
    """File descriptor 1 -> 2 for the block: the process-group setup's native libraries print connection
    notices on stdout (gloo: "[Gloo] Rank r is connected to ..."), which must not mix into rank 0's one
    JSON line (bench.py)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def init(backend=None, device=None):
    """Initialise the default process group when running under torch.distributed.run."""
    rank, ws, local = world()
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            shared = torch.cuda.device_count() < int(os.environ.get("LOCAL_WORLD_SIZE", ws))
            backend = "nccl" if torch.cuda.is_available() and not shared else "gloo"
        with _stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group(backend, device_id=device)
            else:
                dist.init_process_group(backend)
            barrier(device)  # connections made here (lazily connecting backends print at their first collective)
    return rank, ws, local


def barrier(device=None):
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl" and device is not None:
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def max_over_ranks(value, device=None):
    """Max of a host float over all ranks (the bench's job time is the slowest rank's)."""
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_images(local, global_batch):
    """All-gather every rank's [b_r, C, H, W] shard into the full [global_batch, C, H, W] batch
    (returned on every rank; rank 0 is the consumer). Uneven shards are padded to the largest."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    ws = dist.get_world_size()
    sizes = [shard_range(global_batch, r, ws) for r in range(ws)]
    cap = max(hi - lo for lo, hi in sizes)
    src = local if dist.get_backend() == "nccl" else local.cpu()  # gloo: host buffers
    pad = src.new_zeros((cap,) + tuple(src.shape[1:]))
    pad[: src.shape[0]] = src
    out = src.new_empty((ws * cap,) + tuple(src.shape[1:]))
    dist.all_gather_into_tensor(out, pad.contiguous())
    full = torch.cat([out[r * cap: r * cap + (hi - lo)] for r, (lo, hi) in enumerate(sizes)], 0)
    return full.to(local.device)
