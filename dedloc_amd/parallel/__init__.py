"""Process-group management for the collaboration's data plane.

One OS process per GPU peer; all peers of a node share ONE world communicator (RCCL over xGMI on
GPUs, gloo on CPU) created at start-up.  Averaging groups are arbitrary subsets of it driven by
point-to-point operations, so matchmaking never creates communicators.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


def env_rank_world():
    rank = int(os.environ.get("RANK", os.environ.get("LOCAL_RANK", "0")))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_world(backend: Optional[str] = None, timeout_s: float = 600.0, device: Optional[torch.device] = None):
    """Initialise (or reuse) the world process group from torchrun-style env variables.

    Returns (rank, world_size, device).  A single process without MASTER_ADDR runs without a
    process group (world size 1; averaging is then skipped, as in the reference's 1-peer case).
    """
    rank, world, local = env_rank_world()
    if device is None:
        if torch.cuda.is_available():
            device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        else:
            device = torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
        # the first P2P batch must not be the first collective on the communicator
        t = torch.zeros(1, device=device)
        dist.all_reduce(t)
    return rank, world, device


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def shutdown_world():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
