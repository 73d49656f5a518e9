"""Data-plane communicators for an open-membership collaboration.

There is no launch-time world: a peer is a process with a DHT client and (normally) one GPU.  Every
matchmade averaging group builds its own communicator through the DHT (``comm.GroupCommunicators``:
native RCCL for all-GPU groups, gloo when a CPU peer is a member), so a process that never took
part in any launch — a volunteer, a respawned spot instance — joins the next round like any other
peer.  The only process-local input is which GPU to use.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .comm import CommError, GlooGroupComm, GroupCommunicators, RcclGroupComm, pairwise_rccl, rccl_available

__all__ = ["CommError", "GlooGroupComm", "GroupCommunicators", "RcclGroupComm", "pairwise_rccl", "rccl_available",
           "local_device"]


def local_device(device: Optional[torch.device] = None) -> torch.device:
    """This peer's device: ``device`` if given, else GPU ``LOCAL_RANK`` (the launcher's per-process
    GPU index, 0 by default) when a GPU is visible, else the CPU.  Sets the current HIP device."""
    if device is None:
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        else:
            device = torch.device("cpu")
    device = torch.device(device)
    if device.type == "cuda":
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(device)
    return device
