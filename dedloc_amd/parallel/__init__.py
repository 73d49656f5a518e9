"""Process-group management for the collaboration's data plane.

One OS process per GPU peer.  The world process group (RCCL over xGMI on GPUs, gloo on CPU) is
created at start-up for bootstrap, barriers and its key-value store; averaging rounds run on
*group communicators* (``GroupCommunicators``): one RCCL/gloo communicator per (member set,
data-plane epoch), created by the members only, through the world store, the first time that set
is matchmade.  A data-plane failure (a member stalls past ``averaging_timeout``) aborts that
communicator — outstanding send/recv operations die with it instead of being matched by the next
round — and bumps the epoch, so the next round between those peers runs on a fresh communicator.
With a stable membership (the common case on one node) the communicator is created once and
reused for every round.
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
from collections import OrderedDict
from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def env_rank_world():
    rank = int(os.environ.get("RANK", os.environ.get("LOCAL_RANK", "0")))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_world(backend: Optional[str] = None, timeout_s: float = 600.0, device: Optional[torch.device] = None,
               force: bool = False):
    """Initialise (or reuse) the world process group from torchrun-style env variables.

    Returns (rank, world_size, device).  A single process runs without a process group (world
    size 1; averaging is then skipped, as in the reference's 1-peer case) unless ``force``.
    """
    rank, world, local = env_rank_world()
    if device is None:
        if torch.cuda.is_available():
            device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        else:
            device = torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if device.type == "cuda" else "gloo")
        # no device_id: a world communicator bound to a device makes torch create every later group
        # with ncclCommSplit, a collective over ALL world ranks, which member-only group creation
        # (GroupCommunicators) would hang in; unbound, each group gets its own ncclCommInitRank
        # among its members (the current device is set above)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
        # the first P2P batch must not be the first collective on the communicator
        t = torch.zeros(1, device=device)
        dist.all_reduce(t)
    return rank, world, device


logger = logging.getLogger(__name__)


class GroupCommunicators:
    """Cache of per-(members, epoch) process groups over the world store (see module docstring).

    ``get`` must be called by every member of ``ranks`` with the same arguments (the matchmade
    group's member list and epoch are identical on all members); non-members never call it."""

    def __init__(self, timeout_s: float = 120.0, max_cached: int = 8):
        self.timeout = datetime.timedelta(seconds=max(1.0, float(timeout_s)))
        self.max_cached = max_cached
        self._cache: "OrderedDict[Tuple[Tuple[int, ...], int], object]" = OrderedDict()
        self._lock = threading.Lock()
        self.created = 0
        self.aborted = 0

    @staticmethod
    def _key(ranks: Sequence[int], epoch: int):
        return tuple(sorted(int(r) for r in ranks)), int(epoch)

    def get(self, ranks: Sequence[int], epoch: int):
        key = self._key(ranks, epoch)
        with self._lock:
            pg = self._cache.get(key)
            if pg is not None:
                self._cache.move_to_end(key)
                return pg
            # older epochs of the same member set are dead for good: release them
            for old in [k for k in self._cache if k[0] == key[0] and k[1] < key[1]]:
                self._drop(old)
            while len(self._cache) >= self.max_cached:
                self._drop(next(iter(self._cache)))
            pg = _new_member_group(list(key[0]), f"dedloc_avg_e{key[1]}_" + "-".join(map(str, key[0])), self.timeout)
            self._cache[key] = pg
            self.created += 1
            return pg

    def invalidate(self, ranks: Sequence[int], epoch: int):
        with self._lock:
            key = self._key(ranks, epoch)
            if key in self._cache:
                self._drop(key)

    def _drop(self, key):
        pg = self._cache.pop(key)
        abort_group(pg)
        self.aborted += 1

    def close(self):
        with self._lock:
            for k in list(self._cache):
                self._drop(k)


def _new_member_group(ranks, name: str, timeout: datetime.timedelta):
    """A process group over ``ranks`` created by its members only (torch's ``new_group`` with local
    synchronisation names groups by their rank set, which cannot express epochs)."""
    import torch.distributed.distributed_c10d as c10d

    default_pg = c10d._get_default_group()
    backend, store = c10d._world.pg_map[default_pg]
    me = dist.get_rank()
    assert me in ranks, "only members create a group communicator"
    if default_pg.bound_device_id is not None:
        raise RuntimeError("the world process group is bound to a device: group communicators would be created by "
                           "ncclCommSplit over all world ranks (init the world with parallel.init_world)")
    pg, _ = c10d._new_process_group_helper(len(ranks), ranks.index(me), ranks, backend, store, name, timeout=timeout,
                                           group_desc=name)
    c10d._world.pg_group_ranks[pg] = {g: i for i, g in enumerate(ranks)}
    # RCCL: the first operation on a communicator must include every member (lazy init); the
    # all-reduce also proves every member has created its end before any P2P traffic is posted
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.zeros(1, device=dev)
    work = dist.all_reduce(t, group=pg, async_op=True)
    if not work.wait(timeout=timeout):
        abort_group(pg)
        raise RuntimeError(f"group communicator {name} did not come up")
    if dev.type == "cuda":
        torch.cuda.current_stream().synchronize()
    return pg


def abort_group(pg):
    """Abort a group communicator (outstanding operations are cancelled, not left to be matched by
    a later round).  gloo has no abort; its group is dropped — a new group uses new connections."""
    import torch.distributed.distributed_c10d as c10d

    try:
        c10d._abort_process_group(pg)
        return
    except Exception as e:  # noqa: BLE001  (gloo: abort unsupported)
        logger.debug(f"abort of {getattr(pg, 'group_name', pg)} unsupported ({e}); dropping it")
    for m in (c10d._world.pg_map, c10d._world.pg_names, c10d._world.pg_group_ranks, c10d._world.pg_backend_config,
              c10d._world.pg_to_tag, c10d._world.pg_coalesce_state):
        m.pop(pg, None)


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def shutdown_world():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
