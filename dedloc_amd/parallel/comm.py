"""Open-membership group communicators for the averaging data plane.

DeDLOC's peers join and leave at any time: a volunteer or a respawned spot instance bootstraps
from the DHT and enters the next averaging round (reference: ``albert/run_trainer.py:236-264``,
``AWS_runner.ipynb:342-370``).  So there is no launch-time world here.  Every communicator is
built by the members of one matchmade group, from scratch, through the control-plane DHT:

* **GPU groups: RCCL** (``csrc/comm/rccl_comm.cpp``).  The group's leader (the member with the
  smallest peer id) calls ``ncclGetUniqueId`` and publishes the 128 bytes under
  ``{prefix}_comm_{token}``; every member then runs a non-blocking ``ncclCommInitRankConfig`` and
  the host polls readiness against the round's deadline.  Transfers are grouped
  ``ncclSend``/``ncclRecv`` on the current HIP stream — all pairs at once, which drives every xGMI
  link of a fully connected 8-GPU node concurrently — and a stalled round is cancelled with
  ``ncclCommAbort``.
* **Groups with a CPU member** (a CPU auxiliary peer, the CPU plumbing configuration): gloo.  The
  leader hosts a ``TCPStore`` on an ephemeral port and publishes its address the same way; GPU
  members stage their tensors through host memory for such a round.

**Reuse without disagreement** (ADVICE r2): a communicator is identified by a *token* — the id of
the matchmaking round that created it — and bound to the sorted member set and backend it was
created for.  Every peer announces the tokens it still holds in its matchmaking info; a round
reuses a token only if EVERY member announced it, otherwise the members create a fresh one keyed
by the new round's group id.  Each peer evicts (and aborts) communicators from its own bounded
cache independently: an eviction on one side simply makes that token non-common, so the members
can never end up on different communicators, and a failed round drops its token on the members
that saw the failure, with the same effect.  With a stable membership the communicator is built
once and reused for every round.
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)

NCCL_SUCCESS, NCCL_IN_PROGRESS = 0, 7
_POLL_S = 1e-4


class CommError(RuntimeError):
    """A group operation failed or missed its deadline; the communicator has been aborted."""


def rccl_available(device: torch.device) -> bool:
    if device.type != "cuda":
        return False
    from ..ops import native_loaded

    return native_loaded() and hasattr(torch.ops, "dedloc_comm") and hasattr(torch.ops.dedloc_comm, "comm_init")


def _left(deadline: Optional[float]) -> float:
    return float("inf") if deadline is None else deadline - time.monotonic()


class RcclGroupComm:
    """One RCCL communicator (native handle) over ``nranks`` GPU peers."""

    backend = "rccl"

    def __init__(self, handle: int, nranks: int, rank: int, device: torch.device):
        self.handle, self.nranks, self.rank, self.device = handle, nranks, rank, device
        self.alive = True

    @staticmethod
    def new_unique_id() -> bytes:
        return bytes(torch.ops.dedloc_comm.unique_id().numpy().tobytes())

    @classmethod
    def create(cls, uid: bytes, nranks: int, rank: int, device: torch.device, deadline: Optional[float]):
        ops = torch.ops.dedloc_comm
        t = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
        h = ops.comm_init(t, nranks, rank, device.index if device.index is not None else torch.cuda.current_device())
        comm = cls(h, nranks, rank, device)
        comm._wait_ready(deadline, "communicator bootstrap")
        return comm

    def _status(self) -> int:
        return int(torch.ops.dedloc_comm.comm_status(self.handle))

    def _fail(self, what: str, code: Optional[int] = None):
        msg = f"RCCL {what} failed"
        if code is not None:
            msg += f": {torch.ops.dedloc_comm.error_string(code)} ({code})"
        self.abort()
        raise CommError(msg)

    def _wait_ready(self, deadline: Optional[float], what: str):
        while True:
            st = self._status()
            if st == NCCL_SUCCESS:
                return
            if st != NCCL_IN_PROGRESS:
                self._fail(what, st)
            if _left(deadline) <= 0:
                self._fail(what + " (deadline)")
            time.sleep(_POLL_S)

    def p2p(self, sends: Sequence[torch.Tensor], send_peers: Sequence[int], recvs: Sequence[torch.Tensor],
            recv_peers: Sequence[int], deadline: Optional[float], tag: int = 0):
        """All sends and receives as one RCCL group on the current stream; returns when they have
        completed on the device, or aborts the communicator and raises at ``deadline``."""
        if not self.alive:
            raise CommError("communicator was aborted")
        rc = int(torch.ops.dedloc_comm.group_p2p(self.handle, list(sends), [int(p) for p in send_peers],
                                                 list(recvs), [int(p) for p in recv_peers]))
        if rc not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
            self._fail("group send/recv", rc)
        self._wait_ready(deadline, "group send/recv enqueue")
        ev = torch.cuda.Event()
        ev.record()
        n = 0
        while not ev.query():
            n += 1
            if n % 64 == 0:
                st = self._status()
                if st not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
                    self._fail("group send/recv", st)
            if _left(deadline) <= 0:
                self._fail("group send/recv (deadline)")
            time.sleep(_POLL_S)

    def abort(self):
        if self.alive:
            self.alive = False
            torch.ops.dedloc_comm.comm_abort(self.handle)


# gloo has no abort: a group whose operation timed out is parked here instead of being destroyed
# (destroying a process group with an operation still posted can block its destructor)
_GLOO_GRAVEYARD: List[object] = []


class GlooGroupComm:
    """A gloo process group over ``nranks`` peers (CPU peers, or any group with one)."""

    backend = "gloo"

    def __init__(self, pg, nranks: int, rank: int, store=None):
        self.pg, self.nranks, self.rank = pg, nranks, rank
        self.store = store  # the leader keeps its TCPStore server alive with the group
        self.alive = True

    @classmethod
    def create(cls, store, nranks: int, rank: int, timeout_s: float, keep_store=None):
        pg = dist.ProcessGroupGloo(store, rank, nranks, datetime.timedelta(seconds=max(1.0, timeout_s)))
        return cls(pg, nranks, rank, keep_store)

    def p2p(self, sends, send_peers, recvs, recv_peers, deadline: Optional[float], tag: int = 0):
        if not self.alive:
            raise CommError("communicator was aborted")
        host_sends = [s.detach().cpu() if s.is_cuda else s.detach().contiguous() for s in sends]
        host_recvs = [torch.empty(r.shape, dtype=r.dtype) if r.is_cuda else r for r in recvs]
        works = []
        try:
            for t, p in zip(host_recvs, recv_peers):
                if t.numel():
                    works.append(self.pg.recv([t], int(p), tag))
            for t, p in zip(host_sends, send_peers):
                if t.numel():
                    works.append(self.pg.send([t], int(p), tag))
            for w in works:
                left = _left(deadline)
                if left <= 0:
                    raise CommError("gloo group send/recv (deadline)")
                ok = w.wait(datetime.timedelta(seconds=min(left, 3600.0)))
                if ok is False:
                    raise CommError("gloo group send/recv (deadline)")
        except CommError:
            self.abort()
            raise
        except RuntimeError as e:
            self.abort()
            raise CommError(f"gloo group send/recv failed: {e}") from e
        for r, h in zip(recvs, host_recvs):
            if r is not h:
                r.copy_(h)

    def abort(self):
        if self.alive:
            self.alive = False
            _GLOO_GRAVEYARD.append(self.pg)


class _Entry:
    __slots__ = ("comm", "key", "members")

    def __init__(self, comm, key, members):
        self.comm, self.key, self.members = comm, key, members


class GroupCommunicators:
    """Per-peer cache of group communicators, bootstrapped through the DHT (see module docstring).

    ``get`` must be called by every member of a matchmade group with the same member list and group
    id (the matchmaking result); it returns ``(comm, comm_rank_of)`` where ``comm_rank_of`` maps a
    member's peer id to its rank in the communicator (the rank order is the sorted peer ids, fixed
    for the communicator's lifetime, independent of each round's join order)."""

    def __init__(self, dht, prefix: str, peer_id: bytes, device: torch.device, timeout_s: float = 60.0,
                 max_cached: int = 8, host: str = "127.0.0.1"):
        self.dht, self.prefix, self.peer_id = dht, prefix, bytes(peer_id)
        self.device = torch.device(device)
        self.timeout_s = float(timeout_s)
        self.max_cached = max(1, int(max_cached))
        self.host = host
        self._cache: "OrderedDict[str, _Entry]" = OrderedDict()
        self._lock = threading.RLock()
        self.created = 0
        self.aborted = 0
        self.rccl_create_failures = 0  # consecutive RCCL communicators that never came up

    # ------------------------------------------------------------------ matchmaking info
    # After this many consecutive RCCL communicators failed to come up (a broken RCCL install or
    # transport on this host), the peer announces gloo: every later group it joins runs over
    # host-staged gloo — slower, but the collaboration keeps averaging instead of losing every
    # round to the bootstrap deadline.  DEDLOC_DATA_PLANE=gloo forces that from the start.
    RCCL_FALLBACK_AFTER = 3

    @property
    def backend(self) -> str:
        if os.environ.get("DEDLOC_DATA_PLANE", "").lower() == "gloo":
            return "gloo"
        if self.rccl_create_failures >= self.RCCL_FALLBACK_AFTER:
            return "gloo"
        return "rccl" if rccl_available(self.device) else "gloo"

    def announce(self) -> Dict:
        """The fields this peer adds to its matchmaking info."""
        with self._lock:
            return {"backend": self.backend, "comms": list(self._cache.keys())}

    # ------------------------------------------------------------------ communicator for a group
    def get(self, members: Sequence[Tuple[bytes, Dict]], group_id: bytes, deadline: Optional[float] = None):
        pids = sorted(bytes(pid) for pid, _ in members)
        assert self.peer_id in pids, "only members build a group communicator"
        backend = "rccl" if all(info.get("backend") == "rccl" for _, info in members) else "gloo"
        key = (tuple(pids), backend)
        rank_of = {pid: i for i, pid in enumerate(pids)}
        with self._lock:
            common = None
            for _, info in members:
                toks = set(info.get("comms") or ())
                common = toks if common is None else (common & toks)
            candidates = sorted(t for t in (common or ()) if t in self._cache and self._cache[t].key == key)
            if candidates:
                tok = candidates[-1]
                self._cache.move_to_end(tok)
                return self._cache[tok].comm, rank_of
            # a member set we share no live communicator with: build one for this round's group id
            while len(self._cache) >= self.max_cached:
                self._drop(next(iter(self._cache)))
            tok = bytes(group_id).hex()
            if deadline is None:
                deadline = time.monotonic() + self.timeout_s
            comm = self._create(tok, backend, len(pids), rank_of[self.peer_id], deadline)
            self._cache[tok] = _Entry(comm, key, pids)
            self.created += 1
            return comm, rank_of

    def _rendezvous_key(self, tok: str) -> str:
        return f"{self.prefix}_comm_{tok}"

    def _publish(self, tok: str, value: Dict):
        from ..dht import get_dht_time

        self.dht.store(self._rendezvous_key(tok), value, get_dht_time() + max(30.0, 2 * self.timeout_s))

    def _await(self, tok: str, deadline: float) -> Dict:
        delay = 2e-3
        while True:
            rec = self.dht.get(self._rendezvous_key(tok), latest=True)
            if rec is not None and isinstance(rec.value, dict):
                return rec.value
            if _left(deadline) <= 0:
                raise CommError(f"group {tok[:12]}: the leader never published the communicator bootstrap")
            time.sleep(delay)
            delay = min(0.05, delay * 1.5)

    def _create(self, tok: str, backend: str, n: int, rank: int, deadline: float):
        leader = rank == 0
        if backend == "rccl":
            if leader:
                uid = RcclGroupComm.new_unique_id()
                self._publish(tok, {"uid": uid})
            else:
                uid = bytes(self._await(tok, deadline)["uid"])
            try:  # a healthy bootstrap takes seconds: a broken one should not hold the whole round
                boot = time.monotonic() + float(os.environ.get("DEDLOC_RCCL_BOOTSTRAP_S", "30"))
                boot = boot if deadline is None else min(deadline, boot)
                comm = RcclGroupComm.create(uid, n, rank, self.device, boot)
            except Exception:  # CommError (deadline) or an RCCL init error raised by the op
                self.rccl_create_failures += 1
                if self.rccl_create_failures == self.RCCL_FALLBACK_AFTER:
                    logger.warning(f"{self.rccl_create_failures} RCCL group communicators in a row did not come "
                                   f"up; this peer now averages over host-staged gloo groups")
                raise
            self.rccl_create_failures = 0
            return comm
        timeout = max(1.0, _left(deadline))
        store_td = datetime.timedelta(seconds=timeout)
        if leader:
            server = dist.TCPStore(self.host, 0, n, True, store_td, wait_for_workers=False)
            self._publish(tok, {"host": self.host, "port": int(server.port)})
            store = server
        else:
            rv = self._await(tok, deadline)
            server = None
            store = dist.TCPStore(rv["host"], int(rv["port"]), n, False, store_td)
        try:
            return GlooGroupComm.create(dist.PrefixStore(tok, store), n, rank, max(1.0, _left(deadline)),
                                        keep_store=server)
        except RuntimeError as e:
            raise CommError(f"gloo group {tok[:12]} did not come up: {e}") from e

    # ------------------------------------------------------------------ failure handling
    def invalidate(self, comm) -> None:
        """Abort ``comm`` and forget it (its token stops being announced, so the next round between
        these peers builds a fresh communicator)."""
        with self._lock:
            for tok, e in list(self._cache.items()):
                if e.comm is comm:
                    self._drop(tok)
                    return
        comm.abort()

    def _drop(self, tok: str):
        e = self._cache.pop(tok)
        try:
            e.comm.abort()
        except Exception as ex:  # noqa: BLE001
            logger.debug(f"abort of communicator {tok[:12]} failed: {ex}")
        self.aborted += 1

    def close(self):
        with self._lock:
            for tok in list(self._cache):
                self._drop(tok)


def pairwise_rccl(uid: bytes, rank: int, device: torch.device, deadline: Optional[float]) -> RcclGroupComm:
    """A 2-rank RCCL communicator for a one-off transfer (peer state download): the receiver made
    ``uid`` and is rank 1, the donor rank 0."""
    return RcclGroupComm.create(uid, 2, rank, device, deadline)
