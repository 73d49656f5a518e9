"""Open-membership group communicators for the averaging data plane.

DeDLOC's peers join and leave at any time: a volunteer or a respawned spot instance bootstraps
from the DHT and enters the next averaging round (reference: ``albert/run_trainer.py:236-264``,
``AWS_runner.ipynb:342-370``).  So there is no launch-time world here.  Every communicator is
built by the members of one matchmade group, from scratch, through the control-plane DHT:

* **GPU groups: RCCL** (``csrc/comm/rccl_comm.cpp``).  The group's leader (the member with the
  smallest peer id) calls ``ncclGetUniqueId`` and publishes the 128 bytes under
  ``{prefix}_comm_{token}``; every member then runs a non-blocking ``ncclCommInitRankConfig`` and
  polls readiness against the round's deadline.  Transfers are grouped ``ncclSend``/``ncclRecv``
  on the caller's HIP stream — all pairs at once, which drives every xGMI link of a fully
  connected 8-GPU node concurrently — and a stalled round is cancelled with ``ncclCommAbort``.
* **All-CPU groups** (the CPU plumbing configuration): gloo.  The leader hosts a ``TCPStore`` on
  an ephemeral port and publishes its address the same way.
* **Mixed groups** (GPU trainers plus CPU auxiliary peers, the reference fleet's shape:
  ``AWS_runner.ipynb:26-30``): ``HybridGroupComm`` — the GPU members keep RCCL among themselves and
  only the pairs with a CPU member go over gloo (host-staged on the GPU side).  The averager's
  load balancing gives a CPU member a part proportional to its bandwidth, so the GPU members stage
  only that small share through host memory.

Every RCCL call (and every gloo send/recv) runs on the process's data-plane owner thread
(``comm_worker.CommWorker``): the classes below only build jobs and wait for them.

**Reuse without disagreement**: a communicator is identified by a *token* — the id of the
matchmaking round that created it — and bound to the sorted member set and backend it was
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
import socket
import threading
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import comm_worker as cw
from .comm_worker import CommError, CommWorker

logger = logging.getLogger(__name__)

__all__ = ["CommError", "RcclGroupComm", "GlooGroupComm", "HybridGroupComm", "GroupCommunicators", "pairwise_rccl",
           "rccl_available", "routable_host"]


def rccl_available(device: torch.device) -> bool:
    if device.type != "cuda":
        return False
    from ..ops import native_loaded

    return native_loaded() and hasattr(torch.ops, "dedloc_comm") and hasattr(torch.ops.dedloc_comm, "comm_init")


def _left(deadline: Optional[float]) -> float:
    return float("inf") if deadline is None else deadline - time.monotonic()


def _caller_stream(device: torch.device):
    return torch.cuda.current_stream(device) if device.type == "cuda" else None


class RcclGroupComm:
    """One RCCL communicator (native handle) over ``nranks`` GPU peers."""

    backend = "rccl"

    def __init__(self, handle: int, nranks: int, rank: int, device: torch.device):
        self.handle, self.nranks, self.rank, self.device = handle, nranks, rank, device
        self.alive = True

    @staticmethod
    def new_unique_id() -> bytes:
        return cw.unique_id()

    @classmethod
    def create(cls, uid: bytes, nranks: int, rank: int, device: torch.device, deadline: Optional[float]):
        dev_index = device.index if device.index is not None else (
            torch.cuda.current_device() if device.type == "cuda" else 0)
        h = CommWorker.get().run(lambda: cw.init_job(uid, nranks, rank, dev_index, deadline))
        return cls(h, nranks, rank, device)

    def p2p(self, sends: Sequence[torch.Tensor], send_peers: Sequence[int], recvs: Sequence[torch.Tensor],
            recv_peers: Sequence[int], deadline: Optional[float], tag: int = 0):
        """All sends and receives as one RCCL group on the caller's current stream (of this
        communicator's device); returns when they have completed on the device, or aborts the
        communicator and raises at ``deadline``."""
        if not self.alive:
            raise CommError("communicator was aborted")
        stream = _caller_stream(self.device)
        try:
            CommWorker.get().run(lambda: cw.p2p_job(self.handle, self.device, stream, sends, send_peers, recvs,
                                                    recv_peers, deadline))
        except CommError:
            self.alive = False  # the job aborted the communicator
            raise

    def p2p_job(self, sends, send_peers, recvs, recv_peers, deadline, stream):
        """The same transfer as a job (for a caller already composing jobs: HybridGroupComm)."""
        return cw.p2p_job(self.handle, self.device, stream, sends, send_peers, recvs, recv_peers, deadline)

    def abort(self):
        if self.alive:
            self.alive = False
            CommWorker.get().run(lambda: cw.abort_job(self.handle))


# gloo has no abort: a group whose operation timed out is parked here instead of being destroyed
# (destroying a process group with an operation still posted can block its destructor)
_GLOO_GRAVEYARD: List[object] = []


class GlooGroupComm:
    """A gloo process group over ``nranks`` peers (all-CPU groups, and the CPU side of mixed ones)."""

    backend = "gloo"

    def __init__(self, pg, nranks: int, rank: int, store=None):
        self.pg, self.nranks, self.rank = pg, nranks, rank
        self.store = store  # the leader keeps its TCPStore server alive with the group
        self.alive = True

    @classmethod
    def create(cls, store, nranks: int, rank: int, timeout_s: float, keep_store=None):
        pg = dist.ProcessGroupGloo(store, rank, nranks, datetime.timedelta(seconds=max(1.0, timeout_s)))
        return cls(pg, nranks, rank, keep_store)

    @staticmethod
    def stage(sends, recvs):
        """Host copies of device tensors (synchronous on the caller's stream, after its producers)."""
        host_sends = [s.detach().cpu() if s.is_cuda else s.detach().contiguous() for s in sends]
        host_recvs = [torch.empty(r.shape, dtype=r.dtype) if r.is_cuda else r for r in recvs]
        return host_sends, host_recvs

    @staticmethod
    def unstage(recvs, host_recvs):
        for r, h in zip(recvs, host_recvs):
            if r is not h:
                r.copy_(h)

    def p2p_job(self, host_sends, send_peers, host_recvs, recv_peers, deadline, tag):
        return cw.gloo_p2p_job(self.pg, host_sends, send_peers, host_recvs, recv_peers, deadline, tag)

    def p2p(self, sends, send_peers, recvs, recv_peers, deadline: Optional[float], tag: int = 0):
        if not self.alive:
            raise CommError("communicator was aborted")
        host_sends, host_recvs = self.stage(sends, recvs)
        try:
            CommWorker.get().run(lambda: self.p2p_job(host_sends, send_peers, host_recvs, recv_peers, deadline, tag))
        except CommError:
            self.abort()
            raise
        self.unstage(recvs, host_recvs)

    def abort(self):
        if self.alive:
            self.alive = False
            _GLOO_GRAVEYARD.append(self.pg)


def _both(a, b):
    """Step two jobs until both are done (the RCCL and gloo halves of a mixed group's transfer)."""
    done_a = done_b = False
    err = None
    while not (done_a and done_b):
        for which in (0, 1):
            if (done_a, done_b)[which]:
                continue
            try:
                next(a if which == 0 else b)
            except StopIteration:
                if which == 0:
                    done_a = True
                else:
                    done_b = True
            except CommError as e:
                err = err or e
                if which == 0:
                    done_a = True
                else:
                    done_b = True
        if not (done_a and done_b):
            yield
    if err is not None:
        raise err


class HybridGroupComm:
    """A mixed group: RCCL among its GPU members, gloo for every pair with a CPU member.

    Peers are numbered like every group communicator (sorted peer ids of the whole group);
    ``rccl_rank`` maps a member's group rank to its rank in the GPU members' RCCL communicator
    (None for a CPU member)."""

    backend = "rccl+gloo"

    def __init__(self, rccl: Optional[RcclGroupComm], gloo: GlooGroupComm, rccl_rank: List[Optional[int]],
                 rank: int, device: torch.device):
        self.rccl, self.gloo, self.rccl_rank = rccl, gloo, rccl_rank
        self.nranks, self.rank, self.device = len(rccl_rank), rank, device
        self.alive = True

    def _split(self, tensors, peers):
        fast, slow = ([], []), ([], [])
        for t, p in zip(tensors, peers):
            if self.rccl is not None and self.rccl_rank[int(p)] is not None:
                fast[0].append(t)
                fast[1].append(self.rccl_rank[int(p)])
            else:
                slow[0].append(t)
                slow[1].append(int(p))
        return fast, slow

    def p2p(self, sends, send_peers, recvs, recv_peers, deadline: Optional[float], tag: int = 0):
        if not self.alive:
            raise CommError("communicator was aborted")
        (fs, fsp), (ss, ssp) = self._split(sends, send_peers)
        (fr, frp), (sr, srp) = self._split(recvs, recv_peers)
        host_sends, host_recvs = GlooGroupComm.stage(ss, sr)
        stream = _caller_stream(self.device)
        jobs = []
        if fs or fr:
            jobs.append(lambda: self.rccl.p2p_job(fs, fsp, fr, frp, deadline, stream))
        if host_sends or host_recvs:
            jobs.append(lambda: self.gloo.p2p_job(host_sends, ssp, host_recvs, srp, deadline, tag))
        try:
            if len(jobs) == 2:
                CommWorker.get().run(lambda: _both(jobs[0](), jobs[1]()))
            elif jobs:
                CommWorker.get().run(jobs[0])
        except CommError:
            self.abort()
            raise
        GlooGroupComm.unstage(sr, host_recvs)

    def abort(self):
        if self.alive:
            self.alive = False
            if self.rccl is not None:
                try:
                    self.rccl.abort()
                except Exception as e:  # noqa: BLE001
                    logger.debug(f"abort of the RCCL half failed: {e}")
            self.gloo.abort()


class _Entry:
    __slots__ = ("comm", "key", "members")

    def __init__(self, comm, key, members):
        self.comm, self.key, self.members = comm, key, members


def routable_host(listen_host: str) -> str:
    """The address other machines can reach this peer's servers at: the listen address itself when
    it is specific, else the host's outbound interface (no packet is sent: a UDP socket is only
    connected to learn the route), else loopback."""
    if listen_host not in ("", "0.0.0.0", "::", "[::]"):
        return listen_host
    env = os.environ.get("DEDLOC_ANNOUNCE_HOST")
    if env:
        return env
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            ip = s.getsockname()[0]
            if ip and not ip.startswith("0."):
                return ip
    except OSError:
        pass
    return "127.0.0.1"


class GroupCommunicators:
    """Per-peer cache of group communicators, bootstrapped through the DHT (see module docstring).

    ``get`` must be called by every member of a matchmade group with the same member list and group
    id (the matchmaking result); it returns ``(comm, comm_rank_of)`` where ``comm_rank_of`` maps a
    member's peer id to its rank in the communicator (the rank order is the sorted peer ids, fixed
    for the communicator's lifetime, independent of each round's join order)."""

    # After this many consecutive RCCL communicators failed to come up BECAUSE OF THIS PEER (its own
    # RCCL stack reported an error: a broken install or transport on this host — not a deadline,
    # which another member's death or preemption can cause), the peer announces gloo: every later
    # group it joins runs over host-staged gloo.  The fallback is retried after
    # RCCL_RETRY_AFTER_S seconds.  DEDLOC_DATA_PLANE=gloo forces gloo from the start.
    RCCL_FALLBACK_AFTER = int(os.environ.get("DEDLOC_RCCL_FALLBACK_AFTER", "3"))
    RCCL_RETRY_AFTER_S = 300.0
    # Communicators abandoned during their bootstrap stay quarantined (comm_core.h) until RCCL's
    # init thread lets go of them.  Repeated churn during bootstraps could pile them up (each holds
    # sockets and an init thread), so past this many the peer stops building new RCCL communicators
    # and averages over gloo until the reaper has brought the count back down.
    MAX_QUARANTINED = int(os.environ.get("DEDLOC_RCCL_MAX_QUARANTINED", "16"))

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
        self.rccl_create_failures = 0  # consecutive RCCL communicators this peer could not bring up
        self._gpu_id: Optional[str] = None
        self._fallback_since: Optional[float] = None
        self._quarantine_warned = False

    # ------------------------------------------------------------------ matchmaking info
    @property
    def backend(self) -> str:
        if os.environ.get("DEDLOC_DATA_PLANE", "").lower() == "gloo":
            return "gloo"
        if self.rccl_create_failures >= self.RCCL_FALLBACK_AFTER:
            if time.monotonic() - (self._fallback_since or 0.0) < self.RCCL_RETRY_AFTER_S:
                return "gloo"
            self.rccl_create_failures = self.RCCL_FALLBACK_AFTER - 1  # one more try
        if not rccl_available(self.device):
            return "gloo"
        q = self.quarantined
        if q >= self.MAX_QUARANTINED:
            if not self._quarantine_warned:
                self._quarantine_warned = True
                logger.warning(f"{q} RCCL communicators are quarantined (bootstraps abandoned by churn); "
                               f"averaging over gloo until they are reaped")
            return "gloo"
        self._quarantine_warned = False
        return "rccl"

    @property
    def quarantined(self) -> int:
        """RCCL communicators of this process waiting for their bootstrap to end (comm_core.h)."""
        w = cw.CommWorker._instance
        return int(w.quarantined) if w is not None else 0

    @property
    def gpu_id(self) -> Optional[str]:
        """Host + device identity: RCCL takes one rank per device, so peers that share a GPU (a
        protocol emulation on a small box) cannot be ranks of one communicator."""
        if self._gpu_id is None and self.device.type == "cuda":
            props = torch.cuda.get_device_properties(self.device)
            uid = getattr(props, "uuid", None)
            self._gpu_id = f"{socket.gethostname()}/{uid if uid is not None else self.device.index}"
        return self._gpu_id

    def announce(self) -> Dict:
        """The fields this peer adds to its matchmaking info."""
        with self._lock:
            backend = self.backend
            return {"backend": backend, "comms": list(self._cache.keys()),
                    "gpu": self.gpu_id if backend == "rccl" else None}

    @staticmethod
    def rccl_members(members: Sequence[Tuple[bytes, Dict]]) -> List[bytes]:
        """Sorted peer ids of the members that take an RCCL rank: every member announcing rccl,
        except that of several members on one device only the first (in peer-id order) does — the
        others join the group's gloo side like CPU members."""
        seen, out = set(), []
        for pid, info in sorted(members, key=lambda m: bytes(m[0])):
            if info.get("backend") != "rccl":
                continue
            gpu = info.get("gpu")
            if gpu is not None:
                if gpu in seen:
                    continue
                seen.add(gpu)
            out.append(bytes(pid))
        return out

    @classmethod
    def group_backend(cls, members: Sequence[Tuple[bytes, Dict]]) -> str:
        n_rccl = len(cls.rccl_members(members))
        if n_rccl == len(members):
            return "rccl"
        return "hybrid" if n_rccl >= 2 else "gloo"

    # ------------------------------------------------------------------ communicator for a group
    def get(self, members: Sequence[Tuple[bytes, Dict]], group_id: bytes, deadline: Optional[float] = None):
        pids = sorted(bytes(pid) for pid, _ in members)
        assert self.peer_id in pids, "only members build a group communicator"
        backend = self.group_backend(members)
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
            # the DHT's matchmaking returns an integer round id (bytes(int) would be that many zero bytes)
            tok = f"{group_id:016x}" if isinstance(group_id, int) else bytes(group_id).hex()
            if deadline is None:
                deadline = time.monotonic() + self.timeout_s
            if backend == "hybrid":
                comm = self._create_hybrid(tok, pids, self.rccl_members(members), deadline)
            else:
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

    def _create_rccl(self, tok: str, n: int, rank: int, deadline: float) -> RcclGroupComm:
        if rank == 0:
            uid = RcclGroupComm.new_unique_id()
            self._publish(tok, {"uid": uid})
        else:
            uid = bytes(self._await(tok, deadline)["uid"])
        try:  # a healthy bootstrap takes seconds: a broken one should not hold the whole round
            boot = time.monotonic() + float(os.environ.get("DEDLOC_RCCL_BOOTSTRAP_S", "30"))
            boot = boot if deadline is None else min(deadline, boot)
            comm = RcclGroupComm.create(uid, n, rank, self.device, boot)
        except CommError as e:
            if e.local:  # this peer's RCCL failed; a deadline may be another member's doing
                self.rccl_create_failures += 1
                if self.rccl_create_failures == self.RCCL_FALLBACK_AFTER:
                    self._fallback_since = time.monotonic()
                    logger.warning(f"{self.rccl_create_failures} RCCL group communicators in a row failed on this "
                                   f"peer; it averages over host-staged gloo for the next "
                                   f"{self.RCCL_RETRY_AFTER_S:.0f} s")
            raise
        self.rccl_create_failures = 0
        return comm

    def _create_gloo(self, tok: str, n: int, rank: int, deadline: float) -> GlooGroupComm:
        timeout = max(1.0, _left(deadline))
        store_td = datetime.timedelta(seconds=timeout)
        if rank == 0:
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

    def _create(self, tok: str, backend: str, n: int, rank: int, deadline: float):
        if backend == "rccl":
            return self._create_rccl(tok, n, rank, deadline)
        return self._create_gloo(tok, n, rank, deadline)

    def _create_hybrid(self, tok: str, pids: List[bytes], gpu: List[bytes], deadline: float) -> HybridGroupComm:
        rank = pids.index(self.peer_id)
        rccl_rank = [gpu.index(p) if p in gpu else None for p in pids]
        rccl = None
        if self.peer_id in gpu:
            rccl = self._create_rccl(tok + "r", len(gpu), gpu.index(self.peer_id), deadline)
        try:
            gloo = self._create_gloo(tok + "g", len(pids), rank, deadline)
        except CommError:
            if rccl is not None:
                rccl.abort()
            raise
        return HybridGroupComm(rccl, gloo, rccl_rank, rank, self.device)

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
