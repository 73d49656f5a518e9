"""Cross-process stand-in for the native RCCL operators (``torch.ops.dedloc_comm``) — TEST ONLY.

``tests/test_comm_fake_rccl.py`` pins the protocol around RCCL with "ranks" that are threads of one
process.  This module is its cross-process counterpart ("what's missing" 1): separate
peer processes — ``bench.py --gpus 8 --cpu_test``, or the churn peers of ``tests/xproc/peer.py`` —
run the REAL data-plane code (``parallel/comm.py``, ``comm_worker.py``, the butterfly all-reduce,
the state server) with only the bottom layer replaced: communicators and grouped send/recv go
through a mailbox directory shared by the processes (tmpfs) instead of RCCL over xGMI.

It keeps the semantics the Python side depends on:

* **non-blocking bootstrap** — ``comm_init`` registers the rank and returns at once; ``comm_status``
  reports ``ncclInProgress`` until every rank of the unique id has registered (plus a few polls);
* **non-blocking grouped send/recv, matched per (communicator, sender, receiver) in order** — a
  send is a message file ``m-<src>-<dst>-<seq>``, complete only once the receiver has consumed it
  (rendezvous, like a real send to a peer that never posts the receive); receives complete when
  their file appears;
* **a member that never arrives / dies** — its files never appear, so the others poll until the
  round's deadline and abort (``DEDLOC_XPROC_DIE_AT_P2P=k`` makes this process SIGKILL itself in
  its k-th grouped call, after posting half of its sends: a peer dying mid-round);
* **asynchronous errors** — ``DEDLOC_XPROC_ERROR_AT_P2P=k``: the k-th grouped call's communicator
  reports ``ncclSystemError`` from then on;
* **release = abort, except while the bootstrap is in flight (quarantine, reaped later)** — the
  rule of ``csrc/comm/comm_core.h``.

Installed into a process by ``tests/xproc/sitecustomize.py`` when ``DEDLOC_XPROC_RCCL_DIR`` names
the mailbox directory; per-process counters are written to ``<dir>/stats-<pid>.json`` at exit.
"""
from __future__ import annotations

import atexit
import json
import os
import signal
import threading
from collections import Counter

import numpy as np
import torch

SUCCESS, SYSTEM_ERROR, INVALID_ARGUMENT, IN_PROGRESS = 0, 2, 4, 7
RELEASE_ABORTED, RELEASE_QUARANTINED, RELEASE_UNKNOWN = 0, 1, 2


def _write_atomic(path: str, t: torch.Tensor):
    tmp = f"{path}.tmp{os.getpid()}"
    t.detach().reshape(-1).contiguous().view(torch.uint8).numpy().tofile(tmp)
    os.replace(tmp, path)


class _Comm:
    __slots__ = ("key", "n", "rank", "polls", "ready", "recvs", "sends", "sseq", "rseq", "error", "quarantined")

    def __init__(self, key, n, rank, polls):
        self.key, self.n, self.rank, self.polls = key, n, rank, polls
        self.ready = False          # status() has reported success once (the bootstrap completed)
        self.recvs = []             # (tensor, message path) still to arrive
        self.sends = []             # message paths the receiver has not consumed yet
        self.sseq, self.rseq = Counter(), Counter()
        self.error = 0
        self.quarantined = False


class FsRccl:
    """The operator surface of ``csrc/comm/rccl_comm.cpp`` over a shared mailbox directory."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(root, exist_ok=True)
        self.lock = threading.Lock()
        self.next = 1
        self.comms = {}
        self.calls = Counter()
        self.die_at = int(os.environ.get("DEDLOC_XPROC_DIE_AT_P2P", "0"))
        self.error_at = int(os.environ.get("DEDLOC_XPROC_ERROR_AT_P2P", "0"))
        self.init_polls = int(os.environ.get("DEDLOC_XPROC_INIT_POLLS", "2"))
        atexit.register(self._dump)

    # ---------------------------------------------------------------- helpers
    def _dir(self, key: str) -> str:
        return os.path.join(self.root, key)

    def _joined(self, c: _Comm) -> bool:
        d = self._dir(c.key)
        return all(os.path.exists(os.path.join(d, f"joined-{r}")) for r in range(c.n))

    def _msg(self, c: _Comm, src: int, dst: int, seq: int) -> str:
        return os.path.join(self._dir(c.key), f"m-{src}-{dst}-{seq}")

    def _dump(self):
        try:
            with open(os.path.join(self.root, f"stats-{os.getpid()}.json"), "w") as f:
                json.dump({"calls": dict(self.calls), "live": sum(not c.quarantined for c in self.comms.values()),
                           "quarantined": sum(c.quarantined for c in self.comms.values())}, f)
        except OSError:
            pass

    # ---------------------------------------------------------------- operators
    def unique_id(self):
        self.calls["unique_id"] += 1
        return torch.frombuffer(bytearray(os.urandom(128)), dtype=torch.uint8)

    def comm_init(self, uid, n, rank, dev):
        self.calls["comm_init"] += 1
        key = bytes(uid.numpy().tobytes())[:16].hex()
        os.makedirs(self._dir(key), exist_ok=True)
        open(os.path.join(self._dir(key), f"joined-{int(rank)}"), "w").close()
        with self.lock:
            h = self.next
            self.next += 1
            self.comms[h] = _Comm(key, int(n), int(rank), self.init_polls)
        return h

    def comm_status(self, h):
        self.calls["comm_status"] += 1
        with self.lock:
            c = self.comms.get(int(h))
            if c is None or c.quarantined:
                return INVALID_ARGUMENT
            if c.error:
                return c.error
            if not c.ready:
                if not self._joined(c):
                    return IN_PROGRESS
                if c.polls > 0:
                    c.polls -= 1
                    return IN_PROGRESS
                c.ready = True
            still = []
            for t, path in c.recvs:
                if os.path.exists(path):
                    raw = torch.from_numpy(np.fromfile(path, dtype=np.uint8))
                    flat = t.view(-1)
                    if raw.numel() != flat.numel() * flat.element_size():
                        c.error = SYSTEM_ERROR  # a size mismatch is a protocol bug: surface it as an RCCL error
                        return c.error
                    flat.copy_(raw.view(flat.dtype))
                    os.unlink(path)
                else:
                    still.append((t, path))
            c.recvs = still
            c.sends = [p for p in c.sends if os.path.exists(p)]
            return SUCCESS if not (c.recvs or c.sends) else IN_PROGRESS

    def group_p2p(self, h, sends, send_peers, recvs, recv_peers):
        self.calls["group_p2p"] += 1
        with self.lock:
            c = self.comms.get(int(h))
            if c is None or c.quarantined or not c.ready:
                return INVALID_ARGUMENT
            k = self.calls["group_p2p"]
            posted = [(t, int(p)) for t, p in zip(sends, send_peers) if t.numel()]
            if self.die_at and k == self.die_at:
                for t, p in posted[: max(1, len(posted) // 2)]:
                    _write_atomic(self._msg(c, c.rank, p, c.sseq[p]), t)
                    c.sseq[p] += 1
                os.kill(os.getpid(), signal.SIGKILL)
            if self.error_at and k == self.error_at:
                c.error = SYSTEM_ERROR
                return IN_PROGRESS  # reported asynchronously, by the next status poll
            for t, p in posted:
                path = self._msg(c, c.rank, p, c.sseq[p])
                c.sseq[p] += 1
                _write_atomic(path, t)
                c.sends.append(path)
            for t, p in zip(recvs, recv_peers):
                if t.numel():
                    p = int(p)
                    c.recvs.append((t, self._msg(c, p, c.rank, c.rseq[p])))
                    c.rseq[p] += 1
            return IN_PROGRESS

    def comm_release(self, h):
        self.calls["comm_release"] += 1
        with self.lock:
            c = self.comms.get(int(h))
            if c is None:
                return RELEASE_UNKNOWN
            if not c.ready and not c.error and not self._joined(c):
                c.quarantined = True
                self.calls["quarantined"] += 1
                return RELEASE_QUARANTINED
            self._abort(int(h), c)
            return RELEASE_ABORTED

    def _abort(self, h: int, c: _Comm):
        for p in c.sends:  # an abort cancels what was posted
            try:
                os.unlink(p)
            except OSError:
                pass
        self.comms.pop(h, None)
        self.calls["aborted"] += 1

    def comm_reap(self):
        self.calls["comm_reap"] += 1
        with self.lock:
            for h, c in list(self.comms.items()):
                if c.quarantined and self._joined(c):
                    self._abort(h, c)
            return sum(c.quarantined for c in self.comms.values())

    def comm_quarantined(self):
        with self.lock:
            return sum(c.quarantined for c in self.comms.values())

    def error_string(self, code):
        return f"xproc mailbox error {int(code)}"


_INSTALLED = None


def install(root: str) -> FsRccl:
    """Route this process's data plane through the mailbox (the way the in-process ``fake``
    fixture of tests/test_comm_fake_rccl.py does)."""
    global _INSTALLED
    if _INSTALLED is None:
        from dedloc_amd.parallel import comm as C
        from dedloc_amd.parallel import comm_worker as W

        _INSTALLED = FsRccl(root)
        W._ops = lambda: _INSTALLED
        C.rccl_available = lambda dev: True
    return _INSTALLED
