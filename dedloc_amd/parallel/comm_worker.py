"""The data plane's owner thread: every RCCL call of this process is issued here.

The reference's averager is its own process (hivemind spawns it from CollaborativeOptimizer,
``albert/run_trainer.py:251-264``), so all of a peer's transfers come from one place.  Here a peer
is one process, and the transfers are requested by several threads: the trainer (gradient rounds),
the delayed-parameter round, and the state server (one thread per joining peer).  They all submit
*jobs* to one ``CommWorker`` per process, which alone calls ``torch.ops.dedloc_comm``
(communicator bootstrap, grouped send/recv, abort) and the gloo send/recv of mixed groups.

A job is a generator: it issues its calls and ``yield``s whenever it has to wait (a communicator
still connecting, a transfer still on the device, a gloo work item still pending).  The worker
steps every live job round-robin, so a state download served to a joiner progresses while a
gradient round is in flight instead of queueing behind it — and a job can never block the worker:
each one carries its own deadline and aborts its communicator when the deadline passes.

The calling thread passes its current HIP stream with the job: RCCL enqueues the transfer on it,
behind the pack kernels the caller already queued there, and completion is tracked with an event
recorded on that stream (on the communicator's device, whatever device the worker thread has
current).
"""
from __future__ import annotations

import collections
import logging
import threading
import time
from concurrent.futures import Future
from typing import Callable, Generator, Optional, Sequence

import torch

logger = logging.getLogger(__name__)

NCCL_SUCCESS, NCCL_IN_PROGRESS = 0, 7
POLL_S = 1e-4


def _ops():
    """The native RCCL operators (``csrc/comm/rccl_comm.cpp``); tests substitute a fake."""
    return torch.ops.dedloc_comm


class CommError(RuntimeError):
    """A group operation failed or missed its deadline; the communicator has been aborted.

    ``local`` is True when this peer's own RCCL stack reported the error (an init or enqueue error
    code), False when the failure can be the other members' doing (a deadline)."""

    def __init__(self, msg: str, local: bool = False):
        super().__init__(msg)
        self.local = local


def _left(deadline: Optional[float]) -> float:
    return float("inf") if deadline is None else deadline - time.monotonic()


Job = Generator[None, None, object]


class CommWorker:
    """One thread that owns the data plane of this process (see module docstring)."""

    _instance: Optional["CommWorker"] = None
    _instance_lock = threading.Lock()

    def __init__(self):
        self._queue: "collections.deque[tuple[Job, Future]]" = collections.deque()
        self._cv = threading.Condition()
        self._thread = threading.Thread(target=self._loop, daemon=True, name="comm-worker")
        self.jobs_run = 0
        self.quarantined = 0  # communicators waiting for their bootstrap to end before the abort
        self._thread.start()

    @classmethod
    def get(cls) -> "CommWorker":
        with cls._instance_lock:
            if cls._instance is None or not cls._instance._thread.is_alive():
                cls._instance = cls()
            return cls._instance

    def in_worker(self) -> bool:
        return threading.current_thread() is self._thread

    def submit(self, job: Job) -> Future:
        fut: Future = Future()
        with self._cv:
            self._queue.append((job, fut))
            self._cv.notify()
        return fut

    def run(self, make_job: Callable[[], Job]):
        """Run a job to completion and return its result (re-raising its exception).  Called from
        the worker itself (a job that needs another job's result), it runs inline."""
        job = make_job()
        if self.in_worker():
            return _drain(job)
        return self.submit(job).result()

    def note_quarantined(self):
        self.quarantined += 1

    REAP_PERIOD_S = 0.5

    def _reap(self):
        try:
            self.quarantined = int(_ops().comm_reap())
        except Exception as e:  # noqa: BLE001
            logger.debug(f"comm_reap failed: {e}")
            self.quarantined = 0

    def _loop(self):
        active = []
        last_reap = time.monotonic()
        while True:
            with self._cv:
                while not self._queue and not active:
                    if not self.quarantined:
                        self._cv.wait()
                        continue
                    self._cv.wait(self.REAP_PERIOD_S)
                    if not self._queue:
                        break
                while self._queue:
                    active.append(self._queue.popleft())
            if self.quarantined and time.monotonic() - last_reap >= self.REAP_PERIOD_S:
                last_reap = time.monotonic()
                self._reap()
            still = []
            for job, fut in active:
                try:
                    next(job)
                    still.append((job, fut))
                except StopIteration as done:
                    self.jobs_run += 1
                    fut.set_result(done.value)
                except BaseException as e:  # noqa: BLE001  (delivered to the submitting thread)
                    self.jobs_run += 1
                    fut.set_exception(e)
            active = still
            if active:
                time.sleep(POLL_S)


def _drain(job: Job):
    while True:
        try:
            next(job)
        except StopIteration as done:
            return done.value
        time.sleep(POLL_S)


# ---------------------------------------------------------------------------------------------
# RCCL jobs (the only callers of torch.ops.dedloc_comm)
# ---------------------------------------------------------------------------------------------

def unique_id() -> bytes:
    return CommWorker.get().run(lambda: _unique_id_job())


def _unique_id_job():
    return bytes(_ops().unique_id().numpy().tobytes())
    yield  # noqa: unreachable — makes this a generator


def _error(code: int) -> str:
    try:
        return f"{_ops().error_string(int(code))} ({code})"
    except Exception:  # noqa: BLE001
        return f"code {code}"


QUARANTINED = 1


def _abort(handle: int):
    """Release a failed or finished communicator: ncclCommAbort, unless its non-blocking bootstrap
    is still in flight — then the native registry quarantines it (RCCL's init thread still owns
    it) and the worker reaps it once the bootstrap has ended (``comm_core.h``)."""
    try:
        if int(_ops().comm_release(int(handle))) == QUARANTINED:
            CommWorker.get().note_quarantined()
    except Exception as e:  # noqa: BLE001
        logger.debug(f"comm_release({handle}) failed: {e}")


def _sync_quarantined():
    try:
        w = CommWorker.get()
        w.quarantined = max(w.quarantined, int(_ops().comm_quarantined()))
    except Exception as e:  # noqa: BLE001
        logger.debug(f"comm_quarantined failed: {e}")


def _wait_ready(handle: int, deadline: Optional[float], what: str):
    """Poll the communicator until its last call has been enqueued (ncclSuccess)."""
    ops = _ops()
    while True:
        st = int(ops.comm_status(handle))
        if st == NCCL_SUCCESS:
            return
        if st != NCCL_IN_PROGRESS:
            _abort(handle)
            raise CommError(f"RCCL {what} failed: {_error(st)}", local=True)
        if _left(deadline) <= 0:
            _abort(handle)
            raise CommError(f"RCCL {what} failed (deadline)")
        yield


def init_job(uid: bytes, nranks: int, rank: int, device_index: int, deadline: Optional[float]):
    """ncclCommInitRankConfig (non-blocking) and the wait for the bootstrap; returns the handle."""
    t = torch.frombuffer(bytearray(uid), dtype=torch.uint8)
    try:
        h = int(_ops().comm_init(t, int(nranks), int(rank), int(device_index)))
    except RuntimeError as e:
        # a synchronous init failure may leave a half-built communicator quarantined in the native
        # registry (comm_core.cpp): let the worker know, so that it keeps reaping
        _sync_quarantined()
        raise CommError(f"RCCL communicator init failed: {e}", local=True) from e
    yield from _wait_ready(h, deadline, "communicator bootstrap")
    return h


def p2p_job(handle: int, device: torch.device, stream, sends: Sequence[torch.Tensor], send_peers: Sequence[int],
            recvs: Sequence[torch.Tensor], recv_peers: Sequence[int], deadline: Optional[float]):
    """One grouped send/recv on ``stream``; returns once it has completed on the device."""
    ops = _ops()
    if stream is not None:
        with torch.cuda.stream(stream):
            rc = int(ops.group_p2p(handle, list(sends), [int(p) for p in send_peers], list(recvs),
                                   [int(p) for p in recv_peers]))
    else:
        rc = int(ops.group_p2p(handle, list(sends), [int(p) for p in send_peers], list(recvs),
                               [int(p) for p in recv_peers]))
    if rc not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
        _abort(handle)
        raise CommError(f"RCCL group send/recv failed: {_error(rc)}", local=True)
    yield from _wait_ready(handle, deadline, "group send/recv enqueue")
    if device.type != "cuda":
        return  # host communicators (tests): ready == transferred
    ev = torch.cuda.Event()
    ev.record(stream)
    n = 0
    while not ev.query():
        n += 1
        if n % 64 == 0:
            st = int(ops.comm_status(handle))
            if st not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
                _abort(handle)
                raise CommError(f"RCCL group send/recv failed: {_error(st)}", local=True)
        if _left(deadline) <= 0:
            _abort(handle)
            raise CommError("RCCL group send/recv failed (deadline)")
        yield


def abort_job(handle: int):
    _abort(handle)
    return None
    yield  # noqa: unreachable


# ---------------------------------------------------------------------------------------------
# gloo send/recv (groups with a CPU member).  gloo work items only complete inside a blocking
# wait(), so the waits run on a short-lived helper thread and the job polls that thread: the worker
# itself never blocks.  (gloo holds no device state; the single-owner rule is about RCCL.)
# ---------------------------------------------------------------------------------------------

def gloo_p2p_job(pg, sends, send_peers, recvs, recv_peers, deadline: Optional[float], tag: int):
    import datetime

    # the k-th transfer between two peers gets its own tag (the two sides list a pair's transfers in
    # the same order, as RCCL matches them), so several tensors per pair never cross
    seen = collections.Counter()

    def tag_for(kind, p):
        k = seen[(kind, int(p))]
        seen[(kind, int(p))] += 1
        return tag * 1024 + k

    works = []
    try:
        for t, p in zip(recvs, recv_peers):
            if t.numel():
                works.append(pg.recv([t], int(p), tag_for("r", p)))
        for t, p in zip(sends, send_peers):
            if t.numel():
                works.append(pg.send([t], int(p), tag_for("s", p)))
    except RuntimeError as e:
        raise CommError(f"gloo group send/recv failed: {e}") from e
    outcome = {}

    def wait_all():
        try:
            for w in works:
                left = _left(deadline)
                if left <= 0:
                    raise CommError("gloo group send/recv failed (deadline)")
                if w.wait(datetime.timedelta(seconds=min(left, 3600.0))) is False:
                    raise CommError("gloo group send/recv failed (deadline)")
        except CommError as e:
            outcome["error"] = e
        except RuntimeError as e:
            outcome["error"] = CommError(f"gloo group send/recv failed: {e}")

    waiter = threading.Thread(target=wait_all, daemon=True, name="gloo-wait")
    waiter.start()
    while waiter.is_alive():
        yield
    if "error" in outcome:
        raise outcome["error"]
