"""The RCCL data-plane logic on CPU, against a fake ``torch.ops.dedloc_comm``.

Multi-rank RCCL cannot run on a one-GPU box, so the host-side protocol around it is pinned here:
the comm worker's jobs (parallel/comm_worker.py), the butterfly all-reduce over ``RcclGroupComm``,
the RCCL state-download path, and the mixed RCCL + gloo group.  The fake matches sends to receives
per (communicator, sender, receiver) pair in order, as RCCL does, and can be told to report
``ncclInProgress`` for a number of polls (non-blocking enqueue), to raise an asynchronous error on
one member, or to never see a member's operations (a dead peer).

Parity note: the fake checks the protocol (who sends what to whom, polling, abort on deadline and
on error), not RCCL itself; a real multi-GPU run is the only check of the latter.
"""
import threading
import time
from collections import defaultdict, deque

import pytest
import torch

import dedloc_amd.ops  # noqa: F401  (dedloc:: CPU kernels: pack / reduce_delta / unpack)
from dedloc_amd.averaging.allreduce import GroupSpec, butterfly_allreduce
from dedloc_amd.parallel import comm as C
from dedloc_amd.parallel import comm_worker as W

SUCCESS, IN_PROGRESS, SYSTEM_ERROR = 0, 7, 2


class FakeRccl:
    """A process-local stand-in for the native operators of csrc/comm/rccl_comm.cpp."""

    def __init__(self, init_polls=2, enqueue_polls=2):
        self.lock = threading.Lock()
        self.next = 1
        self.comms = {}           # handle -> dict(uid, n, rank, polls, pending recvs, error)
        self.joined = defaultdict(set)
        self.mail = defaultdict(deque)  # (uid, src, dst) -> tensors in send order
        self.init_polls, self.enqueue_polls = init_polls, enqueue_polls
        self.aborted = set()
        self.quarantine = set()   # released while still bootstrapping: aborted by comm_reap later
        self.mute = set()         # (uid, rank): this member's operations never arrive (dead peer)
        self.calls = defaultdict(int)
        self.threads = set()

    def _note(self, name):
        self.calls[name] += 1
        self.threads.add(threading.current_thread().name)

    def unique_id(self):
        self._note("unique_id")
        return torch.randint(0, 256, (128,), dtype=torch.uint8)

    def comm_init(self, uid, n, rank, dev):
        self._note("comm_init")
        key = bytes(uid.numpy().tobytes())
        with self.lock:
            h = self.next
            self.next += 1
            self.comms[h] = {"uid": key, "n": n, "rank": rank, "polls": self.init_polls, "recvs": [], "error": 0}
            self.joined[key].add(rank)
        return h

    def comm_status(self, h):
        self._note("comm_status")
        with self.lock:
            c = self.comms[h]
            if c["error"]:
                return c["error"]
            if len(self.joined[c["uid"]]) < c["n"]:
                return IN_PROGRESS
            if c["polls"] > 0:
                c["polls"] -= 1
                return IN_PROGRESS
            still = []
            for t, src in c["recvs"]:
                box = self.mail[(c["uid"], src, c["rank"])]
                if box:
                    t.copy_(box.popleft())
                else:
                    still.append((t, src))
            c["recvs"] = still
            return SUCCESS if not still else IN_PROGRESS

    def group_p2p(self, h, sends, send_peers, recvs, recv_peers):
        self._note("group_p2p")
        with self.lock:
            c = self.comms[h]
            if (c["uid"], c["rank"]) not in self.mute:
                for t, p in zip(sends, send_peers):
                    if t.numel():
                        self.mail[(c["uid"], c["rank"], p)].append(t.detach().clone())
            c["recvs"] += [(t, p) for t, p in zip(recvs, recv_peers) if t.numel()]
            c["polls"] = self.enqueue_polls
        return IN_PROGRESS

    def _in_progress(self, c):
        return len(self.joined[c["uid"]]) < c["n"]

    def comm_release(self, h):
        """comm_core.h's rule: abort, unless the bootstrap is still in flight (quarantine)."""
        self._note("comm_release")
        with self.lock:
            c = self.comms.get(h)
            if c is not None and self._in_progress(c) and not c["error"]:
                self.quarantine.add(h)
                return 1
            self.aborted.add(h)
            self.quarantine.discard(h)
            return 0

    def comm_reap(self):
        self._note("comm_reap")
        with self.lock:
            for h in list(self.quarantine):
                if not self._in_progress(self.comms[h]):
                    self.quarantine.discard(h)
                    self.aborted.add(h)
            return len(self.quarantine)

    def comm_quarantined(self):
        return len(self.quarantine)

    def error_string(self, code):
        return f"fake error {code}"


@pytest.fixture
def fake(monkeypatch):
    f = FakeRccl()
    monkeypatch.setattr(W, "_ops", lambda: f)
    monkeypatch.setattr(C, "rccl_available", lambda dev: True)
    return f


def _run_ranks(n, fn):
    out, errs = {}, {}

    def body(r):
        try:
            out[r] = fn(r)
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,), name=f"rank{r}") for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    return out, errs


def test_butterfly_over_rccl_nonuniform_parts_and_weights(fake):
    """Three members, LP-style unequal parts (one member owns none), unequal weights, FLOAT16 wire:
    every member ends with the weighted fp32 mean (to fp16 accuracy), and every RCCL call was made
    on the comm worker thread."""
    n, V = 3, 1000
    uid = W.unique_id()
    xs = [torch.randn(V, generator=torch.Generator().manual_seed(r)) for r in range(n)]
    weights = [1.0, 2.5, 0.5]
    parts = [600, 0, 400]
    expected = sum(w * x for w, x in zip(weights, xs)) / sum(weights)

    def rank(r):
        comm = C.RcclGroupComm.create(uid, n, r, torch.device("cpu"), time.monotonic() + 20)
        x = xs[r].clone()
        spec = GroupSpec(ranks=list(range(n)), part_sizes=parts, weights=[weights[r] if k == r else 0.0 for k in range(n)],
                         contributes=[True] * n, my_index=r)
        butterfly_allreduce([x], spec, "FLOAT16", comm=comm, timeout=20)
        comm.abort()
        return x

    out, errs = _run_ranks(n, rank)
    assert not errs, errs
    for r in range(n):
        torch.testing.assert_close(out[r], expected, rtol=2e-3, atol=2e-3)
    assert fake.threads == {"comm-worker"}, fake.threads  # the single RCCL owner
    assert fake.calls["group_p2p"] == 2 * n and fake.calls["comm_release"] == n and len(fake.aborted) == n


def test_async_error_while_polling_aborts_and_raises(fake):
    """An asynchronous RCCL error reported while a transfer is polled: the job aborts the
    communicator and the caller gets a CommError flagged as this peer's own (local) failure."""
    uid = W.unique_id()

    def rank(r):
        comm = C.RcclGroupComm.create(uid, 2, r, torch.device("cpu"), time.monotonic() + 20)
        if r == 0:
            fake.comms[comm.handle]["error"] = SYSTEM_ERROR
        buf = torch.zeros(8)
        comm.p2p([torch.ones(8)], [1 - r], [buf], [1 - r], time.monotonic() + 3)
        return comm

    out, errs = _run_ranks(2, rank)
    assert isinstance(errs.get(0), C.CommError) and errs[0].local, errs
    assert "fake error" in str(errs[0])
    assert any(fake.comms[h]["rank"] == 0 for h in fake.aborted)


def test_dead_member_is_aborted_at_the_deadline(fake):
    """A member that never sends (dead peer): the live member's transfer is aborted at the round's
    deadline — not later, and flagged as not this peer's fault (no RCCL fallback counting)."""
    uid = W.unique_id()
    fake.mute.add((uid, 1))

    def rank(r):
        comm = C.RcclGroupComm.create(uid, 2, r, torch.device("cpu"), time.monotonic() + 20)
        if r == 1:
            return None  # posts nothing, ever
        t0 = time.monotonic()
        try:
            comm.p2p([torch.ones(8)], [1], [torch.zeros(8)], [1], time.monotonic() + 1.0)
        finally:
            fake_elapsed.append(time.monotonic() - t0)
        return comm

    fake_elapsed = []
    out, errs = _run_ranks(2, rank)
    assert isinstance(errs.get(0), C.CommError) and not errs[0].local, errs
    assert 0.9 < fake_elapsed[0] < 2.0, fake_elapsed
    assert len(fake.aborted) == 1


def test_state_download_over_rccl_path(fake):
    """The state server's 'R' mode (a donor sends its snapshot over a one-off 2-rank communicator
    the requester bootstrapped): header over TCP, tensors through the comm worker."""
    from dedloc_amd.averaging.averager import StateServer, download_state

    state = [torch.randn(300), torch.arange(10, dtype=torch.float32)]
    srv = StateServer(lambda: ({"step": 7}, [t.clone() for t in state]), "127.0.0.1:0", device=torch.device("cpu"))
    try:
        meta, tensors = download_state(srv.endpoint, timeout=20, device=torch.device("cpu"), allow_rccl=True)
        t0 = time.monotonic()
        while srv.served["R"] < 1 and time.monotonic() - t0 < 10:  # the server counts after its send
            time.sleep(0.01)
    finally:
        srv.shutdown()
    assert meta["_mode"] == "R" and meta["step"] == 7 and srv.served["R"] == 1
    for a, b in zip(tensors, state):
        torch.testing.assert_close(a, b)
    assert fake.threads == {"comm-worker"}


@pytest.mark.timeout(120)
def test_mixed_group_keeps_gpu_members_on_rccl(fake):
    """Two RCCL-capable members + one CPU (gloo) member: the group communicator is hybrid — the
    GPU pair's transfers go through RCCL, only the pairs with the CPU member over gloo — and the
    average is exact."""
    from dedloc_amd.dht import DHT

    root = DHT(listen_on="127.0.0.1:*")
    dhts = [DHT(initial_peers=[root.endpoint], listen=False) for _ in range(3)]
    names = [b"gpu-a", b"gpu-b", b"cpu-c"]
    members = [(b"gpu-a", {"backend": "rccl", "comms": []}), (b"gpu-b", {"backend": "rccl", "comms": []}),
               (b"cpu-c", {"backend": "gloo", "comms": []})]
    xs = [torch.full((96,), float(r + 1)) for r in range(3)]
    try:
        def rank(r):
            g = C.GroupCommunicators(dhts[r], "mixed", names[r], torch.device("cpu"), timeout_s=30)
            comm, rank_of = g.get(members, b"round-0")
            assert comm.backend == "rccl+gloo"
            pids = [m for m, _ in members]
            spec = GroupSpec(ranks=[rank_of[p] for p in pids], part_sizes=[40, 40, 16],
                             weights=[1.0 if k == r else 0.0 for k in range(3)], contributes=[True] * 3, my_index=r)
            x = xs[r].clone()
            butterfly_allreduce([x], spec, "NONE", comm=comm, timeout=20)
            g.close()
            return x, comm.rccl is not None

        out, errs = _run_ranks(3, rank)
        assert not errs, errs
        for r in range(3):
            torch.testing.assert_close(out[r][0], torch.full((96,), 2.0))
        assert [out[r][1] for r in range(3)] == [True, True, False]
        # RCCL carried the GPU pair's traffic: exactly one 2-rank communicator was built
        assert fake.calls["comm_init"] == 2
    finally:
        for d in dhts:
            d.shutdown()
        root.shutdown()


def test_peers_sharing_a_gpu_take_one_rccl_rank():
    """RCCL takes one rank per device: of several members announcing the same GPU only the first (in
    peer-id order) is an RCCL member, the rest join the group's gloo side — so 8 peers emulated on one
    GPU average over gloo instead of failing communicator set-up every round, and 2 GPUs with 4
    peers each form a hybrid group with one RCCL rank per GPU."""
    G = C.GroupCommunicators
    one_gpu = [(bytes([65 + i]), {"backend": "rccl", "gpu": "host/gpu0"}) for i in range(8)]
    assert G.rccl_members(one_gpu) == [b"A"] and G.group_backend(one_gpu) == "gloo"
    two_gpus = [(bytes([65 + i]), {"backend": "rccl", "gpu": f"host/gpu{i % 2}"}) for i in range(8)]
    assert G.rccl_members(two_gpus) == [b"A", b"B"] and G.group_backend(two_gpus) == "hybrid"
    distinct = [(bytes([65 + i]), {"backend": "rccl", "gpu": f"host/gpu{i}"}) for i in range(4)]
    assert G.group_backend(distinct) == "rccl"
    # members that announce no device identity (older peers) keep the previous rule
    legacy = [(b"x", {"backend": "rccl"}), (b"y", {"backend": "rccl"}), (b"z", {"backend": "gloo"})]
    assert G.rccl_members(legacy) == [b"x", b"y"] and G.group_backend(legacy) == "hybrid"


def test_abandoned_bootstrap_is_quarantined_then_reaped(fake):
    """A member that never arrives: the bootstrap is abandoned at its deadline, but the
    communicator is NOT aborted while RCCL's init thread may still own it (the round-4 SIGSEGV on
    the driver's box came out of this path).  It is quarantined, and the comm worker aborts it as
    soon as the bootstrap ends (here: the late member finally shows up)."""
    uid = W.unique_id()
    t0 = time.monotonic()
    with pytest.raises(C.CommError) as ei:
        C.RcclGroupComm.create(uid, 2, 0, torch.device("cpu"), time.monotonic() + 0.5)
    assert time.monotonic() - t0 < 5 and not ei.value.local
    (h,) = fake.comms
    assert h in fake.quarantine and h not in fake.aborted
    assert W.CommWorker.get().quarantined >= 1
    with fake.lock:  # the missing member bootstraps late: RCCL's init ends, the reaper may abort
        fake.joined[fake.comms[h]["uid"]].add(1)
    t0 = time.monotonic()
    while h not in fake.aborted and time.monotonic() - t0 < 10:
        time.sleep(0.05)
    assert h in fake.aborted and not fake.quarantine
    assert fake.threads == {"comm-worker"}


def test_same_device_donor_answers_over_tcp(fake):
    """A requester on the donor's own GPU (peers sharing a device) is served over TCP, and no
    communicator is ever initialised for it (RCCL takes one rank per device)."""
    from dedloc_amd.averaging.averager import StateServer, download_state

    state = [torch.randn(64)]
    srv = StateServer(lambda: ({"step": 3}, [t.clone() for t in state]), "127.0.0.1:0", device=torch.device("cpu"),
                      gpu_id="host/gpu0")
    try:
        meta, tensors = download_state(srv.endpoint, timeout=20, device=torch.device("cpu"), allow_rccl=True,
                                       gpu_id="host/gpu0")
        assert meta["_mode"] == "T" and fake.calls["comm_init"] == 0
        torch.testing.assert_close(tensors[0], state[0])
        # another device on the same host: the RCCL path
        meta, tensors = download_state(srv.endpoint, timeout=20, device=torch.device("cpu"), allow_rccl=True,
                                       gpu_id="host/gpu1")
        assert meta["_mode"] == "R" and fake.calls["comm_init"] == 2
        torch.testing.assert_close(tensors[0], state[0])
    finally:
        srv.shutdown()


def test_legacy_uid_only_request_is_served_without_stalling(fake):
    """a requester on the pre-GPU-identity format sends ``STATER`` + the unique id only;
    the donor must answer it at once (the extended request has its own mode byte, ``G``) instead of
    waiting for a GPU-identity field that never comes."""
    import socket
    import struct

    import msgpack

    from dedloc_amd.averaging.averager import StateServer

    state = [torch.randn(50)]
    srv = StateServer(lambda: ({"step": 2}, [t.clone() for t in state]), "127.0.0.1:0", device=torch.device("cpu"),
                      transfer_timeout=10)
    try:
        uid = C.RcclGroupComm.new_unique_id()
        host, port = srv.endpoint.split(":")
        t0 = time.monotonic()
        with socket.create_connection((host, int(port)), timeout=10) as s:
            s.sendall(b"STATER" + uid)
            (hl,) = struct.unpack("<Q", s.recv(8, socket.MSG_WAITALL))
            header = msgpack.unpackb(s.recv(hl, socket.MSG_WAITALL), raw=False)
            assert header["mode"] == "R" and time.monotonic() - t0 < 5
            out = torch.empty(50)
            comm = C.pairwise_rccl(uid, 1, torch.device("cpu"), time.monotonic() + 10)
            comm.p2p([], [], [out], [0], time.monotonic() + 10)
            comm.abort()
        torch.testing.assert_close(out, state[0])
    finally:
        srv.shutdown()
