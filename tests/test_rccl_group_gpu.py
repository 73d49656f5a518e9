"""The native RCCL data plane (csrc/comm/rccl_comm.cpp, parallel/comm.py) on one GPU, in a child
process with no torch.distributed world at all:

* a communicator bootstrapped through the DHT by ``GroupCommunicators`` (the leader publishes the
  unique id), non-blocking init polled to readiness, grouped send/recv (to itself: a one-rank
  group) with host-polled completion, reuse of the cached communicator, abort;
* a bootstrap whose second member never arrives is abandoned at the deadline (the host never
  hangs in ncclCommInitRank); the communicator is QUARANTINED, not aborted, while RCCL's init
  thread still owns it (csrc/comm/comm_core.h) — aborting an in-flight bootstrap, or putting two
  ranks of one device into a communicator, is what SIGSEGV'd this child on the driver's box in
  round 4 (GPUTEST_r04.json);
* a peer state download between two peers on ONE device: the donor's record names its GPU, so the
  requester goes straight to the TCP stream (no communicator is ever initialised for it) and the
  exact tensors arrive (on a multi-GPU node the RCCL path carries a download between devices).

The child runs with faulthandler on every thread and prints a flushed marker around each phase,
so a native crash names its phase and the Python stacks of all threads.

Multi-rank RCCL traffic between GPUs needs a multi-GPU node (the driver's scaling bench); the
CPU/gloo multi-process tests cover the protocol with any number of ranks."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import faulthandler, os, sys, time, torch
    faulthandler.enable(file=sys.stderr, all_threads=True)
    def mark(m):
        print("@@", m, flush=True)
    import torch.distributed as dist
    import dedloc_amd.ops
    from dedloc_amd.dht import DHT
    from dedloc_amd.parallel import CommError, GroupCommunicators, RcclGroupComm, local_device, rccl_available
    from dedloc_amd.parallel.comm_worker import CommWorker
    dev = local_device()
    assert not dist.is_initialized()
    assert rccl_available(dev), "the native RCCL data plane must be built into _C.so"
    root = DHT(listen_on="127.0.0.1:*")
    comms = GroupCommunicators(root, "rccl-test", b"solo", dev, timeout_s=60)
    members = [(b"solo", comms.announce())]
    assert members[0][1]["backend"] == "rccl"
    mark("bootstrap 1-rank")
    comm, rank_of = comms.get(members, b"round-1")
    assert comm.backend == "rccl" and rank_of == {b"solo": 0} and comms.created == 1
    src = torch.arange(1 << 20, device=dev, dtype=torch.float16)
    dst = torch.zeros_like(src)
    mark("p2p")
    comm.p2p([src], [0], [dst], [0], time.monotonic() + 30)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    # the next round announces the token and reuses the communicator
    members = [(b"solo", comms.announce())]
    comm2, _ = comms.get(members, b"round-2")
    assert comm2 is comm and comms.created == 1
    mark("abort ready communicator")
    comms.invalidate(comm)
    assert comms.aborted == 1 and not comm.alive
    assert torch.ops.dedloc_comm.comm_count() == 0
    # a member that never shows up: the bootstrap is abandoned at the deadline
    mark("abandoned bootstrap")
    uid = RcclGroupComm.new_unique_id()
    t0 = time.monotonic()
    try:
        RcclGroupComm.create(uid, 2, 0, dev, time.monotonic() + 5.0)
        raise SystemExit("a 2-rank communicator came up with one rank")
    except CommError as e:
        waited = time.monotonic() - t0
        assert waited < 30, waited
        print("abandoned bootstrap after", round(waited, 2), "s:", e, flush=True)
    mark("after abandon")
    # quarantined, not aborted: RCCL's init thread may still be waiting for the missing member
    assert torch.ops.dedloc_comm.comm_count() == 0
    assert torch.ops.dedloc_comm.comm_quarantined() == 1 and CommWorker.get().quarantined >= 1
    # state download between two peers of one GPU: straight to TCP, no communicator at all
    mark("state download")
    from dedloc_amd.averaging.averager import DecentralizedAverager
    x = torch.randn(3_000_000, device=dev)
    m = torch.randn(3_000_000, device=dev)
    donor = DecentralizedAverager([x, m], root, "rccl-test", peer_id=b"donor", device=dev,
                                  listen_on="127.0.0.1:*")
    donor.publish_state_sharing(5).result(timeout=30)
    rx = DecentralizedAverager([torch.zeros_like(x), torch.zeros_like(m)], root, "rccl-test", peer_id=b"rx",
                               device=dev, listen_on="127.0.0.1:*", allow_state_sharing=False)
    meta, tensors = rx.load_state_from_peers(timeout=30)
    assert meta["step"] == 5
    assert torch.equal(tensors[0].to(dev), x) and torch.equal(tensors[1].to(dev), m)
    print("download", rx.last_download, flush=True)
    t0 = time.monotonic()
    while donor.state_server.served["T"] < 1 and time.monotonic() - t0 < 10:  # counted after the send
        time.sleep(0.01)
    assert rx.last_download["mode"] == "T" and donor.state_server.served == {"R": 0, "T": 1}
    assert torch.ops.dedloc_comm.comm_count() == 0 and torch.ops.dedloc_comm.comm_quarantined() == 1
    mark("shutdown")
    donor.shutdown(); rx.shutdown(); comms.close(); root.shutdown()
    print("RCCL_NATIVE_OK", flush=True)
""")


@pytest.mark.timeout(240)
def test_native_rccl_group_comm_lifecycle(cuda):
    env = dict(os.environ, PYTHONPATH=ROOT, LOCAL_RANK="0")
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=220)
    print(r.stdout[-3000:])
    assert r.returncode == 0 and "RCCL_NATIVE_OK" in r.stdout, (r.stdout[-3000:], r.stderr[-5000:])
