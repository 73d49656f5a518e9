"""RCCL group-communicator plumbing on one GPU (a world of one rank, in a child process): member-only
group creation without ncclCommSplit, batched P2P with host-polled completion (the path the
butterfly uses), and abort of a group communicator — the NCCL-specific code the CPU/gloo
multi-process tests cannot reach."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import os, time, torch, torch.distributed as dist
    import dedloc_amd.ops
    from dedloc_amd.parallel import init_world, GroupCommunicators, abort_group
    from dedloc_amd.averaging.allreduce import _run_p2p
    rank, world, dev = init_world(force=True)
    assert dist.get_backend() == "nccl" and dev.type == "cuda"
    assert dist.distributed_c10d._get_default_group().bound_device_id is None
    comms = GroupCommunicators(timeout_s=60)
    pg = comms.get([0], 0)
    assert dist.get_backend(pg) == "nccl"
    src = torch.arange(1024, device=dev, dtype=torch.float16)
    dst = torch.zeros_like(src)
    _run_p2p([dist.P2POp(dist.isend, src, 0, group=pg), dist.P2POp(dist.irecv, dst, 0, group=pg)],
             time.monotonic() + 30, pg)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert comms.get([0], 0) is pg and comms.created == 1
    comms.invalidate([0], 0)
    assert comms.aborted == 1
    pg2 = comms.get([0], 1)
    dst.zero_()
    _run_p2p([dist.P2POp(dist.isend, src, 0, group=pg2), dist.P2POp(dist.irecv, dst, 0, group=pg2)],
             time.monotonic() + 30, pg2)
    torch.cuda.synchronize()
    assert torch.equal(src, dst) and comms.created == 2
    comms.close()
    dist.destroy_process_group()
    print("RCCL_GROUP_OK", flush=True)
""")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(180)
def test_rccl_group_communicator_lifecycle(cuda):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0 and "RCCL_GROUP_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
