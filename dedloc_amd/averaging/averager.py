"""DecentralizedAverager / TrainingAverager (hivemind 0.9.x equivalents).

In-process design (no helper processes, no host staging of the averaged tensors):
  * matchmaking through the control-plane DHT (``DHT.join_group``): a group closes at
    ``target_group_size``, when every live peer of the collaboration has joined, or when the
    ``averaging_expiration`` window of its first member ends;
  * the data plane is the butterfly all-reduce (``allreduce.butterfly_allreduce``) with LP-balanced
    parts and FLOAT16/BFLOAT16 wire compression, on a communicator the group's members build
    through the DHT (``parallel.GroupCommunicators``: RCCL between GPU peers, gloo when a CPU peer
    is a member).  Nothing depends on a launch-time world, so any process that can reach the DHT
    — a late volunteer, a respawned spot instance — averages in the next round it joins.  A failed
    round aborts its communicator; members reuse a communicator only while all of them still hold
    it;
  * state sharing: every peer with ``allow_state_sharing`` runs a state server (``listen_on``) and
    advertises it under ``{prefix}_state_sharing``; ``load_state_from_peers`` downloads (metadata,
    tensors) from the freshest donor — GPU to GPU over a one-off RCCL communicator, or streamed over
    TCP for CPU peers (``StateServer``).
"""
from __future__ import annotations

import logging
import socket
import struct
import threading
import time
from concurrent.futures import Future
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import msgpack
import torch

from ..dht import DHT, get_dht_time, parse_endpoint
from ..parallel import comm as _comm
from ..parallel.comm import CommError, GroupCommunicators, RcclGroupComm, pairwise_rccl, routable_host
from .allreduce import GroupSpec, WIRE_DTYPES, butterfly_allreduce
from .load_balancing import load_balance_peers

logger = logging.getLogger(__name__)

_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16, "int64": torch.int64}


_CHUNK = 32 << 20  # bytes per host-staging chunk of a GPU tensor sent over TCP


def _recv_exact(sock, n):
    buf = bytearray(n)
    _recv_into(sock, memoryview(buf))
    return bytes(buf)


def _recv_into(sock, view: memoryview):
    got, n = 0, len(view)
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k


def _byte_view(t: torch.Tensor) -> memoryview:
    """Zero-copy bytes of a contiguous CPU tensor."""
    return memoryview(t.reshape(-1).view(torch.uint8).numpy())


class StateServer:
    """Serves ``get_state() -> (metadata, [tensors])`` to joining peers.

    Request: ``b"STATE" + mode`` with mode ``G`` (followed by a 128-byte RCCL unique id made by the
    requester, then the requester's GPU identity as a 2-byte length + UTF-8), ``R`` (the unique id
    only: the format of peers from before the GPU identity existed, still accepted) or ``T``.  RCCL takes
    one rank per device, so a requester on the donor's own GPU is always answered over TCP: two
    ranks of one device are never put into a communicator (that only exercises RCCL's error and
    abort path, which crashed a peer on the driver's box in round 4).  A GPU donor answers an ``R`` request by sending the snapshot device-to-
    device over a 2-rank RCCL communicator on its own HIP stream (no host staging at all); otherwise
    the tensors are streamed over TCP — GPU tensors through two pinned host chunks (the D2H copy of
    chunk i+1 overlaps the socket send of chunk i), CPU tensors straight from their storage (no
    ``tobytes`` copies).  The trainer only ever blocks for the snapshot itself: ``get_state`` clones
    the state on the device under the optimizer's step lock and the transfer runs outside it."""

    def __init__(self, get_state: Callable[[], Tuple[Dict, List[torch.Tensor]]], listen_on: str = "0.0.0.0:0",
                 device: Optional[torch.device] = None, transfer_timeout: float = 120.0,
                 gpu_id: Optional[str] = None):
        host, port = parse_endpoint(listen_on.replace("*", "0"))
        bind = "0.0.0.0" if listen_on.startswith(("0.0.0.0", "[::]", "*")) else host
        self.get_state = get_state
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.transfer_timeout = transfer_timeout
        self.gpu_id = gpu_id
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((bind, port))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        # the address published through the DHT: routable from other machines
        self.endpoint = f"{routable_host(bind)}:{self.port}"
        self.served = {"R": 0, "T": 0}
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True, name="state-server")
        self.thread.start()

    def _loop(self):
        while not self._stop.is_set():
            try:
                conn, _ = self.sock.accept()
            except OSError:
                break
            threading.Thread(target=self._serve, args=(conn,), daemon=True, name="state-transfer").start()

    def _serve(self, conn):
        try:
            with conn:
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                req = _recv_exact(conn, 6)
                if req[:5] != b"STATE":
                    return
                uid, their_gpu = None, None
                if req[5:6] in (b"R", b"G"):
                    uid = _recv_exact(conn, 128)
                if req[5:6] == b"G":
                    (n,) = struct.unpack("<H", _recv_exact(conn, 2))
                    their_gpu = _recv_exact(conn, n).decode() if n else None
                if self.device.type == "cuda":
                    torch.cuda.set_device(self.device)
                meta, tensors = self.get_state()
                same_device = their_gpu is not None and their_gpu == self.gpu_id
                rccl = (uid is not None and not same_device and _comm.rccl_available(self.device)
                        and all(t.device == self.device for t in tensors))
                descs = [(str(t.dtype).replace("torch.", ""), list(t.shape)) for t in tensors]
                header = msgpack.packb({"metadata": meta, "tensors": descs, "mode": "R" if rccl else "T"},
                                       use_bin_type=True)
                conn.sendall(struct.pack("<Q", len(header)) + header)
                if rccl:
                    self._send_rccl(uid, tensors)
                    self.served["R"] += 1
                else:
                    self._send_tcp(conn, tensors)
                    self.served["T"] += 1
        except Exception as e:  # noqa: BLE001
            logger.warning(f"state transfer failed: {e}")

    def _send_rccl(self, uid: bytes, tensors: List[torch.Tensor]):
        deadline = time.monotonic() + self.transfer_timeout
        comm = pairwise_rccl(uid, 0, self.device, deadline)
        try:
            if self.device.type == "cuda":
                ready = torch.cuda.Event()
                ready.record()  # the snapshot clones were queued on this thread's current stream
                stream = torch.cuda.Stream(self.device)
                with torch.cuda.stream(stream):
                    stream.wait_event(ready)
                    comm.p2p([t.reshape(-1) for t in tensors], [1] * len(tensors), [], [], deadline)
            else:
                comm.p2p([t.reshape(-1) for t in tensors], [1] * len(tensors), [], [], deadline)
        finally:
            comm.abort()

    def _send_tcp(self, conn, tensors: List[torch.Tensor]):
        staging, stream = None, None
        for t in tensors:
            nbytes = t.numel() * t.element_size()
            conn.sendall(struct.pack("<Q", nbytes))
            if not t.is_cuda:
                if nbytes:
                    conn.sendall(_byte_view(t.detach().contiguous()))
                continue
            if staging is None:
                staging = [torch.empty(_CHUNK, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
                stream = torch.cuda.Stream(t.device)
                ready = torch.cuda.Event()
                ready.record()
                stream.wait_event(ready)
            flat = t.detach().reshape(-1).view(torch.uint8)
            events, offs = [], list(range(0, nbytes, _CHUNK))
            with torch.cuda.stream(stream):
                for i, off in enumerate(offs[:2]):
                    n = min(_CHUNK, nbytes - off)
                    staging[i % 2][:n].copy_(flat[off:off + n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    events.append(ev)
                for i, off in enumerate(offs):
                    n = min(_CHUNK, nbytes - off)
                    events[i].synchronize()
                    conn.sendall(_byte_view(staging[i % 2])[:n])
                    j = i + 2
                    if j < len(offs):  # refill this buffer with chunk i+2 while chunk i+1 is sent
                        m = min(_CHUNK, nbytes - offs[j])
                        staging[j % 2][:m].copy_(flat[offs[j]:offs[j] + m], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(stream)
                        events.append(ev)

    def shutdown(self):
        self._stop.set()
        try:
            self.sock.close()
        except OSError:
            pass


def download_state(endpoint: str, timeout: float = 60.0, device: Optional[torch.device] = None,
                   allow_rccl: bool = True, gpu_id: Optional[str] = None):
    """(metadata, tensors) from a state server.  A GPU requester asks for the RCCL transfer (the
    tensors arrive on ``device``) and names its GPU (``gpu_id``: a donor on the same device answers
    over TCP); otherwise the tensors arrive over TCP into host memory.  The metadata carries the
    transfer mode under ``_mode`` ("R" or "T")."""
    host, port = parse_endpoint(endpoint)
    device = torch.device(device) if device is not None else torch.device("cpu")
    uid = RcclGroupComm.new_unique_id() if allow_rccl and _comm.rccl_available(device) else None
    deadline = time.monotonic() + timeout
    with socket.create_connection((host, port), timeout=timeout) as s:
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if uid is not None:
            g = (gpu_id or "").encode()
            s.sendall(b"STATEG" + uid + struct.pack("<H", len(g)) + g)
        else:
            s.sendall(b"STATET")
        (hl,) = struct.unpack("<Q", _recv_exact(s, 8))
        header = msgpack.unpackb(_recv_exact(s, hl), raw=False)
        descs = [(_DT[dt], shape) for dt, shape in header["tensors"]]
        if header.get("mode") == "R":
            out = [torch.empty(shape, dtype=dt, device=device) for dt, shape in descs]
            comm = pairwise_rccl(uid, 1, device, deadline)
            try:
                comm.p2p([], [], [t.reshape(-1) for t in out], [0] * len(out), deadline)
            finally:
                comm.abort()
            return dict(header["metadata"], _mode="R"), out
        out = []
        for dt, shape in descs:
            (nb,) = struct.unpack("<Q", _recv_exact(s, 8))
            t = torch.empty(shape, dtype=dt)
            if nb:
                _recv_into(s, _byte_view(t))
            out.append(t)
        return dict(header["metadata"], _mode="T"), out


class DecentralizedAverager:
    def __init__(self, averaged_tensors: Sequence[torch.Tensor], dht: DHT, prefix: str, *, peer_id: bytes,
                 target_group_size: int = 256, min_group_size: int = 2, averaging_expiration: float = 5.0,
                 averaging_timeout: float = 30.0, compression: str = "FLOAT16", throughput: Optional[float] = None,
                 client_mode: bool = False, auxiliary: bool = False, allow_state_sharing: bool = True,
                 listen_on: str = "0.0.0.0:*", metadata_expiration: float = 30.0, device: Optional[torch.device] = None,
                 max_cached_comms: int = 8, emulate_transfer_delay: bool = False, **_unused):
        self.averaged_tensors = list(averaged_tensors)
        self.dht, self.prefix, self.peer_id = dht, prefix, bytes(peer_id)
        self.target_group_size, self.min_group_size = target_group_size, min_group_size
        self.averaging_expiration, self.averaging_timeout = averaging_expiration, averaging_timeout
        if compression not in WIRE_DTYPES:
            raise ValueError(f"unknown compression {compression}; expected one of {sorted(WIRE_DTYPES)}")
        self.compression = compression
        self.throughput = throughput
        self.client_mode, self.auxiliary = client_mode, auxiliary
        self.allow_state_sharing = allow_state_sharing and not auxiliary
        self.metadata_expiration = metadata_expiration
        if device is None:
            device = self.averaged_tensors[0].device if self.averaged_tensors else torch.device("cpu")
        self.device = torch.device(device)
        host = parse_endpoint(listen_on.replace("*", "0").replace("[::]", "0.0.0.0"))[0]
        self.host = routable_host(host)  # published for gloo rendezvous: reachable by other machines
        self.comms = GroupCommunicators(dht, prefix, self.peer_id, self.device,
                                        timeout_s=max(30.0, 2 * averaging_timeout), max_cached=max_cached_comms,
                                        host=self.host)
        self.lock_averaged_tensors = threading.RLock()
        self.last_group: Optional[Dict] = None
        self.state_server = StateServer(self._serve_state, listen_on.replace("[::]", "0.0.0.0"), device=self.device,
                                        gpu_id=self.comms.gpu_id) if self.allow_state_sharing else None
        self.local_step_for_state = 0
        self.last_download: Optional[Dict] = None
        self.emulate_transfer_delay = emulate_transfer_delay

    # ------------------------------------------------------------------ averaging
    # Load balancing in a mixed group (GPU trainers on RCCL + CPU peers on gloo), in the Mbps unit of
    # the reference's --bandwidth: an RCCL member's link is one xGMI link (~153 GB/s); a CPU member
    # keeps its declared --bandwidth, or DEFAULT_HOST_MBPS (a 10 Gb/s host link) when it declared
    # none.  The LP minimises the round's slowest member, so a CPU member gets a part only when its
    # link is fast enough not to become that member: with xGMI peers that means a CPU auxiliary
    # needs a declared --bandwidth comparable to xGMI, otherwise it owns no part (it then neither
    # sends nor receives — it cannot slow the GPU members down).
    XGMI_MBPS = 1.2e6
    DEFAULT_HOST_MBPS = 1.0e4

    @classmethod
    def group_bandwidths(cls, infos: Sequence[Dict], pids: Sequence[bytes], on_rccl) -> List[Optional[float]]:
        """Per-member throughputs for the LP (``on_rccl``: peer ids on the RCCL side of a mixed
        group, None for a homogeneous group, whose undeclared members get the mean of the declared
        ones — all equal when nobody declared)."""
        bws = [i.get("bandwidth") for i in infos]
        if on_rccl is None:
            return bws
        return [(cls.XGMI_MBPS if (b is None or b > 0) else 0.0) if p in on_rccl
                else (cls.DEFAULT_HOST_MBPS if b is None else b) for b, p in zip(bws, pids)]

    def _info(self, weight: Optional[float], gather: Optional[Dict[str, Any]]) -> Dict:
        bw = 0.0 if self.client_mode else self.throughput  # None: not declared
        info = {"bandwidth": bw, "weight": weight, "aux": self.auxiliary, "gather": gather or {}}
        info.update(self.comms.announce())
        return info

    def _join(self, info: Dict, expected_group_size: int, key_suffix: str):
        window = self.averaging_expiration
        t0 = time.perf_counter()
        ok, gid, members = self.dht.join_group(f"{self.prefix}_averaging{key_suffix}".encode(), self.peer_id, info,
                                               self.target_group_size, self.min_group_size, expected_group_size,
                                               window, timeout=window + 10.0)
        return ok, gid, members, time.perf_counter() - t0

    def prejoin(self, expected_group_size: int = 0, gather: Optional[Dict[str, Any]] = None,
                key_suffix: str = "") -> Future:
        """Start matchmaking for the next round in the background and return its future, to be passed
        to ``step(prejoined=...)``.  The collaborative optimizer calls this when the NEXT micro-step
        will complete the global batch (``albert/arguments.py:67-70``, batch_size_lead: "begin
        looking for group in advance"), so the group forms while that micro-step computes.  The
        weight is not known yet and need not be: weights travel with the data (allreduce.py)."""
        fut: Future = Future()
        info = self._info(None if not self.auxiliary else 0.0, gather)

        def run():
            try:
                fut.set_result(self._join(info, expected_group_size, key_suffix))
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)

        threading.Thread(target=run, daemon=True, name="prejoin").start()
        return fut

    def step(self, weight=1.0, timeout: Optional[float] = None, expected_group_size: int = 0,
             gather: Optional[Dict[str, Any]] = None, tensors: Optional[Sequence[torch.Tensor]] = None,
             sources: Optional[Sequence[torch.Tensor]] = None, key_suffix: str = "",
             prejoined: Optional[Future] = None) -> Optional[Dict]:
        """Matchmake and average.  Returns {"group_id", "size", "gathered"} or None on failure.

        ``tensors`` overrides the averaged set for this round (e.g. gradients only), ``sources`` packs
        snapshots instead of the live tensors, ``key_suffix`` selects an independent matchmaking key
        (so a delayed parameter round never mixes with a gradient round), ``prejoined`` is a
        ``prejoin`` future whose group this round uses (a fresh matchmaking if it failed)."""
        tensors = list(tensors) if tensors is not None else self.averaged_tensors
        # a device-scalar weight (CollaborativeOptimizer's finite-sample count) travels as is
        weight = 0.0 if self.auxiliary else (weight if isinstance(weight, torch.Tensor) else float(weight))
        t_wait = time.perf_counter()
        res = None
        if prejoined is not None:
            try:
                res = prejoined.result(timeout=self.averaging_expiration + 15.0)
                if not res[0] or len(res[2]) < self.min_group_size:
                    res = None
            except Exception as e:  # noqa: BLE001
                logger.info(f"matchmaking ahead of the step failed ({e}); joining now")
                res = None
        if res is None:
            try:
                res = self._join(self._info(weight if not isinstance(weight, torch.Tensor) else None, gather),
                                 expected_group_size, key_suffix)
            except Exception as e:  # noqa: BLE001
                logger.warning(f"matchmaking failed: {e}")
                return None
        ok, gid, members, t_match_total = res
        t_match = time.perf_counter() - t_wait  # matchmaking time this step actually waited for
        if not ok or len(members) < self.min_group_size:
            logger.info(f"averaging round failed: group of {len(members)} < {self.min_group_size}")
            return None
        infos = [m[1] for m in members]
        pids = [bytes(m[0]) for m in members]
        my_index = pids.index(self.peer_id)
        V = sum(t.numel() for t in tensors)
        hybrid = GroupCommunicators.group_backend(members) == "hybrid"
        bws = self.group_bandwidths(infos, pids, set(GroupCommunicators.rccl_members(members)) if hybrid else None)
        parts = load_balance_peers(V, bws, min_size=0)
        if not any(not i["aux"] for i in infos):
            return None
        t0 = time.perf_counter()
        deadline = time.monotonic() + (timeout or self.averaging_timeout)
        comm = None
        try:
            comm, rank_of = self.comms.get(members, gid, deadline)
            spec = GroupSpec(ranks=[rank_of[p] for p in pids], part_sizes=list(parts),
                             weights=[weight if k == my_index else 0.0 for k in range(len(pids))],
                             contributes=[not i["aux"] for i in infos], my_index=my_index)
            with self.lock_averaged_tensors:
                butterfly_allreduce(tensors, spec, self.compression, comm=comm,
                                    timeout=max(1e-3, deadline - time.monotonic()), sources=sources)
        except (CommError, RuntimeError) as e:
            # the communicator may still hold posted operations: it is aborted and forgotten, so the
            # next round between these peers runs on a fresh one
            logger.warning(f"all-reduce failed ({e}); skipping this round")
            if comm is not None:
                self.comms.invalidate(comm)
            return None
        bw = bws[my_index]
        if self.emulate_transfer_delay and bw is not None and bw > 0:  # emulate the volunteer's link (AWS_runner wondershaper caps)
            from ..emulation.heterogeneity import emulated_transfer_seconds

            wire_bytes = torch.empty(0, dtype=WIRE_DTYPES[self.compression]).element_size()
            want = 2 * emulated_transfer_seconds(V, wire_bytes, len(members), parts[my_index] / max(1, V), bw)
            spent = time.perf_counter() - t0
            if want > spent:
                time.sleep(want - spent)
        self.last_group = {"group_id": gid, "size": len(members), "gathered": [i["gather"] for i in infos],
                           "matchmaking_s": t_match, "matchmaking_total_s": t_match_total,
                           "prejoined": prejoined is not None, "allreduce_s": time.perf_counter() - t0,
                           "parts": list(parts), "backend": comm.backend if comm is not None else None}
        return self.last_group

    # ------------------------------------------------------------------ state sharing
    def get_current_state(self) -> Tuple[Dict, List[torch.Tensor]]:
        with self.lock_averaged_tensors:
            return {"step": self.local_step_for_state}, [t.detach().clone() for t in self.averaged_tensors]

    def _serve_state(self):
        return self.get_current_state()

    def publish_state_sharing(self, step: int):
        """Advertise this peer's state server (asynchronous DHT store: the returned future resolves
        once the record is stored)."""
        if self.state_server is None:
            return None
        self.local_step_for_state = step
        return self.dht.store(f"{self.prefix}_state_sharing",
                              {"endpoint": self.state_server.endpoint, "step": int(step), "gpu": self.comms.gpu_id},
                              get_dht_time() + self.metadata_expiration, subkey=self.peer_id, return_future=True)

    def load_state_from_peers(self, timeout: float = 15.0, min_step: int = 0):
        """(metadata, tensors) from the freshest state-sharing peer whose advertised step is at least
        ``min_step``, or None if nobody qualifies (peers that are not ahead have nothing to give: a
        fresh collaboration of peers all at step 0 starts at once instead of downloading in a circle)."""
        rec = self.dht.get(f"{self.prefix}_state_sharing", latest=True)
        if rec is None or not isinstance(rec.value, dict):
            return None
        donors = []
        for sub, v in rec.value.items():
            if sub == self.peer_id or not isinstance(v.value, dict):
                continue
            if int(v.value.get("step", 0)) < min_step:
                continue
            donors.append((v.value.get("step", 0), v.value["endpoint"], v.value.get("gpu")))
        mine = self.comms.gpu_id
        for step, ep, gpu in sorted(donors, key=lambda d: (d[0], d[1]), reverse=True):
            # RCCL only between two different devices (one rank per device): a donor on our own GPU
            # — peers sharing a device in a protocol emulation — streams over TCP straight away
            rccl_ok = _comm.rccl_available(self.device) and not (gpu is not None and gpu == mine)
            for rccl in ((True, False) if rccl_ok else (False,)):
                try:
                    t0 = time.perf_counter()
                    meta, tensors = download_state(ep, timeout=timeout, device=self.device, allow_rccl=rccl,
                                                   gpu_id=mine)
                    self.last_download = {"endpoint": ep, "mode": meta.pop("_mode", "T"),
                                          "bytes": sum(t.numel() * t.element_size() for t in tensors),
                                          "seconds": time.perf_counter() - t0}
                    logger.info(f"downloaded state (step {meta.get('step')}) from {ep}: {self.last_download}")
                    return meta, tensors
                except Exception as e:  # noqa: BLE001
                    logger.warning(f"failed to download state from {ep} ({'RCCL' if rccl else 'TCP'}): {e}")
        return None

    def shutdown(self):
        if self.state_server is not None:
            self.state_server.shutdown()
        self.comms.close()
