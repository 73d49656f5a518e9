"""DecentralizedAverager / TrainingAverager (hivemind 0.9.x equivalents).

In-process design (no helper processes, no host staging of the averaged tensors):
  * matchmaking through the control-plane DHT (``DHT.join_group``): a group closes at
    ``target_group_size``, when every live peer of the collaboration has joined, or when the
    ``averaging_expiration`` window of its first member ends;
  * the data plane is the butterfly all-reduce (``allreduce.butterfly_allreduce``) with LP-balanced
    parts and FLOAT16/BFLOAT16 wire compression, on a group communicator keyed by (member set,
    data-plane epoch) (``parallel.GroupCommunicators``).  Every member announces its epoch in its
    matchmaking info and the group runs on epoch max(announced), so all members pick the same
    communicator; a failed round aborts that communicator and the member moves to epoch + 1, which
    forces a fresh communicator the next time it averages with any of those peers;
  * state sharing: every peer with ``allow_state_sharing`` runs a small TCP state server
    (``listen_on``) and advertises it under ``{prefix}_state_sharing``; ``load_state_from_peers``
    downloads (metadata, tensors) from the freshest donor.
"""
from __future__ import annotations

import logging
import socket
import struct
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import msgpack
import numpy as np
import torch
import torch.distributed as dist

from ..dht import DHT, get_dht_time, parse_endpoint
from .allreduce import AllreduceException, GroupSpec, WIRE_DTYPES, butterfly_allreduce
from .load_balancing import load_balance_peers

logger = logging.getLogger(__name__)

_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16, "int64": torch.int64}


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k
    return bytes(buf)


class StateServer:
    """Serves ``get_state() -> (metadata, [tensors])`` to joining peers over TCP."""

    def __init__(self, get_state: Callable[[], Tuple[Dict, List[torch.Tensor]]], listen_on: str = "0.0.0.0:0"):
        host, port = parse_endpoint(listen_on.replace("*", "0"))
        bind = "0.0.0.0" if listen_on.startswith(("0.0.0.0", "[::]", "*")) else host
        self.get_state = get_state
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((bind, port))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        self.endpoint = f"{'127.0.0.1' if bind == '0.0.0.0' else bind}:{self.port}"
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True, name="state-server")
        self.thread.start()

    def _loop(self):
        while not self._stop.is_set():
            try:
                conn, _ = self.sock.accept()
            except OSError:
                break
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn):
        try:
            with conn:
                req = _recv_exact(conn, 5)
                if req != b"STATE":
                    return
                meta, tensors = self.get_state()
                descs = [(str(t.dtype).replace("torch.", ""), list(t.shape)) for t in tensors]
                header = msgpack.packb({"metadata": meta, "tensors": descs}, use_bin_type=True)
                conn.sendall(struct.pack("<Q", len(header)) + header)
                for t in tensors:
                    arr = t.detach().contiguous().cpu()
                    conn.sendall(struct.pack("<Q", arr.numel() * arr.element_size()))
                    conn.sendall(arr.view(torch.uint8).numpy().tobytes() if arr.dtype == torch.bfloat16
                                 else arr.numpy().tobytes())
        except Exception as e:  # noqa: BLE001
            logger.debug(f"state transfer failed: {e}")

    def shutdown(self):
        self._stop.set()
        try:
            self.sock.close()
        except OSError:
            pass


def download_state(endpoint: str, timeout: float = 60.0):
    host, port = parse_endpoint(endpoint)
    with socket.create_connection((host, port), timeout=timeout) as s:
        s.sendall(b"STATE")
        (hl,) = struct.unpack("<Q", _recv_exact(s, 8))
        header = msgpack.unpackb(_recv_exact(s, hl), raw=False)
        tensors = []
        for dtype, shape in header["tensors"]:
            (nb,) = struct.unpack("<Q", _recv_exact(s, 8))
            raw = bytearray(_recv_exact(s, nb))
            t = torch.frombuffer(raw, dtype=_DT[dtype]).reshape(shape) if nb else torch.empty(shape, dtype=_DT[dtype])
            tensors.append(t)
        return header["metadata"], tensors


class DecentralizedAverager:
    def __init__(self, averaged_tensors: Sequence[torch.Tensor], dht: DHT, prefix: str, *, peer_id: bytes,
                 target_group_size: int = 256, min_group_size: int = 2, averaging_expiration: float = 5.0,
                 averaging_timeout: float = 30.0, compression: str = "FLOAT16", throughput: Optional[float] = None,
                 client_mode: bool = False, auxiliary: bool = False, allow_state_sharing: bool = True,
                 listen_on: str = "0.0.0.0:*", metadata_expiration: float = 30.0, pg=None, rank: Optional[int] = None,
                 emulate_transfer_delay: bool = False, **_unused):
        self.averaged_tensors = list(averaged_tensors)
        self.dht, self.prefix, self.peer_id = dht, prefix, peer_id
        self.target_group_size, self.min_group_size = target_group_size, min_group_size
        self.averaging_expiration, self.averaging_timeout = averaging_expiration, averaging_timeout
        if compression not in WIRE_DTYPES:
            raise ValueError(f"unknown compression {compression}; expected one of {sorted(WIRE_DTYPES)}")
        self.compression = compression
        self.throughput = throughput
        self.client_mode, self.auxiliary = client_mode, auxiliary
        self.allow_state_sharing = allow_state_sharing and not auxiliary
        self.metadata_expiration = metadata_expiration
        self.pg = pg
        self.epoch = 0
        self.comms = None
        if pg is None:
            from ..parallel import GroupCommunicators

            self.comms = GroupCommunicators(timeout_s=max(60.0, 2 * averaging_timeout))
        self.rank = rank if rank is not None else (dist.get_rank() if dist.is_available() and dist.is_initialized() else 0)
        self.lock_averaged_tensors = threading.RLock()
        self.last_group: Optional[Dict] = None
        self.state_server = StateServer(self._serve_state, listen_on.replace("[::]", "0.0.0.0")) \
            if self.allow_state_sharing else None
        self.local_step_for_state = 0
        self.emulate_transfer_delay = emulate_transfer_delay

    # ------------------------------------------------------------------ averaging
    def step(self, weight: float = 1.0, timeout: Optional[float] = None, expected_group_size: int = 0,
             gather: Optional[Dict[str, Any]] = None, tensors: Optional[Sequence[torch.Tensor]] = None,
             sources: Optional[Sequence[torch.Tensor]] = None, key_suffix: str = "") -> Optional[Dict]:
        """Matchmake and average.  Returns {"group_id", "size", "gathered"} or None on failure.

        ``tensors`` overrides the averaged set for this round (e.g. gradients only), ``sources`` packs
        snapshots instead of the live tensors, ``key_suffix`` selects an independent matchmaking key
        (so a delayed parameter round never mixes with a gradient round)."""
        tensors = list(tensors) if tensors is not None else self.averaged_tensors
        if not (dist.is_available() and dist.is_initialized()):
            logger.warning("averaging requires the collaboration's world communicator; skipping")
            return None
        weight = 0.0 if self.auxiliary else float(weight)
        bw = 0.0 if self.client_mode else (self.throughput if self.throughput is not None else 1.0)
        info = {"rank": self.rank, "bandwidth": bw, "weight": weight, "aux": self.auxiliary, "gather": gather or {},
                "epoch": self.epoch}
        window = self.averaging_expiration
        t_join = time.perf_counter()
        try:
            ok, gid, members = self.dht.join_group(f"{self.prefix}_averaging{key_suffix}".encode(), self.peer_id, info,
                                                   self.target_group_size, self.min_group_size,
                                                   expected_group_size, window, timeout=window + 10.0)
        except Exception as e:  # noqa: BLE001
            logger.warning(f"matchmaking failed: {e}")
            return None
        t_match = time.perf_counter() - t_join
        if not ok or len(members) < self.min_group_size:
            logger.info(f"averaging round failed: group of {len(members)} < {self.min_group_size}")
            return None
        infos = [m[1] for m in members]
        my_index = [m[0] for m in members].index(self.peer_id)
        V = sum(t.numel() for t in tensors)
        parts = load_balance_peers(V, [i["bandwidth"] for i in infos], min_size=0)
        spec = GroupSpec(ranks=[i["rank"] for i in infos], part_sizes=list(parts),
                         weights=[i["weight"] for i in infos], contributes=[not i["aux"] for i in infos],
                         my_index=my_index)
        if sum(w for w, c in zip(spec.weights, spec.contributes) if c) <= 0:
            return None
        epoch = max(int(i.get("epoch", 0)) for i in infos)
        self.epoch = max(self.epoch, epoch)
        t0 = time.perf_counter()
        try:
            pg = self.pg if self.pg is not None else self.comms.get(spec.ranks, epoch)
            with self.lock_averaged_tensors:
                butterfly_allreduce(tensors, spec, self.compression, pg=pg,
                                    timeout=timeout or self.averaging_timeout, sources=sources)
        except (AllreduceException, RuntimeError) as e:
            # the communicator may still hold posted operations: abort it and move to a new epoch
            # so no later round can be matched against them
            logger.warning(f"all-reduce failed ({e}); skipping this round (data-plane epoch {epoch} -> {epoch + 1})")
            if self.comms is not None:
                self.comms.invalidate(spec.ranks, epoch)
            self.epoch = max(self.epoch, epoch + 1)
            return None
        if self.emulate_transfer_delay and bw > 0:  # emulate the volunteer's link (AWS_runner wondershaper caps)
            from ..emulation.heterogeneity import emulated_transfer_seconds

            wire_bytes = torch.empty(0, dtype=WIRE_DTYPES[self.compression]).element_size()
            want = 2 * emulated_transfer_seconds(V, wire_bytes, len(members), parts[my_index] / max(1, V), bw)
            spent = time.perf_counter() - t0
            if want > spent:
                time.sleep(want - spent)
        self.last_group = {"group_id": gid, "size": len(members), "gathered": [i["gather"] for i in infos],
                           "matchmaking_s": t_match, "allreduce_s": time.perf_counter() - t0, "parts": list(parts)}
        return self.last_group

    # ------------------------------------------------------------------ state sharing
    def get_current_state(self) -> Tuple[Dict, List[torch.Tensor]]:
        with self.lock_averaged_tensors:
            return {"step": self.local_step_for_state}, [t.detach().clone() for t in self.averaged_tensors]

    def _serve_state(self):
        return self.get_current_state()

    def publish_state_sharing(self, step: int):
        if self.state_server is None:
            return
        self.local_step_for_state = step
        self.dht.store(f"{self.prefix}_state_sharing", {"endpoint": self.state_server.endpoint, "step": int(step)},
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
            donors.append((v.value.get("step", 0), v.value["endpoint"]))
        for step, ep in sorted(donors, reverse=True):
            try:
                meta, tensors = download_state(ep, timeout=timeout)
                logger.info(f"downloaded state (step {meta.get('step')}) from {ep}")
                return meta, tensors
            except Exception as e:  # noqa: BLE001
                logger.warning(f"failed to download state from {ep}: {e}")
        return None

    def shutdown(self):
        if self.state_server is not None:
            self.state_server.shutdown()
        if self.comms is not None:
            self.comms.close()
