"""DHT: the collaboration's control plane (hivemind.DHT replacement).

API kept from the reference call sites (``albert/run_trainer.py:236-243``, ``run_first_peer.py:159-177``,
``run_aux.py:229-236``, ``swav/run_initial_dht_node.py:35-38``):

    dht = DHT(initial_peers=["host:port"], listen=True, listen_on="0.0.0.0:*", endpoint=None,
              start=True, record_validators=[...])
    dht.store(key, value, expiration_time, subkey=None, return_future=False) -> bool
    dht.get(key, latest=False) -> Optional[ValueWithExpiration]   (dict keys -> {subkey: VWE})
    dht.port, dht.endpoint, get_dht_time()

Architecture (single node, MI355X-first, not Kademlia): every listening peer runs a native server
(``csrc/runtime/dht_server.cpp`` loaded from ``_dht.so``) holding a full replica of the (small)
key space.  Writes go to every known replica, reads merge replicas by latest expiration, so the
collaboration survives the loss of any node, including the root.  Replicas discover each other
through the reserved ``_dht_nodes`` key.  Matchmaking (``join_group``) is served by the primary
replica (lowest endpoint that answers), which every peer therefore agrees on.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import os
import socket
import struct
import threading
import time
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import msgpack

from .validation import RecordValidatorBase, CompositeValidator

DHT_NODES_KEY = b"_dht_nodes"
_OP_PING, _OP_STORE, _OP_GET, _OP_JOIN, _OP_KEYS, _OP_STATS = 1, 2, 3, 4, 5, 6


def get_dht_time() -> float:
    """Shared clock of the collaboration (all peers are on one node: wall clock)."""
    return time.time()


@dataclass
class ValueWithExpiration:
    value: Any
    expiration_time: float

    def __iter__(self):  # allows `value, expiration = vwe`
        return iter((self.value, self.expiration_time))


# ----------------------------------------------------------------------------- native server
_SO = None


def _lib():
    global _SO
    if _SO is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_dht.so")
        if not os.path.exists(path):
            from .. import _build

            _build.build()
        _SO = ctypes.CDLL(path)
        _SO.dht_server_start.restype = ctypes.c_void_p
        _SO.dht_server_start.argtypes = [ctypes.c_char_p, ctypes.c_int]
        _SO.dht_server_port.argtypes = [ctypes.c_void_p]
        _SO.dht_server_stop.argtypes = [ctypes.c_void_p]
    return _SO


class NativeServer:
    """In-process handle of the C++ control-plane server (runs on its own threads)."""

    def __init__(self, host: str = "0.0.0.0", port: int = 0):
        lib = _lib()
        self._h = lib.dht_server_start(host.encode(), int(port))
        if not self._h:
            raise OSError(f"could not start DHT server on {host}:{port}")
        self.port = lib.dht_server_port(self._h)

    def shutdown(self):
        if self._h:
            _lib().dht_server_stop(self._h)
            self._h = None


def parse_endpoint(ep: str) -> Tuple[str, int]:
    ep = ep.strip()
    if ep.startswith("["):  # [::]:port
        host, _, port = ep[1:].rpartition("]:")
        host = "127.0.0.1" if host in ("::", "") else host
    else:
        host, _, port = ep.rpartition(":")
    if host in ("0.0.0.0", "", "*", "::"):
        host = "127.0.0.1"
    return host, int(port) if port not in ("*", "") else 0


# ----------------------------------------------------------------------------- wire client
class _Conn:
    def __init__(self, endpoint: str, timeout: float):
        host, port = parse_endpoint(endpoint)
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def call(self, op: int, payload: bytes, timeout: Optional[float]) -> bytes:
        self.sock.settimeout(timeout)
        msg = bytes([op]) + payload
        self.sock.sendall(struct.pack("<I", len(msg)) + msg)
        hdr = self._recv(4)
        (n,) = struct.unpack("<I", hdr)
        return self._recv(n)

    def _recv(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("DHT server closed the connection")
            buf += chunk
        return bytes(buf)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


def _b(x) -> bytes:
    if isinstance(x, bytes):
        return x
    if isinstance(x, str):
        return x.encode()
    return msgpack.packb(x, use_bin_type=True)


def _pb(x: bytes) -> bytes:
    return struct.pack("<I", len(x)) + x


class _Reader:
    def __init__(self, data: bytes):
        self.d, self.i = data, 0

    def u8(self):
        v = self.d[self.i]
        self.i += 1
        return v

    def u32(self):
        (v,) = struct.unpack_from("<I", self.d, self.i)
        self.i += 4
        return v

    def u64(self):
        (v,) = struct.unpack_from("<Q", self.d, self.i)
        self.i += 8
        return v

    def f64(self):
        (v,) = struct.unpack_from("<d", self.d, self.i)
        self.i += 8
        return v

    def bytes(self):
        n = self.u32()
        v = self.d[self.i:self.i + n]
        self.i += n
        return v


class DHTClient:
    """Thread-safe RPC client to one server endpoint (one socket per calling thread)."""

    def __init__(self, endpoint: str, timeout: float = 5.0):
        self.endpoint = endpoint
        self.timeout = timeout
        self._local = threading.local()

    def _conn(self) -> _Conn:
        c = getattr(self._local, "conn", None)
        if c is None:
            c = self._local.conn = _Conn(self.endpoint, self.timeout)
        return c

    def _call(self, op, payload, timeout=None):
        try:
            return self._conn().call(op, payload, self.timeout if timeout is None else timeout)
        except (OSError, ConnectionError):
            c = getattr(self._local, "conn", None)
            if c is not None:
                c.close()
            self._local.conn = None
            raise

    def ping(self) -> bool:
        return self._call(_OP_PING, b"")[:1] == b"\x01"

    def store_raw(self, key: bytes, subkey: Optional[bytes], value: bytes, expiration: float) -> bool:
        payload = _pb(key) + bytes([subkey is not None]) + _pb(subkey or b"") + _pb(value) + struct.pack("<d", expiration)
        return self._call(_OP_STORE, payload)[:1] == b"\x01"

    def get_raw(self, key: bytes):
        r = _Reader(self._call(_OP_GET, _pb(key)))
        kind = r.u8()
        if kind == 0:
            return None
        if kind == 1:
            return ("plain", r.bytes(), r.f64())
        n = r.u32()
        return ("dict", {r.bytes(): (r.bytes(), r.f64()) for _ in range(n)})

    def join(self, group_key: bytes, peer_id: bytes, info: bytes, target: int, min_size: int, expected: int,
             window: float, timeout: float):
        payload = (_pb(group_key) + _pb(peer_id) + _pb(info) + struct.pack("<IIId", target, min_size, expected, window))
        r = _Reader(self._call(_OP_JOIN, payload, timeout=timeout))
        failed = r.u8()
        gid = r.u64()
        n = r.u32()
        members = [(r.bytes(), r.bytes()) for _ in range(n)]
        return (not failed), gid, members

    def keys(self, prefix: bytes = b"") -> List[bytes]:
        r = _Reader(self._call(_OP_KEYS, _pb(prefix)))
        return [r.bytes() for _ in range(r.u32())]

    def stats(self) -> Dict[str, int]:
        r = _Reader(self._call(_OP_STATS, b""))
        return dict(keys=r.u64(), stores=r.u64(), gets=r.u64(), groups=r.u64())


# ----------------------------------------------------------------------------- DHT facade
class DHT:
    """Replicated control-plane DHT with hivemind-compatible ``store``/``get``."""

    def __init__(self, initial_peers: Sequence[str] = (), listen: bool = True, listen_on: str = "0.0.0.0:*",
                 endpoint: Optional[str] = None, start: bool = True,
                 record_validators: Iterable[RecordValidatorBase] = (), client_mode: Optional[bool] = None,
                 rpc_timeout: float = 5.0, replica_refresh: float = 10.0, authorizer=None, **_ignored):
        if client_mode is not None:
            listen = not client_mode
        self.initial_peers = [p for p in (initial_peers or []) if p]
        self.listen = listen
        self.listen_on = listen_on
        self.endpoint_host = None
        if endpoint:
            self.endpoint_host = parse_endpoint(endpoint.replace("*", "0"))[0]
        record_validators = list(record_validators)
        if authorizer is not None:  # token-based access control (dht/auth.py)
            from .auth import AuthorizedRecordValidator

            record_validators.append(AuthorizedRecordValidator(authorizer))
        self.validator = CompositeValidator(record_validators)
        self.rpc_timeout = rpc_timeout
        self.replica_refresh = replica_refresh
        self._server: Optional[NativeServer] = None
        self._clients: Dict[str, DHTClient] = {}
        self._lock = threading.Lock()
        self._pool = cf.ThreadPoolExecutor(max_workers=8, thread_name_prefix="dht")
        self._stop = threading.Event()
        self._refresher: Optional[threading.Thread] = None
        self.port: Optional[int] = None
        self.endpoint: Optional[str] = None
        self._started = time.time()
        self._birth: Dict[str, float] = {}
        if start:
            self.run_in_background()

    # ------------------------------------------------------------------ lifecycle
    def run_in_background(self, await_ready: bool = True):
        if self.listen:
            host, port = parse_endpoint(self.listen_on.replace("*", "0"))
            bind_host = "0.0.0.0" if self.listen_on.split(":")[0] in ("0.0.0.0", "[", "[::]", "*", "") or \
                self.listen_on.startswith("[::]") else host
            self._server = NativeServer(bind_host, port)
            self.port = self._server.port
            adv = self.endpoint_host or ("127.0.0.1" if bind_host == "0.0.0.0" else bind_host)
            self.endpoint = f"{adv}:{self.port}"
            self._birth[self.endpoint] = self._started
            self._add_replica(self.endpoint)
        for p in self.initial_peers:
            self._add_replica(p)
        if not self._clients:
            raise ValueError("DHT needs either listen=True or at least one reachable initial peer")
        if self.port is None:  # client mode: report the port of the first initial peer
            self.port = parse_endpoint(self.initial_peers[0])[1]
        self._sync_replicas()
        self._announce()
        self._refresher = threading.Thread(target=self._refresh_loop, daemon=True, name="dht-refresh")
        self._refresher.start()

    def shutdown(self):
        self._stop.set()
        if self._server is not None:
            try:
                self._raw_store_all(DHT_NODES_KEY, self.endpoint.encode(), msgpack.packb(None), get_dht_time() + 1)
            except Exception:  # noqa: BLE001
                pass
            self._server.shutdown()
            self._server = None
        self._pool.shutdown(wait=False, cancel_futures=True)

    def is_alive(self) -> bool:
        return not self._stop.is_set()

    # ------------------------------------------------------------------ replica management
    def _add_replica(self, ep: str):
        with self._lock:
            if ep not in self._clients:
                self._clients[ep] = DHTClient(ep, timeout=self.rpc_timeout)

    def replicas(self) -> List[str]:
        with self._lock:
            return sorted(self._clients)

    def _announce(self):
        if self.endpoint:
            self._raw_store_all(DHT_NODES_KEY, self.endpoint.encode(),
                                msgpack.packb([self.endpoint, self._started]),
                                get_dht_time() + 3 * self.replica_refresh)

    def _sync_replicas(self):
        r = self._merged_get(DHT_NODES_KEY)
        if r is not None and r[0] == "dict":
            for sub, (val, _exp) in r[1].items():
                rec = msgpack.unpackb(val)
                if rec:
                    ep, started = rec
                    self._birth[ep] = started
                    self._add_replica(ep)
            # gossip the membership table back to every replica, so a node that bootstraps from ANY
            # replica (not only the oldest) learns the whole replica set immediately
            for sub, (val, exp) in r[1].items():
                self._raw_store_all(DHT_NODES_KEY, sub, val, exp)

    def _refresh_loop(self):
        while not self._stop.wait(self.replica_refresh):
            try:
                self._announce()
                self._sync_replicas()
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------------ raw ops
    def _raw_store_all(self, key: bytes, subkey: Optional[bytes], value: bytes, exp: float) -> bool:
        clients = list(self._clients.values())
        futs = [self._pool.submit(c.store_raw, key, subkey, value, exp) for c in clients]
        ok = False
        for f in futs:
            try:
                ok = f.result(timeout=self.rpc_timeout + 1) or ok
            except Exception:  # noqa: BLE001
                pass
        return ok

    def _merged_get(self, key: bytes):
        clients = list(self._clients.values())
        futs = [self._pool.submit(c.get_raw, key) for c in clients]
        plain, merged = None, {}
        for f in futs:
            try:
                r = f.result(timeout=self.rpc_timeout + 1)
            except Exception:  # noqa: BLE001
                continue
            if r is None:
                continue
            if r[0] == "plain":
                if plain is None or r[2] > plain[1]:
                    plain = (r[1], r[2])
            else:
                for sub, (val, exp) in r[1].items():
                    if sub not in merged or exp > merged[sub][1]:
                        merged[sub] = (val, exp)
        if merged:
            if plain is not None and plain[1] > max(e for _, e in merged.values()):
                return ("plain",) + plain
            return ("dict", merged)
        if plain is not None:
            return ("plain",) + plain
        return None

    # ------------------------------------------------------------------ public API
    def store(self, key, value, expiration_time: float, subkey=None, return_future: bool = False, **_kw):
        """Store ``value`` (msgpack-serialisable) under key[/subkey] until ``expiration_time``.

        With ``return_future`` the record is signed (RSA, ~1.5 ms of big-integer arithmetic for an
        owned subkey), validated and stored on the node's pool: a trainer publishing its state or
        metrics at a global step does not spend that time on its own critical path."""
        kb, sb = _b(key), (None if subkey is None else _b(subkey))
        vb = msgpack.packb(value, use_bin_type=True)
        if return_future:
            return self._pool.submit(self._sign_and_store, kb, sb, vb, expiration_time)
        return self._sign_and_store(kb, sb, vb, expiration_time)

    def _sign_and_store(self, kb: bytes, sb: Optional[bytes], vb: bytes, expiration_time: float) -> bool:
        vb = self.validator.sign_value(kb, sb, vb, expiration_time)
        if not self.validator.validate(kb, sb, vb, expiration_time):
            return False
        return self._raw_store_all(kb, sb, vb, expiration_time)

    def get(self, key, latest: bool = False, return_future: bool = False, **_kw):
        """Freshest live value of ``key`` across replicas (``latest`` is always honoured)."""
        if return_future:
            return self._pool.submit(self.get, key, latest)
        kb = _b(key)
        r = self._merged_get(kb)
        if r is None:
            return None
        if r[0] == "plain":
            _, vb, exp = r
            if not self.validator.validate(kb, None, vb, exp):
                return None
            return ValueWithExpiration(msgpack.unpackb(self.validator.strip_value(kb, None, vb), raw=False), exp)
        out = {}
        for sub, (vb, exp) in r[1].items():
            if not self.validator.validate(kb, sub, vb, exp):
                continue
            val = msgpack.unpackb(self.validator.strip_value(kb, sub, vb), raw=False)
            out[sub] = ValueWithExpiration(val, exp)
        if not out:
            return None
        return ValueWithExpiration(out, max(v.expiration_time for v in out.values()))

    def primary(self) -> DHTClient:
        """Replica used for matchmaking: the OLDEST live replica.

        Every node learns all older replicas when it starts (it syncs ``_dht_nodes`` from its initial
        peers), so all peers agree on the oldest live one without waiting for replica discovery —
        a newcomer can never split matchmaking by being "lowest".
        """
        order = sorted(self.replicas(), key=lambda ep: (self._birth.get(ep, float("inf")), ep))
        for ep in order:
            c = self._clients[ep]
            try:
                if c.ping():
                    return c
            except Exception:  # noqa: BLE001
                continue
        raise ConnectionError("no DHT replica reachable")

    def join_group(self, group_key: bytes, peer_id: bytes, info: dict, target_size: int, min_size: int,
                   expected_size: int, window: float, timeout: float):
        """Matchmaking (App. A.4): returns (ok, group_id, [(peer_id, info_dict)...]) in join order."""
        cli = self.primary()
        conn = DHTClient(cli.endpoint, timeout=timeout)  # dedicated socket: the call blocks
        try:
            ok, gid, members = conn.join(_b(group_key), peer_id, msgpack.packb(info, use_bin_type=True),
                                         target_size, min_size, expected_size, window, timeout)
        finally:
            c = getattr(conn._local, "conn", None)
            if c is not None:
                c.close()
        return ok, gid, [(pid, msgpack.unpackb(inf, raw=False)) for pid, inf in members]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()
