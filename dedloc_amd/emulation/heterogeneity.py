"""Per-peer heterogeneity profiles (variable micro-batch, compute speed, bandwidth, client mode).

``aws_fleet_profiles`` reproduces the shape of the reference's ALBERT fleet
(``albert/AWS_runner.ipynb:26-34``: 16 T4 workers on g4dn.xlarge/2xlarge with bandwidth caps
4x200, 8x100, 4x50 Mbps, ``:269``) scaled to the GPUs of one node; the sahajBERT contributor mix
(``sahajbert/contributor_notebook.ipynb:50-61``: micro-batch 4 on T4/P100 else 1, client mode) is
available through ``client_every``.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence


@dataclass
class PeerProfile:
    micro_batch: Optional[int] = None     # None -> the run's --per_device_train_batch_size
    slowdown: float = 1.0                 # >1: the peer's step takes this many times longer (duty cycle)
    throttle: float = 0.0                 # extra fixed seconds per step
    bandwidth: Optional[float] = None     # Mbps reported to the load-balancing LP
    client_mode: bool = False
    churn: Optional[str] = None           # churn schedule (see emulation/churn.py)
    extra: dict = field(default_factory=dict)


def select_for_rank(values: Optional[str], rank: int, cast=float, sep: str = ","):
    """Pick entry ``rank`` (cyclically) of a per-rank list flag like ``--peer_batch_sizes 32,16,8``."""
    if values is None or values == "":
        return None
    items = [v.strip() for v in values.split(sep)]
    v = items[rank % len(items)]
    if v in ("", "-", "none", "None"):
        return None
    return cast(v)


def profile_for_rank(rank: int, peer_batch_sizes: Optional[str] = None, peer_slowdowns: Optional[str] = None,
                     peer_bandwidths: Optional[str] = None, peer_client_mode: Optional[str] = None,
                     peer_churn: Optional[str] = None) -> PeerProfile:
    return PeerProfile(micro_batch=select_for_rank(peer_batch_sizes, rank, int),
                       slowdown=select_for_rank(peer_slowdowns, rank, float) or 1.0,
                       bandwidth=select_for_rank(peer_bandwidths, rank, float),
                       client_mode=bool(select_for_rank(peer_client_mode, rank, int) or 0),
                       churn=select_for_rank(peer_churn, rank, str, sep=";"))


def aws_fleet_profiles(n: int, client_every: int = 0) -> List[PeerProfile]:
    """n GPU peers with the AWS runner's bandwidth bands (200/100/100/50 pattern) and a 2:1 mix of
    fast/slow instances (g4dn.2xlarge vs xlarge: ~1.0 vs ~1.3 relative step time)."""
    bands = [200.0, 100.0, 100.0, 50.0]
    out = []
    for i in range(n):
        out.append(PeerProfile(bandwidth=bands[i % len(bands)], slowdown=1.0 if i % 3 else 1.3,
                               client_mode=bool(client_every) and (i % client_every == client_every - 1)))
    return out


class StepThrottle:
    """Makes a peer emulate slower hardware: after a step that took ``t`` seconds, idle for
    ``(slowdown - 1) * t + throttle`` seconds.  The GPU is synchronised first so ``t`` is real."""

    def __init__(self, slowdown: float = 1.0, throttle: float = 0.0, sync=None):
        self.slowdown, self.throttle = float(slowdown), float(throttle)
        self.sync = sync
        self._t = None

    @property
    def active(self) -> bool:
        return self.slowdown > 1.0 or self.throttle > 0.0

    def begin(self):
        if self.active:
            self._t = time.perf_counter()

    def end(self):
        if not self.active or self._t is None:
            return 0.0
        if self.sync is not None:
            self.sync()
        dt = time.perf_counter() - self._t
        idle = max(0.0, (self.slowdown - 1.0) * dt) + self.throttle
        if idle > 0:
            time.sleep(idle)
        return idle


def emulated_transfer_seconds(vector_elems: int, wire_bytes: int, group_size: int, my_fraction: float,
                              bandwidth_mbps: float) -> float:
    """Per-direction transfer time of one butterfly round for a member owning ``my_fraction`` of the
    vector under the LP cost model: (1 + (N-2) w_i) * V * bytes / bandwidth."""
    if bandwidth_mbps <= 0 or group_size <= 1:
        return 0.0
    volume = (1 + (group_size - 2) * my_fraction) * vector_elems * wire_bytes
    return volume / (bandwidth_mbps * 1e6 / 8)


def cycle(values: Sequence, n: int) -> list:
    return [values[i % len(values)] for i in range(n)]
