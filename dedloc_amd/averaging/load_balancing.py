"""Load balancing of butterfly all-reduce parts (hivemind.averaging.load_balancing).

Each member i of a group with throughput b_i (the reference's ``--bandwidth``; 0 for client-mode
peers that cannot aggregate) receives a fraction w_i of the averaged vector to reduce.  Member i
moves (1 - w_i) V as a sender plus (N - 1) w_i V as an aggregator per direction, so the round time
is max_i (1 + (N - 2) w_i) / b_i.  hivemind minimises that max with an LP.  The LP is degenerate
whenever one member is slow enough to be the bottleneck at w = 0 (a CPU peer next to xGMI peers:
every split among the others is optimal, and a solver returns a vertex — one member takes the
whole vector).  So the min-max is solved by water-filling instead, which picks the balanced
optimum: a level T with w_i = max(0, (T b_i - 1) / (N - 2)) and sum w = 1 (bisection on T).
Members whose link is too slow to finish a share within T get none, every other member finishes
exactly at T, and the round's max time equals the LP optimum.  With N <= 2 the time does not depend
on w; parts are then proportional to b.  Shares below ``min_size`` elements are dropped and the
rest rounded to integers with Hagenbach-Bischoff (largest remainder) so the parts sum exactly to
the vector size.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def optimize_parts_lp(vector_size: int, throughputs: Sequence[Optional[float]], min_size: int = 0) -> np.ndarray:
    b = np.asarray([np.nan if t is None else float(t) for t in throughputs], dtype=np.float64)
    n = len(b)
    if n == 0:
        return np.zeros(0, dtype=np.int64)
    if np.isnan(b).any():  # unknown throughput -> mean of the known ones (or 1)
        known = b[~np.isnan(b)]
        b[np.isnan(b)] = known[known > 0].mean() if (known > 0).any() else 1.0
    if n == 1 or (b > 0).sum() <= 1:
        w = (b > 0).astype(np.float64) if (b > 0).any() else np.full(n, 1.0 / n)
        return hagenbach_bischoff(vector_size, w / w.sum())
    active = b > 0
    if n <= 2:
        w = np.where(active, b, 0.0)
    else:
        w = _water_fill(np.where(active, b, 0.0), n - 2)
    w = np.clip(w, 0.0, None)
    if min_size > 0:
        small = w * vector_size < min_size
        if (~small).any():
            w[small] = 0.0
    return hagenbach_bischoff(vector_size, w / w.sum())


def _water_fill(b: np.ndarray, k: int) -> np.ndarray:
    """w_i = max(0, (T b_i - 1) / k) with sum w = 1 (b_i = 0: w_i = 0)."""
    def total(t):
        return np.clip((t * b - 1.0) / k, 0.0, None).sum()

    lo, hi = 0.0, (1.0 + k) / b[b > 0].min()  # at hi every active member holds >= 1 share
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if total(mid) < 1.0:
            lo = mid
        else:
            hi = mid
    w = np.clip((hi * b - 1.0) / k, 0.0, None)
    return w / w.sum()


def hagenbach_bischoff(total: int, fractions: np.ndarray) -> np.ndarray:
    """Largest-remainder apportionment: integer parts summing exactly to ``total``."""
    fractions = np.asarray(fractions, dtype=np.float64)
    raw = fractions * total
    parts = np.floor(raw).astype(np.int64)
    remainder = int(total - parts.sum())
    if remainder > 0:
        order = np.argsort(-(raw - parts), kind="stable")
        parts[order[:remainder]] += 1
    return parts


def load_balance_peers(vector_size: int, throughputs: Sequence[Optional[float]], min_size: int = 0):
    return tuple(int(x) for x in optimize_parts_lp(vector_size, throughputs, min_size))
