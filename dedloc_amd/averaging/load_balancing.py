"""Load balancing of butterfly all-reduce parts (hivemind.averaging.load_balancing).

Each member i of a group with throughput b_i (the reference's ``--bandwidth``; 0 for client-mode
peers that cannot aggregate) receives a fraction w_i of the averaged vector to reduce.  Member i
moves (1 - w_i) V as a sender plus (N - 1) w_i V as an aggregator per direction, so the round time
is max_i (1 + (N - 2) w_i) / b_i.  We solve  min xi  s.t.  xi >= (1 + (N-2) w_i) / b_i,
sum w = 1, w >= 0, w_i = 0 where b_i = 0  (a <=9-variable LP; scipy HiGHS), drop shares below
``min_size`` elements and round to integers with Hagenbach-Bischoff (largest remainder) so the
parts sum exactly to the vector size.
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
    if np.allclose(b[active], b[active][0]) and active.all():
        w = np.full(n, 1.0 / n)
    else:
        from scipy.optimize import linprog

        # variables: w_0..w_{n-1}, xi ; minimise xi
        c = np.zeros(n + 1)
        c[-1] = 1.0
        A_ub, b_ub = [], []
        for i in range(n):
            if not active[i]:
                continue
            row = np.zeros(n + 1)
            row[i] = (n - 2) / b[i]
            row[-1] = -1.0
            A_ub.append(row)
            b_ub.append(-1.0 / b[i])
        A_eq = np.zeros((1, n + 1))
        A_eq[0, :n] = 1.0
        bounds = [(0.0, None) if active[i] else (0.0, 0.0) for i in range(n)] + [(0.0, None)]
        res = linprog(c, A_ub=np.asarray(A_ub), b_ub=np.asarray(b_ub), A_eq=A_eq, b_eq=[1.0], bounds=bounds,
                      method="highs")
        w = res.x[:n] if res.success else active / active.sum()
    w = np.clip(w, 0.0, None)
    if min_size > 0:
        small = w * vector_size < min_size
        if (~small).any():
            w[small] = 0.0
    return hagenbach_bischoff(vector_size, w / w.sum())


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
