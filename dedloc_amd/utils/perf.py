"""Per-phase GPU timers on HIP events (vissl ``PerfTimer``/``PerfStats``, ``vissl/utils/perf_stats.py:12-250``,
SURVEY.md §2.3 V20 / §5.1).

``with stats.phase("fwd_bwd"):`` records a start/end event pair on the current stream without
synchronising; ``stats.report()`` returns the mean milliseconds per phase over the occurrences that
have completed since the previous report, without waiting for the device (host wall time is used
on CPU).  With
``sample_every`` = k only every k-th iteration (``next_iteration()``) is timed: timing events are
queue markers, and at SwAV's ~1000 kernels / 21 ms iteration eight of them per iteration cost ~0.5%.
"""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Tuple

import torch


class PerfStats:
    def __init__(self, device=None, enabled: bool = True, sample_every: int = 1):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.cuda = self.device.type == "cuda" and torch.cuda.is_available()
        self.enabled = enabled
        self.sample_every = max(1, int(sample_every))
        self._tick = 0
        self._events: Dict[str, List[Tuple]] = defaultdict(list)

    def next_iteration(self):
        self._tick += 1

    @contextmanager
    def phase(self, name: str):
        if not self.enabled or self._tick % self.sample_every:
            yield
            return
        if self.cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._events[name].append((s, e))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._events[name].append((t0, time.perf_counter()))

    def report(self, block: bool = False) -> Dict[str, float]:
        """Mean ms per phase occurrence over the occurrences that have completed since the last
        report (and their number).  Without ``block`` it never waits for the device: occurrences
        still in flight stay for the next report (a synchronising report at every global step
        drained the GPU queue there and idled it while the host refilled it)."""
        out = {}
        for name, evs in self._events.items():
            if not evs:
                continue
            if self.cuda:
                if block:
                    evs[-1][1].synchronize()
                done = 0
                while done < len(evs) and evs[done][1].query():
                    done += 1
                ms = [s.elapsed_time(e) for s, e in evs[:done]]
            else:
                done = len(evs)
                ms = [(e - s) * 1e3 for s, e in evs]
            del evs[:done]
            if ms:
                out[f"{name}_ms"] = sum(ms) / len(ms)
                out[f"{name}_n"] = len(ms)
        return out
