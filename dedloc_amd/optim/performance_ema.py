"""PerformanceEMA — the reference's throughput meter (hivemind).

EMA of *seconds per sample* with bias correction; ``pause()`` excludes averaging time.  Each peer
publishes ``samples_per_second`` (albert/run_trainer.py:145-152) and the coordinator sums them into
the whole-collaboration "performance" (albert/run_first_peer.py:197,208) — the BASELINE metric.

On a GPU peer the host runs ahead of the device, so host-clock intervals between ``update`` calls
are not the time the samples took: a host that waits for the device at one point (e.g. the global
step) hands that step's device time to the wrong interval, or to none.  ``DeviceStepTimer`` feeds
the EMA from micro-step completion events instead: each micro-step's interval is the device time
between its end and the previous micro-step's end, and the only interval excluded is the global
step itself (from the last micro-step's end to the end of averaging + optimizer), which is
exactly what ``pause()`` excludes in the reference.
"""
from __future__ import annotations

import collections
import time
from contextlib import contextmanager
from threading import Lock
from typing import Callable, Optional


class PerformanceEMA:
    def __init__(self, alpha: float = 0.1, eps: float = 1e-20, clock=time.perf_counter):
        self.alpha, self.eps, self.clock = alpha, eps, clock
        self.ema_seconds_per_sample = 0.0
        self.num_updates = 0
        self.samples_per_second = 0.0
        self.timestamp = clock()
        self.paused = False
        self.lock = Lock()

    def update(self, num_processed: int, interval: Optional[float] = None) -> float:
        """Account ``num_processed`` samples finished since the previous update (or reset), or, with
        ``interval``, processed in that many seconds (measured elsewhere: ``DeviceStepTimer``)."""
        assert interval is not None or not self.paused, "PerformanceEMA is paused"
        with self.lock:
            if interval is None:
                now = self.clock()
                dt = max(0.0, now - self.timestamp)
                self.timestamp = now
            else:
                dt = max(0.0, float(interval))
            if num_processed <= 0:
                return self.samples_per_second
            sps = dt / num_processed
            self.ema_seconds_per_sample = self.alpha * sps + (1 - self.alpha) * self.ema_seconds_per_sample
            self.num_updates += 1
            adjusted = self.ema_seconds_per_sample / (1 - (1 - self.alpha) ** self.num_updates)
            self.samples_per_second = 1.0 / max(adjusted, self.eps)
            return self.samples_per_second

    def reset_timer(self):
        with self.lock:
            self.timestamp = self.clock()

    @contextmanager
    def pause(self):
        """Time spent inside is not counted (the timer restarts on exit)."""
        was = self.paused
        self.paused = True
        try:
            yield
        finally:
            self.paused = was
            self.reset_timer()

    def __repr__(self):
        return f"PerformanceEMA(alpha={self.alpha}, samples_per_second={self.samples_per_second:.2f})"


class DeviceStepTimer:
    """Feeds a ``PerformanceEMA`` from device completion events (see module docstring).

    ``step_done(n)`` records an event on the current stream after a micro-step of ``n`` samples has
    been queued; ``resume()`` records a marker after work that must not count (the global step, a
    state download); ``poll()`` folds every completed micro-step into the EMA, in order, without
    ever waiting for the device.  ``event_factory`` makes timing events (tests pass fakes)."""

    def __init__(self, ema: PerformanceEMA, event_factory: Optional[Callable[[], object]] = None):
        self.ema = ema
        if event_factory is None:
            import torch

            event_factory = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        self._make = event_factory
        self._queue: "collections.deque" = collections.deque()  # (event, samples or None = marker)
        self._prev = None
        self.updates = 0
        self.last = None  # the most recently recorded event

    def _record(self, samples):
        ev = self._make()
        ev.record()
        self._queue.append((ev, samples))
        self.last = ev

    def step_done(self, samples: int):
        self._record(int(samples))

    def resume(self):
        self._record(None)

    def poll(self) -> float:
        while self._queue:
            ev, samples = self._queue[0]
            if not ev.query():
                break
            self._queue.popleft()
            if samples is not None and self._prev is not None and samples > 0:
                self.ema.update(samples, interval=self._prev.elapsed_time(ev) / 1e3)
                self.updates += 1
            self._prev = ev
        return self.ema.samples_per_second
