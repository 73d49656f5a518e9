"""PerformanceEMA — the reference's throughput meter (hivemind).

EMA of *seconds per sample* with bias correction; ``pause()`` excludes averaging time.  Each peer
publishes ``samples_per_second`` (albert/run_trainer.py:145-152) and the coordinator sums them into
the whole-collaboration "performance" (albert/run_first_peer.py:197,208) — the BASELINE metric.
"""
from __future__ import annotations

import time
from contextlib import contextmanager
from threading import Lock


class PerformanceEMA:
    def __init__(self, alpha: float = 0.1, eps: float = 1e-20, clock=time.perf_counter):
        self.alpha, self.eps, self.clock = alpha, eps, clock
        self.ema_seconds_per_sample = 0.0
        self.num_updates = 0
        self.samples_per_second = 0.0
        self.timestamp = clock()
        self.paused = False
        self.lock = Lock()

    def update(self, num_processed: int) -> float:
        """Account ``num_processed`` samples finished since the previous update (or reset)."""
        assert not self.paused, "PerformanceEMA is paused"
        with self.lock:
            now = self.clock()
            dt = max(0.0, now - self.timestamp)
            self.timestamp = now
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
