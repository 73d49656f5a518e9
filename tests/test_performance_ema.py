"""PerformanceEMA fed from device completion events (optim/performance_ema.py).

The reference's throughput metric is Σ PerformanceEMA.samples_per_second over peers
(albert/run_trainer.py:145, albert/run_first_peer.py:197,208), with averaging time excluded.  A GPU
peer's host runs ahead of the device, so the EMA is fed from micro-step completion events
(``DeviceStepTimer``).  These tests drive it with a fake device clock: every micro-step takes a
known device time, every global step (averaging + optimizer) another, and the host polls at
arbitrary moments — the EMA must equal samples / (device time minus global steps)."""
import pytest

from dedloc_amd.optim.performance_ema import DeviceStepTimer, PerformanceEMA


class FakeDevice:
    """An in-order device queue with a clock: work is enqueued with a duration, an event completes
    when the device clock passes the end of everything enqueued before it."""

    def __init__(self):
        self.queued_until = 0.0  # device time at which everything enqueued so far is done
        self.now = 0.0           # what the host has observed of the device clock

    def enqueue(self, seconds):
        self.queued_until += seconds

    def event(self):
        dev = self

        class Ev:
            t = None

            def record(self):
                self.t = dev.queued_until

            def query(self):
                return dev.now >= self.t

            def elapsed_time(self, other):
                return (other.t - self.t) * 1e3

        return Ev()


@pytest.mark.parametrize("micro_steps", [1, 8])
def test_device_timer_counts_every_micro_step_and_excludes_global_steps(micro_steps):
    dev = FakeDevice()
    ema = PerformanceEMA(alpha=0.1)
    timer = DeviceStepTimer(ema, event_factory=dev.event)
    bs, step_s, global_s = 512, 0.54, 0.12
    counted = 0
    timer.resume()  # start of training (the first micro-step then has a reference point)
    for g in range(12):
        for i in range(micro_steps):
            dev.enqueue(step_s)
            timer.step_done(bs)
            counted += 1
            # the host is one micro-step ahead: it observes the device up to the previous step
            dev.now = dev.queued_until - step_s
            timer.poll()
        dev.enqueue(global_s)  # averaging + optimizer
        timer.resume()
    dev.now = dev.queued_until
    timer.poll()
    assert timer.updates == counted
    expected = bs / step_s
    assert ema.samples_per_second == pytest.approx(expected, rel=0.02)


def test_device_timer_never_blocks_and_keeps_order():
    dev = FakeDevice()
    ema = PerformanceEMA(alpha=0.5)
    timer = DeviceStepTimer(ema, event_factory=dev.event)
    timer.resume()
    for s in (1.0, 2.0, 4.0):
        dev.enqueue(s)
        timer.step_done(100)
    assert timer.poll() == 0.0 and timer.updates == 0  # nothing has completed yet
    dev.now = 3.0  # the first two micro-steps are done, the third is not
    timer.poll()
    assert timer.updates == 2
    dev.now = 7.0
    timer.poll()
    assert timer.updates == 3
    # 3 updates of seconds-per-sample .01, .02, .04 with alpha .5 and bias correction
    e = 0.0
    for n, x in enumerate((0.01, 0.02, 0.04), 1):
        e = 0.5 * x + 0.5 * e
    assert ema.samples_per_second == pytest.approx((1 - 0.5 ** 3) / e, rel=1e-6)


def test_host_clock_path_with_pause_excludes_global_step():
    """The CPU path (host clock, pause() around the global step) on a fake clock: 8 micro-steps of
    1 s and a 0.5 s global step give exactly 1 sample/s per sample of batch."""
    t = [0.0]
    ema = PerformanceEMA(alpha=0.1, clock=lambda: t[0])
    for g in range(5):
        for i in range(8):
            t[0] += 1.0
            ema.update(4)
        with ema.pause():
            t[0] += 0.5
    assert ema.samples_per_second == pytest.approx(4.0, rel=1e-9)
