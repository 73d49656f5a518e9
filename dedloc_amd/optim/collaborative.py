"""CollaborativeOptimizer — global-batch collaborative training (hivemind 0.9.x semantics, SURVEY.md
§2.2 H4-H6, App. A.2; reference call sites albert/run_trainer.py:251-264, run_aux.py:243-262,
run_first_peer.py:97-121, sgd_collaborative.py:145-171).

Peers of different speed accumulate gradients locally until the *collaboration* has processed
``target_batch_size`` samples (tracked through ``{prefix}_progress`` records on the DHT, with an
ETA-driven refresh period), then they average parameters and gradients (sample-weighted,
butterfly all-reduce) and apply one synchronised optimizer step; the LR schedule follows the
global step.  Out-of-sync peers download the state from a donor instead of contributing.

Flat-buffer implementation: gradients arrive in ``opt.flat.grad`` (fp32), the accumulator is one
flat fp32 buffer, and every accumulate/average/apply is a single multi-tensor HIP launch; the
fast path of ``step()`` (most calls) costs one kernel and a few Python statements.

``delay_param_averaging=True`` (BASELINE config 5; not in hivemind 0.9.x): the
global step averages only the gradients synchronously, applies the optimizer, then averages a
snapshot of the parameters on a side HIP stream in a background thread while the next
accumulation proceeds; the result is applied with the delta rule ``p += avg(snap) - snap`` (App. A.7)
at the next ``step()`` that finds the round finished (and always before the next averaging round,
so only one thread drives the communicator at a time).
"""
from __future__ import annotations

import logging
import math
import threading
import time
from dataclasses import dataclass
from typing import Any, Dict, Optional

import torch
from pydantic import BaseModel, StrictBool, StrictFloat, confloat, conint

from ..averaging.averager import DecentralizedAverager
from ..dht import DHT, get_dht_time
from .performance_ema import DeviceStepTimer, PerformanceEMA

logger = logging.getLogger(__name__)


class TrainingState(BaseModel):
    peer_id: bytes
    step: conint(ge=0, strict=True)
    samples_accumulated: conint(ge=0, strict=True)
    samples_per_second: confloat(ge=0.0, strict=True)
    time: StrictFloat
    client_mode: StrictBool
    auxiliary: bool = False


@dataclass
class CollaborationState:
    optimizer_step: int
    samples_accumulated: int
    target_batch_size: int
    num_peers: int
    num_clients: int
    eta_next_step: float
    next_fetch_time: float
    own_samples: int = 0  # this peer's samples as counted in samples_accumulated

    @property
    def ready_for_step(self) -> bool:
        return self.samples_accumulated >= self.target_batch_size or get_dht_time() >= self.eta_next_step

    def register_step(self, local_step: int):
        self.optimizer_step = max(local_step, self.optimizer_step)
        self.samples_accumulated = 0
        self.own_samples = 0
        self.eta_next_step = float("inf")


class CollaborativeOptimizer:
    def __init__(self, opt, *, dht: DHT, prefix: str, target_batch_size: int, batch_size_per_step: Optional[int] = None,
                 scheduler=None, min_refresh_period: float = 0.5, max_refresh_period: float = 30,
                 default_refresh_period: float = 3, expected_drift_peers: float = 3, expected_drift_rate: float = 0.2,
                 performance_ema_alpha: float = 0.1, metadata_expiration: float = 30.0,
                 averaging_timeout: Optional[float] = None, step_tolerance: int = 1, client_mode: bool = False,
                 auxiliary: bool = False, allow_state_sharing: bool = True, verbose: bool = False, start: bool = True,
                 compression_type: str = "FLOAT16", compression: Optional[str] = None, throughput: Optional[float] = None,
                 peer_id: Optional[bytes] = None, max_grad_norm: Optional[float] = None,
                 delay_param_averaging: bool = False, eta_slack: float = 0.0, prejoin: bool = True,
                 **averager_kwargs):
        self.opt, self.dht, self.prefix = opt, dht, prefix
        self.flat = opt.flat
        self.scheduler = scheduler
        self.target_batch_size = target_batch_size
        self.batch_size_per_step = batch_size_per_step
        self.min_refresh_period, self.max_refresh_period = min_refresh_period, max_refresh_period
        self.default_refresh_period = default_refresh_period
        self.expected_drift_peers, self.expected_drift_rate = expected_drift_peers, expected_drift_rate
        self.metadata_expiration = metadata_expiration
        self.averaging_timeout = averaging_timeout or 30.0
        self.step_tolerance = step_tolerance
        self.client_mode, self.auxiliary = client_mode, auxiliary
        self.verbose = verbose
        self.status_loglevel = logging.INFO if verbose else logging.DEBUG
        if peer_id is None:
            import os

            peer_id = f"peer-{os.getpid()}-{id(self):x}".encode()
        self.peer_id = peer_id

        self.accumulator = torch.zeros_like(self.flat.fp32) if not auxiliary else None
        self.local_samples_accumulated = 0
        self.local_steps_accumulated = 0
        self.local_step = 0
        self.performance_ema = PerformanceEMA(alpha=performance_ema_alpha)
        # GPU peers time micro-steps on the device (performance_ema.DeviceStepTimer): the host runs
        # ahead of the GPU, so its clock does not say when samples were processed
        self._device_timer = DeviceStepTimer(self.performance_ema) if self.flat.fp32.is_cuda and not auxiliary else None
        self.last_step_time = None
        self._pending_finite = []  # (host flag, event, batch size, local step) of recent micro-steps
        # [finite samples, finite micro-steps] of the current global batch, counted ON THE DEVICE: the
        # global step's averaging weight and gradient divisor come from here, so it never waits for
        # the host to learn which micro-steps were finite
        self._finite_counts = torch.zeros(2, device=self.flat.fp32.device) if not auxiliary else None
        self._count_vecs: Dict[int, torch.Tensor] = {}
        self.last_group: Optional[Dict] = None
        self.stats = {"global_steps": 0, "averaging_rounds": 0, "averaging_failed": 0, "state_loads": 0,
                      # where a global step's time goes (host clock, seconds, summed over steps): the
                      # wait for the batch's last micro-step on the device, the state fetch,
                      # matchmaking + all-reduce (and each separately), the optimizer launch, the
                      # bookkeeping after it, and the local micro-steps that went into each global batch
                      "wait_s": 0.0, "fetch_s": 0.0, "averaging_s": 0.0, "matchmaking_s": 0.0, "allreduce_s": 0.0,
                      "optimizer_s": 0.0, "tail_s": 0.0, "local_steps": 0}

        self.averager = DecentralizedAverager(
            [self.flat.fp32, self.flat.grad], dht, prefix, peer_id=peer_id,
            compression=compression or compression_type, throughput=throughput, client_mode=client_mode,
            auxiliary=auxiliary, allow_state_sharing=allow_state_sharing, metadata_expiration=metadata_expiration,
            averaging_timeout=self.averaging_timeout, **averager_kwargs)
        self.averager.get_current_state = self._get_current_state
        self._snapshot_lock = threading.Lock()
        self._snapshot_bufs = None
        self._snapshot_readers = []
        self._snapshot_ready = None
        self._snapshot_meta = None
        self._serve_stream = None

        self.eta_slack = float(eta_slack)
        self._prejoin = None  # background matchmaking for the coming global step (_maybe_prejoin)
        self._prejoin_key = None  # (local step, monotonic start) the pending prejoin was made for
        self.prejoin_enabled = prejoin
        self.delay_param_averaging = delay_param_averaging
        self._param_round: Optional[threading.Thread] = None
        self._param_round_result = None
        self._param_done_event = None
        if delay_param_averaging:
            self._param_snapshot = torch.empty_like(self.flat.fp32)
            self._param_delta = torch.empty_like(self.flat.fp32)
            self._side_stream = torch.cuda.Stream(self.flat.fp32.device) if self.flat.fp32.is_cuda else None

        self.lock_collaboration_state = threading.Lock()
        self.lock_local_progress = threading.Lock()
        self.lock_step = threading.RLock()
        self.should_report_progress = threading.Event()
        self.collaboration_state_updated = threading.Event()
        self._stop = threading.Event()
        self.collaboration_state = self.fetch_collaboration_state()
        with self.lock_step:
            self._take_snapshot()
        self._threads = []
        if start:
            for target, name in ((self._report_loop, "progress-reporter"), (self._update_loop, "collab-updater")):
                t = threading.Thread(target=target, daemon=True, name=name)
                t.start()
                self._threads.append(t)
            self.averager.publish_state_sharing(self.local_step)

    # ------------------------------------------------------------------ properties
    @property
    def is_synchronized(self) -> bool:
        return self.local_step >= self.collaboration_state.optimizer_step - self.step_tolerance

    @property
    def is_alive(self) -> bool:
        return not self._stop.is_set()

    # ------------------------------------------------------------------ state
    def _take_snapshot(self):
        """Copy the state a joiner downloads (parameters + optimizer state + step metadata) into the
        snapshot buffers.  Called with ``lock_step`` held, at the end of every global step and state
        load: one device copy on the trainer's stream (~200 MB for ALBERT-large, well under a
        millisecond).  ``_get_current_state`` serves from it without taking ``lock_step``, so a peer
        joining while this one is in the middle of an averaging round gets the last global step's
        state at once instead of waiting for the round (which holds ``lock_step``) to finish."""
        if not self.averager.allow_state_sharing:
            return
        src = [self.flat.fp32] + list(self.opt.state_tensors())
        cuda = self.flat.fp32.is_cuda
        with self._snapshot_lock:
            if self._snapshot_bufs is None:
                self._snapshot_bufs = [torch.empty_like(t) for t in src]
            if cuda:
                for ev in self._snapshot_readers:  # clones of the previous snapshot still in flight
                    torch.cuda.current_stream().wait_event(ev)
            self._snapshot_readers = []
            for d, t in zip(self._snapshot_bufs, src):
                d.copy_(t.detach(), non_blocking=True)
            self._snapshot_ready = None
            if cuda:
                self._snapshot_ready = torch.cuda.Event()
                self._snapshot_ready.record()
            self._snapshot_meta = {"step": int(self.local_step), "opt_step": int(self.opt.step_count),
                                   "lr_sched": self.scheduler.state_dict() if self.scheduler is not None else None}

    def _get_current_state(self):
        """The latest global step's state (``_take_snapshot``), cloned on the calling thread's own
        stream; never waits for ``lock_step``."""
        with self._snapshot_lock:
            if self._snapshot_bufs is None:  # no snapshot yet (state sharing off): the live state
                with self.lock_step:
                    meta = {"step": int(self.local_step), "opt_step": int(self.opt.step_count),
                            "lr_sched": self.scheduler.state_dict() if self.scheduler is not None else None}
                    return meta, [self.flat.fp32.detach().clone()] + [t.detach().clone()
                                                                      for t in self.opt.state_tensors()]
            meta = dict(self._snapshot_meta)
            if self._snapshot_ready is None:
                return meta, [t.clone() for t in self._snapshot_bufs]
            dev = self.flat.fp32.device
            if self._serve_stream is None:
                self._serve_stream = torch.cuda.Stream(dev)
            with torch.cuda.stream(self._serve_stream):
                self._serve_stream.wait_event(self._snapshot_ready)
                tensors = [t.clone() for t in self._snapshot_bufs]
                done = torch.cuda.Event()
                done.record(self._serve_stream)
            self._snapshot_readers.append(done)
            # the caller continues on its own current stream (the RCCL / TCP sender): order it after
            # the clones
            torch.cuda.current_stream(dev).wait_event(done)
        return meta, tensors

    @torch.no_grad()
    def load_state_from_peers(self, **kwargs) -> bool:
        """Download params + optimizer state from the freshest donor (App. A.7)."""
        self._finish_param_round(apply=False)
        self._drop_prejoin()  # a group matched for the step we are leaving is not ours any more
        # download WITHOUT holding lock_step: our own state server takes that lock to snapshot the
        # state it serves, so two peers loading from each other would otherwise block each other
        kwargs.setdefault("min_step", self.local_step + 1 if self.local_step > 0 or self.is_synchronized else 0)
        res = self.averager.load_state_from_peers(**kwargs)
        with self.lock_step:
            if res is None:
                # nobody shares state: keep our parameters but adopt the collaboration's step, otherwise
                # an out-of-sync peer would retry forever without contributing
                if self.local_step < self.collaboration_state.optimizer_step:
                    self.local_step = self.collaboration_state.optimizer_step
                    self.update_scheduler()
                logger.log(self.status_loglevel, "no peers to load state from; keeping local state")
                return False
            meta, tensors = res
            mine = [self.flat.fp32] + list(self.opt.state_tensors())
            if len(tensors) != len(mine) or any(t.numel() != m.numel() for t, m in zip(tensors, mine)):
                raise ValueError(f"the donor's state ({[t.numel() for t in tensors]} elements) does not match this "
                                 f"peer's model and optimizer ({[m.numel() for m in mine]}): different configs?")
            self.flat.fp32.copy_(tensors[0].to(self.flat.fp32.device))
            for dst, src in zip(self.opt.state_tensors(), tensors[1:]):
                dst.copy_(src.to(dst.device))
            self.opt.step_count = int(meta.get("opt_step", self.opt.step_count))
            self.local_step = max(self.local_step, int(meta.get("step", 0)))
            self.flat.refresh_bf16()
            self._reset_accumulators()
            self.update_scheduler()
            self.stats["state_loads"] += 1
            self._take_snapshot()
            if self._device_timer is not None:
                self._device_timer.resume()
            self.averager.publish_state_sharing(self.local_step)
        dl = self.averager.last_download or {}
        logger.warning(f"downloaded state from peers: step {self.local_step}, {dl.get('bytes', 0) / 2**20:.0f} MiB in "
                       f"{dl.get('seconds', 0.0):.2f}s over {'RCCL' if dl.get('mode') == 'R' else 'TCP'}")
        return True

    def _reset_accumulators(self):
        if self.accumulator is not None:
            self.accumulator.zero_()
        if self._finite_counts is not None:
            self._finite_counts.zero_()
        with self.lock_local_progress:
            self.local_samples_accumulated = 0
            self.local_steps_accumulated = 0

    def update_scheduler(self):
        if self.scheduler is not None:
            while self.scheduler._step_count < self.local_step:
                self.scheduler.step()

    # ------------------------------------------------------------------ training step
    def zero_grad(self, *args, **kwargs):
        self.opt.zero_grad()

    def _count_finite(self, finite: Optional[torch.Tensor], batch_size: int):
        """[samples, steps] += [batch_size, 1] x finite, on the device (one launch)."""
        vec = self._count_vecs.get(batch_size)
        if vec is None:
            vec = self._count_vecs[batch_size] = torch.tensor([float(batch_size), 1.0],
                                                              device=self._finite_counts.device)
        if finite is None:
            self._finite_counts.add_(vec)
        else:
            self._finite_counts.addcmul_(vec, finite.reshape(1).to(torch.float32))

    def _track_finite(self, finite: torch.Tensor, batch_size: int):
        """Remember a micro-step's device-side finite flag (1 = finite).  The reference's GradScaler
        skips ``step()`` for a non-finite step, so its samples never count toward the global batch;
        here the gradient is already zeroed on the device, and once the flag has reached the host the
        step's samples and its micro-step are taken back out of the local counts (``_resolve_finite``)
        — without a per-step host sync."""
        if not finite.is_cuda:
            self._pending_finite.append((finite.reshape(-1)[:1].clone(), None, batch_size, self.local_step))
            return
        host = torch.empty(1, dtype=finite.dtype, pin_memory=True)
        host.copy_(finite.reshape(-1)[:1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending_finite.append((host, ev, batch_size, self.local_step))

    def _resolve_finite(self, block: bool):
        while self._pending_finite:
            host, ev, bs, step = self._pending_finite[0]
            if ev is not None:
                if block:
                    ev.synchronize()
                elif not ev.query():
                    return
            self._pending_finite.pop(0)
            if float(host[0]) == 0.0 and step == self.local_step:
                with self.lock_local_progress:
                    self.local_samples_accumulated = max(0, self.local_samples_accumulated - bs)
                    self.local_steps_accumulated = max(0, self.local_steps_accumulated - 1)
                    self.stats["nonfinite_steps"] = self.stats.get("nonfinite_steps", 0) + 1

    def step(self, batch_size: Optional[int] = None, finite: Optional[torch.Tensor] = None, **kwargs):
        """Accumulate this step's gradients; run a global step when the collaboration is ready.

        ``finite``: the micro-step's device-side finite flag; a step whose flag reads 0 (its gradient
        was zeroed by the caller) does not count toward the global batch (``_track_finite``)."""
        if self.batch_size_per_step is None:
            if batch_size is None:
                raise ValueError("specify batch_size_per_step or pass batch_size")
            self.batch_size_per_step = batch_size
        batch_size = batch_size if batch_size is not None else self.batch_size_per_step

        if not self.is_synchronized:
            logger.log(self.status_loglevel, "peer is out of sync; loading state from peers")
            self._drop_prejoin()
            self.load_state_from_peers()
            return None
        if self.last_step_time is not None and get_dht_time() - self.last_step_time > self.metadata_expiration:
            logger.warning(f"training step took {get_dht_time() - self.last_step_time:.1f}s, longer than "
                           f"metadata_expiration; other peers may have considered this one dead")

        with self.lock_local_progress:
            torch.ops.dedloc.axpby(self.accumulator, self.flat.grad, 1.0, batch_size / self.batch_size_per_step)
            self.local_samples_accumulated += batch_size
            self.local_steps_accumulated += 1
            if self._device_timer is None:
                self.performance_ema.update(num_processed=batch_size)
            self.should_report_progress.set()
        self._count_finite(finite, batch_size)
        if finite is not None:
            self._track_finite(finite, batch_size)
        self._resolve_finite(block=False)
        if self._device_timer is not None:
            self._device_timer.step_done(batch_size)
            self._device_timer.poll()

        if self._param_round is not None and not self._param_round.is_alive():
            self._finish_param_round()
        fresh = False
        if not self._ready(batch_size) and self._imminent():
            # the matchmaking for this step is already under way (a prejoin made at this local step):
            # this micro-step is expected to complete the global batch.  The host runs a micro-step
            # ahead of the GPU, so the other peers' reports of THEIR last micro-step are typically
            # not in our view yet: wait until this micro-step has finished on the device (the global
            # step needs its gradient anyway), then look again with a fresh view — instead of
            # queueing one more micro-step per peer past the target batch.
            t_wait = time.perf_counter()
            if self._device_timer is not None and self._device_timer.last is not None:
                self._device_timer.last.synchronize()
            self.stats["wait_s"] = self.stats.get("wait_s", 0.0) + time.perf_counter() - t_wait
            self._refresh_state()
            fresh = True
        if not self._ready(batch_size):
            self._maybe_prejoin(batch_size)
            return None

        logger.log(self.status_loglevel, f"beginning global optimizer step #{self.collaboration_state.optimizer_step}")
        self._finish_param_round()
        if not fresh:
            self._refresh_state()
        if not self.is_synchronized:
            self._drop_prejoin()
            self.load_state_from_peers()
            return None

        with self.performance_ema.pause(), self.lock_collaboration_state, self.lock_step:
            cs = self.collaboration_state
            # grads = accumulator / local_steps (hivemind apply_accumulated_grads_), counting finite
            # micro-steps only — the count is a device scalar: no host sync here
            torch.ops.dedloc.axpby(self.flat.grad, self.accumulator, 0.0, 1.0, None, self._finite_counts[1:2])
            group = None
            t_avg = time.perf_counter()
            prejoined = self._take_prejoin()
            if cs.num_peers > 1 or prejoined is not None:
                mean_samples = self.target_batch_size / max(1, cs.num_peers)
                # the finite samples of this global batch / the mean per peer, as a device scalar
                # that travels with the data (allreduce.py)
                weight = self._finite_counts[0:1] * (1.0 / mean_samples)
                group = self.averager.step(weight=weight, timeout=self.averaging_timeout,
                                           expected_group_size=cs.num_peers + self._num_aux(),
                                           gather={"step": int(self.local_step)},
                                           tensors=[self.flat.grad] if self.delay_param_averaging else None,
                                           prejoined=prejoined)
                self.stats["averaging_rounds"] += 1
                if group is None:
                    self.stats["averaging_failed"] += 1
                    logger.log(self.status_loglevel, "Skipped averaging: collaboration consists of this peer only "
                                                     "or the round failed; applying local gradients")
                else:
                    self._adopt_group_step(group)
                    # successful rounds per data plane ("rccl" / "gloo" / "rccl+gloo"): bench.py checks
                    # that a multi-GPU run averaged over RCCL, not over a silent gloo fallback
                    key = f"rounds_{group.get('backend')}"
                    self.stats[key] = self.stats.get(key, 0) + 1
            else:
                logger.log(self.status_loglevel, "Skipped averaging: collaboration consists of this peer alone")
            t_opt = time.perf_counter()
            self.opt.step()
            if self.delay_param_averaging and group is not None:
                self._start_param_round(weight, cs.num_peers + self._num_aux())
            self.stats["averaging_s"] += t_opt - t_avg
            if group is not None:
                self.stats["matchmaking_s"] = self.stats.get("matchmaking_s", 0.0) + group.get("matchmaking_s", 0.0)
                self.stats["allreduce_s"] = self.stats.get("allreduce_s", 0.0) + group.get("allreduce_s", 0.0)
            t_tail = time.perf_counter()
            self.stats["optimizer_s"] += t_tail - t_opt  # launch time (kernels run async)
            self.stats["local_steps"] += self.local_steps_accumulated
            self._reset_accumulators()
            self.collaboration_state.register_step(self.local_step + 1)
            self.local_step += 1
            self.update_scheduler()
            self.last_group = group
            self.stats["global_steps"] += 1
            self.should_report_progress.set()
            self._take_snapshot()
            if self._device_timer is not None:  # the global step's device time is not counted
                self._device_timer.resume()
        self.averager.publish_state_sharing(self.local_step)
        self.last_step_time = get_dht_time()
        logger.log(self.status_loglevel, f"optimizer step #{self.local_step} done")
        self._prejoin_next(batch_size, cs.num_peers)
        # bookkeeping after the optimizer launch: counters, scheduler, snapshot copy, state-sharing
        # record, the next round's prejoin
        self.stats["tail_s"] = self.stats.get("tail_s", 0.0) + time.perf_counter() - t_tail
        return group

    def _adopt_group_step(self, group: Dict):
        """After a successful round, take the largest step any member gathered (hivemind 0.9.x:
        "update our current step if we averaged with another peer that was ahead of us").  The
        members now hold the same parameters, so they continue with the same step counter: without
        this a peer that lags one step behind (inside ``step_tolerance``, e.g. after an early global
        step some peers took alone) stays one behind for the whole run, and its prejoined groups
        never line up with the others' at the end of a run."""
        steps = [g.get("step") for g in group.get("gathered") or () if isinstance(g, dict)]
        steps = [s for s in steps if isinstance(s, int)]
        if steps and max(steps) > self.local_step:
            self.stats["steps_adopted"] = self.stats.get("steps_adopted", 0) + max(steps) - self.local_step
            self.local_step = max(steps)

    def _ready(self, batch_size: int) -> bool:
        return (self.collaboration_state.ready_for_step or self._ready_exact()
                or self._ready_within_slack(batch_size))

    def _imminent(self) -> bool:
        """A prejoin made at this local step is pending, and this step has not waited yet: the wait
        for the device happens at most once per global step (a slower collaboration would otherwise
        keep the host from running ahead of the GPU on every following micro-step)."""
        if self._prejoin is None or self._prejoin_key is None or self._prejoin_key[0] != int(self.local_step):
            return False
        if getattr(self, "_imminent_step", None) == int(self.local_step):
            return False
        self._imminent_step = int(self.local_step)
        return True

    def _refresh_state(self):
        t_fetch = time.perf_counter()
        self.collaboration_state = self.fetch_collaboration_state()
        self.stats["fetch_s"] += time.perf_counter() - t_fetch
        self.collaboration_state_updated.set()

    def _start_prejoin(self, expected_group_size: int):
        self._prejoin = self.averager.prejoin(expected_group_size=expected_group_size,
                                              gather={"step": int(self.local_step)})
        self._prejoin_key = (int(self.local_step), time.monotonic())

    def _drop_prejoin(self):
        """Forget a pending prejoin (its group, if one forms, will fail its round for the other
        members exactly as a peer leaving a hivemind group does — never later, with a stale group)."""
        if self._prejoin is not None:
            self.stats["prejoins_dropped"] = self.stats.get("prejoins_dropped", 0) + 1
        self._prejoin, self._prejoin_key = None, None

    def _take_prejoin(self):
        """The pending prejoin future if it still belongs to THIS global step: made at the current
        local step and no older than one matchmaking window plus the averaging timeout (a group
        its members have long since abandoned is never passed to the averager)."""
        fut, key = self._prejoin, self._prejoin_key
        self._prejoin, self._prejoin_key = None, None
        if fut is None:
            return None
        step, t0 = key
        max_age = self.averager.averaging_expiration + self.averaging_timeout
        if step != int(self.local_step) or time.monotonic() - t0 > max_age:
            self.stats["prejoins_dropped"] = self.stats.get("prejoins_dropped", 0) + 1
            return None
        return fut

    def _prejoin_next(self, batch_size: int, num_peers: int):
        """Right after a global step: when one micro-step of every peer completes the next global
        batch (num_peers x batch_size >= target, e.g. 8 peers x 512 samples at 4096), the next global
        step begins right after this peer's next micro-step — _maybe_prejoin, which runs only between
        micro-steps, never sees that moment — so matchmaking for it starts now and runs while the
        micro-step computes."""
        if self._prejoin is not None or not self.prejoin_enabled or self.delay_param_averaging or num_peers < 2:
            return
        if num_peers * batch_size < self.target_batch_size:
            return
        self._start_prejoin(num_peers + self._num_aux())

    def _maybe_prejoin(self, batch_size: int):
        """Begin matchmaking now when the NEXT local step will start the global step (the
        reference's ``batch_size_lead``: "begin looking for group in advance", albert/arguments.py:
        67-70).  With one micro-step per global step (8 peers x 512 samples) the group then forms
        while that micro-step computes instead of after it."""
        if self._prejoin is not None or not self.prejoin_enabled or self.delay_param_averaging:
            return
        cs = self.collaboration_state
        if cs.num_peers < 2 or cs.optimizer_step > self.local_step:
            return
        own_next = cs.samples_accumulated - cs.own_samples + self.local_samples_accumulated + batch_size
        soon = own_next >= self.target_batch_size
        sps = self.performance_ema.samples_per_second
        if not soon and sps > 0:
            soon = get_dht_time() + batch_size / sps * (1.0 + self.eta_slack) >= cs.eta_next_step
        if soon:
            self._start_prejoin(cs.num_peers + self._num_aux())

    def _ready_exact(self) -> bool:
        """The collaboration's sample count with OUR part brought up to date: the fetched state counts
        our samples as of our last progress report, but we know our current count exactly.  A single
        peer therefore steps exactly at the target (with only the stale count it ran one extra local
        step per global step, +12.5% samples at 8 local steps), and with more peers the others' stale
        counts only ever delay, never advance, the step."""
        cs = self.collaboration_state
        if cs.optimizer_step > self.local_step:
            # we are behind: our samples belong to an older step and must not count toward this
            # one (the resynchronisation rule handles a peer that is behind)
            return False
        total = cs.samples_accumulated - cs.own_samples + self.local_samples_accumulated
        return total >= self.target_batch_size

    def _ready_within_slack(self, batch_size: int) -> bool:
        """ETA slack (``eta_slack`` > 0, not in hivemind 0.9.x): start the global step now when the
        collaboration's predicted ETA lies less than ``eta_slack`` of one local step ahead.  With the
        reference rule every peer enters averaging at the first step boundary AFTER the ETA, so the
        group waits for the peer whose boundary falls last (close to a whole local step with many
        peers); entering at the boundary nearest to the ETA halves that wait, and the global batch
        stays the target on average (the weights use each peer's actual sample count)."""
        if self.eta_slack <= 0 or self.performance_ema.samples_per_second <= 0:
            return False
        cs = self.collaboration_state
        if cs.num_peers < 2 or cs.optimizer_step > self.local_step:
            return False
        step_time = batch_size / self.performance_ema.samples_per_second
        return get_dht_time() + self.eta_slack * step_time >= cs.eta_next_step

    def step_aux(self, **kwargs):
        """Auxiliary peer: join the averaging rounds as a reducer only (run_aux.py:260-262).

        Like hivemind, an auxiliary peer never publishes training progress (it must not move the
        collaboration's global step or ETA); it announces itself under ``{prefix}_aux`` so that
        trainers wait for it during matchmaking, and it adopts the step gathered from its group.
        """
        self._announce_aux()
        if not self.collaboration_state.ready_for_step:
            return None
        self.collaboration_state = self.fetch_collaboration_state()
        self.collaboration_state_updated.set()
        with self.lock_collaboration_state, self.lock_step:
            group, current = None, max(self.local_step, self.collaboration_state.optimizer_step)
            if self.collaboration_state.num_peers >= 1:
                expected = self.collaboration_state.num_peers + self._num_aux()
                group = self.averager.step(weight=0.0, timeout=self.averaging_timeout, expected_group_size=expected,
                                           tensors=[self.flat.grad] if self.delay_param_averaging else None)
                if group is not None and self.delay_param_averaging:  # help with the delayed parameter round
                    self.averager.step(weight=0.0, timeout=self.averaging_timeout, expected_group_size=expected,
                                       tensors=[self.flat.fp32], key_suffix="_params")
                if group is not None:
                    steps = [g.get("step") for g in group["gathered"] if isinstance(g.get("step"), int)]
                    current = max([current] + steps)
            self.collaboration_state.register_step(current + 1)
            self.local_step = current + 1
            self.last_group = group
        return group

    def _announce_aux(self):
        now = get_dht_time()
        if now - getattr(self, "_last_aux_announce", 0.0) > self.metadata_expiration / 3:
            self._last_aux_announce = now
            self.dht.store(f"{self.prefix}_aux", True, now + self.metadata_expiration, subkey=self.peer_id,
                           return_future=True)

    def _num_aux(self, max_age: Optional[float] = None) -> int:
        """Live auxiliary peers (``{prefix}_aux``).  Cached: the collaboration-state updater thread
        refreshes it, so a global step does not spend a synchronous DHT lookup on it."""
        max_age = max(self.min_refresh_period, 2.0) if max_age is None else max_age
        cached = getattr(self, "_aux_cache", None)
        if cached is not None and time.monotonic() - cached[1] <= max_age:
            return cached[0]
        rec = self.dht.get(f"{self.prefix}_aux", latest=True)
        n = 0
        if rec is not None and isinstance(rec.value, dict):
            n = sum(1 for k, v in rec.value.items() if v.value is True and k != self.peer_id)
        self._aux_cache = (n, time.monotonic())
        return n

    # ------------------------------------------------------------------ churn
    def leave(self):
        """Stop participating: finish any background round, drop local progress and tombstone our
        progress record so the collaboration's ETA and peer count exclude us immediately."""
        self._finish_param_round(apply=False)
        self._drop_prejoin()
        self._reset_accumulators()
        self._left = True
        try:
            self.dht.store(f"{self.prefix}_progress", None, get_dht_time() + self.metadata_expiration,
                           subkey=self.peer_id)
        except Exception:  # noqa: BLE001
            pass

    def rejoin(self):
        self._left = False
        self.collaboration_state = self.fetch_collaboration_state()
        self.load_state_from_peers()
        self.performance_ema.reset_timer()
        if self._device_timer is not None:
            self._device_timer.resume()
        self.should_report_progress.set()

    # ------------------------------------------------------------------ delayed parameter averaging
    def _start_param_round(self, weight: float, expected_group_size: int):
        self._param_snapshot.copy_(self.flat.fp32)
        self._param_delta.zero_()
        ready = None
        if self._side_stream is not None:
            ready = torch.cuda.Event()
            ready.record()
            self._param_done_event = torch.cuda.Event()

        def run():
            try:
                if self._side_stream is not None:
                    with torch.cuda.stream(self._side_stream):
                        self._side_stream.wait_event(ready)
                        res = self.averager.step(weight=weight, timeout=self.averaging_timeout,
                                                 expected_group_size=expected_group_size, tensors=[self._param_delta],
                                                 sources=[self._param_snapshot], key_suffix="_params")
                        self._param_done_event.record(self._side_stream)
                else:
                    res = self.averager.step(weight=weight, timeout=self.averaging_timeout,
                                             expected_group_size=expected_group_size, tensors=[self._param_delta],
                                             sources=[self._param_snapshot], key_suffix="_params")
            except Exception as e:  # noqa: BLE001
                logger.warning(f"delayed parameter averaging failed: {e}")
                res = None
            self._param_round_result = res

        self._param_round_result = None
        self._param_round = threading.Thread(target=run, daemon=True, name="param-averaging")
        self._param_round.start()

    def _finish_param_round(self, apply: bool = True):
        if self._param_round is None:
            return
        self._param_round.join()
        self._param_round = None
        res, self._param_round_result = self._param_round_result, None
        if self._param_done_event is not None:
            torch.cuda.current_stream().wait_event(self._param_done_event)
        if res is None or not apply:
            self.stats["param_rounds_failed"] = self.stats.get("param_rounds_failed", 0) + int(res is None)
            return
        ops = torch.ops.dedloc
        with self.lock_step:
            ops.axpby(self.flat.fp32, self._param_delta, 1.0, 1.0)  # p += avg(snapshot) - snapshot
            self.flat.refresh_bf16()
            self._take_snapshot()
        self.stats["param_rounds"] = self.stats.get("param_rounds", 0) + 1

    # ------------------------------------------------------------------ background threads
    # Progress records are signed (dht/crypto.py, big-integer RSA holding the GIL ~1.5 ms per record):
    # stored after every micro-step they would take the trainer thread's GIL ~50 times a second at
    # SwAV's 21 ms iterations.  One record per this interval at most still refreshes every peer's
    # ETA far faster than a global step (seconds), and a micro-step slower than it reports each time.
    min_report_interval = 0.1

    def _report_loop(self):
        last = 0.0
        while not self._stop.is_set():
            self.should_report_progress.wait()
            wait = last + self.min_report_interval - time.monotonic()
            if wait > 0 and self._stop.wait(wait):
                break
            self.should_report_progress.clear()
            if self._stop.is_set():
                break
            if not self.auxiliary and not getattr(self, "_left", False):
                last = time.monotonic()
                self.report_training_progress()

    def report_training_progress(self):
        with self.lock_local_progress:
            st = TrainingState(peer_id=self.peer_id, step=int(self.local_step),
                               samples_accumulated=int(self.local_samples_accumulated),
                               samples_per_second=float(self.performance_ema.samples_per_second),
                               time=float(get_dht_time()), client_mode=bool(self.client_mode),
                               auxiliary=bool(self.auxiliary))
        try:
            self.dht.store(f"{self.prefix}_progress", st.model_dump(), get_dht_time() + self.metadata_expiration,
                           subkey=self.peer_id)
        except Exception as e:  # noqa: BLE001
            logger.debug(f"progress report failed: {e}")

    def _update_loop(self):
        while not self._stop.is_set():
            delay = max(0.0, self.collaboration_state.next_fetch_time - get_dht_time())
            if self.collaboration_state_updated.wait(delay):
                self.collaboration_state_updated.clear()
                continue
            if self._stop.is_set():
                break
            try:
                with self.lock_collaboration_state:
                    self.collaboration_state = self.fetch_collaboration_state()
                self._num_aux(max_age=0.0)  # refresh the cached auxiliary count off the critical path
            except Exception as e:  # noqa: BLE001
                logger.debug(f"collaboration state update failed: {e}")

    def fetch_collaboration_state(self) -> CollaborationState:
        now = get_dht_time()
        rec = self.dht.get(f"{self.prefix}_progress", latest=True)
        peers = []
        if rec is not None and isinstance(rec.value, dict):
            for sub, v in rec.value.items():
                try:
                    peers.append(TrainingState.model_validate(v.value))
                except Exception:  # noqa: BLE001
                    continue
        if not peers:
            local_eta = max(0, self.target_batch_size - self.local_samples_accumulated) / max(
                self.performance_ema.samples_per_second, 1e-9)
            local = self.local_samples_accumulated
            return CollaborationState(self.local_step, local, self.target_batch_size,
                                      num_peers=0, num_clients=0, eta_next_step=now + local_eta,
                                      next_fetch_time=now + self.default_refresh_period, own_samples=local)
        num_peers = len(peers)
        num_clients = sum(p.client_mode for p in peers)
        global_step = max(0, self.local_step, *[p.step for p in peers if not p.client_mode] or [0])
        total_sps = sum(p.samples_per_second for p in peers)
        samples_acc, est, own = 0, 0.0, 0
        for p in peers:
            if p.step == global_step:
                samples_acc += p.samples_accumulated
                est += p.samples_accumulated + max(0.0, now - p.time) * p.samples_per_second
                if p.peer_id == self.peer_id:
                    own = p.samples_accumulated
        eta = max(0.0, self.target_batch_size - est) / max(total_sps, 1e-9)
        expected_max_peers = max(num_peers + self.expected_drift_peers, num_peers * (1 + self.expected_drift_rate))
        refresh = eta * num_peers / expected_max_peers
        next_fetch = now + min(max(refresh, self.min_refresh_period), self.max_refresh_period)
        return CollaborationState(global_step, samples_acc, self.target_batch_size, num_peers, num_clients,
                                  eta_next_step=now + eta, next_fetch_time=next_fetch, own_samples=own)

    # ------------------------------------------------------------------ misc
    def state_dict(self) -> Dict[str, Any]:
        return {"opt": self.opt.state_dict(), "local_step": self.local_step,
                "scheduler": self.scheduler.state_dict() if self.scheduler is not None else None}

    def load_state_dict(self, sd: Dict[str, Any]):
        self.opt.load_state_dict(sd["opt"])
        self.local_step = int(sd.get("local_step", self.local_step))
        if self.scheduler is not None and sd.get("scheduler"):
            self.scheduler.load_state_dict(sd["scheduler"])

    def shutdown(self):
        try:
            self._finish_param_round(apply=False)
        except Exception:  # noqa: BLE001
            pass
        self._stop.set()
        self.should_report_progress.set()
        self.collaboration_state_updated.set()
        try:  # tombstone own progress entry
            self.dht.store(f"{self.prefix}_progress", None, get_dht_time() + self.metadata_expiration,
                           subkey=self.peer_id)
        except Exception:  # noqa: BLE001
            pass
        self.averager.shutdown()

    def __del__(self):
        try:
            self._stop.set()
        except Exception:  # noqa: BLE001
            pass
