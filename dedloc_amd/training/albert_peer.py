"""ALBERT collaborative trainer peer — the engine behind ``run_trainer`` (albert/run_trainer.py:210-293,
sahajbert/run_trainer.py:215-300).

Replaces the reference's HF ``Trainer`` + ``CollaborativeCallback`` + ``NoOpScheduler`` stack with
an explicit loop over device-resident batches:

  HF step = gradient_accumulation_steps micro-batches (fwd + bwd into the flat fp32 grad buffer)
          -> clip_grad_norm(max_grad_norm) + finite flag (one fused kernel pair, no host sync)
          -> CollaborativeOptimizer.step(batch_size)  (accumulate; global step when ready)
          -> zero_grad
          -> callback: publish LocalMetrics to {prefix}_metrics when the collaborative step changes

Deliberate differences from the reference: non-finite gradients are dropped on
the device (the reference's state_dict-alias rollback is a no-op, C.1); the loss is accumulated
on the device and read once per collaborative step instead of once per step.
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import time
from pathlib import Path
from typing import Dict, Optional

import torch

from ..data.sop_dataset import DiskSOPStream, StreamingSOPStream, is_sop_dataset, parse_sources
from ..data.synthetic_mlm import SyntheticSOPStream, peer_seed
from ..dht import DHT, get_dht_time
from ..emulation import ChurnController, StepThrottle, parse_churn_schedule, profile_for_rank
from ..metrics import LocalMetrics, make_validators
from ..models.albert import AlbertConfig, AlbertForPreTraining
from ..optim.collaborative import CollaborativeOptimizer
from ..optim.lamb import FusedLamb, get_linear_schedule_with_warmup
from ..utils.perf import PerfStats

logger = logging.getLogger(__name__)


def latest_checkpoint(output_dir: str) -> Optional[Path]:
    return max(Path(output_dir).glob("checkpoint*"), default=None, key=os.path.getctime)


def get_model(training_args, config: AlbertConfig) -> AlbertForPreTraining:
    """Resume from the newest output_dir/checkpoint* (by ctime) else random init (run_trainer.py:56-70)."""
    ckpt = latest_checkpoint(training_args.output_dir)
    if ckpt is not None and (ckpt / "config.json").exists():
        logger.info(f"Loading model from {ckpt}")
        return AlbertForPreTraining.from_pretrained(str(ckpt))
    logger.info("Training from scratch")
    return AlbertForPreTraining(config)


def build_optimizer(model: AlbertForPreTraining, training_args):
    opt = FusedLamb(model.flat, lr=training_args.learning_rate,
                    betas=(training_args.adam_beta1, training_args.adam_beta2), eps=training_args.adam_epsilon,
                    weight_decay=training_args.weight_decay, clamp_value=training_args.clamp_value, debias=True,
                    no_decay=model.no_decay_names())
    sched = get_linear_schedule_with_warmup(opt, training_args.warmup_steps, training_args.max_steps)
    return opt, sched


class AlbertPeer:
    """Everything one GPU peer owns: model, optimizer, DHT node, collaborative optimizer, data."""

    def __init__(self, training_args, dataset_args, collab_args, device, rank: int = 0,
                 dht: Optional[DHT] = None, auxiliary: bool = False, publish_only_synchronized: bool = False,
                 impl: str = "dedloc"):
        self.args, self.dargs, self.cargs = training_args, dataset_args, collab_args
        self.device = torch.device(device)
        # per-rank heterogeneity (emulation/heterogeneity.py): micro-batch, speed, bandwidth, client mode
        prof = profile_for_rank(rank, getattr(training_args, "peer_batch_sizes", None),
                                getattr(training_args, "peer_slowdowns", None),
                                getattr(collab_args, "peer_bandwidths", None),
                                getattr(collab_args, "peer_client_mode", None),
                                getattr(training_args, "peer_churn", None))
        if prof.micro_batch:
            training_args.per_device_train_batch_size = prof.micro_batch
        if prof.bandwidth is not None:
            collab_args.bandwidth = prof.bandwidth
        if prof.client_mode:
            collab_args.client_mode = True
        self.throttle = StepThrottle(slowdown=prof.slowdown * getattr(training_args, "slowdown", 1.0),
                                     throttle=training_args.throttle,
                                     sync=torch.cuda.synchronize if self.device.type == "cuda" else None)
        self.churn = ChurnController(parse_churn_schedule(prof.churn or training_args.churn_schedule), time.time())
        self.auxiliary = auxiliary
        self.publish_only_synchronized = publish_only_synchronized
        torch.manual_seed(training_args.seed)
        config = AlbertConfig.from_pretrained(dataset_args.config_path)
        if getattr(dataset_args, "vocab_size", None):
            config.vocab_size = dataset_args.vocab_size
        self.impl = impl
        if impl == "eager":  # PyTorch-eager reference stack (training/eager_baseline.py)
            from .eager_baseline import EagerAlbertModel, EagerLamb

            self.model = EagerAlbertModel(config, self.device)
            a = training_args
            self.opt = EagerLamb(self.model.flat, lr=a.learning_rate, betas=(a.adam_beta1, a.adam_beta2),
                                 eps=a.adam_epsilon, weight_decay=a.weight_decay, clamp_value=a.clamp_value,
                                 debias=True, no_decay=self.model.no_decay_names())
            self.scheduler = get_linear_schedule_with_warmup(self.opt, a.warmup_steps, a.max_steps)
        else:
            self.model = get_model(training_args, config)
            disk = getattr(dataset_args, "dataset_path", None)
            self._stream_tokenizer = None
            if getattr(dataset_args, "stream_sources", None):
                from transformers import AutoTokenizer

                self._stream_tokenizer = AutoTokenizer.from_pretrained(dataset_args.tokenizer_path)
                self.model.resize_token_embeddings(len(self._stream_tokenizer))
            elif is_sop_dataset(disk):  # run_trainer.py: model.resize_token_embeddings(len(tokenizer))
                with open(os.path.join(disk, "sop_meta.json")) as f:
                    self.model.resize_token_embeddings(int(json.load(f)["vocab_size"]))
            self.model.materialize(self.device)
            self.model.train()
            self.opt, self.scheduler = build_optimizer(self.model, training_args)
        ca = collab_args
        validators, self.local_public_key = make_validators(ca.experiment_prefix)
        self.dht = dht or DHT(initial_peers=ca.initial_peers, listen=not ca.client_mode, listen_on=ca.dht_listen_on,
                              endpoint=ca.endpoint, start=True, record_validators=validators)
        self.batch_size_per_step = training_args.per_device_train_batch_size * training_args.gradient_accumulation_steps
        self.collab_opt = CollaborativeOptimizer(
            self.opt, dht=self.dht, scheduler=self.scheduler, prefix=ca.experiment_prefix,
            compression_type=ca.compression, batch_size_per_step=self.batch_size_per_step,
            throughput=ca.bandwidth, target_batch_size=ca.target_batch_size - ca.batch_size_lead,
            client_mode=ca.client_mode, verbose=True, start=True, auxiliary=auxiliary,
            allow_state_sharing=not auxiliary, peer_id=self.local_public_key,
            averaging_expiration=ca.averaging_expiration, averaging_timeout=ca.averaging_timeout,
            listen_on=ca.listen_on, min_refresh_period=ca.min_refresh_period, max_refresh_period=ca.max_refresh_period,
            default_refresh_period=ca.default_refresh_period, expected_drift_peers=ca.expected_drift_peers,
            expected_drift_rate=ca.expected_drift_rate, performance_ema_alpha=ca.performance_ema_alpha,
            target_group_size=ca.target_group_size, metadata_expiration=ca.metadata_expiration, device=self.device,
            delay_param_averaging=getattr(ca, "delay_param_averaging", False),
            emulate_transfer_delay=getattr(ca, "emulate_transfer_delay", False), eta_slack=getattr(ca, "eta_slack", 0.0))
        self.statistics_expiration = ca.statistics_expiration
        seed = peer_seed(self.local_public_key, training_args.seed)
        if getattr(self, "_stream_tokenizer", None) is not None:
            # sahajBERT: lazily merged text sources, shuffle buffer and tokenization seeded per peer
            logger.info(f"streaming SOP instances from {dataset_args.stream_sources}")
            self.data = StreamingSOPStream(parse_sources(dataset_args.stream_sources), self._stream_tokenizer,
                                           training_args.per_device_train_batch_size, seed=seed % (2 ** 31),
                                           device=self.device, max_seq_length=training_args.seq_length)
        elif is_sop_dataset(getattr(dataset_args, "dataset_path", None)):
            # a tokenized corpus built by data/sop_dataset.py (the reference's albert_tokenized_wikitext)
            logger.info(f"training on the tokenized dataset at {dataset_args.dataset_path}")
            self.data = DiskSOPStream(dataset_args.dataset_path, training_args.per_device_train_batch_size,
                                      seed=seed, device=self.device)
        else:
            self.data = SyntheticSOPStream(training_args.per_device_train_batch_size, training_args.seq_length,
                                           self.model.config.vocab_size, seed=seed, device=self.device,
                                           mask_mode=getattr(dataset_args, "mask_mode", "fixed"),
                                           length_mode=getattr(dataset_args, "length_mode", "full"))
        flat = self.model.flat
        self._clip_part = torch.zeros(256, device=self.device)
        self._clip_out = torch.zeros(3, device=self.device)  # [norm, finite, 1 - finite]
        self._loss_sum = torch.zeros((), device=self.device)
        self.mini_steps = 0
        self.samples = 0
        self.total_samples_processed = 0
        self.last_reported_collaboration_step = -1
        self.hf_step = 0
        self.metrics_log = []
        self._pending_metrics = []  # (pinned host loss, event, record fields) awaiting the device
        self._flat = flat
        self.perf = PerfStats(self.device, enabled=bool(getattr(training_args, "perf_timers", True)))

    # ------------------------------------------------------------------ one HF step
    def train_step(self):
        a = self.args
        ga = a.gradient_accumulation_steps
        self.throttle.begin()
        for _ in range(ga):
            with self.perf.phase("data"):
                batch = self.data.next_batch()
            with self.perf.phase("fwd_bwd"):
                out = self.model(batch["input_ids"], batch["attention_mask"], batch["token_type_ids"],
                                 labels=batch.get("labels"), sentence_order_label=batch["sentence_order_label"],
                                 mlm_positions=batch.get("mlm_positions"), mlm_labels=batch.get("mlm_labels"))
                loss = out["loss"] / ga if ga > 1 else out["loss"]
                loss.backward()
            self._loss_sum += loss.detach()
        finite = None
        if self.impl == "eager":
            if a.max_grad_norm:
                torch.nn.utils.clip_grad_norm_(self.model.module.parameters(), a.max_grad_norm)
        else:
            torch.ops.dedloc.grad_norm_clip(self._flat.grad, float(a.max_grad_norm or 0.0), self._clip_part,
                                            self._clip_out)
            self._drop_if_nonfinite()
            finite = self._clip_out[1:2]
        with self.perf.phase("collab_step"):  # accumulate (+ averaging + optimizer on global steps)
            self.collab_opt.step(batch_size=self.batch_size_per_step, finite=finite)
        self.opt.zero_grad()
        self.mini_steps += 1
        self.hf_step += 1
        self._pace()
        self.throttle.end()
        self.on_step_end()
        ev = self.churn.due(self.collab_opt.local_step, time.time())
        if ev is not None:
            self.drop_out(ev.duration, restart=ev.mode == "restart")

    def _pace(self):
        """Keep the host at most one micro-step ahead of the GPU: wait for the PREVIOUS step's end
        event (the queue still holds this step, so the GPU never idles).  Progress reports and the
        PerformanceEMA then count samples the device has actually processed, which the
        collaboration's ETA (and so the moment every peer enters averaging) depends on — the
        reference gets the same effect from its per-step host syncs (params_are_finite)."""
        if self.device.type != "cuda":
            return
        ev = torch.cuda.Event()
        ev.record()
        prev, self._step_event = getattr(self, "_step_event", None), ev
        if prev is not None:
            prev.synchronize()

    # ------------------------------------------------------------------ churn (emulation/churn.py)
    def drop_out(self, duration: float, restart: bool = False):
        """Leave the collaboration for ``duration`` s (tombstone progress so the others re-plan at
        once); with ``restart`` also lose all local state like a respawned spot instance."""
        co = self.collab_opt
        logger.warning(f"churn: leaving for {duration:.1f}s (restart={restart}) at step {co.local_step}")
        co.leave()
        if restart:
            with torch.no_grad():
                self._flat.fp32.normal_(0.0, 0.02)
                self._flat.refresh_bf16()
                for t in co.opt.state_tensors():
                    t.zero_()
            co.opt.step_count = 0
            co.local_step = 0
            self.hf_step = 0
        time.sleep(duration)
        co.rejoin()
        self.stats_churn = getattr(self, "stats_churn", 0) + 1

    def _drop_if_nonfinite(self):
        # device-side: zero the whole step's gradient when the finite flag is 0 (no host sync)
        torch.ops.dedloc.axpby(self._flat.grad, self._flat.grad, 0.0, 0.0, self._clip_out[2:3])

    def on_step_end(self):
        """CollaborativeCallback.on_step_end (albert/run_trainer.py:130-170): when the collaborative
        step changes, publish LocalMetrics to ``{prefix}_metrics``.  The loss lives on the device;
        its value is copied to pinned host memory behind this step and the record is published once
        the copy has landed (at a later micro-step, never by waiting for the GPU: a read here drained
        the queue at every global step and idled the device while the host refilled it)."""
        co = self.collab_opt
        if co.local_step != self.last_reported_collaboration_step:
            self.last_reported_collaboration_step = co.local_step
            self.total_samples_processed += self.samples
            if self._loss_sum.is_cuda:
                host = torch.empty((), dtype=torch.float32, pin_memory=True)
                host.copy_(self._loss_sum, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            else:
                host, ev = self._loss_sum.clone(), None
            lg = co.last_group or {}
            self._pending_metrics.append((host, ev, dict(
                step=int(co.local_step), samples_accumulated=int(self.samples), mini_steps=int(self.mini_steps),
                hf_step=self.hf_step, lr=self.opt.param_groups[0]["lr"], group=lg.get("size"),
                matchmaking_s=lg.get("matchmaking_s"), allreduce_s=lg.get("allreduce_s"), parts=lg.get("parts"),
                synchronized=co.is_synchronized, contribution=self.total_samples_processed)))
            self._loss_sum.zero_()  # on the stream, after the copy
            self.mini_steps = 0
        self.flush_metrics()
        self.samples = co.local_samples_accumulated
        if self.args.save_steps and self.hf_step % self.args.save_steps == 0:
            self.save_checkpoint()

    def flush_metrics(self, block: bool = False):
        """Publish every pending LocalMetrics record whose loss has reached the host (in order)."""
        co = self.collab_opt
        while self._pending_metrics:
            host, ev, info = self._pending_metrics[0]
            if ev is not None:
                if block:
                    ev.synchronize()
                elif not ev.query():
                    return
            self._pending_metrics.pop(0)
            loss = float(host)
            stats = LocalMetrics(step=info["step"], samples_per_second=float(co.performance_ema.samples_per_second),
                                 samples_accumulated=info["samples_accumulated"], loss=loss,
                                 mini_steps=info["mini_steps"])
            logger.info(f"Step {info['step']}")
            logger.info(f"Your current contribution: {info['contribution']} samples")
            if info["mini_steps"]:
                logger.info(f"Local loss: {loss / info['mini_steps']:.5f}")
            if (not self.publish_only_synchronized) or info["synchronized"]:
                self.dht.store(co.prefix + "_metrics", stats.model_dump(),
                               expiration_time=get_dht_time() + self.statistics_expiration,
                               subkey=self.local_public_key, return_future=True)
            rec = dict(stats.model_dump(), time=time.time(), hf_step=info["hf_step"], lr=info["lr"],
                       group=info["group"], matchmaking_s=info["matchmaking_s"], allreduce_s=info["allreduce_s"],
                       parts=info["parts"], **self.perf.report())
            self.metrics_log.append(rec)
            if self.args.metrics_file:
                with open(self.args.metrics_file, "a") as f:
                    f.write(json.dumps(rec) + "\n")

    # ------------------------------------------------------------------ checkpoints (HF layout)
    def save_checkpoint(self):
        out = Path(self.args.output_dir) / f"checkpoint-{self.hf_step}"
        self.model.save_pretrained(str(out))
        torch.save(self.collab_opt.opt.state_dict(), out / "optimizer.pt")
        torch.save({}, out / "scheduler.pt")  # NoOpScheduler state (albert/run_trainer.py:203-204)
        with open(out / "trainer_state.json", "w") as f:
            json.dump({"global_step": self.hf_step, "collaborative_step": self.collab_opt.local_step}, f)
        ckpts = sorted(Path(self.args.output_dir).glob("checkpoint-*"), key=os.path.getctime)
        for old in ckpts[:-self.args.save_total_limit] if self.args.save_total_limit else []:
            shutil.rmtree(old, ignore_errors=True)

    def train(self, max_steps: Optional[int] = None, stop_after_global_steps: Optional[int] = None,
              max_seconds: Optional[float] = None):
        logger.warning("Loading state from peers")
        self.collab_opt.load_state_from_peers()
        t0 = time.time()
        max_steps = max_steps or self.args.max_steps
        start_global = self.collab_opt.local_step
        while self.hf_step < max_steps:
            self.train_step()
            if stop_after_global_steps is not None and self.collab_opt.local_step - start_global >= stop_after_global_steps:
                break
            if max_seconds is not None and time.time() - t0 > max_seconds:
                break
        self.flush_metrics(block=True)

    def shutdown(self):
        try:
            self.flush_metrics(block=True)
        except Exception as e:  # noqa: BLE001
            logger.debug(f"final metrics flush failed: {e}")
        self.collab_opt.shutdown()
        self.dht.shutdown()
