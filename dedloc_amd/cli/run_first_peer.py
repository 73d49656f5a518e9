#!/usr/bin/env python
"""Coordinator / first peer (albert/run_first_peer.py:149-218).

* hosts the DHT root and prints ``Running DHT root at {address}:{port}``;
* every ``refresh_period`` seconds reads ``{prefix}_metrics`` and, when the collaboration's step
  advances, aggregates loss (sum loss / sum mini_steps), alive peers, samples and
  **performance = sum of the peers' samples_per_second** (the reference's whole-collaboration
  throughput, BASELINE metric) — logged to stdout / a JSONL file (wandb is optional: no network).
  A record is also written when the number of alive peers changes within a step (a peer joining
  or leaving; the reference logs on step changes only, so a peer whose first report lands after
  the collaboration's last step change never appeared in its log);
* every ``save_checkpoint_step_interval`` steps pulls the latest state from the peers and, when
  ``repo_path`` is set and ``upload_interval`` has elapsed, writes the HF checkpoint
  (config.json + pytorch_model.bin) + ``optimizer_state.pt`` there and commits it if the directory
  is a git repository (push only if a remote exists).
"""
from __future__ import annotations

import json
import logging
import os
import subprocess
import sys
import time
from dataclasses import asdict

import torch
from transformers import HfArgumentParser

from ..dht import DHT
from ..metrics import LocalMetrics, make_validators
from ..models.albert import AlbertConfig, AlbertForPreTraining
from ..optim.collaborative import CollaborativeOptimizer
from ..optim.lamb import FusedLamb
from .arguments import AveragerArguments, CollaborativeOptimizerArguments, CoordinatorArguments

logger = logging.getLogger(__name__)


class CheckpointHandler:
    def __init__(self, coordinator_args: CoordinatorArguments, collab_optimizer_args, averager_args, dht: DHT,
                 local_public_key: bytes):
        self.save_checkpoint_step_interval = coordinator_args.save_checkpoint_step_interval
        self.repo_path = coordinator_args.repo_path
        self.upload_interval = coordinator_args.upload_interval
        self.previous_step = -1
        config = AlbertConfig.from_pretrained(coordinator_args.model_config_path)
        if coordinator_args.vocab_size:
            config.vocab_size = coordinator_args.vocab_size
        self.model = AlbertForPreTraining(config)
        self.model.materialize(torch.device(coordinator_args.device or "cpu"))
        opt = FusedLamb(self.model.flat, lr=0.00176, weight_decay=0.01, clamp_value=10000.0, debias=True,
                        no_decay=self.model.no_decay_names())
        ca = collab_optimizer_args
        av = asdict(averager_args)
        self.collaborative_optimizer = CollaborativeOptimizer(
            opt=opt, dht=dht, prefix=coordinator_args.experiment_prefix, compression_type=ca.compression,
            throughput=ca.bandwidth, target_batch_size=ca.target_batch_size - ca.batch_size_lead,
            client_mode=ca.client_mode, verbose=True, start=False, allow_state_sharing=False,
            peer_id=local_public_key + b"#coordinator", **av)
        self.previous_timestamp = time.time()

    def is_time_to_save_state(self, cur_step):
        if self.save_checkpoint_step_interval is None:
            return False
        return cur_step - self.previous_step >= self.save_checkpoint_step_interval

    def save_state(self, cur_step):
        try:
            self.collaborative_optimizer.load_state_from_peers()
        except ValueError as e:  # a replica that does not match the peers' model: keep hosting the DHT
            logger.error(f"cannot take the peers' state into the coordinator's replica: {e}")
        self.previous_step = cur_step

    def is_time_to_upload(self):
        if self.repo_path is None:
            return False
        return self.upload_interval is None or time.time() - self.previous_timestamp >= self.upload_interval

    def upload_checkpoint(self, current_loss):
        self.model.save_pretrained(self.repo_path)
        torch.save(self.collaborative_optimizer.opt.state_dict(), f"{self.repo_path}/optimizer_state.pt")
        self.previous_timestamp = time.time()
        if not os.path.isdir(os.path.join(self.repo_path, ".git")):
            return
        try:
            subprocess.run("git add --all", shell=True, check=True, cwd=self.repo_path)
            step = self.collaborative_optimizer.local_step
            subprocess.run(f"git commit -m 'Step {step}, loss {current_loss:.3f}'", shell=True, check=True,
                           cwd=self.repo_path)
            remotes = subprocess.run("git remote", shell=True, capture_output=True, text=True, cwd=self.repo_path)
            if remotes.stdout.strip():
                subprocess.run("git push", shell=True, check=True, cwd=self.repo_path)
        except subprocess.CalledProcessError as e:
            logger.warning(f"Error while uploading model: {e}")


def aggregate(metrics_dict) -> dict:
    metrics = [LocalMetrics.model_validate(v.value) for v in metrics_dict.values()]
    latest_step = max(m.step for m in metrics)
    sum_loss = sum(m.loss for m in metrics)
    sum_mini = sum(m.mini_steps for m in metrics)
    return {"step": latest_step, "loss": sum_loss / max(sum_mini, 1), "alive peers": len(metrics),
            "samples": sum(m.samples_accumulated for m in metrics),
            "performance": sum(m.samples_per_second for m in metrics)}


def main(argv=None):
    parser = HfArgumentParser((CoordinatorArguments, CollaborativeOptimizerArguments, AveragerArguments))
    coordinator_args, collab_optimizer_args, averager_args = parser.parse_args_into_dataclasses(
        list(sys.argv[1:] if argv is None else argv))
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(name)s -   %(message)s", level=logging.INFO)
    if coordinator_args.address is None:
        coordinator_args.address = "127.0.0.1"  # single-node collaboration: no public-IP lookup
    experiment_prefix = coordinator_args.experiment_prefix
    validators, local_public_key = make_validators(experiment_prefix)
    dht = DHT(start=True, listen_on=coordinator_args.dht_listen_on, endpoint=f"{coordinator_args.address}:*",
              initial_peers=coordinator_args.initial_peers, record_validators=validators)
    logger.info(f"Running DHT root at {coordinator_args.address}:{dht.port}")
    print(f"Running DHT root at {coordinator_args.address}:{dht.port}", flush=True)
    if coordinator_args.wandb_project is not None:
        logger.warning("wandb logging requested but there is no network; metrics go to stdout/metrics_file")
    current_step, alive = 0, 0
    checkpoint_handler = CheckpointHandler(coordinator_args, collab_optimizer_args, averager_args, dht,
                                           local_public_key)
    t0 = time.time()
    try:
        while coordinator_args.max_runtime is None or time.time() - t0 < coordinator_args.max_runtime:
            metrics_dict = dht.get(experiment_prefix + "_metrics", latest=True)
            if metrics_dict is not None and isinstance(metrics_dict.value, dict) and metrics_dict.value:
                agg = aggregate(metrics_dict.value)
                step_changed = agg["step"] != current_step
                if step_changed or agg["alive peers"] != alive:
                    logger.info(f"Got metrics from {agg['alive peers']} peers")
                    current_step, alive = agg["step"], agg["alive peers"]
                    rec = dict(agg, time=time.time())
                    if coordinator_args.metrics_file:
                        with open(coordinator_args.metrics_file, "a") as f:
                            f.write(json.dumps(rec) + "\n")
                    if step_changed and checkpoint_handler.is_time_to_save_state(current_step):
                        checkpoint_handler.save_state(current_step)
                        if checkpoint_handler.is_time_to_upload():
                            checkpoint_handler.upload_checkpoint(agg["loss"])
                    logger.info(f"Step #{current_step}\tloss = {agg['loss']:.5f}\tperformance = "
                                f"{agg['performance']:.1f} samples/s\talive peers = {agg['alive peers']}")
            logger.debug("Peer is still alive...")
            time.sleep(coordinator_args.refresh_period)
    finally:
        checkpoint_handler.collaborative_optimizer.shutdown()
        dht.shutdown()


if __name__ == "__main__":
    main()
