"""Volunteer entry point: the sahajBERT contributor notebook as one command (SURVEY.md D15;
reference ``sahajbert/contributor_notebook.ipynb`` cell 2).

The notebook installs hivemind, signs the volunteer in with Hugging Face, sizes the micro-batch from
the GPU model (4 on T4/P100-class cards, else 1) and launches ``run_trainer.py --client_mode`` with
its fixed collaboration flags (averaging_expiration 10, statistics_expiration 120, batch_size_lead
400, gradient_accumulation_steps 1, seed 42, logging every 100 steps, run name = user name).  Here
there is nothing to install and no network: the coordinator address is given directly (or printed by
``run_first_peer``), the micro-batch is sized from the MI355X's HBM instead of the card's name, and the
trainer runs in this process (no exec; one peer per GPU).

    python -m dedloc_amd.cli.contributor --initial_peers 127.0.0.1:PORT --experiment_prefix bengali_MAIN
    python -m dedloc_amd.cli.contributor ... --dry_run        # print the run_trainer arguments only
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List


def micro_batch_for_device(device: str = "cuda", seq_length: int = 512) -> int:
    """ALBERT-large micro-batch for the volunteer's accelerator: the notebook keys it on the card name;
    here on free memory (~1 GiB per sequence of 512 tokens incl. activations, at most 256 — the
    measured throughput plateau on MI355X, profiles/README.md), 1 on the CPU."""
    if device == "cpu":
        return 1
    import torch

    if not torch.cuda.is_available():
        return 1
    free, _ = torch.cuda.mem_get_info()
    per_seq = (1 << 30) * seq_length / 512
    mb = int(free * 0.7 // per_seq)
    p2 = 1
    while p2 * 2 <= min(256, max(1, mb)):
        p2 *= 2
    return p2


def trainer_argv(a, micro_batch: int) -> List[str]:
    argv = ["--sahajbert", "--client_mode",
            "--averaging_expiration", "10", "--statistics_expiration", "120",
            "--batch_size_lead", "400", "--per_device_train_batch_size", str(micro_batch),
            "--gradient_accumulation_steps", "1", "--logging_steps", "100",
            "--run_name", a.username, "--output_dir", a.output_dir, "--experiment_prefix", a.experiment_prefix,
            "--seed", "42"]
    if a.initial_peers:
        argv += ["--initial_peers", *a.initial_peers]
    if a.device:
        argv += ["--device", a.device]
    return argv + list(a.extra)


def main(argv=None):
    ap = argparse.ArgumentParser(description="join a sahajBERT collaboration as a client-mode volunteer")
    ap.add_argument("--initial_peers", nargs="*", default=[], help="coordinator / DHT endpoints (host:port)")
    ap.add_argument("--experiment_prefix", default="bengali_MAIN")
    ap.add_argument("--username", default=os.environ.get("USER", "volunteer"))
    ap.add_argument("--output_dir", default="./outputs")
    ap.add_argument("--device", default=None, help="cuda (default when available) or cpu")
    ap.add_argument("--micro_batch", type=int, default=None, help="override the device-sized micro-batch")
    ap.add_argument("--dry_run", action="store_true", help="print the run_trainer arguments and exit")
    ap.add_argument("extra", nargs=argparse.REMAINDER, help="further run_trainer flags after --")
    a = ap.parse_args(argv)
    if a.extra and a.extra[0] == "--":
        a.extra = a.extra[1:]
    mb = a.micro_batch or micro_batch_for_device(a.device or "cuda")
    args = trainer_argv(a, mb)
    if a.dry_run:
        print(json.dumps({"micro_batch": mb, "run_trainer": args}))
        return 0
    from .run_trainer import main as run_trainer_main

    run_trainer_main(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
