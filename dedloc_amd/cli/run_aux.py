#!/usr/bin/env python
"""Auxiliary peer (albert/run_aux.py:206-262): contributes no gradients, only helps averaging as a
reducer (``auxiliary=True``, ``allow_state_sharing=False``), calling ``step_aux()`` every 0.5 s.
Unlike the reference it carries no dead trainer callback code."""
from __future__ import annotations

import logging
import sys
import time

from transformers import HfArgumentParser

from .arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments
from .run_trainer import setup_logging

logger = logging.getLogger(__name__)


def main(argv=None):
    parser = HfArgumentParser((AlbertTrainingArguments, DatasetArguments, CollaborationArguments))
    training_args, dataset_args, collaboration_args = parser.parse_args_into_dataclasses(
        list(sys.argv[1:] if argv is None else argv))
    if len(collaboration_args.initial_peers) == 0:
        raise ValueError("Please specify at least one network endpoint in initial peers.")
    import torch

    import os

    from ..parallel import local_device
    from ..training.albert_peer import AlbertPeer

    rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = local_device(None if training_args.device is None else torch.device(training_args.device))
    setup_logging(rank)
    peer = AlbertPeer(training_args, dataset_args, collaboration_args, device, rank=rank, auxiliary=True)
    try:
        start = peer.collab_opt.local_step
        while True:
            time.sleep(0.5)
            peer.collab_opt.step_aux()
            if (training_args.stop_after_global_steps is not None
                    and peer.collab_opt.local_step - start >= training_args.stop_after_global_steps):
                break
    finally:
        peer.shutdown()


if __name__ == "__main__":
    main()
