#!/usr/bin/env python
"""GPU trainer peer (albert/run_trainer.py + sahajbert/run_trainer.py equivalent).

    # one peer per GPU; peers of one node share an RCCL world (torchrun-style env):
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m dedloc_amd.cli.run_trainer \\
        --experiment_prefix albert --initial_peers 127.0.0.1:PORT --per_device_train_batch_size 32 ...

Same flags as the reference (HfArgumentParser over the dataclasses in cli/arguments.py).  With
``--sahajbert`` the sahajBERT variant applies: initial peers optional, vocabulary 31995, streaming
variable-length data, metrics published only while synchronized (sahajbert/run_trainer.py:164).
"""
from __future__ import annotations

import logging
import sys

from transformers import HfArgumentParser

from .arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments

logger = logging.getLogger(__name__)


def setup_logging(rank: int):
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(name)s -   %(message)s", datefmt="%m/%d/%Y %H:%M:%S",
                        level=logging.INFO if rank == 0 else logging.WARNING)


def main(argv=None, sahajbert: bool = False):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--sahajbert" in argv:
        argv.remove("--sahajbert")
        sahajbert = True
    parser = HfArgumentParser((AlbertTrainingArguments, DatasetArguments, CollaborationArguments))
    training_args, dataset_args, collaboration_args = parser.parse_args_into_dataclasses(argv)
    import os

    from ..parallel import local_device

    # the launcher's per-process GPU index doubles as this peer's slot in the heterogeneity profiles
    rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = local_device(None if training_args.device is None else __import__("torch").device(training_args.device))
    setup_logging(rank)
    logger.info(f"Found {len(collaboration_args.initial_peers)} initial peers: {collaboration_args.initial_peers}")
    if not sahajbert and len(collaboration_args.initial_peers) == 0:
        raise ValueError("Please specify at least one network endpoint in initial peers.")
    if sahajbert:
        dataset_args.vocab_size = dataset_args.vocab_size or 31995
        dataset_args.length_mode = "wikitext" if dataset_args.length_mode == "full" else dataset_args.length_mode
        dataset_args.mask_mode = "hf" if dataset_args.mask_mode == "fixed" else dataset_args.mask_mode
        assert not training_args.do_eval, "local evaluation is not supported (yet)"
    from ..training.albert_peer import AlbertPeer

    peer = AlbertPeer(training_args, dataset_args, collaboration_args, device, rank=rank,
                      publish_only_synchronized=sahajbert)
    try:
        if training_args.do_train:
            peer.train(max_steps=training_args.max_steps,
                       stop_after_global_steps=training_args.stop_after_global_steps)
    finally:
        peer.shutdown()


if __name__ == "__main__":
    main()
