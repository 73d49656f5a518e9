#!/usr/bin/env python
"""Collaborative SwAV trainer peer (replaces ``swav/vissl/tools/run_distributed_engines.py:21-58`` +
the vissl launcher/engine/trainer).

Accepts the reference's override spelling (swav/README.md:17-31)::

    python -m dedloc_amd.cli.run_swav config=pretrain/swav/swav_1node_resnet_submit \\
        config.DATA.TRAIN.BATCHSIZE_PER_REPLICA=64 +config.OPTIMIZER.lr=2.4 \\
        +config.OPTIMIZER.dht_initial_peers='["127.0.0.1:1337"]' --max_iterations 1000

One process per GPU (torchrun-style env for several peers on one node); each process is one
collaborative peer, exactly like the reference's world_size=1 vissl jobs.
"""
from __future__ import annotations

import argparse
import logging
import sys

from ..utils.config import load_config, parse_cli

logger = logging.getLogger(__name__)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    name, overrides, rest = parse_cli(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--max_iterations", type=int, default=None)
    ap.add_argument("--stop_after_global_steps", type=int, default=None)
    ap.add_argument("--max_seconds", type=float, default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--print_config", action="store_true")
    args = ap.parse_args(rest)
    cfg = load_config(name, overrides)
    if args.print_config:
        import json

        print(json.dumps(cfg.to_dict(), indent=2))
        return
    import torch

    import os

    from ..parallel import local_device

    rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = local_device(None if args.device is None else torch.device(args.device))
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(name)s -   %(message)s",
                        level=logging.INFO if rank == 0 else logging.WARNING)
    from ..training.swav_peer import SwavPeer

    peer = SwavPeer(cfg, device, rank=rank)
    try:
        peer.maybe_resume()
        peer.train(max_iterations=args.max_iterations, stop_after_global_steps=args.stop_after_global_steps,
                   max_seconds=args.max_seconds)
    finally:
        peer.shutdown()


if __name__ == "__main__":
    main()
