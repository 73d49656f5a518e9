#!/usr/bin/env python
"""Standalone DHT root (swav/run_initial_dht_node.py:15-40): prints "Running DHT root at ip:port"
and keeps its routing view fresh with a periodic random lookup."""
from __future__ import annotations

import argparse
import time
import uuid

from ..dht import DHT


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--address", type=str, default=None,
                        help="this machine's network address (defaults to 127.0.0.1: single-node collaboration)")
    parser.add_argument("--listen_on", type=str, default="0.0.0.0:*", help="interface:port to listen on")
    parser.add_argument("--refresh_period", type=float, default=30, help="seconds between liveness lookups")
    parser.add_argument("--max_runtime", type=float, default=None, help="exit after this many seconds")
    args = parser.parse_args(argv)
    address = args.address or "127.0.0.1"
    dht = DHT(start=True, listen_on=args.listen_on, endpoint=f"{address}:*")
    print(f"Running DHT root at {address}:{dht.port}", flush=True)
    t0 = time.time()
    try:
        while args.max_runtime is None or time.time() - t0 < args.max_runtime:
            dht.get(uuid.uuid4().bytes, latest=True)
            time.sleep(min(args.refresh_period, args.max_runtime or args.refresh_period))
    finally:
        dht.shutdown()


if __name__ == "__main__":
    main()
