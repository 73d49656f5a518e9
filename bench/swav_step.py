"""SwAV ResNet-50 local-iteration throughput of one GPU peer (the SwAV experiment's unit of work).

One iteration = synthetic multi-crop generation (2x224 + 6x96, on the GPU) + forward over the 8 crops
+ Sinkhorn/SwAV loss + backward + gradient accumulation into the collaborative accumulator +
prototype normalisation; the LARC-SGD update runs once per collaborative step (target 32768 samples),
so it is timed separately and amortised.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dedloc_amd.dht import DHT  # noqa: E402
from dedloc_amd.training.swav_peer import SwavPeer  # noqa: E402
from dedloc_amd.utils.config import load_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4, help="untimed iterations (first-call allocations, graph capture)")
    ap.add_argument("--grouped", action="store_true", help="one trunk pass per crop resolution")
    ap.add_argument("--queue", action="store_true", help="queue active (3840 rows in Sinkhorn)")
    ap.add_argument("--graph", action="store_true", help="capture trunk+head fwd/bwd as HIP graphs")
    ap.add_argument("--sequential", action="store_true", help="the two resolution passes on one stream")
    ap.add_argument("--splits", default=None, help="concurrent passes per resolution, e.g. 2,1 (whole crops each)")
    ap.add_argument("--cfg", action="append", default=[], help="extra config override, e.g. config.HOOKS.PERF_STATS=false")
    ap.add_argument("--model_attr", action="append", default=[],
                    help="NAME=INT: set a SwAVModel class attribute for an A/B (e.g. dgrad_weights_stream=0)")
    ap.add_argument("--no_prefetch", action="store_true", help="generate each batch in line (no side-stream prefetch)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ov = [f"config.DATA.TRAIN.BATCHSIZE_PER_REPLICA={args.batch}", f"config.OPTIMIZER.batch_size_for_tracking={args.batch}",
          "config.OPTIMIZER.target_batch_size=100000000", f"config.MODEL.SINGLE_PASS_EVERY_CROP={not args.grouped}",
          f"config.LOSS.swav_loss.queue.start_iter={0 if args.queue else 10**9}", "config.CHECKPOINT.DIR=/tmp/swav_bench", f"config.MODEL.CUDA_GRAPH={args.graph}",
          f"config.MODEL.CONCURRENT_PASSES={not args.sequential}", f"config.DATA.TRAIN.PREFETCH={not args.no_prefetch}"]
    ov += args.cfg
    if args.splits:
        ov.append(f"config.MODEL.CONCURRENT_SPLITS=[{args.splits}]")
    cfg = load_config("swav_1node_resnet_submit", ov)
    from dedloc_amd.models.resnet_swav import SwAVModel

    for kv in args.model_attr:
        k, v = kv.split("=")
        assert hasattr(SwAVModel, k), k
        setattr(SwAVModel, k, type(getattr(SwAVModel, k))(int(v)))
    dht = DHT(start=True)
    peer = SwavPeer(cfg, dev, dht=dht)
    try:
        for i in range(args.warmup):
            t0 = time.perf_counter()
            peer.train_step()
            torch.cuda.synchronize()
            print(f"warmup {i}: {time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)
        t = time.perf_counter()
        for _ in range(args.iters):
            peer.train_step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.iters
        t = time.perf_counter()
        for _ in range(5):
            peer.data.next_batch()
        torch.cuda.synchronize()
        data_ms = (time.perf_counter() - t) / 5 * 1e3
        t = time.perf_counter()
        for _ in range(5):
            peer.opt.step()
        torch.cuda.synchronize()
        opt_ms = (time.perf_counter() - t) / 5 * 1e3
        print(json.dumps({"metric": "swav_rn50_local_samples_per_sec_per_gpu", "value": args.batch / dt,
                          "ms_per_iter": dt * 1e3, "data_ms": data_ms, "larc_sgd_step_ms": opt_ms,
                          "batch": args.batch, "crops": "2x224+6x96", "grouped": args.grouped, "queue": args.queue, "hip_graph": args.graph,
                          "concurrent_passes": not args.sequential, "splits": args.splits, "prefetch": not args.no_prefetch,
                          "peak_mem_gb": torch.cuda.max_memory_allocated() / 2**30}))
    finally:
        peer.shutdown()
        dht.shutdown()


if __name__ == "__main__":
    main()
