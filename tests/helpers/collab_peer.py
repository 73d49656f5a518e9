"""TEST ONLY: one ALBERT collaboration peer (a small config) driven step by step, for the
multi-process tests: the cross-process RCCL rehearsal (tests/test_xproc_rccl.py: run with
``tests/xproc`` on PYTHONPATH and ``DEDLOC_XPROC_RCCL_DIR`` set, so its data plane is the real RCCL
code path over the mailbox stand-in) and the delayed-parameter-averaging GPU test
(tests/test_delayed_averaging_gpu.py: peers sharing one GPU, gloo data plane).

After every global step it appends one JSON record to ``<out>/peer-<name>.jsonl`` and saves the
averaged tensors of every successful gradient round (taken right after the all-reduce, before the
optimizer step) to ``<out>/<name>-s<step>.pt``, so the test can check that the members of a round
ended with the same average."""
from __future__ import annotations

import argparse
import json
import os
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", required=True)
    ap.add_argument("--cfg", required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--target", type=int, default=16)
    ap.add_argument("--averaging_timeout", type=float, default=8.0)
    ap.add_argument("--averaging_expiration", type=float, default=2.0)
    ap.add_argument("--metadata_expiration", type=float, default=6.0)
    ap.add_argument("--join", action="store_true", help="a late joiner: load the state from a peer first")
    ap.add_argument("--barrier", action="store_true",
                    help="write <out>/ready-<name> once built, then wait for <out>/go (all peers start together)")
    ap.add_argument("--gate", default="go", help="the file name --barrier waits for")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--micro_batch", type=int, default=2)
    ap.add_argument("--seq_len", type=int, default=64)
    ap.add_argument("--compression", default="NONE")
    ap.add_argument("--delay_param_averaging", action="store_true")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--aux", action="store_true",
                    help="an auxiliary (reducer-only) peer: step_aux() every 0.1 s until <out>/stop exists")
    ap.add_argument("--final", action="store_true",
                    help="at the end: finish (and apply) a pending delayed parameter round, save the final "
                         "parameters and the counters to <out>/<name>-final.pt")
    args = ap.parse_args()

    from dedloc_amd.cli.arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments
    from dedloc_amd.training.albert_peer import AlbertPeer

    targs = AlbertTrainingArguments(per_device_train_batch_size=args.micro_batch, gradient_accumulation_steps=1,
                                    seq_length=args.seq_len, save_steps=0, seed=7,
                                    output_dir=os.path.join(args.out, f"hf-{args.name}"),
                                    metrics_file=os.path.join(args.out, f"metrics-{args.name}.jsonl"))
    if args.lr is not None:
        targs.learning_rate, targs.warmup_steps = args.lr, 1
    dargs = DatasetArguments(config_path=args.cfg)
    cargs = CollaborationArguments(experiment_prefix="xproc", initial_peers=[args.root], dht_listen_on="127.0.0.1:*",
                                   target_batch_size=args.target, compression=args.compression,
                                   listen_on="127.0.0.1:*", delay_param_averaging=args.delay_param_averaging,
                                   averaging_expiration=args.averaging_expiration,
                                   averaging_timeout=args.averaging_timeout,
                                   metadata_expiration=args.metadata_expiration, min_refresh_period=0.2,
                                   default_refresh_period=0.5)
    peer = AlbertPeer(targs, dargs, cargs, torch.device(args.device), rank=0, auxiliary=args.aux)
    co = peer.collab_opt
    log = open(os.path.join(args.out, f"peer-{args.name}.jsonl"), "a")
    inner = co.averager.step

    def step(*a, **kw):
        res = inner(*a, **kw)
        if res is not None:
            torch.save({"params": co.flat.fp32.clone(), "grads": co.flat.grad.clone(), "group_id": res["group_id"],
                        "size": res["size"]}, os.path.join(args.out, f"{args.name}-s{co.local_step}.pt"))
        return res

    co.averager.step = step
    if args.barrier:
        open(os.path.join(args.out, f"ready-{args.name}"), "w").close()
        while not os.path.exists(os.path.join(args.out, args.gate)):
            time.sleep(0.05)
    if args.join:
        ok = co.load_state_from_peers()
        log.write(json.dumps({"event": "join", "ok": bool(ok), "step": co.local_step,
                              "download": co.averager.last_download, "t": time.time()}) + "\n")
        log.flush()
    if args.aux:
        while not os.path.exists(os.path.join(args.out, "stop")):
            g = co.step_aux()
            if g is not None:
                log.write(json.dumps({"event": "aux_round", "step": co.local_step, "size": g.get("size"),
                                      "group_id": g.get("group_id"), "backend": g.get("backend"),
                                      "t": time.time()}) + "\n")
                log.flush()
            time.sleep(0.1)
        peer.shutdown()
        return
    last = co.local_step
    while co.local_step < args.steps:
        peer.train_step()
        if co.local_step != last:
            last = co.local_step
            g = co.last_group or {}
            comms = co.averager.comms
            log.write(json.dumps({"event": "step", "step": co.local_step, "size": g.get("size"),
                                  "group_id": g.get("group_id"), "backend": g.get("backend"),
                                  "failed": co.stats["averaging_failed"], "rounds": co.stats["averaging_rounds"],
                                  "created": comms.created, "aborted": comms.aborted,
                                  "quarantined": comms.quarantined, "t": time.time()}) + "\n")
            log.flush()
    if args.final:
        co._finish_param_round()
        if co.flat.fp32.is_cuda:
            torch.cuda.synchronize()
        torch.save({"params": co.flat.fp32.cpu(), "stats": {k: float(v) for k, v in co.stats.items()},
                    "side_stream": co.delay_param_averaging and co._side_stream is not None},
                   os.path.join(args.out, f"{args.name}-final.pt"))
    log.write(json.dumps({"event": "done", "step": co.local_step, "t": time.time()}) + "\n")
    log.flush()
    peer.shutdown()


if __name__ == "__main__":
    main()
