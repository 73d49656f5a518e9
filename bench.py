#!/usr/bin/env python
"""Headline benchmark: whole-node samples/sec of collaborative ALBERT-large MLM+SOP pre-training.

Metric/config from BASELINE.json: "samples/sec (whole node) ALBERT-large MLM pretrain at 1/2/4/8
peers".  One process per GPU = one collaboration peer (run_trainer semantics): bf16 compute,
synthetic WikiText-103-shaped SOP instances (seq 512, 15 % MLM), random-init albert-large-v2
weights, LAMB + linear-warmup schedule, target_batch_size 4096 samples per collaborative step,
FLOAT16 butterfly averaging of parameters + gradients over RCCL between all peers, exactly as the
reference's CollaborativeOptimizer does it (nothing is skipped inside the timed region).

A bench "step" = ONE collaborative (global) optimizer step = 4096 samples summed over all peers.
The total work per step is fixed as N grows, so scaling is "strong".

    python bench.py                         # 1 GPU
    python bench.py --gpus 8                # 8 peers, one per GPU: this script starts them itself
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8   # same, launched by torchrun
    python bench.py --model swav            # BASELINE config 3 (collaborative SwAV ResNet-50), same contract

The default single-GPU run also measures BASELINE config 3 in a child process (after the timed ALBERT
region) and reports it under the ``swav`` key of the same JSON line (``--swav 0`` turns that off).

Peers are independent processes, one per GPU, as in the reference's fleet (each AWS worker runs its
own run_trainer, albert/AWS_runner.ipynb:293-297).  Without a launcher (no WORLD_SIZE in the
environment) ``--gpus N`` makes this script start the N peer processes itself, before it touches
the GPU, each with RANK / LOCAL_RANK / WORLD_SIZE set the way torchrun sets them (peer i on GPU i).
Two peers on one device are refused unless ``--allow_shared_device`` is given; the JSON line then
reports ``physical_gpus`` (distinct devices actually used) next to ``n_gpus`` (peers).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "samples/sec (whole node) ALBERT-large MLM pretrain at 1/2/4/8 peers"
# Measured PyTorch-eager reference on MI355X: the reference's compute stack (HF AlbertForPreTraining,
# bf16 autocast, SDPA attention, per-tensor torch LAMB, clip_grad_norm_) driven by this repo's
# collaborative engine — `python bench.py --impl eager` (training/eager_baseline.py), samples/s per
# GPU at N=1 in its best micro-batch: 64 -> 263.48, 128 -> 272.02, 256 runs out of the 288 GB (HF
# materialises the full [B*S, 30000] MLM logits; BASELINE.md "Measured MI355X results",
# profiles/bench_eager_mb128.log).  vs_baseline = value / (this x N).
EAGER_BASELINE_SPS_PER_GPU = 272.02
# The SwAV counterpart (--model swav --impl eager: training/swav_eager.py, stock nn modules with one
# trunk pass per crop, vissl-formula loss, apex-LARC SGD in torch ops, same collaborative engine and
# GPU multi-crop data), samples/s per GPU at N=1, b=64, measured on MI355X
# (profiles/r4_bench_swav_eager_n1.log).
EAGER_SWAV_SPS_PER_GPU = 619.19


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="albert", choices=["albert", "swav"],
                    help="albert = the headline (BASELINE.json metric); swav = BASELINE config 3, collaborative "
                         "SwAV ResNet-50 (b=64 per peer, 2x224+6x96 crops, LARC-SGD, target 32768, groups of 4)")
    ap.add_argument("--steps", type=int, default=3, help="timed collaborative steps")
    ap.add_argument("--warmup", type=int, default=1, help="untimed collaborative steps")
    ap.add_argument("--micro_batch", type=int, default=None,
                    help="per-peer micro-batch (default: min(512, target / peers), at least 64 — measured on "
                         "MI355X 64: 905, 128: 935, 256: 940 samples/s per micro-step, 512 +0.8%% over 256 on one "
                         "box (about 170 GB of activations, fits the 288 GB HBM); with the ETA slack the 8-peer "
                         "protocol efficiency does not drop with fewer micro-steps per global step (1 micro-step: "
                         "89.5%% vs 2: 87.8%% in the CPU emulation, profiles/README.md), so the largest "
                         "micro-batch wins)")
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--seq_len", type=int, default=512)
    ap.add_argument("--target_batch_size", type=int, default=None,
                    help="samples per collaborative step (default: 4096 ALBERT, 32768 SwAV — the reference values)")
    ap.add_argument("--compression", default="FLOAT16")
    ap.add_argument("--impl", default="dedloc", choices=["dedloc", "eager"],
                    help="eager = the reference's compute on stock PyTorch (ALBERT: HF AlbertForPreTraining + "
                         "per-tensor torch LAMB; SwAV: training/swav_eager.py) — the measured baselines")
    ap.add_argument("--cpu_test", default=None, metavar="CONFIG_DIR",
                    help="plumbing test only: run on CPU/gloo with the tiny ALBERT config in CONFIG_DIR (with "
                         "--model swav the value is ignored: full ResNet-50, use a tiny --micro_batch) — exercises "
                         "the multi-rank orchestration of this script; not a measurement")
    ap.add_argument("--throttle", type=float, default=0.0,
                    help="emulation only: idle seconds added after every micro-step (with --cpu_test, stands in "
                         "for GPU compute time when studying the collaboration protocol's overheads)")
    ap.add_argument("--allow_shared_device", action="store_true",
                    help="let several peers share one GPU (protocol emulation on a small box); the JSON line "
                         "reports physical_gpus < n_gpus.  Without it, more peers than visible GPUs is an error")
    ap.add_argument("--swav", type=int, default=1,
                    help="with the default single-GPU ALBERT run: also measure BASELINE config 3 (--model swav) in a "
                         "fresh child process after the timed region (this process frees its memory first), and report it under the "
                         "'swav' key (the headline keys are unchanged; a child failure only sets swav.error).  0: off")
    ap.add_argument("--swav_steps", type=int, default=3, help="timed collaborative steps of the SwAV child run")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(args) -> int:
    """Start ``args.gpus`` peer processes (this script again, with torchrun's environment: RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT) and wait for them; rank 0 prints the JSON line.
    Called before anything initialises the GPU (``device_count`` does not), and the children are
    started as subprocesses, never by exec."""
    n = args.gpus
    if not args.cpu_test:
        visible = torch.cuda.device_count()
        if n > visible and not args.allow_shared_device:
            print(f"bench.py: --gpus {n} needs {n} GPUs but {visible} are visible; one peer per GPU is the "
                  f"measured configuration (pass --allow_shared_device to emulate {n} peers on "
                  f"{max(visible, 1)} device(s))", file=sys.stderr)
            return 2
    env = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), start_new_session=True))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"bench.py: peer process {p.pid} exited with {code}; stopping the others", file=sys.stderr)
                    for q in pending:
                        os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    return rc if rc >= 0 else 128 - rc


_BACKEND_CODE = {"rccl": 0, "gloo": 1, "rccl+gloo": 2}
_BACKEND_NAME = {v: k for k, v in _BACKEND_CODE.items()}


def rccl_fallback(dev_type: str, world: int, physical: int, rccl_rounds, other_rounds) -> bool:
    """N > 1 peers on N distinct GPUs must average over RCCL: a silent fallback to host-staged gloo
    (a broken RCCL on the box) must not become the scaling number — such a run exits non-zero.  The
    check is over every successful round of the timed region, per peer: any round over gloo or a
    mixed group, or a peer with no RCCL round at all, fails the run (a single failed round — e.g. a
    straggler at the very end — does not).  Peers sharing a device (``--allow_shared_device``) and
    CPU plumbing runs are exempt."""
    if not (dev_type == "cuda" and world > 1 and physical == world):
        return False
    return any(o > 0 for o in other_rounds) or any(r == 0 for r in rccl_rounds)


def _swav_child(args) -> dict:
    """BASELINE config 3 in a child process (``bench.py --model swav``): its own CUDA context, run
    after the parent's timed region and once the parent has freed its memory (the parent only
    waits), started as a subprocess — never by exec from a process that initialised the GPU."""
    cmd = [sys.executable, os.path.abspath(__file__), "--model", "swav", "--gpus", "1", "--steps", str(args.swav_steps),
           "--warmup", "1", "--swav", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return {"error": "timeout after 900 s", "cmd": " ".join(cmd[1:])}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}: {r.stderr.strip()[-400:]}", "cmd": " ".join(cmd[1:])}
    out = json.loads(lines[-1])
    keep = ("metric", "value", "unit", "vs_baseline", "ms_per_step", "steps", "warmup", "config", "data_plane",
            "ema_samples_per_s_sum", "first_microstep_s")
    return dict({k: out.get(k) for k in keep}, wall_s=round(time.perf_counter() - t0, 1), cmd=" ".join(cmd[1:]))


def _protocol_breakdown(gathered, keys):
    out = {}
    for i, k in enumerate(keys[:-1]):
        vals = [float(g[3 + i]) / max(1.0, float(g[3 + len(keys) - 1])) for g in gathered]
        out[k.replace("_s", "_ms") if k.endswith("_s") else k] = round(
            sum(vals) / len(vals) * (1e3 if k.endswith("_s") else 1.0), 3)
    return out


def _albert_peer(args, rank, world, dev, root_ep):
    """The headline: one ALBERT-large run_trainer peer (AlbertPeer) per GPU."""
    if args.target_batch_size is None:
        args.target_batch_size = 4096
    if args.micro_batch is None:
        args.micro_batch = 2 if args.cpu_test else min(512, max(64, args.target_batch_size // world))
    from dedloc_amd.cli.arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments
    from dedloc_amd.training.albert_peer import AlbertPeer

    targs = AlbertTrainingArguments(per_device_train_batch_size=args.micro_batch,
                                    gradient_accumulation_steps=args.grad_accum, seq_length=args.seq_len,
                                    save_steps=0, output_dir=f"/tmp/dedloc_bench_{os.getpid()}", seed=1234,
                                    throttle=args.throttle)
    dargs = DatasetArguments(config_path=args.cpu_test or "albert-large-v2")
    cargs = CollaborationArguments(experiment_prefix="bench", initial_peers=[root_ep], dht_listen_on="127.0.0.1:*",
                                   target_batch_size=args.target_batch_size, compression=args.compression,
                                   listen_on="127.0.0.1:*", averaging_expiration=5.0, averaging_timeout=60.0,
                                   min_refresh_period=0.2, default_refresh_period=0.5)
    if args.impl == "eager":
        dargs.mask_mode = "hf"
    peer = AlbertPeer(targs, dargs, cargs, dev, rank=rank, dht=None, impl=args.impl)

    def describe(value, world):
        return {"metric": METRIC, "value": round(value, 2), "unit": "samples/s", "higher_is_better": True,
                "scaling": "strong",
                "vs_baseline": (round(value / (EAGER_BASELINE_SPS_PER_GPU * world), 3)
                                if EAGER_BASELINE_SPS_PER_GPU else None),
                "dtype": "bf16", "data": "synthetic (WikiText-103 SOP shapes, seq 512, 15% MLM; random-init weights)",
                "config": {"model": "albert-large-v2", "global_batch": args.target_batch_size,
                           "seq_len": args.seq_len, "parallelism": f"collaborative-dp{world}",
                           "micro_batch": args.micro_batch, "grad_accum": args.grad_accum,
                           "compression": args.compression, "optimizer": "LAMB", "impl": args.impl}}
    return peer, args.micro_batch * args.grad_accum, describe


def _swav_peer(args, rank, dev, root_ep):
    """BASELINE config 3: one collaborative SwAV ResNet-50 peer (SwavPeer, the reference's
    sgd_collaborative + vissl train step) per GPU, with the reference's recipe values (local batch 64,
    target 32768 samples per collaborative step, LARC-SGD, FLOAT16 wire, matchmaking groups of 4)."""
    if args.target_batch_size is None:
        args.target_batch_size = 32768
    b = args.micro_batch or 64
    from dedloc_amd.training.swav_peer import SwavPeer
    from dedloc_amd.utils.config import load_config

    ov = [f"config.DATA.TRAIN.BATCHSIZE_PER_REPLICA={b}", f"config.OPTIMIZER.batch_size_for_tracking={b}",
          f"config.OPTIMIZER.target_batch_size={args.target_batch_size}",
          f"config.OPTIMIZER.compression={args.compression}",
          f'config.OPTIMIZER.dht_initial_peers=["{root_ep}"]', f"config.CHECKPOINT.DIR=/tmp/dedloc_swav_bench_{os.getpid()}",
          "config.CHECKPOINT.AUTO_RESUME=false", "config.CHECKPOINT.CHECKPOINT_ITER_FREQUENCY=0"]
    if args.cpu_test:
        # plumbing runs: eight full ResNet-50 peers share the host's CPUs, so one global step can take
        # longer than the GPU recipe's 30 s metadata expiration — peers would count each other dead —
        # and a peer's last micro-step can end well past the 5 s matchmaking window of its partition's
        # first member, which then closes a group without it (a group of another composition: a new
        # communicator, and a failed round for the late peer)
        ov += ["config.OPTIMIZER.metadata_expiration=300", "config.OPTIMIZER.averaging_timeout=120",
               "config.OPTIMIZER.averaging_expiration=30"]
    cfg = load_config("swav_1node_resnet_submit", ov)
    peer = SwavPeer(cfg, dev, rank=rank, impl=args.impl)

    def describe(value, world):
        base = EAGER_SWAV_SPS_PER_GPU
        return {"metric": "samples/sec (whole node) SwAV ResNet-50 at 1/2/4/8 peers", "value": round(value, 2),
                "unit": "samples/s", "higher_is_better": True, "scaling": "strong",
                "vs_baseline": round(value / (base * world), 3) if base else None,
                "dtype": "bf16", "data": "synthetic (ImageNet-224-sized image pool, 2x224 + 6x96 multi-crop on the "
                                         "GPU; random-init weights)",
                "config": {"model": "swav-resnet50", "global_batch": args.target_batch_size, "batch_per_peer": b,
                           "crops": "2x224+6x96", "parallelism": f"collaborative-dp{world}",
                           "compression": args.compression, "optimizer": "LARC-SGD", "impl": args.impl,
                           "target_group_size": int(cfg.OPTIMIZER.target_group_size)}}
    return peer, b, describe


def _harness_world(cpu: bool):
    """The BENCH HARNESS's own process group (gloo, host-side): barriers around the timed region,
    the DHT root's address, and the max-over-ranks reduction.  The collaboration itself never sees
    it — peers find each other through the DHT and build their RCCL communicators there
    (dedloc_amd/parallel/comm.py)."""
    from dedloc_amd.parallel import local_device

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = local_device(torch.device("cpu") if cpu else None)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import datetime

        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=1800))
    return rank, world, dev


def _device_id(dev: torch.device) -> str:
    if dev.type != "cuda":
        return "cpu"
    props = torch.cuda.get_device_properties(dev)
    uuid = getattr(props, "uuid", None)
    return str(uuid) if uuid is not None else f"{props.name}:{dev.index}"


def _physical_devices(dev, world: int):
    """Distinct devices used by the peers (gathered over the harness group)."""
    ids = [None] * world
    if world > 1:
        dist.all_gather_object(ids, _device_id(dev))
    else:
        ids = [_device_id(dev)]
    return ids


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_self_launch(args))
    # the SwAV child run (BASELINE config 3) happens AFTER the timed ALBERT region, once this process
    # has released its GPU memory, so the headline is measured on a cool, idle device
    want_swav = (args.swav and args.model == "albert" and args.impl == "dedloc" and not args.cpu_test
                 and args.gpus == 1 and "WORLD_SIZE" not in os.environ and torch.cuda.device_count() > 0)
    logging.basicConfig(level=logging.INFO if args.verbose else logging.WARNING,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    rank, world, dev = _harness_world(cpu=bool(args.cpu_test))

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev_ids = _physical_devices(dev, world)
    physical = len({d for d in dev_ids if d != "cpu"})
    if dev.type == "cuda" and physical < world and not args.allow_shared_device:
        if rank == 0:
            print(f"bench.py: {world} peers on {physical} GPU(s): two peers would share a device; pass "
                  f"--allow_shared_device to emulate that", file=sys.stderr)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(2)
    from dedloc_amd.dht import DHT

    # control plane: rank 0 hosts the DHT root, everyone else bootstraps from it
    root = DHT(listen_on="127.0.0.1:*") if rank == 0 else None
    ep = [root.endpoint if root is not None else None]
    if world > 1:
        dist.broadcast_object_list(ep, src=0)
    if args.model == "swav":
        peer, bs, describe = _swav_peer(args, rank, dev, ep[0])
    else:
        peer, bs, describe = _albert_peer(args, rank, world, dev, ep[0])
    co = peer.collab_opt

    def run_until(step):
        n = 0
        while co.local_step < step:
            peer.train_step()
            n += bs
        return n

    if world > 1:
        dist.barrier()
    co.load_state_from_peers()  # joins the collaboration like run_trainer does (on_train_begin)
    if world > 1:
        dist.barrier()
    base = co.local_step
    first_s = None
    if args.warmup > 0:  # the first micro-step alone: lazy start-up (module loads, allocations) cost
        sync()
        t_first = time.perf_counter()
        peer.train_step()
        sync()
        first_s = time.perf_counter() - t_first
    run_until(base + args.warmup)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    keys = ("wait_s", "fetch_s", "averaging_s", "matchmaking_s", "allreduce_s", "optimizer_s", "tail_s", "local_steps",
            "global_steps")
    st0 = {k: co.stats.get(k, 0.0) for k in keys}
    st0_rounds = (co.stats.get("rounds_rccl", 0), co.stats.get("rounds_gloo", 0) + co.stats.get("rounds_rccl+gloo", 0))
    t0 = time.perf_counter()
    samples = run_until(base + args.warmup + args.steps)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    if hasattr(peer, "flush_metrics"):
        peer.flush_metrics(block=True)
    if co._device_timer is not None:  # fold the timed region's last micro-steps into the EMA
        co._device_timer.poll()
    ema = co.performance_ema.samples_per_second
    comms = co.averager.comms
    rccl_rounds = co.stats.get("rounds_rccl", 0) - st0_rounds[0]
    other_rounds = co.stats.get("rounds_gloo", 0) + co.stats.get("rounds_rccl+gloo", 0) - st0_rounds[1]
    stats = torch.tensor([samples, dt, ema] + [co.stats.get(k, 0.0) - st0[k] for k in keys]
                         + [comms.created, comms.aborted, comms.quarantined, float(_BACKEND_CODE.get(
                             (co.last_group or {}).get("backend"), -1)), co.stats["averaging_failed"],
                            rccl_rounds, other_rounds],
                         dtype=torch.float64)
    if world > 1:
        gathered = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(gathered, stats)
    else:
        gathered = [stats]
    total_samples = sum(float(g[0]) for g in gathered)
    max_dt = max(float(g[1]) for g in gathered)
    ema_sum = sum(float(g[2]) for g in gathered)
    n0 = 3 + len(keys)
    per_peer = {"comms_created": [int(g[n0]) for g in gathered], "comms_aborted": [int(g[n0 + 1]) for g in gathered],
                "comms_quarantined": [int(g[n0 + 2]) for g in gathered],
                "data_plane": [_BACKEND_NAME.get(int(g[n0 + 3])) for g in gathered],
                "averaging_failed": [int(g[n0 + 4]) for g in gathered],
                # successful timed-region rounds per peer: over RCCL / over gloo or mixed groups
                "rounds_rccl": [int(g[n0 + 5]) for g in gathered], "rounds_other": [int(g[n0 + 6]) for g in gathered]}
    fallback = rccl_fallback(dev.type, world, physical, per_peer["rounds_rccl"], per_peer["rounds_other"])
    if rank == 0:
        value = total_samples / max_dt
        out = dict(describe(value, world), n_gpus=world, steps=args.steps, warmup=args.warmup,
                   ms_per_step=round(max_dt / args.steps * 1e3, 2))
        out.update({
               "physical_gpus": physical, "peers": world,
               "data_plane": (co.last_group or {}).get("backend"),
               "first_microstep_s": None if first_s is None else round(first_s, 3),
               "ema_samples_per_s_sum": round(ema_sum, 2), "averaging_rounds": co.stats["averaging_rounds"],
               "averaging_failed": co.stats["averaging_failed"],
               # timed-region breakdown, mean over peers: host ms per global step waiting for the
               # batch's last micro-step, in the state fetch, matchmaking + all-reduce (and each),
               # the optimizer launch and the bookkeeping after it; local micro-steps per global step
               "protocol": _protocol_breakdown(gathered, keys),
               "last_group": {k: v for k, v in (co.last_group or {}).items() if k != "gathered"},
               "per_peer": per_peer})
        if fallback:
            out["error"] = (f"data plane is not RCCL on every peer: rounds over RCCL {per_peer['rounds_rccl']}, "
                            f"over gloo / mixed groups {per_peer['rounds_other']}")
        if want_swav:
            import gc

            peer.shutdown()
            peer = co = None
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()  # the child gets the device's memory back
            out["swav"] = _swav_child(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    if peer is not None:
        peer.shutdown()
    if root is not None:
        root.shutdown()
    if world > 1:
        dist.destroy_process_group()
    if fallback:
        if rank == 0:
            print(f"bench.py: {world} peers on {physical} GPUs did not all average over RCCL (rounds over RCCL "
                  f"{per_peer['rounds_rccl']}, over gloo / mixed {per_peer['rounds_other']}); failing the run",
                  file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
