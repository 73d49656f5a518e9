#!/usr/bin/env python
"""Single-node collaboration launcher — the MI355X stand-in for ``albert/AWS_runner.ipynb`` (SURVEY.md
§2.1 D9): one coordinator (DHT root + metrics aggregation, ``run_first_peer``), N GPU trainer peers and
A auxiliary peers, all on one node, with the AWS fleet's heterogeneity injected per rank.

    python -m dedloc_amd.cli.launch_collaboration --n_trainers 8 --fleet aws --duration 600 \\
        --experiment_prefix albert -- --per_device_train_batch_size 32 --target_batch_size 4096

Everything after ``--`` is passed to every trainer (and aux peer).  Trainers and aux peers share one
torch.distributed world (the data plane: RCCL over xGMI), trainer i on GPU i, aux peer j on GPU
``n_trainers + j`` (the reference used CPU aux instances; here they are reducer-only processes on
spare GPUs: an RCCL communicator cannot hold two ranks on one device, so trainers + aux peers must
not exceed the node's GPUs).
The coordinator is not part of the world (it only reads metrics and downloads state over TCP).
This process never touches the GPU itself; children are plain subprocesses.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

from ..emulation.heterogeneity import aws_fleet_profiles


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fleet_flags(fleet: str, n: int, client_every: int = 0):
    if fleet == "uniform":
        return []
    profs = aws_fleet_profiles(n, client_every=client_every)
    return ["--peer_bandwidths", ",".join(f"{p.bandwidth:g}" for p in profs),
            "--peer_slowdowns", ",".join(f"{p.slowdown:g}" for p in profs),
            "--peer_client_mode", ",".join(str(int(p.client_mode)) for p in profs)]


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--n_trainers", type=int, default=8)
    ap.add_argument("--n_aux", type=int, default=0)
    ap.add_argument("--n_gpus", type=int, default=None,
                    help="GPUs on this node (default: n_trainers + n_aux, one per peer)")
    ap.add_argument("--experiment_prefix", default="albert")
    ap.add_argument("--fleet", choices=["uniform", "aws"], default="uniform")
    ap.add_argument("--client_every", type=int, default=0, help="every k-th trainer runs in client mode")
    ap.add_argument("--duration", type=float, default=None, help="stop everything after this many seconds")
    ap.add_argument("--log_dir", default="collab_logs")
    ap.add_argument("--sahajbert", action="store_true")
    ap.add_argument("--no_coordinator", action="store_true")
    ap.add_argument("--coordinator_refresh", type=float, default=5.0, help="coordinator metrics poll period (s)")
    args = ap.parse_args(argv)
    log_dir = Path(args.log_dir)
    log_dir.mkdir(parents=True, exist_ok=True)
    py = sys.executable
    env0 = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
                PYTHONUNBUFFERED="1")
    procs = []

    def spawn(cmd, log, env):
        f = open(log_dir / log, "w")
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, start_new_session=True)
        procs.append((p, f, log))
        return p

    # 1. coordinator (DHT root)
    if args.no_coordinator:
        root = None
    else:
        spawn([py, "-m", "dedloc_amd.cli.run_first_peer", "--experiment_prefix", args.experiment_prefix,
               "--dht_listen_on", "0.0.0.0:*", "--refresh_period", str(args.coordinator_refresh),
               "--metrics_file", str(log_dir / "coordinator_metrics.jsonl"),
               *(["--max_runtime", str(args.duration)] if args.duration else [])], "coordinator.log", env0)
        root = None
        t0 = time.time()
        while root is None and time.time() - t0 < 300:
            time.sleep(0.5)
            for line in (log_dir / "coordinator.log").read_text().splitlines():
                if line.startswith("Running DHT root at"):
                    root = line.split()[-1]
        if root is None:
            raise RuntimeError("coordinator did not start; see coordinator.log")
        print(f"coordinator DHT root at {root}", flush=True)

    # 2. trainer + aux world
    world = args.n_trainers + args.n_aux
    n_gpus = args.n_gpus or world
    if world > n_gpus:
        raise SystemExit(f"{args.n_trainers} trainers + {args.n_aux} aux peers need {world} GPUs (one RCCL rank per "
                         f"device), the node has {n_gpus}")
    port = _free_port()
    common = ["--experiment_prefix", args.experiment_prefix, *(["--initial_peers", root] if root else [])]
    common += fleet_flags(args.fleet, args.n_trainers, args.client_every) + extra
    for r in range(world):
        aux = r >= args.n_trainers
        env = dict(env0, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        mod = "dedloc_amd.cli.run_aux" if aux else "dedloc_amd.cli.run_trainer"
        cmd = [py, "-m", mod, *common, *(["--sahajbert"] if args.sahajbert and not aux else [])]
        spawn(cmd, f"{'aux' if aux else 'trainer'}{r}.log", env)
    print(f"launched {args.n_trainers} trainers + {args.n_aux} aux peers; logs in {log_dir}", flush=True)

    # 3. supervise: stop at duration, or when every trainer has exited
    t0 = time.time()
    rc = 0
    try:
        while True:
            time.sleep(1.0)
            trainers = [p for p, _, log in procs if log.startswith("trainer")]
            if all(p.poll() is not None for p in trainers):
                rc = max((p.returncode or 0) for p in trainers)
                break
            if args.duration is not None and time.time() - t0 > args.duration:
                break
    finally:
        for p, f, _ in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGTERM)
        deadline = time.time() + 30
        for p, f, _ in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
            f.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())
