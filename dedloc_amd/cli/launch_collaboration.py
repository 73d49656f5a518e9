#!/usr/bin/env python
"""Single-node collaboration launcher — the MI355X stand-in for ``albert/AWS_runner.ipynb`` (SURVEY.md
§2.1 D9): one coordinator (DHT root + metrics aggregation, ``run_first_peer``), N GPU trainer peers and
A auxiliary peers, with the AWS fleet's heterogeneity injected per peer slot and its spot churn
(preemption + the respawn loop of ``AWS_runner.ipynb:342-370``) reproduced at process level.

    python -m dedloc_amd.cli.launch_collaboration --n_trainers 8 --n_aux 4 --fleet aws --duration 600 \\
        --kill_schedule 120:3,300:5 --respawn --respawn_delay 30 \\
        --experiment_prefix albert -- --per_device_train_batch_size 32 --target_batch_size 4096

Everything after ``--`` is passed to every trainer (and aux peer).  There is no launch-time world:
every peer is an independent process that bootstraps from the coordinator's DHT and averages over
communicators its matchmade groups build themselves (``parallel/comm.py``), so a killed trainer can
be replaced by a brand-new process (new peer id) that downloads the state and joins the next round.

* trainer i runs on GPU i (``LOCAL_RANK=i``, also its heterogeneity slot), or on the CPU with
  ``--cpu`` (plumbing / tests);
* auxiliary peers run on the CPU by default, like the reference's ``r5.large`` aux instances
  (``AWS_runner.ipynb:30, 186-217``): they need no spare GPU; a round that contains one runs over
  gloo.  ``--aux_device gpu`` puts them on GPUs ``n_trainers..`` instead;
* ``--kill_schedule T:i[,T:i...]`` SIGKILLs trainer i T seconds after launch (a spot preemption: no
  clean-up, no tombstone); with ``--respawn`` every trainer that dies is restarted as a fresh process
  in its slot after ``--respawn_delay`` seconds.  Events go to ``launcher_events.jsonl``.

This process never touches the GPU itself; children are plain subprocesses.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
from pathlib import Path

from ..emulation.heterogeneity import aws_fleet_profiles


def fleet_flags(fleet: str, n: int, client_every: int = 0):
    if fleet == "uniform":
        return []
    profs = aws_fleet_profiles(n, client_every=client_every)
    return ["--peer_bandwidths", ",".join(f"{p.bandwidth:g}" for p in profs),
            "--peer_slowdowns", ",".join(f"{p.slowdown:g}" for p in profs),
            "--peer_client_mode", ",".join(str(int(p.client_mode)) for p in profs)]


def parse_kill_schedule(spec):
    out = []
    for item in (spec or "").split(","):
        if item.strip():
            t, slot = item.split(":")
            out.append((float(t), int(slot)))
    return sorted(out)


class _Proc:
    def __init__(self, name, cmd, env, log_dir: Path, generation: int):
        self.name, self.cmd, self.env, self.generation = name, cmd, env, generation
        self.log_path = log_dir / (f"{name}.log" if generation == 0 else f"{name}.gen{generation}.log")
        self.f = open(self.log_path, "w")
        self.p = subprocess.Popen(cmd, stdout=self.f, stderr=subprocess.STDOUT, env=env, start_new_session=True)
        self.started = time.time()
        self.killed = False  # ended by the kill schedule (a scripted preemption), not by itself

    def alive(self):
        return self.p.poll() is None

    def kill(self, sig=signal.SIGKILL):
        if self.alive():
            try:
                os.killpg(self.p.pid, sig)
            except ProcessLookupError:
                pass


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--n_trainers", type=int, default=8)
    ap.add_argument("--n_aux", type=int, default=0)
    ap.add_argument("--n_gpus", type=int, default=None, help="GPUs on this node (default: one per GPU peer)")
    ap.add_argument("--cpu", action="store_true", help="run the trainers on the CPU (plumbing / tests)")
    ap.add_argument("--allow_shared_device", action="store_true",
                    help="more GPU peers than --n_gpus: peer slot i runs on GPU i %% n_gpus (protocol emulation on "
                         "a small box; peers on one device average over gloo, RCCL takes one rank per device)")
    ap.add_argument("--aux_device", choices=["cpu", "gpu"], default="cpu")
    ap.add_argument("--experiment_prefix", default="albert")
    ap.add_argument("--model_config_path", default=None, help="model config for the coordinator's replica")
    ap.add_argument("--fleet", choices=["uniform", "aws"], default="uniform")
    ap.add_argument("--client_every", type=int, default=0, help="every k-th trainer runs in client mode")
    ap.add_argument("--duration", type=float, default=None, help="stop everything after this many seconds")
    ap.add_argument("--kill_schedule", default=None, help="T:slot[,T:slot...] — SIGKILL trainer `slot` at T s")
    ap.add_argument("--respawn", action="store_true", help="restart dead trainers as fresh processes")
    ap.add_argument("--respawn_delay", type=float, default=30.0)
    ap.add_argument("--min_run_s", type=float, default=30.0,
                    help="a trainer that exits on its own (non-zero) sooner than this after starting is a fast "
                         "failure: its respawn delay doubles each time (capped at 10 x respawn_delay)")
    ap.add_argument("--max_fast_failures", type=int, default=5,
                    help="stop respawning a slot after this many consecutive fast failures (a bad config or "
                         "import error would otherwise restart forever)")
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
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env0.pop(k, None)
    events = open(log_dir / "launcher_events.jsonl", "a")
    t_start = time.time()

    def event(kind, **kw):
        events.write(json.dumps(dict(kind=kind, t=round(time.time() - t_start, 3), **kw)) + "\n")
        events.flush()
        print(f"[launcher +{time.time() - t_start:7.1f}s] {kind} {kw}", flush=True)

    others = []

    # 1. coordinator (DHT root)
    root = None
    if not args.no_coordinator:
        cmd = [py, "-m", "dedloc_amd.cli.run_first_peer", "--experiment_prefix", args.experiment_prefix,
               "--dht_listen_on", "0.0.0.0:*", "--refresh_period", str(args.coordinator_refresh),
               "--metrics_file", str(log_dir / "coordinator_metrics.jsonl"),
               *(["--model_config_path", args.model_config_path] if args.model_config_path else []),
               *(["--vocab_size", "31995"] if args.sahajbert else []),
               *(["--max_runtime", str(args.duration)] if args.duration else [])]
        coord = _Proc("coordinator", cmd, env0, log_dir, 0)
        others.append(coord)
        t0 = time.time()
        while root is None and time.time() - t0 < 300:
            time.sleep(0.5)
            for line in coord.log_path.read_text().splitlines():
                if line.startswith("Running DHT root at"):
                    root = line.split()[-1]
            if not coord.alive():
                break
        if root is None:
            raise RuntimeError(f"coordinator did not start; see {coord.log_path}")
        event("coordinator", dht_root=root)

    # 2. peers
    n_gpu_peers = (0 if args.cpu else args.n_trainers) + (args.n_aux if args.aux_device == "gpu" else 0)
    n_gpus = args.n_gpus if args.n_gpus is not None else n_gpu_peers
    if n_gpu_peers > n_gpus and not args.allow_shared_device:
        raise SystemExit(f"{n_gpu_peers} GPU peers need {n_gpu_peers} GPUs (one RCCL rank per device), the node has "
                         f"{n_gpus}; run auxiliary peers on the CPU (--aux_device cpu)")
    common = ["--experiment_prefix", args.experiment_prefix, *(["--initial_peers", root] if root else [])]
    common += fleet_flags(args.fleet, args.n_trainers, args.client_every) + extra

    def trainer_cmd(slot):
        dev = ["--device", "cpu"] if args.cpu else []
        return [py, "-m", "dedloc_amd.cli.run_trainer", *common, *dev, *(["--sahajbert"] if args.sahajbert else [])]

    trainers = {}
    for r in range(args.n_trainers):
        trainers[r] = _Proc(f"trainer{r}", trainer_cmd(r), dict(env0, LOCAL_RANK=str(r)), log_dir, 0)
        event("start", slot=r, pid=trainers[r].p.pid, generation=0)
    for j in range(args.n_aux):
        on_gpu = args.aux_device == "gpu"
        env = dict(env0, LOCAL_RANK=str(args.n_trainers + j if on_gpu else 0))
        cmd = [py, "-m", "dedloc_amd.cli.run_aux", *common, *([] if on_gpu else ["--device", "cpu"])]
        others.append(_Proc(f"aux{j}", cmd, env, log_dir, 0))
        event("start_aux", index=j, device="gpu" if on_gpu else "cpu")
    print(f"launched {args.n_trainers} trainers + {args.n_aux} aux peers; logs in {log_dir}", flush=True)

    # 3. supervise: scripted preemptions, respawn loop, stop at duration / when all trainers finished
    kills = parse_kill_schedule(args.kill_schedule)
    respawn_at = {}
    fast_failures, gave_up = {}, set()
    rc = 0
    try:
        while True:
            time.sleep(0.2)
            now = time.time() - t_start
            while kills and kills[0][0] <= now:
                _, slot = kills.pop(0)
                proc = trainers.get(slot)
                if proc is not None and proc.alive():
                    proc.kill(signal.SIGKILL)
                    proc.killed = True
                    event("kill", slot=slot, pid=proc.p.pid, generation=proc.generation)
            for slot, proc in trainers.items():
                if proc.alive() or slot in respawn_at or slot in gave_up or getattr(proc, "handled", False):
                    continue
                proc.handled = True
                code = proc.p.returncode
                finished = code == 0
                if args.respawn and not finished:
                    fast = not proc.killed and time.time() - proc.started < args.min_run_s
                    fast_failures[slot] = fast_failures.get(slot, 0) + 1 if fast else 0
                    if fast_failures[slot] >= args.max_fast_failures:
                        gave_up.add(slot)
                        event("gave_up", slot=slot, returncode=code, fast_failures=fast_failures[slot])
                        continue
                    delay = min(args.respawn_delay * 2 ** fast_failures[slot], 10 * args.respawn_delay)
                    respawn_at[slot] = now + delay
                    event("died", slot=slot, returncode=code, respawn_in=delay, fast_failures=fast_failures[slot])
            for slot, t in list(respawn_at.items()):
                if t <= now:
                    del respawn_at[slot]
                    gen = trainers[slot].generation + 1
                    trainers[slot].f.close()
                    trainers[slot] = _Proc(f"trainer{slot}", trainer_cmd(slot), dict(env0, LOCAL_RANK=str(slot)),
                                           log_dir, gen)
                    event("respawn", slot=slot, pid=trainers[slot].p.pid, generation=gen)
            if not respawn_at and not kills and all(not p.alive() for p in trainers.values()):
                rc = max((p.p.returncode or 0) for p in trainers.values())
                break
            if args.duration is not None and now > args.duration:
                break
    finally:
        for proc in list(trainers.values()) + others:
            proc.kill(signal.SIGTERM)
        deadline = time.time() + 30
        for proc in list(trainers.values()) + others:
            try:
                proc.p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                proc.kill(signal.SIGKILL)
            proc.f.close()
        event("stop")
        events.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())
