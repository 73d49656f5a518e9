"""Cross-process rehearsal of the multi-peer RCCL data plane ("next round" item 1).

RCCL takes one rank per device, so the multi-rank RCCL path cannot run on a one-GPU box — and the
driver's 8-GPU scaling run must not be the first time this code sees more than one process.  Here
separate peer processes run the real data-plane code (``parallel/comm.py`` token reuse and
communicator cache, ``comm_worker.py`` jobs, the butterfly all-reduce, the state server's RCCL
mode) with only ``torch.ops.dedloc_comm`` replaced by the mailbox stand-in of
``tests/xproc/xproc_rccl.py`` (installed by ``tests/xproc/sitecustomize.py``; no production
switch).  What this pins, across processes:

* ``bench.py --gpus 8`` (ALBERT) averages every global step over "rccl" with ONE communicator per
  peer, reused for every round (the token-reuse rule);
* ``bench.py --model swav --gpus 8`` (groups of 4, Moshpit alternating partitions) builds exactly
  TWO communicators per peer (block and stride partitions) and reuses them;
* a peer SIGKILLed in the middle of a round: the 7 survivors abort at the deadline, rebuild a
  7-member communicator and complete an exact next round within the averaging timeout;
* a late joiner downloads the state over the RCCL path (mode "R") between two processes and then
  averages with the others.

Parity note: the stand-in moves bytes through tmpfs, not xGMI; RCCL itself is exercised only by the
GPU tests (tests/test_rccl_group_gpu.py, tests/test_rccl_multi_gpu.py on a 2+ GPU box).
"""
import json
import os
import signal
import subprocess
import sys
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XPROC = os.path.join(ROOT, "tests", "xproc")
PEER = os.path.join(ROOT, "tests", "helpers", "collab_peer.py")


def _env(mbox, **extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=f"{XPROC}:{ROOT}", DEDLOC_XPROC_RCCL_DIR=str(mbox))
    env.update(extra)
    return env


def _tiny_cfg(tmp_path):
    from dedloc_amd.models.albert import AlbertConfig

    cfg = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfg))
    return cfg


def _bench_json(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return json.loads(lines[0])


@pytest.mark.multiproc
@pytest.mark.timeout(300)
def test_bench_eight_peers_albert_one_reused_rccl_communicator(tmp_path):
    cfg = _tiny_cfg(tmp_path)
    cmd = [sys.executable, "bench.py", "--gpus", "8", "--steps", "10", "--warmup", "1", "--cpu_test", str(cfg),
           "--micro_batch", "2", "--seq_len", "64", "--target_batch_size", "16"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280, env=_env(tmp_path / "mbox"))
    out = _bench_json(r)
    pp = out["per_peer"]
    assert out["n_gpus"] == 8 and out["data_plane"] == "rccl"
    assert pp["data_plane"] == ["rccl"] * 8, pp
    assert out["averaging_rounds"] >= 10 and pp["averaging_failed"] == [0] * 8, pp
    assert out["last_group"]["size"] == 8
    assert pp["comms_created"] == [1] * 8 and pp["comms_aborted"] == [0] * 8, pp  # built once, reused
    assert pp["comms_quarantined"] == [0] * 8
    assert min(pp["rounds_rccl"]) >= 10 and pp["rounds_other"] == [0] * 8, pp


@pytest.mark.multiproc
@pytest.mark.timeout(600)
def test_bench_eight_peers_swav_two_partition_communicators(tmp_path):
    # 10 timed + 1 warm-up global steps: >= 10 rounds even when a peer that lagged one step at the
    # start adopts the group's step (one step number fewer to run)
    cmd = [sys.executable, "bench.py", "--model", "swav", "--gpus", "8", "--steps", "10", "--warmup", "1",
           "--cpu_test", "swav", "--micro_batch", "1", "--target_batch_size", "8"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=580, env=_env(tmp_path / "mbox"))
    out = _bench_json(r)
    pp = out["per_peer"]
    assert out["config"]["target_group_size"] == 4 and out["last_group"]["size"] == 4
    assert pp["data_plane"] == ["rccl"] * 8, pp
    assert out["averaging_rounds"] >= 10 and pp["averaging_failed"] == [0] * 8, pp
    # Moshpit groups of 4 over 8 peers alternate between two partitions: one communicator each
    assert pp["comms_created"] == [2] * 8 and pp["comms_aborted"] == [0] * 8, pp


def _records(out, name):
    path = out / f"peer-{name}.jsonl"
    if not path.exists():
        return []
    return [json.loads(ln) for ln in path.read_text().splitlines() if ln.strip()]


def _wait(cond, timeout, procs=()):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if cond():
            return True
        time.sleep(0.2)
    return False


@pytest.mark.multiproc
@pytest.mark.timeout(400)
def test_sigkill_mid_round_survivors_rebuild_and_joiner_downloads_over_rccl(tmp_path):
    from dedloc_amd.dht import DHT

    cfg = _tiny_cfg(tmp_path)
    out = tmp_path / "out"
    out.mkdir()
    mbox = tmp_path / "mbox"
    timeout_s, expiration_s = 8.0, 2.0
    root = DHT(listen_on="127.0.0.1:*")
    procs = {}

    def start(name, *extra, **env):
        cmd = [sys.executable, PEER, "--root", root.endpoint, "--cfg", str(cfg), "--name",
               name, "--out", str(out), "--steps", "24", "--averaging_timeout", str(timeout_s),
               "--averaging_expiration", str(expiration_s), *extra]
        procs[name] = subprocess.Popen(cmd, cwd=ROOT, env=_env(mbox, **env), stdout=subprocess.DEVNULL,
                                       stderr=open(out / f"{name}.err", "w"), start_new_session=True)

    try:
        # p3 dies in its 7th grouped send/recv: the scatter of the 4th round, half of its sends posted
        for i in range(8):
            start(f"p{i}", "--barrier", **({"DEDLOC_XPROC_DIE_AT_P2P": "7"} if i == 3 else {}))
        # the late joiner is built now too (imports take seconds) but joins only after the failure
        start("joiner", "--join", "--barrier", "--gate", "join")
        survivors = [f"p{i}" for i in range(8) if i != 3]
        assert _wait(lambda: all((out / f"ready-{n}").exists() for n in list(procs)), 120)
        (out / "go").touch()  # all eight start training together
        # once the survivors are past the failure, the joiner downloads the state and joins
        assert _wait(lambda: all(any(r.get("step", 0) >= 7 for r in _records(out, n)) for n in survivors), 200), \
            {n: _records(out, n)[-1:] for n in survivors}
        (out / "join").touch()
        for n in survivors + ["joiner"]:
            procs[n].wait(timeout=200)
        assert procs["p3"].wait(timeout=10) == -signal.SIGKILL
        for n in survivors + ["joiner"]:
            assert procs[n].returncode == 0, (n, (out / f"{n}.err").read_text()[-3000:])
    finally:
        for p in procs.values():
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        root.shutdown()

    recs = {n: [r for r in _records(out, n) if r["event"] == "step"] for n in survivors}
    rebuilt, snaps = set(), []
    for n, rs in recs.items():
        # every survivor saw exactly one failed round: the one the dead peer left in the middle
        i = next(k for k, r in enumerate(rs) if r["failed"] > 0)
        assert rs[-1]["failed"] == 1 and 0 < i < len(rs) - 1, (n, rs)
        before, failed, after = rs[i - 1], rs[i], rs[i + 1]
        # until then all eight averaged every step on ONE communicator, built once
        assert all(r["size"] == 8 and r["created"] == 1 for r in rs[:i]), (n, rs[:i])
        # the dead round aborted its communicator (dropped from the cache) ...
        assert failed["aborted"] == 1 and failed["quarantined"] == 0, failed
        # ... and the next round ran on a freshly built 7-member communicator, within the deadline
        assert after["size"] == 7 and after["backend"] == "rccl" and after["created"] == 2, after
        assert after["t"] - failed["t"] < timeout_s + expiration_s + 5.0, (failed, after)
        rebuilt.add(after["group_id"])
        snaps.append(torch.load(out / f"{n}-s{after['step'] - 1}.pt", weights_only=True))
    assert len(rebuilt) == 1, rebuilt
    # an exact round: the 7 members hold the same average
    assert {s["group_id"] for s in snaps} == rebuilt and all(s["size"] == 7 for s in snaps)
    for s in snaps[1:]:
        torch.testing.assert_close(s["params"], snaps[0]["params"], rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(s["grads"], snaps[0]["grads"], rtol=1e-5, atol=1e-7)

    # the joiner: state over the RCCL path from another process, then averaging with the others
    jr = _records(out, "joiner")
    join = [r for r in jr if r["event"] == "join"][0]
    assert join["ok"] and join["download"]["mode"] == "R" and join["step"] >= 7, join
    jsteps = [r for r in jr if r["event"] == "step" and r["size"] == 8]
    assert jsteps, jr
    js = torch.load(out / f"joiner-s{jsteps[-1]['step'] - 1}.pt", weights_only=True)
    p0 = {r["group_id"]: r["step"] for r in recs["p0"]}
    other = torch.load(out / f"p0-s{p0[js['group_id']] - 1}.pt", weights_only=True)
    assert js["group_id"] == other["group_id"]
    torch.testing.assert_close(js["params"], other["params"], rtol=1e-6, atol=1e-7)


def _run_peers(tmp_path, specs, steps=10, timeout_s=8.0, expiration_s=2.0, wait_s=200):
    """Start collab_peer processes (name, extra args, extra env) together through the barrier; the
    trainers run ``steps`` global steps, auxiliary peers run until the trainers are done."""
    from dedloc_amd.dht import DHT

    cfg = _tiny_cfg(tmp_path)
    out = tmp_path / "out"
    out.mkdir()
    root = DHT(listen_on="127.0.0.1:*")
    procs = {}
    try:
        for name, extra, env in specs:
            cmd = [sys.executable, PEER, "--root", root.endpoint, "--cfg", str(cfg), "--name", name, "--out", str(out),
                   "--steps", str(steps), "--averaging_timeout", str(timeout_s), "--averaging_expiration",
                   str(expiration_s), "--barrier", *extra]
            procs[name] = subprocess.Popen(cmd, cwd=ROOT, env=_env(tmp_path / "mbox", **env), stdout=subprocess.DEVNULL,
                                           stderr=open(out / f"{name}.err", "w"), start_new_session=True)
        assert _wait(lambda: all((out / f"ready-{n}").exists() for n in procs), 120)
        (out / "go").touch()
        trainers = [n for n, extra, _ in specs if "--aux" not in extra]
        for n in trainers:
            procs[n].wait(timeout=wait_s)
        (out / "stop").touch()
        for n in procs:
            assert procs[n].wait(timeout=60) == 0, (n, (out / f"{n}.err").read_text()[-3000:])
    finally:
        for p in procs.values():
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
        root.shutdown()
    return out


@pytest.mark.multiproc
@pytest.mark.timeout(300)
def test_mixed_group_gpu_trainers_and_cpu_aux_across_processes(tmp_path):
    """The reference fleet's shape (AWS_runner.ipynb:26-30: GPU trainers + CPU auxiliary peers) across
    processes: three "GPU" trainers on the RCCL stand-in and one auxiliary peer forced to gloo
    (DEDLOC_DATA_PLANE=gloo, a CPU aux) form hybrid groups — RCCL among the trainers, gloo only for
    the pairs with the aux — every round succeeds and the trainers hold the same average."""
    specs = [(f"t{i}", [], {}) for i in range(3)] + [("aux", ["--aux"], {"DEDLOC_DATA_PLANE": "gloo"})]
    out = _run_peers(tmp_path, specs, steps=8)
    recs = {n: [r for r in _records(out, n) if r["event"] == "step"] for n in ("t0", "t1", "t2")}
    for n, rs in recs.items():
        assert rs[-1]["failed"] == 0, (n, rs)
        hybrid = [r for r in rs if r["backend"] == "rccl+gloo"]
        assert len(hybrid) >= 5 and all(r["size"] == 4 for r in hybrid), (n, rs)
        assert rs[-1]["created"] <= 2, rs[-1]  # built once (a second only if the aux joined late)
    aux = [r for r in _records(out, "aux") if r["event"] == "aux_round"]
    assert len(aux) >= 5 and all(r["backend"] == "rccl+gloo" for r in aux), aux
    # an exact round: the trainers of one hybrid round hold the same average
    last = {n: [r for r in rs if r["backend"] == "rccl+gloo"][-1] for n, rs in recs.items()}
    assert len({r["group_id"] for r in last.values()}) == 1, last
    snaps = [torch.load(out / f"{n}-s{r['step'] - 1}.pt", weights_only=True) for n, r in last.items()]
    for s in snaps[1:]:
        torch.testing.assert_close(s["params"], snaps[0]["params"], rtol=1e-6, atol=1e-7)


@pytest.mark.multiproc
@pytest.mark.timeout(300)
def test_asynchronous_rccl_error_fails_one_round_then_rebuilds(tmp_path):
    """An asynchronous RCCL error on one member (ncclSystemError reported by a status poll after its
    grouped call was accepted): that member's round fails AT ONCE (its own RCCL failed: no deadline
    wait), the others' at the round's deadline; they drop the communicator and average on a freshly
    built one in the next round.  (The failed member itself moves on with its local gradients — it
    is ahead for a while, exactly as a hivemind peer whose round failed.)"""
    timeout_s = 8.0
    specs = [(f"p{i}", [], {"DEDLOC_XPROC_ERROR_AT_P2P": "5"} if i == 2 else {}) for i in range(4)]
    out = _run_peers(tmp_path, specs, steps=8, timeout_s=timeout_s)
    recs = {n: [r for r in _records(out, n) if r["event"] == "step"] for n in ("p0", "p1", "p2", "p3")}
    first_fail = {}
    for n, rs in recs.items():
        i = next(k for k, r in enumerate(rs) if r["failed"] > 0)
        assert all(r["size"] == 4 and r["created"] == 1 for r in rs[:i]), (n, rs[:i])
        first_fail[n] = (i, rs[i]["t"])
    # the erroring member failed without waiting for the deadline; the others waited it out
    t_err = first_fail["p2"][1]
    for n in ("p0", "p1", "p3"):
        assert first_fail[n][1] - t_err > timeout_s - 3.0, first_fail
    rebuilt = set()
    for n in ("p0", "p1", "p3"):
        rs, i = recs[n], first_fail[n][0]
        assert rs[-1]["failed"] == 1 and i < len(rs) - 1, (n, rs)
        after = rs[i + 1]
        assert after["size"] >= 3 and after["created"] == 2 and after["backend"] == "rccl", (n, after)
        rebuilt.add(after["group_id"])
    assert len(rebuilt) == 1, rebuilt
