"""bench.py driver contract, exercised on CPU/gloo with a tiny model (multi-rank orchestration:
DHT root broadcast, state download, collaborative steps with averaging, barrier-bracketed timing,
max-over-ranks time, ONE JSON line from rank 0 with the required keys)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.multiproc
@pytest.mark.timeout(400)
@pytest.mark.parametrize("nproc", [2, 4])
def test_bench_multi_rank_cpu_plumbing(tmp_path, nproc):
    from dedloc_amd.models.albert import AlbertConfig

    cfg = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfg))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc), "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(nproc), "--steps", "2", "--warmup", "1",
           "--cpu_test", str(cfg), "--micro_batch", "2", "--seq_len", "64", "--target_batch_size", str(4 * nproc)]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=360, env=env)
    wall = time.time() - t0
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == nproc and out["steps"] == 2 and out["value"] > 0 and out["higher_is_better"] is True
    # every global step (warm-up + timed) averaged over the world communicator with all peers
    assert out["averaging_rounds"] >= 3 and out["averaging_failed"] == 0
    assert out["last_group"]["size"] == nproc
    # timed-region protocol breakdown: every global step took at least one local micro-step
    prot = out["protocol"]
    assert prot["local_steps"] >= 1 and min(prot["fetch_ms"], prot["averaging_ms"], prot["optimizer_ms"]) >= 0
    # a fresh collaboration starts at once (no circular state downloads between step-0 peers) and
    # no step waits out a matchmaking window
    assert out["ms_per_step"] < 4000 and wall < 120, (out["ms_per_step"], wall)


@pytest.mark.multiproc
@pytest.mark.timeout(400)
def test_bench_self_launches_peers_without_torchrun(tmp_path):
    """`python bench.py --gpus 3` (no torchrun, no WORLD_SIZE): the script starts its three peer
    processes itself; they find each other through the DHT, average every global step, and rank 0
    reports 3 peers."""
    from dedloc_amd.models.albert import AlbertConfig

    cfg = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfg))
    cmd = [sys.executable, "bench.py", "--gpus", "3", "--steps", "2", "--warmup", "1", "--cpu_test", str(cfg),
           "--micro_batch", "2", "--seq_len", "64", "--target_batch_size", "12"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=360, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == 3 and out["peers"] == 3 and out["physical_gpus"] == 0
    assert out["averaging_rounds"] >= 3 and out["averaging_failed"] == 0 and out["last_group"]["size"] == 3
    assert out["data_plane"] == "gloo"


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_bench_refuses_more_peers_than_gpus():
    """On a box with fewer GPUs than --gpus, bench.py refuses to put two peers on one device unless
    --allow_shared_device is given (the check runs before any GPU work)."""
    import torch

    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--steps", "1", "--warmup", "0"], cwd=ROOT,
                       capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--allow_shared_device" in r.stderr


@pytest.mark.multiproc
@pytest.mark.timeout(600)
def test_bench_swav_mode_two_ranks_cpu():
    """bench.py --model swav (BASELINE config 3): two collaborative SwAV ResNet-50 peers on CPU/gloo run
    global steps with averaging and rank 0 prints one JSON line with the SwAV metric."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--model", "swav", "--gpus", "2", "--steps", "1",
           "--warmup", "1", "--cpu_test", "swav", "--micro_batch", "2", "--target_batch_size", "8"]
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=560, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["metric"].startswith("samples/sec (whole node) SwAV ResNet-50") and out["n_gpus"] == 2
    assert out["config"]["model"] == "swav-resnet50" and out["config"]["optimizer"] == "LARC-SGD"
    assert out["averaging_rounds"] >= 2 and out["averaging_failed"] == 0 and out["last_group"]["size"] == 2


def test_bench_fails_multi_gpu_runs_that_fell_back_to_gloo():
    """N > 1 peers on N GPUs that did not all average over RCCL make bench.py exit 3
    (the decision; the exit itself needs a multi-GPU box)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_script", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)  # (the bench/ package shadows the name "bench")
    spec.loader.exec_module(bench)
    f = bench.rccl_fallback
    assert f("cuda", 8, 8, [10] * 8, [0] * 7 + [1])          # one round of one peer over gloo
    assert f("cuda", 2, 2, [0, 10], [0, 0])                  # a peer that never averaged over RCCL
    assert not f("cuda", 8, 8, [10] * 8, [0] * 8)
    assert not f("cuda", 8, 8, [10] * 7 + [9], [0] * 8)      # a straggler's last round failed: fine
    assert not f("cuda", 4, 1, [0] * 4, [10] * 4)            # --allow_shared_device: gloo by design
    assert not f("cpu", 8, 0, [10] * 8, [0] * 8)             # CPU plumbing
    assert not f("cuda", 1, 1, [0], [0])                     # one peer averages with nobody
