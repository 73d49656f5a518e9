"""Entry points and checkpoint format (CPU): HF checkpoint interchange with transformers, the
coordinator's aggregation and checkpoint upload, the DHT-root CLI, and BASELINE config 1 (single
ALBERT peer on CPU with a local DHT, batch 1) through the real ``run_trainer`` command line."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tiny_dir(tmp_path, **kw):
    from dedloc_amd.models.albert import AlbertConfig

    cfg = AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64, **kw)
    d = tmp_path / "cfg"
    cfg.save_pretrained(str(d))
    return str(d)


def test_hf_checkpoint_roundtrip_with_transformers(tmp_path):
    import transformers

    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining

    torch.manual_seed(0)
    cfg = AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64)
    ours = AlbertForPreTraining(cfg)
    ours.save_pretrained(str(tmp_path / "ours"))
    hf = transformers.AlbertForPreTraining.from_pretrained(str(tmp_path / "ours"))
    ref = ours.hf_state_dict()
    for k, v in hf.state_dict().items():
        if k in ref:
            assert torch.allclose(v, ref[k].float()), k
    # and back: an HF-saved checkpoint loads into ours
    with torch.no_grad():
        hf.albert.embeddings.LayerNorm.weight.add_(0.5)
    hf.save_pretrained(str(tmp_path / "hf"), safe_serialization=False)
    back = AlbertForPreTraining.from_pretrained(str(tmp_path / "hf"))
    assert torch.allclose(back.hf_state_dict()["albert.embeddings.LayerNorm.weight"],
                          hf.albert.embeddings.LayerNorm.weight.detach())


def test_coordinator_aggregate():
    from dedloc_amd.cli.run_first_peer import aggregate
    from dedloc_amd.dht.node import ValueWithExpiration
    from dedloc_amd.metrics import LocalMetrics

    recs = {b"a": ValueWithExpiration(LocalMetrics(step=4, samples_per_second=10.0, samples_accumulated=32, loss=6.0,
                                                   mini_steps=3).model_dump(), 0.0),
            b"b": ValueWithExpiration(LocalMetrics(step=5, samples_per_second=30.0, samples_accumulated=64, loss=2.0,
                                                   mini_steps=1).model_dump(), 0.0)}
    agg = aggregate(recs)
    assert agg["step"] == 5 and agg["alive peers"] == 2 and agg["samples"] == 96
    assert agg["performance"] == 40.0  # the BASELINE metric: sum of the peers' samples/s
    assert agg["loss"] == pytest.approx(8.0 / 4)


def test_checkpoint_handler_uploads_into_git_repo(tmp_path):
    from dedloc_amd.cli.arguments import AveragerArguments, CollaborativeOptimizerArguments, CoordinatorArguments
    from dedloc_amd.cli.run_first_peer import CheckpointHandler
    from dedloc_amd.dht import DHT

    repo = tmp_path / "repo"
    repo.mkdir()
    subprocess.run(["git", "init", "-q"], cwd=repo, check=True)
    subprocess.run(["git", "config", "user.email", "t@t"], cwd=repo, check=True)
    subprocess.run(["git", "config", "user.name", "t"], cwd=repo, check=True)
    dht = DHT(start=True)
    try:
        ca = CoordinatorArguments(experiment_prefix="ck", model_config_path=_tiny_dir(tmp_path), repo_path=str(repo),
                                  upload_interval=0, save_checkpoint_step_interval=1)
        h = CheckpointHandler(ca, CollaborativeOptimizerArguments(), AveragerArguments(), dht, b"coord")
        assert h.is_time_to_save_state(1)
        h.save_state(1)  # nobody shares state: keeps the local replica
        assert h.is_time_to_upload()
        h.upload_checkpoint(3.25)
        assert (repo / "pytorch_model.bin").exists() and (repo / "optimizer_state.pt").exists()
        log = subprocess.run(["git", "log", "--oneline"], cwd=repo, capture_output=True, text=True).stdout
        assert "loss 3.250" in log
        h.collaborative_optimizer.shutdown()
    finally:
        dht.shutdown()


def test_run_initial_dht_node_cli():
    r = subprocess.run([sys.executable, "-m", "dedloc_amd.cli.run_initial_dht_node", "--listen_on", "127.0.0.1:*",
                        "--refresh_period", "0.2", "--max_runtime", "1"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Running DHT root at 127.0.0.1:" in r.stdout


@pytest.mark.timeout(300)
@pytest.mark.parametrize("sahajbert", [False, True])
def test_run_trainer_single_cpu_peer(tmp_path, sahajbert):
    """BASELINE config 1: one peer on CPU, local DHT root, batch 1, reference flags."""
    from dedloc_amd.dht import DHT

    root = DHT(listen_on="127.0.0.1:*")
    try:
        metrics = tmp_path / "m.jsonl"
        cmd = [sys.executable, "-m", "dedloc_amd.cli.run_trainer", "--experiment_prefix", "cfg1",
               "--initial_peers", root.endpoint, "--device", "cpu", "--config_path", _tiny_dir(tmp_path),
               "--per_device_train_batch_size", "1", "--gradient_accumulation_steps", "2", "--seq_length", "64",
               "--target_batch_size", "4", "--stop_after_global_steps", "2", "--save_steps", "0",
               "--output_dir", str(tmp_path / "out"), "--min_refresh_period", "0.05", "--default_refresh_period",
               "0.1", "--dht_listen_on", "127.0.0.1:*", "--listen_on", "127.0.0.1:*", "--metrics_file", str(metrics)]
        if sahajbert:
            cmd.append("--sahajbert")
        env = dict(os.environ, PYTHONPATH=ROOT)
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        recs = [json.loads(x) for x in metrics.read_text().splitlines()]
        assert max(rec["step"] for rec in recs) >= 2
    finally:
        root.shutdown()


@pytest.mark.multiproc
@pytest.mark.timeout(420)
def test_launch_collaboration_coordinator_trainers_aux_cpu(tmp_path):
    """The single-node launcher (AWS_runner stand-in, D9): coordinator + 2 trainers + 1 auxiliary peer
    on CPU/gloo (no launch-time world: the peers meet through the coordinator's DHT); the trainers finish their global steps and the coordinator's metrics
    file reports both trainers alive (the aux peer publishes no training metrics)."""
    logs = tmp_path / "logs"
    cmd = [sys.executable, "-m", "dedloc_amd.cli.launch_collaboration", "--n_trainers", "2", "--n_aux", "1",
           "--experiment_prefix", "launch", "--log_dir", str(logs), "--duration", "360",
           "--coordinator_refresh", "0.3", "--",
           "--device", "cpu", "--config_path", _tiny_dir(tmp_path), "--per_device_train_batch_size", "2",
           "--seq_length", "64", "--target_batch_size", "8", "--stop_after_global_steps", "6", "--save_steps", "0",
           "--output_dir", str(tmp_path / "out"), "--min_refresh_period", "0.05", "--default_refresh_period", "0.1",
           "--dht_listen_on", "127.0.0.1:*", "--listen_on", "127.0.0.1:*", "--averaging_expiration", "3",
           "--compression", "NONE", "--throttle", "0.05"]
    # --throttle: 6 global steps of the tiny model take ~1 s, less than the start-up skew of two
    # trainer processes on a loaded host; paced steps make the two trainers actually collaborate
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400, env=env)
    tails = {p.name: p.read_text()[-1500:] for p in logs.glob("*.log")}
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:], tails)
    events = [json.loads(x) for x in (logs / "launcher_events.jsonl").read_text().splitlines()]
    assert any(e["kind"] == "coordinator" and e["dht_root"] for e in events), events
    for t in ("trainer0.log", "trainer1.log"):
        assert "Traceback" not in tails[t], tails[t]
    recs = [json.loads(x) for x in (logs / "coordinator_metrics.jsonl").read_text().splitlines()] \
        if (logs / "coordinator_metrics.jsonl").exists() else []
    assert recs and max(rec["step"] for rec in recs) >= 1 and max(rec["alive peers"] for rec in recs) == 2, tails
