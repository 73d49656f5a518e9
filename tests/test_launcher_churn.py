"""Process-level churn through the launcher (reference ``albert/AWS_runner.ipynb:310-320, 342-370``
respawn loop, ``:30, 227`` CPU aux peers): coordinator + 3 CPU trainers + 1 CPU
auxiliary peer; trainer 1 is SIGKILLed (a spot preemption) and the launcher starts a brand-new
process in its slot.  The coordinator's log must show the alive-peer count dipping and recovering
while the collaboration's step keeps increasing, and the respawned process must re-enter through
a state download."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_launcher_kill_and_respawn_with_cpu_aux(tmp_path):
    from dedloc_amd.models.albert import AlbertConfig

    cfg = tmp_path / "cfg"
    AlbertConfig.tiny(num_hidden_layers=2, max_position_embeddings=64).save_pretrained(str(cfg))
    logs = tmp_path / "logs"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    peer_flags = ["--config_path", str(cfg), "--per_device_train_batch_size", "2", "--seq_length", "64",
                  "--target_batch_size", "24", "--throttle", "0.15", "--statistics_expiration", "5",
                  "--metadata_expiration", "5", "--averaging_timeout", "5", "--averaging_expiration", "2",
                  "--min_refresh_period", "0.1", "--default_refresh_period", "0.3", "--max_steps", "1000000",
                  "--save_steps", "0", "--output_dir", str(tmp_path / "out"), "--dht_listen_on", "127.0.0.1:*",
                  "--listen_on", "127.0.0.1:*", "--compression", "FLOAT16"]
    cmd = [sys.executable, "-m", "dedloc_amd.cli.launch_collaboration", "--n_trainers", "3", "--n_aux", "1", "--cpu",
           "--aux_device", "cpu", "--experiment_prefix", "churn", "--model_config_path", str(cfg),
           "--duration", "75", "--kill_schedule", "25:1", "--respawn", "--respawn_delay", "8",
           "--coordinator_refresh", "0.5", "--log_dir", str(logs), "--", *peer_flags]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    events = [json.loads(l) for l in (logs / "launcher_events.jsonl").read_text().splitlines()]
    kinds = [e["kind"] for e in events]
    assert "kill" in kinds and "respawn" in kinds, kinds
    rows = [json.loads(l) for l in (logs / "coordinator_metrics.jsonl").read_text().splitlines()]
    assert rows, "the coordinator saw no metrics"
    alive = [row["alive peers"] for row in rows]
    steps = [row["step"] for row in rows]
    print("alive peers over time:", alive)
    print("steps:", steps)
    assert max(alive[: max(1, len(alive) // 3)]) == 3, alive  # all three trainers reported early on
    i_dip = next((i for i, a in enumerate(alive) if a < 3 and i > 0 and max(alive[:i]) == 3), None)
    assert i_dip is not None, alive  # the preempted peer's record expired ...
    assert max(alive[i_dip:]) >= 3, alive  # ... and the respawned process brought the count back
    # the step kept increasing throughout (the coordinator also writes a row when only the alive
    # count changes, so consecutive rows may share a step)
    assert all(b >= a for a, b in zip(steps, steps[1:])) and steps[-1] > steps[0], steps
    # the respawned trainer is a new process that joined through a state download
    gen1 = (logs / "trainer1.gen1.log").read_text()
    assert "downloaded state" in gen1, gen1[-3000:]
    aux = (logs / "aux0.log").read_text()
    assert "Traceback" not in aux, aux[-3000:]


@pytest.mark.timeout(120)
def test_launcher_gives_up_on_a_trainer_that_always_fails_fast(tmp_path):
    """with --respawn a trainer that always crashes at start (here: a flag run_trainer
    does not know) is restarted with a doubling delay and, after --max_fast_failures consecutive
    fast failures, given up ('gave_up' event) — the launcher then ends instead of restarting it
    forever."""
    logs = tmp_path / "logs"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "dedloc_amd.cli.launch_collaboration", "--n_trainers", "1", "--cpu",
           "--no_coordinator", "--respawn", "--respawn_delay", "0.2", "--min_run_s", "60", "--max_fast_failures", "3",
           "--log_dir", str(logs), "--", "--no_such_flag"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    events = [json.loads(l) for l in (logs / "launcher_events.jsonl").read_text().splitlines()]
    kinds = [e["kind"] for e in events]
    assert kinds.count("respawn") == 2 and kinds[-2:] == ["gave_up", "stop"], kinds
    delays = [e["respawn_in"] for e in events if e["kind"] == "died"]
    assert delays == [0.4, 0.8], delays  # the delay doubles with each fast failure
    assert r.returncode != 0
