"""Contributor entry point (reference sahajbert/contributor_notebook.ipynb): the
notebook's fixed run_trainer flags, client mode, device-sized micro-batch; every generated flag must
parse with the trainer's own argument dataclasses."""
import json
import os
import subprocess
import sys

from dedloc_amd.cli.contributor import main, micro_batch_for_device


def test_contributor_flags_parse_as_run_trainer_arguments(capsys):
    main(["--initial_peers", "127.0.0.1:1234", "--experiment_prefix", "bengali_MAIN", "--username", "robot",
          "--device", "cpu", "--dry_run", "--", "--max_steps", "5"])
    out = json.loads(capsys.readouterr().out)
    argv = out["run_trainer"]
    assert out["micro_batch"] == 1 and argv[0] == "--sahajbert" and "--client_mode" in argv
    from transformers import HfArgumentParser

    from dedloc_amd.cli.arguments import AlbertTrainingArguments, CollaborationArguments, DatasetArguments

    t, d, c = HfArgumentParser((AlbertTrainingArguments, DatasetArguments, CollaborationArguments)) \
        .parse_args_into_dataclasses(argv[1:])
    assert c.client_mode and c.averaging_expiration == 10 and c.statistics_expiration == 120
    assert c.batch_size_lead == 400 and c.initial_peers == ["127.0.0.1:1234"]
    assert t.per_device_train_batch_size == 1 and t.gradient_accumulation_steps == 1 and t.seed == 42
    assert t.max_steps == 5 and c.experiment_prefix == "bengali_MAIN"


def test_micro_batch_sizing_cpu():
    assert micro_batch_for_device("cpu") == 1


def test_contributor_cli_dry_run_subprocess():
    r = subprocess.run([sys.executable, "-m", "dedloc_amd.cli.contributor", "--device", "cpu", "--micro_batch", "8",
                        "--dry_run"], capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["micro_batch"] == 8 and "--per_device_train_batch_size" in out["run_trainer"]


import pytest  # noqa: E402


@pytest.mark.gpu
def test_micro_batch_sizing_gpu(cuda):
    mb = micro_batch_for_device("cuda")
    assert 1 <= mb <= 256 and mb & (mb - 1) == 0  # a power of two up to the measured plateau
