import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "multiproc: spawns several processes (gloo on CPU)")


def record_margin(test: str, **fields):
    """Append a numerics test's measured margins (errors and the bounds they are held to) to a JSONL
    file — ``$DEDLOC_MARGINS_FILE``, default ``gpurun_out/parity_margins.jsonl`` (merged back from a
    GPU box; the committed copy lives under profiles/)."""
    import json
    import time

    path = os.environ.get("DEDLOC_MARGINS_FILE") or os.path.join(ROOT, "gpurun_out", "parity_margins.jsonl")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(dict(test=test, time=time.time(), **fields)) + "\n")
    except OSError:
        pass


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import dedloc_amd.ops as ops

    assert ops.native_loaded(), "gfx950 kernel library must be loaded on a GPU box"
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _isolate_miopen_find():
    """SwavPeer turns on cudnn.benchmark (MIOpen solver search, MODEL.MIOPEN_FIND); restore it after
    every test so later MIOpen reference computations use the same (immediate-mode) solvers."""
    import torch

    saved = torch.backends.cudnn.benchmark
    yield
    torch.backends.cudnn.benchmark = saved
