import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "multiproc: spawns several processes (gloo on CPU)")


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
