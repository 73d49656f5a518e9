"""hipBLASLt plan selection (csrc/host/lt_gemm.cpp): the exhaustive autotune over every supported
solution for large bf16-output GEMMs, the tuning database it writes (DEDLOC_LT_DB_OUT) and reads
back (DEDLOC_LT_DB), and the fallback when a database entry is unusable — each in a child process,
because the database is read once per process."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys, torch
    import dedloc_amd.ops  # noqa: F401
    O = torch.ops.dedloc
    torch.manual_seed(0)
    M, N, K = 8192, 4096, 4096          # 2.7e11 FLOP: above the exhaustive-search threshold
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    b = torch.randn(N, device="cuda")
    y = O.gemm(x, w, b, None, False, True, 0)
    ref = x.float() @ w.float().t() + b
    err = ((y.float() - ref).norm() / ref.norm()).item()
    torch.save(y.cpu(), sys.argv[1])
    print("REL", err, flush=True)
""")


def _run(env_extra, out):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, out], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    rel = float([ln for ln in r.stdout.splitlines() if ln.startswith("REL")][0].split()[1])
    return rel, r.stderr


@pytest.mark.timeout(600)
def test_exhaustive_autotune_database_roundtrip(cuda, tmp_path):
    import torch

    db = tmp_path / "lt_db.txt"
    rel1, err1 = _run({"DEDLOC_LT_DB": str(tmp_path / "none.txt"), "DEDLOC_LT_DB_OUT": str(db),
                       "DEDLOC_LT_EXHAUSTIVE": "1"}, str(tmp_path / "y1.pt"))
    assert rel1 < 1e-2
    assert "[lt] exhaustive tune" in err1
    lines = db.read_text().split("\n")
    entries = [ln.split() for ln in lines if ln.strip()]
    assert entries and all(len(e) == 2 and int(e[1]) >= 0 for e in entries)
    # a second process takes the recorded solution from the database (no tuning) and computes
    # exactly the same result
    rel2, err2 = _run({"DEDLOC_LT_DB": str(db), "DEDLOC_LT_DEBUG": "1"}, str(tmp_path / "y2.pt"))
    assert "tuning database solution" in err2 and "[lt] exhaustive tune" not in err2
    y1 = torch.load(tmp_path / "y1.pt", weights_only=True)
    y2 = torch.load(tmp_path / "y2.pt", weights_only=True)
    assert torch.equal(y1, y2) and rel2 == rel1
    # an unusable entry (solution index out of range) falls back to tuning
    bad = tmp_path / "bad.txt"
    bad.write_text("".join(f"{e[0]} 999999999\n" for e in entries))
    rel3, err3 = _run({"DEDLOC_LT_DB": str(bad), "DEDLOC_LT_DEBUG": "1"}, str(tmp_path / "y3.pt"))
    assert rel3 < 1e-2 and "not usable" in err3
