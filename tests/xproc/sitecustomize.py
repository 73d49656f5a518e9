"""TEST ONLY: with ``DEDLOC_XPROC_RCCL_DIR`` set and this directory on ``PYTHONPATH``, every Python
process of a test run (bench.py peers, churn peers) gets the cross-process RCCL stand-in of
``xproc_rccl.py`` installed before its own code runs.  Production code has no switch for it."""
import os

if os.environ.get("DEDLOC_XPROC_RCCL_DIR"):
    import xproc_rccl

    xproc_rccl.install(os.environ["DEDLOC_XPROC_RCCL_DIR"])
