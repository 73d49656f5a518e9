"""Same-box A/B of two builds of the kernel library: runs a command alternately with the in-tree
_C.so (arm B, the current tree) and with DEDLOC_NATIVE_LIB=<variant> (arm A, built by
``python -m dedloc_amd._build variant NAME REV kernel.hip ...``), ``--rounds`` times, and prints each
run's JSON line tagged with its arm.  Box-to-box spread on this pool is a few percent, so kernel
changes are judged on interleaved runs on one box (cdna_hip_programming.md §5.4 rule 24).

    python bench/ab_native.py --lib ab/_C_base.so --rounds 2 -- python bench.py --steps 3 --warmup 1
"""
import argparse
import json
import os
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=300)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    cmd = args.cmd[1:] if args.cmd and args.cmd[0] == "--" else args.cmd
    for r in range(args.rounds):
        for arm in ("A", "B"):
            env = dict(os.environ)
            if arm == "A":
                env["DEDLOC_NATIVE_LIB"] = os.path.abspath(args.lib)
            else:
                env.pop("DEDLOC_NATIVE_LIB", None)
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.timeout)
            if p.returncode != 0:
                print(f"arm {arm} round {r} failed ({p.returncode}):\n{p.stderr[-3000:]}", file=sys.stderr)
                sys.exit(p.returncode if p.returncode > 0 else 1)
            for ln in p.stdout.splitlines():
                if ln.startswith("{"):
                    d = json.loads(ln)
                    d["arm"], d["round"] = arm, r
                    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
