"""Summarise bench/ab_native.py output: per-arm values of each row kind, and the B-vs-A delta.

    python scripts/ab_summary.py gpurun_out/x_gemm_ab.jsonl [--key g8_us --group gemm]
    python scripts/ab_summary.py gpurun_out/x_step_ab.jsonl --key samples_per_s

Arm A is the variant library (DEDLOC_NATIVE_LIB), arm B the in-tree build.
"""
import argparse
import collections
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--key", default=None, help="value field (default: g8_us, samples_per_s or value)")
    ap.add_argument("--group", default=None, help="field naming the row kind (e.g. gemm)")
    args = ap.parse_args()
    rows = [json.loads(ln) for ln in open(args.path) if ln.startswith("{")]
    if not rows:
        raise SystemExit("no JSON rows")
    key = args.key or next(k for k in ("g8_us", "samples_per_s", "value") if k in rows[0])
    group = args.group or ("gemm" if "gemm" in rows[0] else None)
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        d[r.get(group, "-") if group else "-"][r["arm"]].append(float(r[key]))
    lower_better = key.endswith("_us") or key.startswith("ms")
    for g, v in d.items():
        a, b = v.get("A", []), v.get("B", [])
        if not a or not b:
            continue
        ma, mb = sum(a) / len(a), sum(b) / len(b)
        delta = 100 * (mb - ma) / ma
        tag = "better" if (delta < 0) == lower_better else "worse"
        print(f"{g:24s} A {[round(x, 1) for x in a]}  B {[round(x, 1) for x in b]}  {delta:+.2f}% ({tag})")


if __name__ == "__main__":
    main()
