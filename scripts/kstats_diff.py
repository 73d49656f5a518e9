"""Per-kernel difference of two rocprofv3 ``--kernel-trace --stats`` runs of the same program.

    python scripts/kstats_diff.py gpurun_out/kst_base gpurun_out/kst_new [--top 25]

Reads ``*_kernel_stats.csv`` under each directory and prints, per kernel name, calls and total /
mean time in both runs and the relative change of the total, largest absolute change first.
"""
import argparse
import csv
import glob
import os


def load(d):
    path = glob.glob(os.path.join(d, "**", "*_kernel_stats.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no *_kernel_stats.csv under {d}")
    out = {}
    for r in csv.DictReader(open(path[0])):
        name = r["Name"].replace("(anonymous namespace)::", "")
        name = (name[5:] if name.startswith("void ") else name).split("(")[0][:72]
        calls, tot = int(r["Calls"]), float(r["TotalDurationNs"])
        c0, t0 = out.get(name, (0, 0.0))
        out[name] = (c0 + calls, t0 + tot)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    A, B = load(args.a), load(args.b)
    ta, tb = sum(v[1] for v in A.values()), sum(v[1] for v in B.values())
    print(f"total kernel time: {ta / 1e6:.3f} -> {tb / 1e6:.3f} ms ({100 * (tb - ta) / ta:+.2f}%)")
    names = sorted(set(A) | set(B), key=lambda n: -abs(B.get(n, (0, 0.0))[1] - A.get(n, (0, 0.0))[1]))
    print(f"{'A ms':>8} {'B ms':>8} {'A us/call':>10} {'B us/call':>10} {'calls':>6} {'change':>8}  kernel")
    for n in names[: args.top]:
        (ca, xa), (cb, xb) = A.get(n, (0, 0.0)), B.get(n, (0, 0.0))
        ch = f"{100 * (xb - xa) / xa:+.1f}%" if xa else "new"
        print(f"{xa / 1e6:8.3f} {xb / 1e6:8.3f} {xa / max(ca, 1) / 1e3:10.1f} {xb / max(cb, 1) / 1e3:10.1f} "
              f"{cb:6d} {ch:>8}  {n}")


if __name__ == "__main__":
    main()
