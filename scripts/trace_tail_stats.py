"""Per-kernel stats of the LAST `--window` seconds of a rocprofv3 kernel trace (steady state, after
warm-up / library autotuning), written as a small CSV; the multi-MB trace itself can then be dropped."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("out")
ap.add_argument("--window", type=float, default=2.0, help="seconds of trace to keep (from the end)")
ap.add_argument("--skip_tail", type=float, default=0.0, help="seconds to drop at the very end")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
end = max(int(r["End_Timestamp"]) for r in rows) - int(a.skip_tail * 1e9)
start = end - int(a.window * 1e9)
agg = collections.defaultdict(lambda: [0, 0])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= start and e <= end:
        agg[r["Kernel_Name"]][0] += 1
        agg[r["Kernel_Name"]][1] += e - s
tot = sum(v[1] for v in agg.values())
with open(a.out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([k, n, d, d / n, 100.0 * d / tot])
print(f"window {a.window}s: {sum(v[0] for v in agg.values())} kernels, busy {tot / 1e6:.1f} ms")
