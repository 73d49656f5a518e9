"""Per-kernel summary of a rocprofv3 ``--kernel-trace`` database (``*_results.db``).

Takes the dispatches of the last ``--window_ms`` milliseconds of GPU time (the steady-state tail of a
benchmark loop; 0 = everything) and prints / writes one CSV row per kernel name:
calls, total ms, share of the window's kernel time, mean us, grid, VGPR / AGPR / LDS.

usage: python scripts/rocpd_summary.py gpurun_out/prof/run_results.db [--window_ms 600] [--csv out.csv]
"""
import argparse
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return re.sub(r"\(.*$", "", name)[:110]


def timeline(spans, t0, t1):
    """Union of the kernel intervals (GPU busy with >= 1 kernel), time with >= 2 kernels in flight,
    and the kernel time and busy union of each stream."""
    ev = sorted([(s, 1) for s, _, _ in spans] + [(min(e, t1), -1) for _, e, _ in spans])
    depth, last, busy, overlap = 0, t0, 0.0, 0.0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            overlap += t - last
        depth += d
        last = t
    span = t1 - t0
    print(f"timeline: busy (>=1 kernel) {busy / 1e6:.2f} ms = {100 * busy / span:.1f}% of {span / 1e6:.2f} ms; "
          f">=2 kernels {overlap / 1e6:.2f} ms; idle {(span - busy) / 1e6:.2f} ms")
    per = defaultdict(list)
    for s, e, st in spans:
        per[st].append((s, e))
    for st, iv in sorted(per.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        tot = sum(e - s for s, e in iv)
        print(f"  stream {st}: {len(iv)} kernels, {tot / 1e6:.2f} ms kernel time")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window_ms", type=float, default=0.0)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--from_ms", type=float, default=None, help="window start, ms after the first dispatch")
    ap.add_argument("--to_ms", type=float, default=None, help="window end, ms after the first dispatch")
    ap.add_argument("--timeline", action="store_true",
                    help="also print the window's union busy time, overlap and per-stream kernel time")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, accum_vgpr_count, "
                     "lds_size, stream_id from kernels order by start").fetchall()
    if not rows:
        print("no kernels")
        return 1
    t_first = min(r[1] for r in rows)
    t_end = max(r[2] for r in rows) if a.to_ms is None else t_first + a.to_ms * 1e6
    t0 = t_end - a.window_ms * 1e6 if a.window_ms > 0 else t_first
    if a.from_ms is not None:
        t0 = t_first + a.from_ms * 1e6
    rows = [r for r in rows if r[1] < t_end]
    agg = defaultdict(lambda: [0, 0.0, None])
    busy = 0.0
    for name, s, e, gx, gy, gz, wx, vg, ag, lds, _ in rows:
        if s < t0:
            continue
        k = short(name)
        d = (e - s) / 1e3  # us
        agg[k][0] += 1
        agg[k][1] += d
        agg[k][2] = (gx * gy * gz // max(wx, 1), wx, vg, ag, lds)
        busy += d
    span_ms = (t_end - t0) / 1e6
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"window {span_ms:.1f} ms, kernel time {busy / 1e3:.1f} ms ({100 * busy / 1e3 / span_ms:.1f}% busy), "
          f"{sum(v[0] for v in agg.values())} dispatches")
    print(f"{'ms':>9} {'%':>6} {'calls':>6} {'us/call':>9}  {'wgs':>7} {'wg':>4} {'vgpr':>4} {'agpr':>4} {'lds':>6}  kernel")
    for k, (n, tot, meta) in out[:a.top]:
        wgs, wx, vg, ag, lds = meta
        print(f"{tot / 1e3:9.2f} {100 * tot / busy:6.2f} {n:6d} {tot / n:9.1f}  {wgs:7d} {wx:4d} {vg:4d} {ag:4d} {lds:6d}  {k}")
    if a.timeline:
        timeline([(r[1], r[2], r[10]) for r in rows if r[1] >= t0], t0, t_end)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "total_ms", "pct", "us_per_call", "workgroups", "wg_size", "vgpr", "agpr",
                        "lds"])
            for k, (n, tot, meta) in out:
                w.writerow([k, n, f"{tot / 1e3:.3f}", f"{100 * tot / busy:.2f}", f"{tot / n:.1f}", *meta])
    return 0


if __name__ == "__main__":
    sys.exit(main())
