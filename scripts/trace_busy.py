"""GPU occupancy of a training step from a plain rocprofv3 ``--kernel-trace`` CSV (no counters, so
concurrent dispatches stay concurrent).

The window is the span of the last ``--iters`` occurrences of a once-per-iteration marker kernel
(``--marker``, a substring of its name).  Printed: window length, the union of kernel intervals
(time the GPU runs at least one kernel), the idle gaps longest first, the mean number of kernels in
flight while busy, and per-kernel time with the part of it during which that kernel ran alone.

usage: python scripts/trace_busy.py TRACE.csv --marker sinkhorn --iters 4 [--top 20]
"""
import argparse
import collections
import csv


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", required=True)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--top", type=int, default=20)
    args = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(args.path)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "?")))
    ks.sort()
    marks = [k[0] for k in ks if args.marker in k[2]]
    if len(marks) < args.iters + 1:
        raise SystemExit(f"marker {args.marker!r} seen {len(marks)} times; need iters + 1")
    t0, t1 = marks[-args.iters - 1], marks[-1]
    win = [k for k in ks if k[0] >= t0 and k[0] < t1]
    span = t1 - t0
    # sweep: events sorted by time; busy union, concurrency-weighted time, solo time per kernel
    ev = []
    for i, (s, e, _, _) in enumerate(win):
        ev.append((s, 1, i))
        ev.append((min(e, t1), -1, i))
    ev.sort()
    live = set()
    busy = 0
    weighted = 0
    solo = collections.Counter()
    gaps = []
    prev = t0
    for t, d, i in ev:
        dt = t - prev
        if dt > 0:
            if live:
                busy += dt
                weighted += dt * len(live)
                if len(live) == 1:
                    solo[win[next(iter(live))][2]] += dt
            else:
                gaps.append(dt)
        prev = t
        if d > 0:
            live.add(i)
        else:
            live.discard(i)
    if t1 > prev:
        gaps.append(t1 - prev)
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, n, _ in win:
        tot[n] += min(e, t1) - s
        cnt[n] += 1
    queues = collections.Counter(q for *_, q in win)
    it = args.iters
    print(f"window: {it} iterations, {span / 1e6 / it:.3f} ms each; GPU busy {100 * busy / span:.1f}% "
          f"(idle {(span - busy) / 1e6 / it:.3f} ms/iter in {len(gaps) / it:.0f} gaps); "
          f"mean kernels in flight while busy {weighted / max(busy, 1):.2f}; queues {dict(queues)}")
    gaps.sort(reverse=True)
    print("longest gaps (us):", [round(g / 1e3, 1) for g in gaps[:15]])
    print("gap histogram (us): " + ", ".join(
        f"{lo}-{hi}: {sum(1 for g in gaps if lo * 1e3 <= g < hi * 1e3) / it:.0f}/iter "
        f"({sum(g for g in gaps if lo * 1e3 <= g < hi * 1e3) / 1e3 / it:.0f} us)"
        for lo, hi in ((0, 5), (5, 20), (20, 100), (100, 10 ** 9))))
    print(f"{'ms/iter':>8} {'solo ms':>8} {'calls':>6}  kernel")
    for n, v in tot.most_common(args.top):
        print(f"{v / 1e6 / it:8.3f} {solo[n] / 1e6 / it:8.3f} {cnt[n] / it:6.0f}  {n}")


if __name__ == "__main__":
    main()
