"""LayerNorm forward / backward at the ALBERT-large B=512 shape ([262144, 1024] bf16 rows): µs per call
and the HBM rate of the bytes each call must move (reads + writes, fp32 row stats included).

    python bench/ln_bench.py [--rows 262144] [--D 1024] [--iters 50]

Prints one JSON line; A/B two kernel builds on one box with bench/ab_native.py."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")  # evict the 256 MB MALL between calls
    for a, b in evs:
        flush.zero_()
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--D", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import dedloc_amd.ops  # noqa: F401

    ops = torch.ops.dedloc
    R, D = args.rows, args.D
    x = torch.randn(R, D, device="cuda").bfloat16()
    res = torch.randn(R, D, device="cuda").bfloat16()
    g = torch.rand(D, device="cuda") + 0.5
    b = torch.randn(D, device="cuda")
    dy = torch.randn(R, D, device="cuda").bfloat16()
    dg, db, dsum = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    y, s, mean, rstd = ops.layernorm_fwd(x, res, g, b, 1e-12)
    e = R * D * 2
    out = {"rows": R, "D": D}
    t = timed(lambda: ops.layernorm_fwd(x, None, g, b, 1e-12), args.iters)
    out["fwd_us"], out["fwd_TBps"] = round(t, 1), round((2 * e + 8 * R) / t / 1e6, 3)
    t = timed(lambda: ops.layernorm_fwd(x, res, g, b, 1e-12), args.iters)
    out["fwd_res_us"], out["fwd_res_TBps"] = round(t, 1), round((4 * e + 8 * R) / t / 1e6, 3)
    t = timed(lambda: ops.layernorm_bwd(dy, s, g, mean, rstd, dg, db, True, dsum), args.iters)
    out["bwd_us"], out["bwd_TBps"] = round(t, 1), round((3 * e + 8 * R) / t / 1e6, 3)
    # the streaming ceilings on this box for the same byte counts: a device copy (1 read + 1 write,
    # the forward's traffic) and a 2-read + 1-write add (the backward's)
    t = timed(lambda: y.copy_(x), args.iters)
    out["copy_us"], out["copy_TBps"] = round(t, 1), round(2 * e / t / 1e6, 3)
    t = timed(lambda: torch.add(x, res, out=y), args.iters)
    out["add_us"], out["add_TBps"] = round(t, 1), round(3 * e / t / 1e6, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
