"""One ALBERT-large layer GEMM, launched repeatedly: the unit for `rocprofv3 --pmc` passes and
per-kernel traces (bench/gemm_bench.py times the variants against each other).

usage: python bench/gemm_one.py --gemm ffn1 --kind wgrad [--T 262144] [--iters 20]
kinds: fwd, fwd_gelu (ffn1), dgrad, dgrad_dgelu (ffn2), wgrad
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

O = torch.ops.dedloc
SHAPES = {"qkv": (1024, 3072), "o": (1024, 1024), "ffn1": (1024, 4096), "ffn2": (4096, 1024),
          "emb": (128, 1024), "dec": (128, 30000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", default="ffn1", choices=sorted(SHAPES))
    ap.add_argument("--kind", default="wgrad")
    ap.add_argument("--T", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    K, N = SHAPES[a.gemm]
    T = a.T
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device=dev)
    dy = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
    g = torch.zeros(N, K, device=dev)
    db = torch.zeros(N, device=dev)
    if a.kind == "fwd":
        fn = lambda: O.gemm(x, w, b, None, False, True, 0)  # noqa: E731
    elif a.kind == "fwd_gelu":
        fn = lambda: O.gemm_gelu(x, w, b)  # noqa: E731
    elif a.kind == "dgrad":
        fn = lambda: O.gemm(dy, w, None, None, False, False, 0)  # noqa: E731
    elif a.kind == "dgrad_dgelu":
        f = torch.randn(T, K, device=dev).bfloat16()
        fn = lambda: O.gemm_dgelu(dy, w, f, db)  # noqa: E731
    elif a.kind == "wgrad":
        fn = lambda: O.gemm_acc_f32(dy, x, g, True, False)  # noqa: E731
    else:
        raise SystemExit(f"unknown kind {a.kind}")
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(json.dumps({"gemm": a.gemm, "kind": a.kind, "T": T, "us": round(dt * 1e6, 1),
                      "tflops": round(2.0 * T * N * K / dt / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
