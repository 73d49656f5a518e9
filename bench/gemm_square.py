"""Main-loop comparison at a long reduction (epilogue amortised): gemm8 vs hipBLASLt, M=N=K=8192
and the ALBERT N=1024/3072 shapes with K=8192 (random data, interleaved, one process)."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
import json
import os
import time

import torch

import dedloc_amd.ops  # noqa: F401

O = torch.ops.dedloc


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    dev = torch.device("cuda")
    for M, N, K in [(8192, 8192, 8192), (16384, 3072, 8192), (16384, 1024, 16384)]:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        ts = {"gemm8": [], "lt": []}
        for _ in range(3):
            for v, pol in (("gemm8", "mfma"), ("lt", "lib")):
                os.environ["DEDLOC_GEMM"] = pol
                ts[v].append(timeit(lambda: O.gemm(a, w, None, None, False, True, 0)))
        row = {"M": M, "N": N, "K": K}
        for v, t in ts.items():
            row[v + "_tflops"] = round(2.0 * M * N * K / min(t) / 1e12, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
