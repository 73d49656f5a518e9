"""Weight-gradient GEMM study for ALBERT-large (dW[N,K] += dY[T,N]^T X[T,K], fp32 accumulate).

The shared ALBERT layer's wgrads have few output tiles (1024x4096 = 64 tiles of 256^2) and a very
long token reduction, so they under-fill 256 CUs.  Compares: the current dispatch
(O.gemm_acc_f32), hipBLASLt via ATen (fp32 out, beta=1), hipBLASLt bf16-out + fp32 add, the dedloc
split-K MFMA kernel at several split counts (DEDLOC_GEMM=mfma), and a K-concatenated multi-layer
reduction (what deferring the 24 shared-layer wgrads into one GEMM would cost per layer).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

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
    T = int(os.environ.get("T", 32768))
    dev = torch.device("cuda")
    for name, N, K in [("ffn1(w1)", 4096, 1024), ("ffn2(w2)", 1024, 4096), ("qkv", 3072, 1024), ("o", 1024, 1024)]:
        x = torch.randn(T, K, device=dev).bfloat16()
        dy = torch.randn(T, N, device=dev).bfloat16()
        g = torch.zeros(N, K, device=dev)
        fl = 2.0 * T * N * K
        out = {"gemm": name, "N": N, "K": K, "T": T}

        def rec(key, fn, flops=fl):
            t = min(timeit(fn) for _ in range(2))
            out[key] = f"{t * 1e6:.0f}us/{flops / t / 1e12:.0f}TF"

        os.environ.pop("DEDLOC_GEMM", None)
        rec("current", lambda: O.gemm_acc_f32(dy, x, g, True, False))
        for sp in (1, 2, 4, 8, 16, 32):  # direct hipBLASLt token-split into fp32 slabs, forced split count
            os.environ["DEDLOC_WGRAD_SPLITS"] = str(sp)
            rec(f"lt_split{sp}", lambda: O.gemm_acc_f32(dy, x, g, True, False))
        os.environ.pop("DEDLOC_WGRAD_SPLITS", None)
        if os.environ.get("WGRAD_QUICK"):
            print(json.dumps(out), flush=True)
            continue
        rec("aten_f32", lambda: torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32, out=g))
        rec("aten_bf16+add", lambda: g.add_(torch.mm(dy.t(), x)))
        os.environ["DEDLOC_GEMM"] = "mfma"
        rec("mfma_auto", lambda: O.gemm_acc_f32(dy, x, g, True, False))
        os.environ.pop("DEDLOC_GEMM", None)
        for sp in (2, 4, 8):  # batched split-K through the library: [sp, N, K] partials + a sum
            dyv = dy.view(sp, T // sp, N).transpose(1, 2)
            xv = x.view(sp, T // sp, K)
            rec(f"bmm_split{sp}", lambda: g.add_(torch.bmm(dyv, xv).sum(0)))
            rec(f"bmm_split{sp}_only", lambda: torch.bmm(dyv, xv))
        for L in (2, 4):  # K-concatenated reduction over L layers (per-layer cost reported)
            xx = torch.randn(L * T, K, device=dev).bfloat16()
            dd = torch.randn(L * T, N, device=dev).bfloat16()
            t = min(timeit(lambda: torch.ops.aten.addmm.dtype_out(g, dd.t(), xx, torch.float32, out=g))
                    for _ in range(2))
            out[f"concat{L}_per_layer"] = f"{t / L * 1e6:.0f}us/{fl * L / t / 1e12:.0f}TF"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
