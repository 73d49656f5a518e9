"""ALBERT-large layer GEMMs: dedloc MFMA kernel vs hipBLASLt (same random bf16 data, one process,
interleaved rounds — cdna_hip_programming.md §5.4 rules 24/25)."""
import json
import os
import time

import torch

import dedloc_amd.ops  # noqa: F401

O = torch.ops.dedloc


def timeit(fn, iters=20):
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
    H, I = 1024, 4096
    res = []
    shapes = [("qkv_fwd", H, 3 * H), ("o_fwd", H, H), ("ffn1_fwd", H, I), ("ffn2_fwd", I, H)]
    for name, K, N in shapes:
        x = torch.randn(T, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        dy = torch.randn(T, N, device=dev).bfloat16()
        g = torch.zeros(N, K, device=dev)
        fl = 2.0 * T * N * K
        for kind, fn_ours, fn_lib in [
            ("fwd", lambda: O.gemm(x, w, None, None, False, True, 0), lambda: torch.mm(x, w.t())),
            ("dgrad", lambda: O.gemm(dy, w, None, None, False, False, 0), lambda: torch.mm(dy, w)),
            ("wgrad", lambda: O.gemm_acc_f32(dy, x, g, True, False),
             lambda: torch.ops.aten.addmm.dtype_out(g, dy.t(), x, torch.float32, out=g)),
        ]:
            ts = {"ours": [], "lib": []}
            for _ in range(3):
                ts["ours"].append(timeit(fn_ours))
                ts["lib"].append(timeit(fn_lib))
            t_o, t_l = min(ts["ours"]), min(ts["lib"])
            res.append({"gemm": f"{name}:{kind}", "M": T, "N": N, "K": K, "ours_us": round(t_o * 1e6, 1),
                        "lib_us": round(t_l * 1e6, 1), "ours_tflops": round(fl / t_o / 1e12, 1),
                        "lib_tflops": round(fl / t_l / 1e12, 1)})
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
