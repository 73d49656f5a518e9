"""Weight-gradient GEMM timing, dW = dY^T X ([N_out, K_in]) vs its transpose X^T dY ([K_in, N_out]),
both through gemm_acc_f32 (hipBLASLt token-split slabs), ALBERT-large shapes, T tokens."""
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
    T = int(os.environ.get("T", 131072))
    for name, nout, kin in (("qkv", 3072, 1024), ("o", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)):
        dy = (torch.rand(T, nout, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(T, kin, device="cuda") * 2 - 1).bfloat16()
        g = torch.zeros(nout, kin, device="cuda")
        gt = torch.zeros(kin, nout, device="cuda")
        a = [timeit(lambda: O.gemm_acc_f32(dy, x, g, True, False)) for _ in range(3)]
        b = [timeit(lambda: O.gemm_acc_f32(x, dy, gt, True, False)) for _ in range(3)]
        fl = 2.0 * T * nout * kin
        print(json.dumps({"wgrad": name, "dYtX_us": round(min(a) * 1e6, 1), "XtdY_us": round(min(b) * 1e6, 1),
                          "dYtX_tflops": round(fl / min(a) / 1e12, 1), "XtdY_tflops": round(fl / min(b) / 1e12, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
