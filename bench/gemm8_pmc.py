"""Driver for rocprofv3 --pmc passes over gemm8: one NT (forward-layout) GEMM and one TN
(weight-gradient layout, fp32 slabs) GEMM at the ALBERT FFN shape, T = 32768."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

O = torch.ops.dedloc


def main():
    T, N, K = 32768, 4096, 1024
    x = (torch.rand(T, K, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()
    dy = (torch.rand(T, N, device="cuda") * 2 - 1).bfloat16()
    g = torch.zeros(N, K, device="cuda")
    for _ in range(2):
        O.gemm(x, w, None, None, False, True, 0)
        O.gemm_acc_f32(dy, x, g, True, False)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
