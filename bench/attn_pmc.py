"""Minimal attention driver for rocprofv3 --pmc passes: 3 forward + 3 backward (fused bias) calls
at ALBERT-large B x 16 heads x 512 x 64, no padding."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

O = torch.ops.dedloc


def main():
    B, H, S, D = int(os.environ.get("B", 256)), 16, 512, 64
    dev = torch.device("cuda")
    qkv = torch.randn(B * S, 3 * H * D, device=dev).bfloat16()
    mbias = torch.zeros(B, S, device=dev)
    kvinfo = torch.cat([torch.full((B,), S, dtype=torch.int32, device=dev),
                        torch.ones(1, dtype=torch.int32, device=dev)]).contiguous()
    scale = 1 / math.sqrt(D)
    dbias = torch.zeros(3 * H * D, device=dev)
    for _ in range(3):
        out, lse = O.attn_fwd(qkv, mbias, H, S, scale, kvinfo)
    dout = torch.randn_like(out)
    for _ in range(3):
        O.attn_bwd(qkv, mbias, out, dout, lse, H, S, scale, kvinfo, dbias)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
