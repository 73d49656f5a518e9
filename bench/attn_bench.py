"""Attention kernel micro-benchmark at ALBERT-large shapes (head_dim 64): forward, backward, TFLOP/s.

    python bench/attn_bench.py --batch 64 --heads 16 --seq 512 [--pad 0.25]
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

O = torch.ops.dedloc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pad", type=float, default=0.0, help="fraction of each row that is right padding")
    args = ap.parse_args()
    B, H, S, D = args.batch, args.heads, args.seq, 64
    dev = torch.device("cuda")
    qkv = torch.randn(B * S, 3 * H * D, device=dev).bfloat16()
    n = int(round(S * (1 - args.pad)))
    mask = (torch.arange(S, device=dev)[None] < n).expand(B, S).long()
    mbias = torch.where(mask.bool(), 0.0, -1e30).float().contiguous()
    lens = mask.sum(1).int()
    kvinfo = torch.cat([lens, torch.ones(1, dtype=torch.int32, device=dev)]).contiguous()
    scale = 1 / math.sqrt(D)

    def fwd():
        return O.attn_fwd(qkv, mbias, H, S, scale, kvinfo)

    out, lse = fwd()
    dout = torch.randn_like(out)

    def bwd():
        return O.attn_bwd(qkv, mbias, out, dout, lse, H, S, scale, kvinfo)

    dbias = torch.zeros(3 * H * D, device=dev)

    def bwd_fused_bias():  # the model's call: QKV bias gradient inside the backward
        return O.attn_bwd(qkv, mbias, out, dout, lse, H, S, scale, kvinfo, dbias)

    def bwd_then_colsum():  # the previous form: backward, then a column-sum pass over dqkv
        g = O.attn_bwd(qkv, mbias, out, dout, lse, H, S, scale, kvinfo)
        O.bias_grad(g, dbias, True)
        return g

    res = {}
    for name, fn, flop_mult in (("fwd", fwd, 4), ("bwd", bwd, 10), ("bwd_fused_bias", bwd_fused_bias, 10),
                                ("bwd_then_colsum", bwd_then_colsum, 10)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.iters
        flops = flop_mult * B * H * S * S * D
        res[name] = {"us": round(dt * 1e6, 1), "tflops": round(flops / dt / 1e12, 1)}
    print(json.dumps({"B": B, "H": H, "S": S, "D": D, "pad": args.pad, **res}))


if __name__ == "__main__":
    main()
