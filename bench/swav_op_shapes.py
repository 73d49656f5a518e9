"""Shapes and isolated times of the SwAV iteration's fused data-gradient calls (conv2d_dgrad_bn: the
BN-backward preparation in a conv's data-gradient epilogue), b = 64, 2x224 + 6x96 crops, the
concurrent trunk passes.  Each call is timed on its own stream with events after a device sync, so
the times are isolated-kernel times, not the overlapped iteration's.

    python bench/swav_op_shapes.py
"""
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dedloc_amd.models.resnet_swav import SwAVModel
    from dedloc_amd.utils.flat import FlatParams

    dev = torch.device("cuda", 0)
    CL = torch.channels_last
    torch.manual_seed(0)
    bs = 64
    model = SwAVModel(num_prototypes=3000).to(dev).train()
    flat = FlatParams(model.named_parameters(), device=dev, with_bf16=True, autograd=True, channels_last=True)
    model.bind_flat(flat)
    model.concurrent_passes = True
    g = torch.Generator(device="cpu").manual_seed(1)
    crops = [torch.randn(bs, 3, s, s, generator=g).to(dev).bfloat16().contiguous(memory_format=CL)
             for s, n in ((224, 2), (96, 6)) for _ in range(n)]

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            emb, scores = model(crops)
        (emb.float().sum() + scores.float().sum()).backward()
        model.after_backward()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    orig = torch.ops.dedloc.conv2d_dgrad_bn
    rec = collections.defaultdict(list)

    def timed(*a, **k):
        dy, w = a[0], a[1]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig(*a, **k)
        e1.record()
        torch.cuda.synchronize()
        key = (tuple(dy.shape), tuple(w.shape), int(a[2]), a[6] is not None, a[8] is not None, bool(out[1]))
        rec[key].append(e0.elapsed_time(e1) * 1e3)
        return out

    torch.ops.dedloc.conv2d_dgrad_bn = timed
    try:
        step()
        torch.cuda.synchronize()
    finally:
        torch.ops.dedloc.conv2d_dgrad_bn = orig
    total = sum(sum(v) for v in rec.values())
    for (dys, ws, st, res, y, fused), v in sorted(rec.items(), key=lambda kv: -sum(kv[1])):
        N, K, P, Q = dys
        C = ws[1]
        M = N * P * Q
        print(json.dumps({"dy": dys, "w": ws, "stride": st, "residual": res, "y_mask": y, "fused": fused,
                          "calls": len(v), "us_mean": round(sum(v) / len(v), 1), "share": round(sum(v) / total, 3),
                          "M": M, "N_out": C, "K": K, "bytes_min_MB": round(M * (K + 2 * C + (C if res else 0)
                                                                                 + (C if y else 0)) * 2 / 1e6, 1)}),
              flush=True)
    print(json.dumps({"total_us": round(total, 1)}))


if __name__ == "__main__":
    main()
