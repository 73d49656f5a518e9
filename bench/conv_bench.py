"""Per-shape timing of the implicit-GEMM NHWC conv kernels (csrc/kernels/conv.hip) vs MIOpen.

Collects every conv of the SwAV ResNet-50 trunk for one local iteration (b=64: 2x224 crops batched
as N=128, 6x96 crops as N=384), times forward / dgrad / wgrad of each distinct shape for both
implementations (same bf16 channels-last tensors; MIOpen through torch's convolution ops with
cudnn.benchmark autotuning), and prints one JSON line per shape plus a weighted total per iteration.
"""
import argparse
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

CL = torch.channels_last


def collect_shapes(batch224, batch96):
    """Every conv of the SwAV ResNet-50 trunk (torchvision v1.5 layout: stride on the 3x3) as
    (batch, Cin, H_in, Cout, k, stride, pad) with its count, for both crop resolutions."""
    shapes = Counter()
    for n, s in ((batch224, 224), (batch96, 96)):
        shapes[(n, 3, s, 64, 7, 2, 3)] += 1
        h = ((s + 6 - 7) // 2 + 1 + 2 - 3) // 2 + 1  # stem, then the 3x3/2 max-pool
        cin = 64
        for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            for bi in range(blocks):
                st = stride if bi == 0 else 1
                h2 = (h + 2 - 3) // st + 1
                shapes[(n, cin, h, planes, 1, 1, 0)] += 1
                shapes[(n, planes, h, planes, 3, st, 1)] += 1
                shapes[(n, planes, h2, planes * 4, 1, 1, 0)] += 1
                if bi == 0:
                    shapes[(n, cin, h, planes * 4, 1, st, 0)] += 1
                cin, h = planes * 4, h2
    return shapes


def timeit(fn, iters):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no_miopen", action="store_true", help="time the hand-written kernels only")
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    shapes = collect_shapes(2 * args.batch, 6 * args.batch)
    tot = Counter()
    for (N, Cin, H, Cout, k, stride, pad), count in sorted(shapes.items()):
        x = torch.randn(N, Cin, H, H, device=dev).bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(Cout, Cin, k, k, device=dev) * 0.05).bfloat16().contiguous(memory_format=CL)
        P = (H + 2 * pad - k) // stride + 1
        dy = torch.randn(N, Cout, P, P, device=dev).bfloat16().contiguous(memory_format=CL)
        dw32 = torch.zeros(Cout, Cin, k, k, device=dev).contiguous(memory_format=CL)
        ops = torch.ops.dedloc
        flop = 2.0 * N * P * P * Cout * Cin * k * k
        res = {"shape": [N, Cin, H, Cout, k, stride, pad], "count": count, "gflop": flop / 1e9}
        res["ours_fwd_us"] = timeit(lambda: ops.conv2d_fwd(x, w, stride, pad), args.iters)
        if not args.no_miopen:
            res["miopen_fwd_us"] = timeit(lambda: torch.nn.functional.conv2d(x, w, stride=stride, padding=pad), args.iters)
        if Cin % 64 == 0:
            res["ours_dgrad_us"] = timeit(lambda: ops.conv2d_dgrad(dy, w, stride, pad, H, H), args.iters)
            if not args.no_miopen:
                res["miopen_dgrad_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [stride] * 2, [pad] * 2, [1, 1], False, [0, 0], 1, [True, False, False]), args.iters)
        res["ours_wgrad_us"] = timeit(lambda: ops.conv2d_wgrad(dy, x, dw32, stride, pad), args.iters)
        if not args.no_miopen:
            res["miopen_wgrad_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [stride] * 2, [pad] * 2, [1, 1], False, [0, 0], 1, [False, True, False]), args.iters)
        for k_, v in list(res.items()):
            if k_.endswith("_us"):
                tot[k_] += v * count
                res[k_.replace("_us", "_tflops")] = round(flop / (v * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)
    print(json.dumps({"total_per_iteration_ms": {k: round(v / 1e3, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
