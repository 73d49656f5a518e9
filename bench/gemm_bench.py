"""ALBERT-large layer GEMMs on the hand-written MFMA kernels (gemm8.hip: one 256 x 256 tile per
workgroup, LDS-DMA 8-phase pipeline), per shape at T tokens, random bf16 data
(cdna_hip_programming.md §5.4 rules 24/25).  VARIANTS maps names to environment settings for A/B
builds of future variants; the shipped dispatch is "g8".  Fused epilogues are timed as the op the
model calls (gemm_gelu: bias + GELU; gemm_dgelu: GELU' + bias-gradient column sums).

usage: T=262144 [DGRAD_T=1] [KINDS=fwd,dgrad_wT] python bench/gemm_bench.py [--check]
"""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
import json
import os
import sys
import time

import torch

import dedloc_amd.ops  # noqa: F401

O = torch.ops.dedloc
VARIANTS = {"g8": {}}  # the shipped dispatch (the A/B knobs of rounds 2-3 were removed with their losing forms)


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def set_policy(pol):
    os.environ.update(pol)


def with_policy(pol, fn):
    def run():
        set_policy(pol)
        return fn()
    return run


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    T = int(os.environ.get("T", 32768))
    check = "--check" in sys.argv
    variants = os.environ.get("VARIANTS", "g8").split(",")
    dev = torch.device("cuda")
    H, I = 1024, 4096
    torch.manual_seed(0)
    res = []
    shapes = [("qkv", H, 3 * H), ("o", H, H), ("ffn1", H, I), ("ffn2", I, H)]
    for name, K, N in shapes:
        x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        b = torch.randn(N, device=dev)
        dy = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
        g = torch.zeros(N, K, device=dev)
        db = torch.zeros(N, device=dev)
        if name == "ffn2":  # gemm_dgelu's bias gradient spans its K (= 4096) output columns
            db = torch.zeros(K, device=dev)
        fl = 2.0 * T * N * K
        kinds = [("fwd", lambda: O.gemm(x, w, b, None, False, True, 0)),
                 ("dgrad", lambda: O.gemm(dy, w, None, None, False, False, 0)),
                 ("wgrad", lambda: O.gemm_acc_f32(dy, x, g, True, False))]
        wt = w.t().contiguous()
        if os.environ.get("DGRAD_T"):  # the other weight layout: W^T [in, out] copies (B K-outer
            # in the forward, K-inner in the data gradient)
            kinds.insert(1, ("fwd_wT", lambda: O.gemm(x, wt, b, None, False, False, 0)))
            kinds.insert(3, ("dgrad_wT", lambda: O.gemm(dy, wt, None, None, False, True, 0)))
        if name == "ffn1":
            kinds.append(("fwd_gelu", lambda: O.gemm_gelu(x, w, b)))
            kinds.append(("fwd_gelu_d", lambda: O.gemm_gelu_d(x, w, b)))
            if os.environ.get("DGRAD_T"):
                kinds.append(("fwd_gelu_wT", lambda: O.gemm_gelu(x, wt, b, True)))
        if name == "ffn2":
            f = (torch.randn(T, K, device=dev)).bfloat16()
            kinds.append(("dgrad_dgelu", lambda: O.gemm_dgelu(dy, w, f, db)))
            kinds.append(("dgrad_dmul", lambda: O.gemm_dmul(dy, w, f, db)))
            if os.environ.get("DGRAD_T"):
                w2t = w.t().contiguous()
                kinds.append(("dgrad_dgelu_wT", lambda: O.gemm_dgelu(dy, w2t, f, db, True)))
        only = os.environ.get("KINDS")  # e.g. KINDS=fwd,dgrad_wT: time only these
        for kind, fn in kinds:
            if only and kind not in only.split(","):
                continue
            if check:
                outs = {}
                for v in variants:
                    set_policy(VARIANTS[v])
                    g.zero_()
                    db.zero_()
                    o = fn()
                    o = g.clone() if kind == "wgrad" else (o[1] if isinstance(o, (tuple, list)) else o).clone()
                    outs[v] = (o, db.clone())
                base = outs[variants[-1]]
                for v in variants[:-1]:
                    print(json.dumps({"check": f"{name}:{kind}", "variant": v, "rel_vs_" + variants[-1]: rel(outs[v][0], base[0]),
                                      "dbias_rel": rel(outs[v][1], base[1]) if kind == "dgrad_dgelu" else None}),
                          flush=True)
            ts = {v: [] for v in variants}
            for _ in range(3):
                for v in variants:
                    ts[v].append(timeit(with_policy(VARIANTS[v], fn)))
            row = {"gemm": f"{name}:{kind}", "M": T, "N": N, "K": K}
            for v in variants:
                t = min(ts[v])
                row[f"{v}_us"] = round(t * 1e6, 1)
                row[f"{v}_tflops"] = round(fl / t / 1e12, 1)
            res.append(row)
            print(json.dumps(row), flush=True)
    set_policy({})


if __name__ == "__main__":
    main()
