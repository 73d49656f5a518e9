"""Memory-bound kernels of the ALBERT layer at the B=256 token count (T=131072): achieved HBM rate,
v1 (DEDLOC_EW=1) vs v2 (default), interleaved in one process on random data."""
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
    T = int(os.environ.get("T", 131072))
    dev = torch.device("cuda")
    h = torch.randn(T, 4096, device=dev).bfloat16()
    dy = torch.randn(T, 4096, device=dev).bfloat16()
    dq = torch.randn(T, 3072, device=dev).bfloat16()
    db = torch.zeros(4096, device=dev)
    dbq = torch.zeros(3072, device=dev)
    x = torch.randn(T, 1024, device=dev).bfloat16()
    r = torch.randn(T, 1024, device=dev).bfloat16()
    g = torch.rand(1024, device=dev) + 0.5
    b = torch.randn(1024, device=dev)
    nb = h.numel() * 2
    _, _, mean, rstd = O.layernorm_fwd(x, r, g, b, 1e-12)
    dgam, dbet, dsum = torch.zeros(1024, device=dev), torch.zeros(1024, device=dev), torch.zeros(1024, device=dev)
    cases = [("gelu_fwd", lambda: O.gelu_fwd(h), 2 * nb),
             ("gelu_bwd_colsum", lambda: O.gelu_bwd(dy, h, db), 3 * nb),
             ("bias_grad_3072", lambda: O.bias_grad(dq, dbq, True), dq.numel() * 2),
             ("ln_fwd_res", lambda: O.layernorm_fwd(x, r, g, b, 1e-12), 4 * x.numel() * 2),
             ("ln_bwd", lambda: O.layernorm_bwd(x, r, g, mean, rstd, dgam, dbet, True, dsum), 3 * x.numel() * 2)]
    # numerics: v2 must equal v1 bit for bit on the bf16 outputs
    os.environ["DEDLOC_EW"] = "1"
    y1 = O.gelu_fwd(h)
    db.zero_()
    d1 = O.gelu_bwd(dy, h, db)
    s1 = db.clone()
    os.environ["DEDLOC_EW"] = "2"
    y2 = O.gelu_fwd(h)
    db.zero_()
    d2 = O.gelu_bwd(dy, h, db)
    print(json.dumps({"check": "v2_vs_v1", "gelu_fwd_equal": bool(torch.equal(y1, y2)),
                      "gelu_fwd_rel": float((y1.float() - y2.float()).norm() / y1.float().norm()),
                      "gelu_bwd_equal": bool(torch.equal(d1, d2)),
                      "dbias_rel": float((db - s1).norm() / s1.norm())}), flush=True)
    for name, fn, nbytes in cases:
        ts = {"v1": [], "v2": []}
        for _ in range(3):
            for v in ("v1", "v2"):
                os.environ["DEDLOC_EW"] = v[1]
                ts[v].append(timeit(fn))
        row = {"kernel": name, "T": T}
        for v, t in ts.items():
            row[v + "_us"] = round(min(t) * 1e6, 1)
            row[v + "_TBps"] = round(nbytes / min(t) / 1e12, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
