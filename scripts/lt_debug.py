"""Diagnose the direct hipBLASLt GEMM path against fp32 torch references (GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DEDLOC_LT_DEBUG"] = "1"
import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

O = torch.ops.dedloc
dev = torch.device("cuda")


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


torch.manual_seed(0)
for (M, K, N) in [(256, 256, 768), (1024, 1024, 4096), (4096, 1024, 1024)]:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev).bfloat16()
    ref = x.float() @ w.float().t() + b
    print(M, K, N, "gemm+bias", rel(O.gemm(x, w, b, None, False, True, 0), ref))
    w2 = torch.randn(K, N, device=dev).bfloat16()
    ref2 = r.float() + x.float() @ w2.float()
    print(M, K, N, "gemm+residual", rel(O.gemm(x, w2, None, r, False, False, 0), ref2))
    dy = torch.randn(M, N, device=dev).bfloat16()
    c = torch.randn(N, K, device=dev)
    c0 = c.clone()
    O.gemm_acc_f32(dy, x, c, True, False)
    print(M, K, N, "acc_f32 (dy^T x)", rel(c, c0 + dy.float().t() @ x.float()))
    H, G = O.gemm_gelu(x, w, b)
    print(M, K, N, "gemm_gelu H", rel(H, ref), "G", rel(G, torch.nn.functional.gelu(ref, approximate="tanh")))
    db = torch.zeros(K, device=dev)
    Fh = (torch.randn(M, K, device=dev)).bfloat16()
    dh = O.gemm_dgelu(dy, w2.t().contiguous(), Fh, db) if False else None
    wT = torch.randn(N, K, device=dev).bfloat16()  # dgelu: dy[M,N] . W[N,K] -> [M,K]
    db = torch.zeros(K, device=dev)
    dh = O.gemm_dgelu(dy, wT, Fh, db)
    fr = Fh.float().requires_grad_(True)
    g = torch.nn.functional.gelu(fr, approximate="tanh")
    (gr,) = torch.autograd.grad(g, fr, dy.float() @ wT.float())
    print(M, K, N, "gemm_dgelu dh", rel(dh, gr), "db", rel(db, gr.sum(0)))

# whole tiny ALBERT: per-parameter grads with and without the direct hipBLASLt path
from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining  # noqa: E402

cfg = AlbertConfig.tiny(hidden_size=256, num_attention_heads=4, intermediate_size=1024, embedding_size=128)
grads = {}
for lt in ("1", "0"):
    os.environ["DEDLOC_LT"] = lt
    torch.manual_seed(0)
    m = AlbertForPreTraining(cfg)
    m.materialize(dev)
    m.eval()
    torch.manual_seed(1)
    B, S = 2, 128
    ids = torch.randint(5, cfg.vocab_size, (B, S))
    am = torch.ones(B, S, dtype=torch.long)
    am[1, 100:] = 0
    labels = torch.full((B, S), -100)
    labels[:, 3:20] = ids[:, 3:20]
    out = m(ids.to(dev), am.to(dev), None, labels=labels.to(dev), sentence_order_label=torch.tensor([0, 1], device=dev))
    out["loss"].backward()
    grads[lt] = {n: m.flat.view(m.flat.grad, n).clone() for n in m.flat.names}
    print("lt", lt, "loss", out["loss"].item())
for n in grads["1"]:
    e = rel(grads["1"][n], grads["0"][n])
    if e > 1e-2:
        print(f"  {n}: rel {e:.3e}")
