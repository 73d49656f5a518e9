"""Composed attention (ops.attn_composed_fwd / _bwd) — the path for head sizes outside the fused
kernels' 64 (albert-xlarge-v2: 128) — against a plain PyTorch fp32 reference: outputs, log2-unit
lse, packed dQKV and the QKV bias gradient.  CPU tier runs the same code on CPU bf16 GEMMs; the
GPU tier checks it on the card, against the fused kernels at head_dim 64, and one albert-xlarge
shaped model step."""
import math

import pytest
import torch
import torch.nn.functional as F

import dedloc_amd.ops as ops


def _ref(qkv, mask, H, S, dout):
    T, ld = qkv.shape
    D, B = ld // (3 * H), T // S
    x = qkv.float().reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4).detach().requires_grad_(True)
    bias = torch.where(mask.bool(), 0.0, float("-inf"))[:, None, None, :]
    s = torch.matmul(x[0], x[1].transpose(-1, -2)) / math.sqrt(D) + bias
    lse = torch.logsumexp(s, -1) * math.log2(math.e)
    o = F.scaled_dot_product_attention(x[0], x[1], x[2], attn_mask=bias)
    o = o.permute(0, 2, 1, 3).reshape(T, H * D)
    (g,) = torch.autograd.grad(o, [x], dout.float())
    return o.detach(), lse.detach(), g.permute(1, 3, 0, 2, 4).reshape(T, 3 * H * D)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _check(dev, B, H, S, D, tol=2e-2):
    torch.manual_seed(0)
    qkv = (torch.randn(B * S, 3 * H * D, device=dev) * 1.5).bfloat16()
    mask = torch.ones(B, S, device=dev, dtype=torch.long)
    mask[-1, S - S // 4:] = 0
    mbias = torch.where(mask.bool(), 0.0, -1e30).float()
    dout = torch.randn(B * S, H * D, device=dev).bfloat16()
    scale = 1.0 / math.sqrt(D)
    out, lse = ops.attn_composed_fwd(qkv, mbias, H, S, scale)
    dbias = torch.zeros(3 * H * D, device=dev)
    g = ops.attn_composed_bwd(qkv, mbias, out, dout, lse, H, S, scale, dbias)
    o_ref, lse_ref, g_ref = _ref(qkv, mask, H, S, dout)
    assert out.dtype == torch.bfloat16 and out.shape == (B * S, H * D)
    assert rel(out, o_ref) < tol
    assert (lse - lse_ref).abs().max().item() < 1e-2
    assert g.dtype == torch.bfloat16 and g.shape == qkv.shape
    assert rel(g, g_ref) < 3 * tol
    HD = H * D
    assert rel(dbias[:HD], g_ref[:, :HD].sum(0)) < 3 * tol
    assert dbias[HD:2 * HD].abs().max().item() == 0.0
    assert rel(dbias[2 * HD:], dout.float().sum(0)) < 1e-4
    return qkv, mbias, dout, out, lse, g, dbias


@pytest.mark.parametrize("D", [64, 128])
def test_composed_attention_cpu(D):
    _check("cpu", 2, 2, 64, D)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,S", [(2, 2, 64), (4, 16, 512)])
def test_composed_attention_gpu_head128(cuda, B, H, S):
    _check(cuda, B, H, S, 128)


@pytest.mark.gpu
def test_composed_matches_fused_head64(cuda):
    """At head_dim 64 the composed path and the fused flash kernels agree (same lse convention,
    same packed dQKV layout, same bias-gradient accumulation)."""
    B, H, S, D = 2, 4, 128, 64
    qkv, mbias, dout, out, lse, g, dbias = _check(cuda, B, H, S, D)
    O = torch.ops.dedloc
    out_f, lse_f = O.attn_fwd(qkv, mbias, H, S, 1.0 / math.sqrt(D), None)
    assert rel(out, out_f) < 1e-2
    assert (lse - lse_f).abs().max().item() < 1e-3
    db_f = torch.zeros_like(dbias)
    g_f = O.attn_bwd(qkv, mbias, out_f, dout, lse_f, H, S, 1.0 / math.sqrt(D), None, db_f)
    assert rel(g, g_f) < 2e-2
    assert rel(dbias, db_f) < 2e-2


@pytest.mark.gpu
def test_head128_albert_step(cuda):
    """A small ALBERT with 128-wide heads (albert-xlarge's shape of head) trains on the GPU:
    forward + backward + LAMB through the composed attention, finite loss and gradients, loss drops
    when the same batch is repeated."""
    from dedloc_amd.data.synthetic_mlm import SyntheticSOPStream
    from dedloc_amd.models.albert import AlbertConfig, AlbertForPreTraining
    from dedloc_amd.optim.lamb import FusedLamb

    torch.manual_seed(0)
    cfg = AlbertConfig.tiny(hidden_size=256, num_attention_heads=2, intermediate_size=1024)
    model = AlbertForPreTraining(cfg)
    model.materialize(cuda)
    model.train()
    opt = FusedLamb(model.flat, lr=2e-3, weight_decay=0.01, clamp_value=1e4, no_decay=model.no_decay_names())
    batch = SyntheticSOPStream(4, 128, cfg.vocab_size, seed=0, device=cuda).next_batch()
    losses = []
    for _ in range(8):
        out = model(batch["input_ids"], batch["attention_mask"], batch["token_type_ids"],
                    sentence_order_label=batch["sentence_order_label"], mlm_positions=batch["mlm_positions"],
                    mlm_labels=batch["mlm_labels"])
        out["loss"].backward()
        assert torch.isfinite(model.flat.grad).all()
        opt.step()
        model.flat.grad.zero_()
        losses.append(float(out["loss"].detach()))
    torch.cuda.synchronize()
    assert all(math.isfinite(x) for x in losses) and losses[-1] < losses[0], losses
