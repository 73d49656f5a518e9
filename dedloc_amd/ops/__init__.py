"""Differentiable building blocks over the ``dedloc::`` operators.

Parameter gradients are *accumulated as a side effect* straight into fp32 views of the flat
gradient buffer (``g*`` arguments), Megatron-style "gradient accumulation fusion": autograd only
carries activation gradients, and ALBERT's shared layer simply accumulates its 24 weight-gradient
contributions into the same fp32 view.  Weights are consumed as bf16 views of the flat bf16
parameter copy that the optimizer refreshes after each global step.

Reference parity: these implement the HF ``AlbertForPreTraining`` forward used by
``albert/run_trainer.py:56-70`` — Linear, gelu_new, LayerNorm(eps 1e-12),
scaled-dot-product attention with key padding mask, tanh pooler, cross-entropy.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._lib import load_native, native_loaded  # noqa: F401

OPS = torch.ops.dedloc


def _needs_grad(*xs):
    return any(isinstance(x, torch.Tensor) and x.requires_grad for x in xs)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gw, gb, epilogue):
        ctx.save_for_backward(x, w)
        ctx.gw, ctx.gb = gw, gb
        return OPS.gemm(x, w, b, None, False, True, epilogue)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = OPS.gemm(dy, w, None, None, False, False, 0)
        if ctx.gw is not None:
            OPS.gemm_acc_f32(dy, x, ctx.gw, True, False)
        if ctx.gb is not None:
            OPS.bias_grad(dy, ctx.gb, True)
        return dx, None, None, None, None, None


def linear(x, w, b=None, gw=None, gb=None):
    """y = x @ w.T + b with fp32 gradient accumulation into gw / gb.  x: [M, K] bf16, w: [N, K]."""
    return _Linear.apply(x, w, b, gw, gb, 0)


class _Gelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        ctx.save_for_backward(h)
        return OPS.gelu_fwd(h)

    @staticmethod
    def backward(ctx, dy):
        (h,) = ctx.saved_tensors
        return OPS.gelu_bwd(dy.contiguous(), h)


def gelu_new(h):
    return _Gelu.apply(h)


class _Tanh(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = OPS.tanh_fwd(x)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return OPS.tanh_bwd(dy.contiguous(), y)


def tanh(x):
    return _Tanh.apply(x)


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, gamma, beta, ggamma, gbeta, eps):
        y, s, mean, rstd = OPS.layernorm_fwd(x, res, gamma, beta, eps)
        ctx.save_for_backward(s, gamma, mean, rstd)
        ctx.ggamma, ctx.gbeta, ctx.has_res = ggamma, gbeta, res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        s, gamma, mean, rstd = ctx.saved_tensors
        gg, gb = ctx.ggamma, ctx.gbeta
        if gg is None:
            gg = torch.zeros_like(gamma)
            gb = torch.zeros_like(gamma)
        ds = OPS.layernorm_bwd(dy.contiguous(), s, gamma, mean, rstd, gg, gb, True)
        return ds, (ds if ctx.has_res else None), None, None, None, None, None


def add_layernorm(x, res, gamma, beta, ggamma=None, gbeta=None, eps=1e-12):
    """LayerNorm(x + res) (res may be None); gamma/beta are fp32, grads accumulate into ggamma/gbeta."""
    return _AddLayerNorm.apply(x, res, gamma, beta, ggamma, gbeta, eps)


_LOG2E = math.log2(math.e)


def _bmm_f32(a, b):
    """[N, M, K] x [N, K, P] bf16 -> fp32 without rounding the product through bf16 (the own
    batched GEMM kernel; transposed operands are read in place)."""
    return OPS.bmm(a, b, True)


def _bmm(a, b):
    """[N, M, K] x [N, K, P] bf16 -> bf16 on the own batched GEMM kernel."""
    return OPS.bmm(a, b, False)


def _attn_split(qkv, H, S):
    T, ld = qkv.shape
    D = ld // (3 * H)
    B = T // S
    x = qkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)  # 3, B, H, S, D
    return (x[0].reshape(B * H, S, D), x[1].reshape(B * H, S, D), x[2].reshape(B * H, S, D)), B, D


def attn_composed_fwd(qkv, mbias, H, S, scale):
    """Attention for head sizes outside the fused kernels' 64 (albert-xlarge: 128): batched bf16
    GEMMs with fp32 scores around the ``attn_softmax_fwd`` kernel (scale, key bias, log2-unit
    softmax in one pass) — same inputs / outputs as ``attn_fwd`` (out [B*S, H*D] bf16, lse
    [B, H, S] fp32 in log2 units), but the [B*H, S, S] scores go through HBM."""
    (q, k, v), B, D = _attn_split(qkv, H, S)
    s = _bmm_f32(q, k.transpose(1, 2))
    p, lse = OPS.attn_softmax_fwd(s, mbias, H, scale * _LOG2E)
    del s
    o = _bmm(p, v)
    return o.view(B, H, S, D).transpose(1, 2).reshape(B * S, H * D), lse.view(B, H, S)


def attn_composed_bwd(qkv, mbias, out, dout, lse, H, S, scale, dbias=None):
    """Backward of ``attn_composed_fwd`` (probabilities recomputed from lse by the
    ``attn_softmax_bwd`` kernel, which also forms dS); dQKV in the packed layout, and — like the
    fused backward — the QKV bias gradient accumulated into ``dbias``."""
    (q, k, v), B, D = _attn_split(qkv, H, S)
    do = dout.view(B, S, H, D).transpose(1, 2).reshape(B * H, S, D)
    o = out.view(B, S, H, D).transpose(1, 2).reshape(B * H, S, D)
    s = _bmm_f32(q, k.transpose(1, 2))
    dp = _bmm_f32(do, v.transpose(1, 2))
    delta = (do.float() * o.float()).sum(-1)
    p, ds = OPS.attn_softmax_bwd(s, dp, mbias, lse.reshape(-1).contiguous(), delta.reshape(-1), H,
                                 scale * _LOG2E, scale)
    del s, dp
    dv = _bmm(p.transpose(1, 2), do)
    dq = _bmm(ds, k)
    dk = _bmm(ds.transpose(1, 2), q)
    g = torch.stack([dq, dk, dv], 0).view(3, B, H, S, D).permute(1, 3, 0, 2, 4).reshape(B * S, 3 * H * D)
    if dbias is not None:  # query: colsum dQ; key: 0 (softmax shift invariance); value: colsum dout
        HD = H * D
        dbias[:HD] += g[:, :HD].float().sum(0)
        dbias[2 * HD:] += dout.float().sum(0)
    return g


def _fused_attention(qkv, H):
    return not qkv.is_cuda or qkv.shape[-1] // (3 * H) == 64


def attn_fwd(qkv, mbias, H, S, scale, kvinfo=None):
    """The fused flash kernels for head_dim 64 (CPU: the fp32 reference), else the composed path."""
    if _fused_attention(qkv, H):
        return OPS.attn_fwd(qkv, mbias, H, S, scale, kvinfo)
    return attn_composed_fwd(qkv, mbias, H, S, scale)


def attn_bwd(qkv, mbias, out, dout, lse, H, S, scale, kvinfo=None, dbias=None):
    if _fused_attention(qkv, H):
        return OPS.attn_bwd(qkv, mbias, out, dout, lse, H, S, scale, kvinfo, dbias)
    return attn_composed_bwd(qkv, mbias, out, dout, lse, H, S, scale, dbias)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, mbias, H, S, scale):
        out, lse = attn_fwd(qkv, mbias, H, S, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.mbias, ctx.H, ctx.S, ctx.scale = mbias, H, S, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dqkv = attn_bwd(qkv, ctx.mbias, out, dout.contiguous(), lse, ctx.H, ctx.S, ctx.scale)
        return dqkv, None, None, None, None


def attention(qkv, mbias, num_heads, seq_len, scale=None):
    """Fused self-attention over a packed [B*S, 3*H*D] QKV buffer -> [B*S, H*D].

    ``mbias`` is the [B, S] fp32 additive key bias in log2 units (0 = keep, -1e30 = masked).
    """
    d = qkv.shape[-1] // (3 * num_heads)
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    return _Attention.apply(qkv, mbias, num_heads, seq_len, scale)


class _EmbedLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, tt, wemb, pemb, temb, gamma, beta, gw, gp, gt, ggamma, gbeta, S, eps):
        y, s, mean, rstd = OPS.embed_ln_fwd(ids, tt, wemb, pemb, temb, gamma, beta, S, eps)
        ctx.save_for_backward(ids, s, gamma, mean, rstd)
        ctx.tt = tt
        ctx.grads = (gw, gp, gt, ggamma, gbeta)
        ctx.S = S
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, s, gamma, mean, rstd = ctx.saved_tensors
        gw, gp, gt, gg, gb = ctx.grads
        if gw is not None:
            ds = OPS.layernorm_bwd(dy.contiguous(), s, gamma, mean, rstd, gg, gb, True)
            OPS.embed_bwd(ds, ids, ctx.tt, gw, gp, gt, ctx.S)
        return (None,) * 15


def embed_layernorm(ids, tt, wemb, pemb, temb, gamma, beta, grads=(None,) * 5, eps=1e-12):
    """ALBERT embeddings: LN(word[ids] + pos[arange(S)] + type[tt]) -> [B*S, E] bf16.

    The fp32 master tables are read directly; gradients are scattered into ``grads`` =
    (g_word, g_pos, g_type, g_ln_gamma, g_ln_beta).
    """
    B, S = ids.shape
    anchor = torch.empty(0, device=ids.device, requires_grad=True)
    return _EmbedLN.apply(anchor, ids.reshape(-1).contiguous(), None if tt is None else tt.reshape(-1).contiguous(),
                          wemb, pemb, temb, gamma, beta, *grads, S, eps)


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        loss, dlogits = OPS.xent_fwd_bwd(logits, labels, False, ignore_index)
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (dlogits,) = ctx.saved_tensors
        # the kernel already produced d(mean loss)/dlogits; scale in place by the upstream grad (a
        # no-op on the device when it is 1, the usual loss.backward() seed: no host sync, no pass)
        if dlogits.dtype == torch.bfloat16 and dlogits.is_contiguous():
            OPS.scale_by_(dlogits, dloss.reshape(1).float())
            return dlogits, None, None
        return dlogits.mul_(dloss.to(dlogits.dtype)), None, None


def cross_entropy(logits, labels, ignore_index=-100):
    """Mean token cross-entropy over rows whose label != ignore_index (fused fwd+bwd kernel)."""
    return _CrossEntropy.apply(logits.contiguous(), labels.reshape(-1).contiguous(), ignore_index)


__all__ = [
    "linear", "gelu_new", "tanh", "add_layernorm", "attention", "embed_layernorm", "cross_entropy", "OPS",
    "load_native", "native_loaded",
]

# The gfx950 library is mandatory wherever a GPU is visible (fails loudly otherwise); on a CPU-only
# host the CPU implementations registered in _lib serve the plumbing configuration.
load_native()
