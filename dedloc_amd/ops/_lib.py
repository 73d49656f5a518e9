"""Operator registry: schemas of every ``dedloc::`` op, their CPU implementations and the loader of
the gfx950 library.

Single code path per device: on a GPU tensor the dispatcher can only reach the HIP kernel that
``_C.so`` registers under the CUDA key (loading it is mandatory whenever a GPU is visible — a
missing or stale library raises instead of silently falling back).  The CPU implementations below
exist for the CPU plumbing configuration (BASELINE.json config 1) and for the non-GPU test tier;
they mirror the kernels' numerics contract (bf16 storage, fp32 math).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

LIB = torch.library.Library("dedloc", "DEF")

_SCHEMAS = [
    "layernorm_fwd(Tensor x, Tensor? res, Tensor gamma, Tensor beta, float eps) -> (Tensor, Tensor, Tensor, Tensor)",
    "layernorm_bwd(Tensor dy, Tensor s, Tensor gamma, Tensor mean, Tensor rstd, Tensor(a!) dgamma, Tensor(b!) dbeta, bool accumulate, Tensor(c!)? dsum=None) -> Tensor",
    "gelu_fwd(Tensor h) -> Tensor",
    "gelu_bwd(Tensor dy, Tensor h, Tensor(a!)? dbias=None) -> Tensor",
    "tanh_fwd(Tensor x) -> Tensor",
    "tanh_bwd(Tensor dy, Tensor y) -> Tensor",
    "bias_grad(Tensor dy, Tensor(a!) dbias, bool accumulate) -> ()",
    "cast_bf16(Tensor x, Tensor(a!) out) -> ()",
    "lamb_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor chunk_tensor, Tensor chunk_start, Tensor chunk_len, Tensor tensor_wd, Tensor(d!) norms, float beta1, float beta2, float eps, float step_size, float clamp_value, float grad_scale) -> ()",
    "larc_sgd_step(Tensor(a!) p, Tensor g, Tensor(b!) buf, Tensor chunk_tensor, Tensor chunk_start, Tensor chunk_len, Tensor tensor_wd, Tensor(c!) norms, float lr, float momentum, float trust_coef, float eps, bool clip, bool first_step, float grad_scale) -> ()",
    "grad_norm_clip(Tensor(a!) g, float max_norm, Tensor(b!) part, Tensor(c!) out) -> ()",
    "axpby(Tensor(a!) y, Tensor x, float a, float b, Tensor? flag=None, Tensor? bdiv=None) -> ()",
    "add_slabs_zero_(Tensor(a!) out, Tensor(b!) slabs) -> ()",
    "scale_by_(Tensor(a!) x, Tensor s) -> ()",
    "pack(Tensor src, Tensor(a!) dst, float weight) -> ()",
    "reduce_parts(Tensor parts, int nparts, Tensor(a!) out, float inv_total) -> ()",
    "unpack(Tensor src, Tensor(a!) dst, Tensor? snap, bool add=False) -> ()",
    "reduce_delta(Tensor parts, Tensor weights, Tensor(a!) deltas) -> ()",
    "embed_ln_fwd(Tensor ids, Tensor? tt, Tensor wemb, Tensor pemb, Tensor temb, Tensor gamma, Tensor beta, int S, float eps) -> (Tensor, Tensor, Tensor, Tensor)",
    "embed_bwd(Tensor ds, Tensor ids, Tensor? tt, Tensor(a!) dwemb, Tensor(b!) dpemb, Tensor(c!) dtemb, int S) -> ()",
    "xent_fwd_bwd(Tensor logits, Tensor labels, bool inplace, int ignore_index) -> (Tensor, Tensor)",
    "attn_fwd(Tensor qkv, Tensor? mbias, int H, int S, float scale, Tensor? kvinfo=None) -> (Tensor, Tensor)",
    "attn_bwd(Tensor qkv, Tensor? mbias, Tensor out, Tensor dout, Tensor lse, int H, int S, float scale, "
    "Tensor? kvinfo=None, Tensor(a!)? dbias=None) -> Tensor",
    "attn_softmax_fwd(Tensor s, Tensor? mbias, int H, float c) -> (Tensor, Tensor)",
    "attn_softmax_bwd(Tensor s, Tensor dp, Tensor? mbias, Tensor lse, Tensor delta, int H, float c, float scale) "
    "-> (Tensor, Tensor)",
    "gemm(Tensor a, Tensor b, Tensor? bias, Tensor? residual, bool trans_a, bool trans_b, int epilogue) -> Tensor",
    "bmm(Tensor a, Tensor b, bool out_f32=False) -> Tensor",
    "gemm_acc_f32(Tensor a, Tensor b, Tensor(a!) c, bool trans_a, bool trans_b) -> ()",
    "gemm_acc_f32_shared(Tensor a, Tensor b, Tensor(a!) c, bool trans_a, bool trans_b, bool first, bool last) -> ()",
    "gemm_gelu(Tensor x, Tensor w, Tensor bias, bool trans_w=False) -> (Tensor, Tensor)",
    "sinkhorn(Tensor scores, int bs, float eps, int iters) -> Tensor",
    "swav_ce(Tensor scores, Tensor q, Tensor(a!) dscores, Tensor(b!) loss, float temperature, float scale) -> ()",
    "swav_ce_multi(Tensor scores, Tensor q, int[] crops, Tensor(a!) dscores, Tensor(b!) loss, float temperature, "
    "float scale) -> ()",
    "row_normalize_(Tensor(a!) w) -> ()",
    "maxpool_fwd(Tensor x) -> (Tensor, Tensor)",
    "maxpool_bwd(Tensor dy, Tensor arg, int H, int W) -> Tensor",
    "avgpool_fwd(Tensor x) -> Tensor",
    "avgpool_bwd(Tensor dy, int H, int W) -> Tensor",
    "l2norm_fwd(Tensor x, float eps) -> (Tensor, Tensor)",
    "l2norm_bwd(Tensor dy, Tensor y, Tensor rinv) -> Tensor",
    "multicrop(Tensor pool, Tensor params, int size, int rad, float[] mean, float[] std) -> Tensor",
    "bn_fwd(Tensor x, Tensor? res, Tensor gamma, Tensor beta, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
    "float eps, float momentum, bool relu, int groups=1, Tensor(c!)? sums=None, bool stats_ready=False) "
    "-> (Tensor, Tensor, Tensor)",
    "bn_bwd(Tensor dy, Tensor y, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, bool relu, bool want_dres, "
    "Tensor(a!)? sums=None, Tensor(b!)? dgamma_acc=None, Tensor(c!)? dbeta_acc=None, Tensor? beta=None, "
    "bool stats_ready=False) -> (Tensor, Tensor, Tensor, Tensor)",
    "conv2d_dgrad_bn(Tensor dy, Tensor w, int stride, int pad, int H, int W, Tensor? residual, Tensor x, Tensor? y, "
    "Tensor mean, Tensor rstd, Tensor gamma, Tensor beta, Tensor(a!) sums, int groups, Tensor[]? wds=None) "
    "-> (Tensor, bool)",
    "bn_bwd_prep(Tensor(a!) g, Tensor x, Tensor? y, Tensor mean, Tensor rstd, Tensor gamma, Tensor beta, "
    "Tensor(b!) sums, int groups) -> Tensor",
    "gemm_dgelu(Tensor dy, Tensor w, Tensor F, Tensor(a!) dbias, bool trans_w=False) -> Tensor",
    "gemm_gelu_d(Tensor x, Tensor w, Tensor bias, bool trans_w=False) -> (Tensor, Tensor)",
    "gemm_dmul(Tensor dy, Tensor w, Tensor D, Tensor(a!) dbias, bool trans_w=False) -> Tensor",
    "conv2d_fwd(Tensor x, Tensor w, int stride, int pad, Tensor? cols=None) -> Tensor",
    "conv2d_fwd_stats(Tensor x, Tensor w, int stride, int pad, Tensor(a!) sums, int groups, Tensor? cols=None) "
    "-> Tensor",
    "im2col_stem(Tensor x, int R, int S, int stride, int pad) -> Tensor",
    "conv2d_dgrad(Tensor dy, Tensor w, int stride, int pad, int H, int W, Tensor? residual=None, "
    "Tensor[]? wds=None) -> Tensor",
    "conv2d_dgrad_weights(Tensor w, int stride, int pad) -> Tensor[]",
    "conv2d_dgrad_weights_batched(Tensor[] ws, int[] strides, int[] pads) -> Tensor[]",
    "conv2d_wgrad(Tensor dy, Tensor x, Tensor(a!) dw, int stride, int pad, Tensor? cols=None) -> ()",
]
for _s in _SCHEMAS:
    LIB.define(_s)

_NATIVE = {"loaded": False, "path": None, "error": None}


def _impl(name):
    def deco(fn):
        LIB.impl(name, fn, "CPU")
        return fn

    return deco


def load_native(required: bool | None = None) -> bool:
    """Load ``_C.so`` (the gfx950 kernels).  ``required`` defaults to "a GPU is visible"."""
    if _NATIVE["loaded"]:
        return True
    if required is None:
        required = torch.cuda.is_available()
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # DEDLOC_NATIVE_LIB: an alternative build of the same library (same-box A/B measurements,
    # _build.build_variant); the default is the in-tree _C.so
    path = os.environ.get("DEDLOC_NATIVE_LIB") or os.path.join(pkg, "_C.so")
    try:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (run python -m dedloc_amd._build)")
        torch.ops.load_library(path)
        _NATIVE.update(loaded=True, path=path)
        return True
    except Exception as e:  # noqa: BLE001
        _NATIVE["error"] = repr(e)
        if required:
            raise ImportError(
                "dedloc_amd: the gfx950 kernel library could not be loaded on a GPU machine; refusing to run "
                f"without it ({e})"
            ) from e
        return False


def native_loaded() -> bool:
    return _NATIVE["loaded"]


# ---------------------------------------------------------------------------------------------
# CPU implementations (plumbing / reference numerics: bf16 storage, fp32 math)
# ---------------------------------------------------------------------------------------------
def _bf(x):
    return x.to(torch.bfloat16)


@_impl("layernorm_fwd")
def _ln_fwd_cpu(x, res, gamma, beta, eps):
    s = x.float() if res is None else (x.float() + res.float())
    s_b = _bf(s)
    sf = s_b.float() if res is not None else x.float()
    mean = sf.mean(-1)
    var = ((sf - mean.unsqueeze(-1)) ** 2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    y = (sf - mean.unsqueeze(-1)) * rstd.unsqueeze(-1) * gamma + beta
    D = x.shape[-1]
    return _bf(y), (s_b if res is not None else x), mean.reshape(-1), rstd.reshape(-1)


@_impl("layernorm_bwd")
def _ln_bwd_cpu(dy, s, gamma, mean, rstd, dgamma, dbeta, accumulate, dsum=None):
    D = dy.shape[-1]
    g = dy.float().reshape(-1, D)
    xh = (s.float().reshape(-1, D) - mean.unsqueeze(-1)) * rstd.unsqueeze(-1)
    dg = (g * xh).sum(0)
    db = g.sum(0)
    if accumulate:
        dgamma.add_(dg)
        dbeta.add_(db)
    else:
        dgamma.copy_(dg)
        dbeta.copy_(db)
    gy = g * gamma
    a = gy.mean(-1, keepdim=True)
    b = (gy * xh).mean(-1, keepdim=True)
    ds = _bf(rstd.unsqueeze(-1) * (gy - a - xh * b))
    if dsum is not None:
        dsum.add_(ds.float().sum(0))
    return ds.reshape(dy.shape)


def _gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x.pow(3))))


@_impl("gelu_fwd")
def _gelu_fwd_cpu(h):
    return _bf(_gelu_tanh(h.float()))


@_impl("gelu_bwd")
def _gelu_bwd_cpu(dy, h, dbias=None):
    x = h.float()
    k0, k1 = math.sqrt(2.0 / math.pi), 0.044715
    u = k0 * (x + k1 * x ** 3)
    t = torch.tanh(u)
    d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
    dh = _bf(dy.float() * d)
    if dbias is not None:
        dbias.add_(dh.float().reshape(-1, dh.shape[-1]).sum(0))
    return dh


@_impl("tanh_fwd")
def _tanh_fwd_cpu(x):
    return _bf(torch.tanh(x.float()))


@_impl("tanh_bwd")
def _tanh_bwd_cpu(dy, y):
    t = y.float()
    return _bf(dy.float() * (1 - t * t))


@_impl("bias_grad")
def _bias_grad_cpu(dy, dbias, accumulate):
    s = dy.float().reshape(-1, dy.shape[-1]).sum(0)
    if accumulate:
        dbias.add_(s)
    else:
        dbias.copy_(s)


@_impl("cast_bf16")
def _cast_bf16_cpu(x, out):
    out.copy_(x.to(torch.bfloat16))


def _chunks_iter(chunk_tensor, chunk_start, chunk_len):
    for t, s, n in zip(chunk_tensor.tolist(), chunk_start.tolist(), chunk_len.tolist()):
        yield t, s, n


@_impl("lamb_step")
def _lamb_cpu(p, g, m, v, chunk_tensor, chunk_start, chunk_len, tensor_wd, norms, beta1, beta2, eps, step_size,
              clamp_value, grad_scale):
    norms.zero_()
    wd = tensor_wd.tolist()
    chunks = list(_chunks_iter(chunk_tensor, chunk_start, chunk_len))
    for t, s, n in chunks:
        gi = g[s:s + n] * grad_scale
        m[s:s + n].mul_(beta1).add_(gi, alpha=1 - beta1)
        v[s:s + n].mul_(beta2).addcmul_(gi, gi, value=1 - beta2)
        u = m[s:s + n] / (v[s:s + n].sqrt() + eps) + wd[t] * p[s:s + n]
        norms[2 * t] += (p[s:s + n] ** 2).sum()
        norms[2 * t + 1] += (u ** 2).sum()
    for t, s, n in chunks:
        wn = min(max(math.sqrt(norms[2 * t].item()), 0.0), clamp_value)
        un = math.sqrt(norms[2 * t + 1].item())
        trust = 1.0 if (wn == 0 or un == 0) else wn / un
        u = m[s:s + n] / (v[s:s + n].sqrt() + eps) + wd[t] * p[s:s + n]
        p[s:s + n].add_(u, alpha=-step_size * trust)


@_impl("larc_sgd_step")
def _larc_cpu(p, g, buf, chunk_tensor, chunk_start, chunk_len, tensor_wd, norms, lr, momentum, trust_coef, eps, clip,
              first_step, grad_scale):
    norms.zero_()
    wd = tensor_wd.tolist()
    chunks = list(_chunks_iter(chunk_tensor, chunk_start, chunk_len))
    for t, s, n in chunks:
        norms[2 * t] += (p[s:s + n] ** 2).sum()
        norms[2 * t + 1] += ((g[s:s + n] * grad_scale) ** 2).sum()
    for t, s, n in chunks:
        pn, gn = math.sqrt(norms[2 * t].item()), math.sqrt(norms[2 * t + 1].item())
        a = 1.0
        if pn != 0 and gn != 0:
            a = trust_coef * pn / (gn + pn * wd[t] + eps)
            if clip:
                a = min(a / lr, 1.0)
        d = (g[s:s + n] * grad_scale + wd[t] * p[s:s + n]) * a
        if first_step:
            buf[s:s + n].copy_(d)
        else:
            buf[s:s + n].mul_(momentum).add_(d)
        p[s:s + n].add_(buf[s:s + n], alpha=-lr)


@_impl("grad_norm_clip")
def _clip_cpu(g, max_norm, part, out):
    norm = g.float().norm()
    finite = bool(torch.isfinite(norm))
    out[0] = norm
    out[1] = 1.0 if finite else 0.0
    if out.numel() > 2:
        out[2] = 0.0 if finite else 1.0
    if max_norm > 0 and finite:
        coef = max_norm / (norm.item() + 1e-6)
        if coef < 1:
            g.mul_(coef)


@_impl("scale_by_")
def _scale_by_cpu(x, s):
    x.mul_(s.to(x.dtype))


@_impl("add_slabs_zero_")
def _add_slabs_zero_cpu(out, slabs):
    out.add_(slabs.sum(0).view_as(out))
    slabs.zero_()


@_impl("axpby")
def _axpby_cpu(y, x, a, b, flag=None, bdiv=None):
    if flag is not None and float(flag.reshape(-1)[0]) == 0.0:
        return
    if bdiv is not None:
        b = b / max(1.0, float(bdiv.reshape(-1)[0]))
    r = (y * a if a != 0 else torch.zeros_like(y)) + (x * b if b != 0 else 0.0)
    y.copy_(r)


@_impl("pack")
def _pack_cpu(src, dst, weight):
    v = src * weight
    if dst.dtype == torch.float16:
        v = v.clamp(-65504.0, 65504.0)
    dst.copy_(v.to(dst.dtype))


@_impl("reduce_parts")
def _reduce_cpu(parts, nparts, out, inv_total):
    s = parts.reshape(nparts, -1).float().sum(0) * inv_total
    if out.dtype == torch.float16:
        s = s.clamp(-65504.0, 65504.0)
    out.copy_(s.to(out.dtype))


@_impl("reduce_delta")
def _reduce_delta_cpu(parts, weights, deltas):
    x = parts.float()
    w = weights.float()
    tot = float(w.sum())
    if not tot > 0:  # no weight at all: a no-op round (zero deltas), as the HIP kernel does
        deltas.zero_()
        return
    avg = x[0] + (w[1:, None] * (x[1:] - x[0])).sum(0) * (1.0 / tot)
    d = avg[None, :] - x
    if deltas.dtype == torch.float16:
        d = d.clamp(-65504.0, 65504.0)
    deltas.copy_(d.to(deltas.dtype))


@_impl("unpack")
def _unpack_cpu(src, dst, snap, add=False):
    if add:
        dst.add_(src.float())
    elif snap is None:
        dst.copy_(src.float())
    else:
        dst.add_(src.float() - snap)


@_impl("embed_ln_fwd")
def _embed_fwd_cpu(ids, tt, wemb, pemb, temb, gamma, beta, S, eps):
    T = ids.numel()
    pos = torch.arange(T, device=ids.device) % S
    s = wemb[ids.reshape(-1)] + pemb[pos] + temb[(tt.reshape(-1) if tt is not None else torch.zeros_like(pos))]
    s_b = _bf(s)
    sf = s_b.float()
    mean = sf.mean(-1)
    rstd = torch.rsqrt(((sf - mean[:, None]) ** 2).mean(-1) + eps)
    y = (sf - mean[:, None]) * rstd[:, None] * gamma + beta
    return _bf(y), s_b, mean, rstd


@_impl("embed_bwd")
def _embed_bwd_cpu(ds, ids, tt, dwemb, dpemb, dtemb, S):
    g = ds.float().reshape(-1, ds.shape[-1])
    T = g.shape[0]
    dwemb.index_add_(0, ids.reshape(-1), g)
    pos = torch.arange(T) % S
    dpemb.index_add_(0, pos, g)
    tti = tt.reshape(-1) if tt is not None else torch.zeros(T, dtype=torch.long)
    dtemb.index_add_(0, tti, g)


@_impl("xent_fwd_bwd")
def _xent_cpu(logits, labels, inplace, ignore_index):
    x = logits.float().reshape(-1, logits.shape[-1])
    lab = labels.reshape(-1)
    valid = lab != ignore_index
    cnt = int(valid.sum())
    lse = torch.logsumexp(x, -1)
    safe = torch.where(valid, lab, torch.zeros_like(lab))
    rows = lse - x.gather(1, safe[:, None]).squeeze(1)
    scale = 1.0 / cnt if cnt > 0 else 0.0
    loss = (rows * valid).sum() * scale
    grad = torch.softmax(x, -1)
    grad[torch.arange(x.shape[0]), safe] -= 1.0
    grad = grad * valid[:, None] * scale
    g = _bf(grad).reshape(logits.shape)
    if inplace:
        logits.copy_(g)
        g = logits
    return loss.float(), g


def _attn_probs(qkv, mbias, H, S, scale):
    T, ld = qkv.shape
    D = ld // (3 * H)
    B = T // S
    x = qkv.float().reshape(B, S, 3, H, D)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    if mbias is not None:
        s = s + mbias.reshape(B, 1, 1, S) / math.log2(math.e)
    return q, k, v, s


@_impl("attn_fwd")
def _attn_fwd_cpu(qkv, mbias, H, S, scale, kvinfo=None):
    q, k, v, s = _attn_probs(qkv, mbias, H, S, scale)
    B, _, _, D = q.shape
    lse = torch.logsumexp(s, -1)
    p = torch.softmax(s, -1)
    o = torch.matmul(p, v).transpose(1, 2).reshape(B * S, H * D)
    return _bf(o), (lse * math.log2(math.e)).contiguous()


@_impl("attn_bwd")
def _attn_bwd_cpu(qkv, mbias, out, dout, lse, H, S, scale, kvinfo=None, dbias=None):
    q, k, v, s = _attn_probs(qkv, mbias, H, S, scale)
    B, _, _, D = q.shape
    p = torch.softmax(s, -1)
    do = dout.float().reshape(B, S, H, D).transpose(1, 2)
    o = out.float().reshape(B, S, H, D).transpose(1, 2)
    dv = torch.matmul(p.transpose(-1, -2), do)
    dp = torch.matmul(do, v.transpose(-1, -2))
    delta = (do * o).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    dq = torch.matmul(ds, k) * scale
    dk = torch.matmul(ds.transpose(-1, -2), q) * scale
    g = torch.stack([dq, dk, dv], dim=2)  # B,H,3,S,D
    g = _bf(g.permute(0, 3, 2, 1, 4).reshape(B * S, 3 * H * D))
    if dbias is not None:  # query: colsum(dQ); key: 0 (softmax shift invariance); value: colsum(dout)
        HD = H * D
        dbias[:HD] += g[:, :HD].float().sum(0)
        dbias[2 * HD:] += dout.float().reshape(-1, HD).sum(0)
    return g


def _softmax_logits(s, mbias, H, c):
    S = s.shape[-1]
    x = s.float().reshape(-1, H, S, S) * c
    if mbias is not None:
        x = x + mbias.reshape(-1, 1, 1, S)
    return x.reshape(s.shape)


@_impl("attn_softmax_fwd")
def _attn_softmax_fwd_cpu(s, mbias, H, c):
    x = _softmax_logits(s, mbias, H, c)
    lse = torch.logsumexp(x / math.log2(math.e), -1) * math.log2(math.e)
    return _bf(torch.exp2(x - lse[..., None])), lse.reshape(-1).contiguous()


@_impl("attn_softmax_bwd")
def _attn_softmax_bwd_cpu(s, dp, mbias, lse, delta, H, c, scale):
    p = torch.exp2(_softmax_logits(s, mbias, H, c) - lse.reshape(s.shape[:-1])[..., None])
    return _bf(p), _bf(p * (dp.float() - delta.reshape(s.shape[:-1])[..., None]) * scale)


@_impl("gemm")
def _gemm_cpu(a, b, bias, residual, trans_a, trans_b, epilogue):
    A = a.float().t() if trans_a else a.float()
    Bm = b.float().t() if trans_b else b.float()
    c = A @ Bm
    if bias is not None:
        c = c + bias.float()
    if residual is not None:
        c = c + residual.float()
    if epilogue == 1:
        c = _gelu_tanh(c)
    return _bf(c)


@_impl("gemm_gelu")
def _gemm_gelu_cpu(x, w, bias, trans_w=False):
    h = _bf(x.float() @ (w.float() if trans_w else w.float().t()) + bias.float())
    return h, _bf(_gelu_tanh(h.float()))


@_impl("gemm_dgelu")
def _gemm_dgelu_cpu(dy, w, F, dbias, trans_w=False):
    dg = _bf(dy.float() @ (w.float().t() if trans_w else w.float()))
    return _gelu_bwd_cpu(dg, F, dbias)


def _gelu_grad_tanh(x):
    k0, k1 = 0.7978845608028654, 0.044715
    t = torch.tanh(k0 * (x + k1 * x ** 3))
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)


@_impl("gemm_gelu_d")
def _gemm_gelu_d_cpu(x, w, bias, trans_w=False):
    h = _bf(x.float() @ (w.float() if trans_w else w.float().t()) + bias.float()).float()
    return _bf(_gelu_grad_tanh(h)), _bf(_gelu_tanh(h))


@_impl("gemm_dmul")
def _gemm_dmul_cpu(dy, w, D, dbias, trans_w=False):
    dg = _bf(dy.float() @ (w.float().t() if trans_w else w.float())).float()
    c = _bf(dg * D.float())
    dbias.add_(c.float().sum(0))
    return c


@_impl("gemm_acc_f32")
def _gemm_acc_cpu(a, b, c, trans_a, trans_b):
    A = a.float().t() if trans_a else a.float()
    Bm = b.float().t() if trans_b else b.float()
    c.add_(A @ Bm)


@_impl("gemm_acc_f32_shared")
def _gemm_acc_shared_cpu(a, b, c, trans_a, trans_b, first, last):
    _gemm_acc_cpu(a, b, c, trans_a, trans_b)  # same sum; the slab deferral is a GPU-side schedule


@_impl("sinkhorn")
def _sinkhorn_cpu(scores, bs, eps, iters):
    # vissl distributed_sinkhornknopp (world size 1) on Q = exp((s - max s)/eps)^T
    Q = torch.exp((scores.float() - scores.max()) / eps).t()
    Q = Q / Q.sum()
    K, n = Q.shape
    r = torch.ones(K) / K
    c = torch.ones(n) / n
    curr = Q.sum(1)
    for _ in range(iters):
        Q = Q * (r / curr).unsqueeze(1)
        Q = Q * (c / Q.sum(0)).unsqueeze(0)
        curr = Q.sum(1)
    Q = (Q / Q.sum(0, keepdim=True)).t()
    return Q[-bs:].contiguous()


@_impl("swav_ce")
def _swav_ce_cpu(scores, q, dscores, loss, temperature, scale):
    x = scores.float() / temperature
    logp = torch.log_softmax(x, -1)
    qs = q.sum(-1, keepdim=True)
    loss.add_(-(q * logp).sum() * scale)
    dscores.add_((torch.softmax(x, -1) * qs - q) / temperature * scale)


@_impl("swav_ce_multi")
def _swav_ce_multi_cpu(scores, q, crops, dscores, loss, temperature, scale):
    n_assign, bs, K = q.shape
    nc = scores.shape[0] // bs
    x = scores.float().view(nc, bs, K) / temperature
    lsm = torch.log_softmax(x, dim=-1)
    sm = lsm.exp()
    ds = torch.zeros(nc, bs, K)
    tot = torch.zeros(())
    for i, cid in enumerate(crops):
        for v in range(nc):
            if v == cid:
                continue
            qi = q[i]
            tot = tot - (qi * lsm[v]).sum()
            ds[v] += sm[v] * qi.sum(-1, keepdim=True) - qi
    loss.add_(tot * scale)
    dscores.copy_((ds * (scale / temperature)).view_as(dscores))


@_impl("row_normalize_")
def _row_normalize_cpu(w):
    w.div_(w.norm(dim=1, keepdim=True).clamp_min(1e-12))


@_impl("maxpool_fwd")
def _maxpool_fwd_cpu(x):
    y, idx = F.max_pool2d(x.float(), 3, 2, 1, return_indices=True)
    return y.to(x.dtype).contiguous(memory_format=torch.channels_last), idx


@_impl("maxpool_bwd")
def _maxpool_bwd_cpu(dy, arg, H, W):
    dx = F.max_unpool2d(dy.float(), arg, 3, 2, 1, output_size=(H, W))
    return dx.to(dy.dtype).contiguous(memory_format=torch.channels_last)


@_impl("avgpool_fwd")
def _avgpool_fwd_cpu(x):
    return x.float().mean(dim=(2, 3)).to(x.dtype)


@_impl("avgpool_bwd")
def _avgpool_bwd_cpu(dy, H, W):
    return (dy.float()[:, :, None, None] / (H * W)).expand(dy.shape[0], dy.shape[1], H, W).to(dy.dtype).contiguous(
        memory_format=torch.channels_last)


@_impl("l2norm_fwd")
def _l2norm_fwd_cpu(x, eps):
    xf = x.float()
    r = 1.0 / xf.norm(dim=1).clamp_min(eps)
    return (xf * r[:, None]).to(x.dtype), r


@_impl("l2norm_bwd")
def _l2norm_bwd_cpu(dy, y, rinv):
    g, yf = dy.float(), y.float()
    return ((g - yf * (g * yf).sum(1, keepdim=True)) * rinv[:, None]).to(dy.dtype)


@_impl("multicrop")
def _multicrop_cpu(pool, params, size, rad, mean, std):
    from dedloc_amd.data.multicrop import augment_reference

    return augment_reference(pool, params, size, rad, mean, std)


@_impl("bmm")
def _bmm_cpu(a, b, out_f32=False):
    c = torch.bmm(a.float(), b.float())
    return c if out_f32 else c.to(a.dtype)


@_impl("bn_fwd")
def _bn_fwd_cpu(x, res, gamma, beta, running_mean, running_var, eps, momentum, relu, groups=1, sums=None,
                stats_ready=False):  # the reference recomputes the statistics from x either way
    G = groups
    xf = x.float().reshape(G, x.shape[0] // G, *x.shape[1:])
    R = xf[0].numel() // xf.shape[2]
    mean = xf.mean(dim=(1, 3, 4))                  # [G, C]
    var = xf.var(dim=(1, 3, 4), unbiased=False)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean[:, None, :, None, None]) * (rstd * gamma)[:, None, :, None, None] + beta.view(1, 1, -1, 1, 1)
    y = y.reshape(x.shape)
    if res is not None:
        y = y + res.float()
    if relu:
        y = y.clamp_min(0)
    if running_mean is not None:
        for k in range(G):
            running_mean.mul_(1 - momentum).add_(mean[k], alpha=momentum)
            running_var.mul_(1 - momentum).add_(var[k] * (R / max(R - 1, 1)), alpha=momentum)
    return y.to(x.dtype).contiguous(memory_format=torch.channels_last), mean, rstd


@_impl("conv2d_fwd")
def _conv2d_fwd_cpu(x, w, stride, pad, cols=None):  # cols: a GPU-side stem cache, unused here
    y = F.conv2d(x.float(), w.float(), stride=stride, padding=pad)
    return y.to(x.dtype).contiguous(memory_format=torch.channels_last)


@_impl("conv2d_fwd_stats")
def _conv2d_fwd_stats_cpu(x, w, stride, pad, sums, groups, cols=None):
    y = _conv2d_fwd_cpu(x, w, stride, pad)
    yg = y.float().reshape(groups, -1, *y.shape[1:])
    sums.view(groups, 2, -1).add_(torch.stack([yg.sum(dim=(1, 3, 4)), (yg * yg).sum(dim=(1, 3, 4))], 1))
    return y


@_impl("conv2d_dgrad")
def _conv2d_dgrad_cpu(dy, w, stride, pad, H, W, residual=None, wds=None):  # wds: GPU-side cache
    shape = (dy.shape[0], w.shape[1], H, W)
    dx = torch.nn.grad.conv2d_input(shape, w.float(), dy.float(), stride=stride, padding=pad)
    if residual is not None:
        dx = dx + residual.float()
    return dx.to(dy.dtype).contiguous(memory_format=torch.channels_last)


@_impl("conv2d_dgrad_bn")
def _conv2d_dgrad_bn_cpu(dy, w, stride, pad, H, W, residual, x, y, mean, rstd, gamma, beta, sums, groups, wds=None):
    g = _conv2d_dgrad_cpu(dy, w, stride, pad, H, W, residual).float()
    G, C = groups, x.shape[1]
    shp = (G, x.shape[0] // G, C, H, W)
    xf = x.float().reshape(shp)
    mu, rs = mean.reshape(G, 1, C, 1, 1), rstd.reshape(G, 1, C, 1, 1)
    if y is not None:
        live = y.float().reshape(shp) > 0
    else:
        sc = gamma.view(1, 1, C, 1, 1) * rs
        live = xf * sc + (beta.view(1, 1, C, 1, 1) - mu * sc) > 0
    gg = torch.where(live, g.reshape(shp), torch.zeros((), dtype=torch.float32))
    sums.view(G, 2, C).add_(torch.stack([gg.sum((1, 3, 4)), (gg * (xf - mu) * rs).sum((1, 3, 4))], 1))
    return gg.reshape(x.shape).to(dy.dtype).contiguous(memory_format=torch.channels_last), True


@_impl("bn_bwd_prep")
def _bn_bwd_prep_cpu(g, x, y, mean, rstd, gamma, beta, sums, groups):
    G, C, H, W = groups, x.shape[1], x.shape[2], x.shape[3]
    shp = (G, x.shape[0] // G, C, H, W)
    xf, mu, rs = x.float().reshape(shp), mean.reshape(G, 1, C, 1, 1), rstd.reshape(G, 1, C, 1, 1)
    if y is not None:
        live = y.float().reshape(shp) > 0
    else:
        sc = gamma.view(1, 1, C, 1, 1) * rs
        live = xf * sc + (beta.view(1, 1, C, 1, 1) - mu * sc) > 0
    gg = torch.where(live, g.float().reshape(shp), torch.zeros((), dtype=torch.float32))
    sums.view(G, 2, C).add_(torch.stack([gg.sum((1, 3, 4)), (gg * (xf - mu) * rs).sum((1, 3, 4))], 1))
    g.copy_(gg.reshape(g.shape))
    return g


@_impl("im2col_stem")
def _im2col_stem_cpu(x, R, S, stride, pad):
    # the GPU builds the stem's column matrix once per pass for the forward and the weight gradient;
    # the CPU implementations convolve the image directly, so the "column matrix" they hand through
    # is (a copy of) the image itself (conv2d_wgrad(cols=...) below reads it back)
    return x.clone()


@_impl("conv2d_dgrad_weights")
def _conv2d_dgrad_weights_cpu(w, stride, pad):
    # per parity class (a, b) of a stride-s conv, the contributing taps, transposed to [C][R'][S'][K]
    # (the same tensors as the GPU op; the CPU data gradient does not need them)
    wk = w.permute(0, 2, 3, 1)
    R, S = wk.shape[1], wk.shape[2]
    out = []
    for a in range(stride):
        for b in range(stride):
            r0, s0 = (a + pad) % stride, (b + pad) % stride
            if r0 < R and s0 < S:
                out.append(wk[:, r0::stride, s0::stride, :].permute(3, 1, 2, 0).contiguous())
            else:
                out.append(torch.empty(0, dtype=w.dtype))
    return out


@_impl("conv2d_dgrad_weights_batched")
def _conv2d_dgrad_weights_batched_cpu(ws, strides, pads):
    out = []
    for w, st, pd in zip(ws, strides, pads):
        out += _conv2d_dgrad_weights_cpu(w, st, pd)
    return out


@_impl("conv2d_wgrad")
def _conv2d_wgrad_cpu(dy, x, dw, stride, pad, cols=None):
    src = cols if cols is not None and cols.dim() == 4 else x  # the stem: im2col_stem handed the image
    dw.add_(torch.nn.grad.conv2d_weight(src.float(), dw.shape, dy.float(), stride=stride, padding=pad))


@_impl("bn_bwd")
def _bn_bwd_cpu(dy, y, x, mean, rstd, gamma, relu, want_dres, sums=None, dgamma_acc=None, dbeta_acc=None,
                beta=None, stats_ready=False):  # beta: the GPU kernels' ReLU mask from x; the reference reads y
    # (stats_ready: dy arrives masked — masking it again by y > 0 changes nothing)
    mean2 = mean.reshape(-1, x.shape[1])
    rstd2 = rstd.reshape(-1, x.shape[1])
    G = mean2.shape[0]
    g = dy.float()
    if relu:
        g = torch.where(y.float() > 0, g, torch.zeros_like(g))
    gg = g.reshape(G, x.shape[0] // G, *x.shape[1:])
    xh = (x.float().reshape(gg.shape) - mean2[:, None, :, None, None]) * rstd2[:, None, :, None, None]
    sb = gg.sum(dim=(1, 3, 4))                       # [G, C]
    sgx = (gg * xh).sum(dim=(1, 3, 4))
    R = gg[0].numel() // x.shape[1]
    dx = (gamma * rstd2)[:, None, :, None, None] * (gg - (sb / R)[:, None, :, None, None]
                                                    - xh * (sgx / R)[:, None, :, None, None])
    cl = torch.channels_last
    dres = g.to(x.dtype).contiguous(memory_format=cl) if want_dres else torch.empty(0, dtype=x.dtype)
    dxo = dx.reshape(x.shape).to(x.dtype).contiguous(memory_format=cl)
    if dgamma_acc is not None and dbeta_acc is not None:
        dgamma_acc.add_(sgx.sum(0))
        dbeta_acc.add_(sb.sum(0))
        return dxo, dres, torch.empty(0), torch.empty(0)
    return dxo, dres, sgx.sum(0), sb.sum(0)
