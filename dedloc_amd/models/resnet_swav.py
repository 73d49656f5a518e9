"""SwAV ResNet-50 (vissl trunk + swav_head) for the collaborative SwAV experiment.

Reference: ``swav/vissl/vissl/models/trunks/resnext.py:48-172``
(torchvision Bottleneck ResNet-50, depth 50, width 1), ``swav_prototypes_head.py:10-112``
(MLP 2048-2048(BN,ReLU)-128, L2 normalisation, 3000 prototypes without bias),
``base_ssl_model.py:76-105`` (one trunk pass per crop with SINGLE_PASS_EVERY_CROP, features
concatenated before the head).

MI355X-first choices: channels-last bf16 activations (fp32 master weights live in the flat parameter
buffer and receive their gradients in place), optional per-resolution batching of the crops
(``single_pass_every_crop=False``: 2 trunk passes instead of 8), optional activation checkpointing
per stage (off by default: 288 GB HBM makes the recompute pointless).
Parameter names match torchvision/vissl (``trunk.*``, ``heads.0.*``) for checkpoint interchange.

One code path on every device: each op of the model is a ``torch.ops.dedloc`` operator — the HIP
kernels on the GPU, the CPU implementations registered under the CPU dispatch key in
``ops/_lib.py`` (the plumbing configuration) — exactly like the ALBERT model.  There is no stock
module fallback: an input outside a kernel's contract (not channels-last bf16, an unsupported conv
form) raises.  The BatchNorm statistics ride in the producing convolution's epilogue, the identity
branch's gradient in conv1's data-gradient epilogue, and each BatchNorm+ReLU's backward preparation
in the consuming 1x1 convolution's data gradient (measured in profiles/README.md, round 3).
"""
from __future__ import annotations

from typing import List, Sequence

import os

import torch
import torch.nn as nn

from .. import ops as _ops  # noqa: F401  (registers torch.ops.dedloc.*)
from torch.utils.checkpoint import checkpoint


def deterministic_bn() -> bool:
    """DEDLOC_DETERMINISTIC_BN=1: bitwise-reproducible BatchNorm statistics for parity runs — every
    statistic is one fixed-order reduction (batchnorm.hip ``bn_deterministic``: one block per
    statistics group) instead of fp32 atomics from many blocks, conv / GEMM epilogues and the
    BN-backward preparation links (their atomics from many tiles) are bypassed.  Slow; off by default."""
    return os.environ.get("DEDLOC_DETERMINISTIC_BN", "") == "1"


def join_batch(ts: Sequence[torch.Tensor]) -> torch.Tensor:
    """``torch.cat(ts)`` along the batch dimension, as a zero-copy view when the tensors already lie
    back to back in one storage with equal shapes and strides and a dense batch stride (the multi-crop
    pipeline's ``x.split(b)`` outputs, the graphed iteration's static inputs)."""
    if len(ts) == 1:
        return ts[0]
    t0 = ts[0]
    step = t0.shape[0] * t0.stride(0) * t0.element_size()
    dense = t0.dim() >= 1 and t0.stride(0) == max(1, t0[0].numel()) and (
        t0.is_contiguous() or t0.is_contiguous(memory_format=torch.channels_last))
    if dense and all(t.shape == t0.shape and t.stride() == t0.stride() and t.dtype == t0.dtype
                     and t.device == t0.device and t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr()
                     and t.data_ptr() == t0.data_ptr() + i * step for i, t in enumerate(ts)):
        return t0.as_strided((t0.shape[0] * len(ts),) + tuple(t0.shape[1:]), t0.stride())
    return torch.cat(ts)


def _require_nhwc_bf16(x: torch.Tensor, what: str) -> torch.Tensor:
    """The trunk's activation contract: channels-last bf16 (what every producing kernel writes)."""
    if x.dtype != torch.bfloat16 or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError(f"{what}: expected a channels-last bf16 activation, got {x.dtype} with strides "
                         f"{tuple(x.stride())} for shape {tuple(x.shape)}")
    return x


class _GradLink:
    """Hands the identity-branch gradient of a Bottleneck from bn3's backward (the residual input's
    gradient, which autograd would otherwise add to conv1's data gradient with a separate kernel) to
    conv1's backward, whose data-gradient GEMM adds it in its epilogue.  bn3's backward always runs
    first: conv1's backward depends on it through conv3 -> bn2 -> conv2 -> bn1."""

    __slots__ = ("g", "early")

    def __init__(self):
        self.g = None
        self.early = False  # the consumer ran before the producer (see _ConvNHWC.backward)


class _BnBwdLink:
    """Hands a BatchNorm+ReLU's backward preparation to the conv that consumes its output (1x1: the
    GEMM epilogues; 3x3 / strided: conv.hip's data-gradient epilogue).

    The BN forward records what its backward needs (its input, mean / rstd, gamma / beta, the
    pass workspace's backward sums); the consumer conv's backward then computes its data gradient
    with conv2d_dgrad_bn — the ReLU mask applied and the BN backward's two column sums accumulated in
    the GEMM epilogue — and marks the link done, so the BN backward skips its statistics pass over
    dY and X.  The BN backward always runs after that conv's: its incoming gradient is that
    conv's data gradient.  For bn3 (ReLU after the residual add) the mask comes from the BN output,
    which is the consumer's own input (the next block's conv1)."""

    __slots__ = ("bn", "done")

    def __init__(self):
        self.bn = None
        self.done = False


class _BNAct(torch.autograd.Function):
    """Training-mode BN (+ residual) (+ ReLU) on channels-last bf16 via the fused HIP kernels.

    ``ws``: this call's slices of the trunk pass's pre-zeroed statistics workspace (forward and
    backward sums; one memset per pass instead of two hipMemsetAsync launches per BatchNorm).
    With ``module.inplace_grad`` and fp32 gradient buffers bound to gamma / beta (the flat
    gradient), the backward adds dgamma / dbeta into them directly, like the conv weight gradients,
    so autograd launches no per-pass accumulation adds."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, running_mean, running_var, relu, eps, momentum, groups, ws, module,
                stats_ready=False, link=None, bwd_link=None):
        y, mean, rstd = torch.ops.dedloc.bn_fwd(x, res, gamma, beta, running_mean, running_var, eps, momentum, relu,
                                                groups, None if ws is None else ws[0], stats_ready)
        ctx.save_for_backward(x, y, mean, rstd, gamma, beta)
        ctx.relu, ctx.has_res, ctx.ws, ctx.module = relu, res is not None, ws, module
        ctx.gslot = getattr(module, "_gslot", None)  # a concurrent second pass's gradient buffers
        ctx.link = link if res is not None else None
        ctx.bwd_link = None
        if bwd_link is not None and relu and ws is not None:
            bwd_link.bn = (x, mean, rstd, gamma, beta, ws[1], groups, res is not None)
            bwd_link.done = False
            ctx.bwd_link = bwd_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd, gamma, beta = ctx.saved_tensors
        m = ctx.module
        gw, gb = (m.weight.grad, m.bias.grad) if m is not None else (None, None)
        if ctx.gslot is not None:  # a concurrent trunk pass: its own gradient buffer (SwAVModel)
            gw, gb = ctx.gslot
        acc = (m is not None and m.inplace_grad and gw is not None and gb is not None
               and gw.dtype == torch.float32 and gb.dtype == torch.float32)
        # the consuming conv's epilogue prepared dy (ReLU-masked) and the backward sums (_BnBwdLink)
        ready = ctx.bwd_link is not None and ctx.bwd_link.done
        if ready:
            ctx.bwd_link.done = False
        dx, dres, dgamma, dbeta = torch.ops.dedloc.bn_bwd(dy, y, x, mean, rstd, gamma, ctx.relu, ctx.has_res,
                                                          None if ctx.ws is None else ctx.ws[1],
                                                          gw if acc else None, gb if acc else None,
                                                          # BN+ReLU without a residual: ReLU mask from x, y unread
                                                          beta if (ctx.relu and not ctx.has_res) else None,
                                                          ready)
        if acc:
            dgamma = dbeta = None
        if ctx.link is not None:  # the residual's gradient rides in conv1's data-gradient epilogue
            ctx.link.g, dres = dres, None
        return (dx, dgamma, dbeta, (dres if ctx.has_res else None), None, None, None, None, None, None, None, None,
                None, None, None)


class _ConvNHWC(torch.autograd.Function):
    """Conv2d (no bias, groups 1) on channels-last bf16 through the implicit-GEMM MFMA kernels
    (csrc/kernels/conv.hip).  The weight gradient accumulates in fp32 straight into the parameter's
    bound ``.grad`` (the flat gradient buffer, KRSC layout) when there is one, like the ALBERT layer."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, module, stats=None, groups=1, link=None, bn_link=None, give=None):
        # bf16 copy of the weight (keeps the channels-last KRSC strides), shared by the trunk passes
        # of one SwAVModel.forward (one cast per iteration instead of one per resolution group); the
        # model clears the cache at the start and end of every forward, so an optimizer update
        # between iterations can never be missed
        wb = getattr(module, "_wb_cache", None)
        if wb is None:
            wb = weight.detach().to(torch.bfloat16)
            if module._wb_share:
                module._wb_cache = wb
        # the stem (3 input channels): its im2col column matrix is built once here and kept for the
        # weight gradient (the input image needs no gradient, so the matrix replaces it)
        cols = None
        if x.shape[1] % 64 and not x.requires_grad:
            cols = torch.ops.dedloc.im2col_stem(x, wb.shape[2], wb.shape[3], stride, pad)
        ctx.save_for_backward(x if cols is None else cols, wb)
        ctx.stride, ctx.pad, ctx.module = stride, pad, module
        ctx.has_cols, ctx.xshape, ctx.link, ctx.bn_link = cols is not None, tuple(x.shape), link, bn_link
        ctx.give = give
        ctx.gslot = getattr(module, "_gslot", None)  # a concurrent second pass's weight-gradient buffer
        if stats is not None:  # the consuming BatchNorm's statistics, accumulated by the conv's epilogue
            return torch.ops.dedloc.conv2d_fwd_stats(x, wb, stride, pad, stats, groups, cols)
        return torch.ops.dedloc.conv2d_fwd(x, wb, stride, pad, cols)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        cols = None
        if ctx.has_cols:  # stem: x is only consulted for its shape
            cols = x
            x = torch.empty((), dtype=torch.bfloat16, device=dy.device).expand(ctx.xshape)
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = None
        wds = _dgrad_weights(ctx.module, wb, ctx.stride, ctx.pad) if ctx.needs_input_grad[0] else None
        if ctx.needs_input_grad[0]:
            res = None
            if ctx.link is not None:  # + the block's identity-branch gradient (see _GradLink)
                res, ctx.link.g = ctx.link.g, None
                if res is None:  # the producer has not run (yet): it returns its gradient itself
                    ctx.link.early = True
            bl = ctx.bn_link
            if bl is not None and bl.bn is not None:  # + the producing BN's backward preparation (_BnBwdLink)
                bx, mean, rstd, gamma, beta, sums, G, has_res = bl.bn
                dx, bl.done = torch.ops.dedloc.conv2d_dgrad_bn(dy, wb, ctx.stride, ctx.pad, x.shape[2], x.shape[3],
                                                               res, bx, x if has_res else None, mean, rstd, gamma,
                                                               beta, sums, G, wds)
            else:
                dx = torch.ops.dedloc.conv2d_dgrad(dy, wb, ctx.stride, ctx.pad, x.shape[2], x.shape[3], res, wds)
        if ctx.give is not None and dx is not None and not ctx.give.early:
            # a downsample block's shortcut conv: its data gradient rides in conv1's data-gradient
            # epilogue (conv1 runs later: see Bottleneck.forward) instead of an autograd add of two
            # activation-sized tensors
            ctx.give.g, dx = dx, None
        dw = None
        if ctx.needs_input_grad[1]:
            weight = ctx.module.weight
            g = weight.grad if ctx.gslot is None else ctx.gslot
            if (g is not None and ctx.module.inplace_wgrad and g.dtype == torch.float32
                    and g.permute(0, 2, 3, 1).is_contiguous()):
                torch.ops.dedloc.conv2d_wgrad(dy, x, g, ctx.stride, ctx.pad, cols)  # in place, no AccumulateGrad
            else:
                dw = torch.zeros(weight.shape, dtype=torch.float32, device=weight.device).contiguous(
                    memory_format=torch.channels_last)
                torch.ops.dedloc.conv2d_wgrad(dy, x, dw, ctx.stride, ctx.pad, cols)
                dw = dw.to(weight.dtype)
        return dx, dw, None, None, None, None, None, None, None, None


def _dgrad_weights(module, wb, stride, pad):
    """The tap-transposed data-gradient weights of a conv that takes the implicit-GEMM data-gradient
    path (3x3 and strided convs, 1x1 convs with at most 128 input channels), computed once per
    SwAVModel iteration (``module._wd_token``, renewed by every SwAVModel.forward) and shared by the
    backward of both trunk passes; None elsewhere (the op then transposes per call)."""
    k = wb.shape[2]
    if k == 1 and stride == 1 and (wb.shape[1] > 128 or wb.shape[0] % 64):
        return None  # the 1x1 GEMM route reads the weight as it is
    token = getattr(module, "_wd_token", None)
    if token is None:
        return None
    cached = getattr(module, "_wd_cache", None)
    if cached is not None and cached[0] is token:
        return cached[1]
    wds = torch.ops.dedloc.conv2d_dgrad_weights(wb, stride, pad)
    module._wd_cache = (token, wds)
    return wds


def _dgrad_weights_all(convs):
    """_dgrad_weights of every conv of one iteration that takes precomputed data-gradient weights,
    as ONE batched transpose launch (conv.hip wt_transpose_kernel) instead of one strided-permute
    copy kernel per conv and parity class; the per-conv lists are views of one buffer."""
    todo = []
    for m in convs:
        wb, token = m._wb_cache, getattr(m, "_wd_token", None)
        if wb is None or token is None:
            continue
        K, C, k = wb.shape[0], wb.shape[1], wb.shape[2]
        if k == 1 and m.stride[0] == 1 and (C > 128 or K % 64):
            continue  # the 1x1 GEMM route reads the weight as it is
        if K % 64 or C % 64:
            continue  # the stem: its input takes no gradient
        cached = getattr(m, "_wd_cache", None)
        if cached is not None and cached[0] is token:
            continue
        todo.append(m)
    if not todo:
        return
    outs = torch.ops.dedloc.conv2d_dgrad_weights_batched([m._wb_cache for m in todo], [m.stride[0] for m in todo],
                                                          [m.padding[0] for m in todo])
    i = 0
    for m in todo:
        n = m.stride[0] ** 2
        m._wd_cache = (m._wd_token, list(outs[i:i + n]))
        i += n


class ConvNHWC(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state-dict keys) on the dedloc conv operators (forward,
    dgrad, wgrad): on the GPU the implicit-GEMM MFMA convolution (conv.hip) for 3x3 and strided convs
    and the tiled GEMM kernels (gemm8.hip / gemm.hip) for the 1x1 convs and the stem's im2col matrix;
    on the CPU their registered CPU implementations.  The input is brought to channels-last bf16
    (the trunk's entry takes the images as they come).  There is no MIOpen path."""

    _wb_cache = None    # bf16 weight shared across the trunk passes of one model forward
    _wb_share = False   # set by SwAVModel.forward for the duration of that forward
    _gslot = None       # weight-gradient target of a concurrent second trunk pass (SwAVModel)
    # False: return the weight gradient through autograd instead of adding it into the bound .grad
    # (HIP-graph capture via make_graphed_callables needs every parameter to receive an autograd grad)
    inplace_wgrad = True
    # False: the consuming BatchNorm runs its own statistics pass (tests compare the two orders)
    epilogue_stats = True

    def forward(self, x, bn=None, link=None, bn_link=None, give=None):
        """``bn``: the BNAct that consumes this output.  When it will take its fused path with a
        pass workspace, the conv's epilogue accumulates that BatchNorm's batch statistics and the BN
        forward skips its own statistics pass over the tensor.  ``link``: a _GradLink whose gradient the
        data-gradient epilogue adds (Bottleneck conv1).  ``bn_link``: the _BnBwdLink of the
        BatchNorm+ReLU that produced ``x`` (its backward preparation rides in this conv's data
        gradient).  ``give``: a _GradLink that takes this conv's data gradient instead of autograd
        (a downsample block's shortcut conv, consumed by conv1's data-gradient epilogue)."""
        if not (self.bias is None and self.groups == 1 and self.dilation == (1, 1)
                and self.stride[0] == self.stride[1] and self.padding[0] == self.padding[1]
                and self.padding_mode == "zeros"):
            raise NotImplementedError("ConvNHWC: only the ResNet-50 conv forms (no bias, groups 1, square "
                                      "stride/padding) have kernels")
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if bn is not None and self.epilogue_stats and bn.takes_conv_stats() and not deterministic_bn():
            bn.stats_ready = True
            return _ConvNHWC.apply(x, self.weight, self.stride[0], self.padding[0], self, bn.pass_ws[0],
                                   bn.stat_groups, link, bn_link, give)
        return _ConvNHWC.apply(x, self.weight, self.stride[0], self.padding[0], self, None, 1, link, bn_link,
                               give)


class BNAct(nn.BatchNorm2d):
    """BatchNorm2d with the Bottleneck epilogue fused: ``act(BN(x) [+ res])``.

    Same parameters / buffers / state-dict keys as ``nn.BatchNorm2d``.  In training it runs the
    fused BN operators (csrc/kernels/batchnorm.hip on the GPU: 2 kernels forward, 2 backward, ReLU
    and the residual add folded in) on channels-last bf16 activations; in evaluation the running
    statistics as one scale / shift (``_bn_eval``).
    """

    # False: return dgamma / dbeta through autograd (HIP-graph capture needs an autograd grad for
    # every parameter); True: accumulate into the bound fp32 .grad buffers in the kernel
    inplace_grad = True
    _gslot = None        # (dgamma, dbeta) targets of a concurrent second trunk pass (SwAVModel)
    _rs_override = None  # (running_mean, running_var) stand-ins of that pass (deferred update)

    def __init__(self, num_features, relu: bool = False):
        super().__init__(num_features)
        self.relu = relu
        self.stat_groups = 1  # >1: the batch holds that many crops, each normalised with its own stats
        self.pass_ws = None   # set by ResNet50Trunk.forward: (fwd sums, bwd sums) slices, pre-zeroed
        self.count_deferred = False  # num_batches_tracked is advanced by the trunk, one launch per pass
        self.stats_ready = False  # the producing conv accumulated this call's statistics into pass_ws[0]

    def takes_conv_stats(self) -> bool:
        """True when this BN's next forward runs over a pre-zeroed pass workspace, so the conv
        producing its input can accumulate the batch statistics in its epilogue."""
        return self.training and self.pass_ws is not None

    def forward(self, x, res=None, link=None, bwd_link=None):
        if not self.training:
            self.stats_ready = False
            return _bn_eval(self, x, res, self.relu)
        _require_nhwc_bf16(x, "BNAct input")
        if res is not None:
            _require_nhwc_bf16(res, "BNAct residual")
        G = self.stat_groups
        if not self.count_deferred:
            self.num_batches_tracked.add_(G)
        ws, self.pass_ws = self.pass_ws, None
        ready, self.stats_ready = self.stats_ready and ws is not None, False
        rm, rv = self._rs_override or (self.running_mean, self.running_var)
        return _BNAct.apply(x, self.weight, self.bias, res, rm, rv, self.relu,
                            self.eps, self.momentum, G, ws, self, ready, link, bwd_link)


def _bn_eval(m, x, res, relu: bool):
    """Inference BatchNorm with the running statistics: y = x * scale + shift (+ res) (ReLU), as one
    broadcast expression in the input's layout (not on the training path)."""
    scale = m.weight.float() * torch.rsqrt(m.running_var.float() + m.eps)
    shift = m.bias.float() - m.running_mean.float() * scale
    shp = (1, -1) + (1,) * (x.dim() - 2)
    y = x.float() * scale.view(shp) + shift.view(shp)
    if res is not None:
        y = y + res.float()
    if relu:
        y = y.clamp_min(0)
    return y.to(x.dtype)


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, arg = torch.ops.dedloc.maxpool_fwd(x)
        ctx.save_for_backward(arg)
        ctx.hw = (x.shape[2], x.shape[3])
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        return torch.ops.dedloc.maxpool_bwd(dy, arg, *ctx.hw)


class MaxPool3x3s2(nn.MaxPool2d):
    """The stem's MaxPool2d(3, stride 2, padding 1) on channels-last bf16 activations (pool.hip on
    the GPU; the backward routes each gradient to its window's recorded maximum)."""

    def __init__(self):
        super().__init__(3, stride=2, padding=1)

    def forward(self, x):
        return _MaxPool.apply(_require_nhwc_bf16(x, "max-pool input"))


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return torch.ops.dedloc.avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return torch.ops.dedloc.avgpool_bwd(dy.to(torch.bfloat16), *ctx.hw)


def global_avgpool(x):
    """AdaptiveAvgPool2d(1) + flatten -> [N, C] of channels-last bf16 activations (pool.hip)."""
    return _AvgPool.apply(_require_nhwc_bf16(x, "average-pool input"))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = ConvNHWC(inplanes, planes, 1, bias=False)
        self.bn1 = BNAct(planes, relu=True)
        self.conv2 = ConvNHWC(planes, planes, 3, stride=stride, padding=1, bias=False)  # ResNet v1.5
        self.bn2 = BNAct(planes, relu=True)
        self.conv3 = ConvNHWC(planes, planes * 4, 1, bias=False)
        self.bn3 = BNAct(planes * 4, relu=True)  # relu(bn3(conv3) + identity), add fused
        self.downsample = downsample

    def forward(self, x):
        link = None
        # the previous block's bn3 backward preparation can ride in conv1's data gradient only when
        # that gradient is the whole gradient of x: identity block, identity gradient linked in
        in_link = getattr(x, "_dedloc_bn_link", None)
        fused_bwd = x.requires_grad and torch.is_grad_enabled() and not deterministic_bn()
        # bn1's backward preparation stays in the BN backward: in the 3x3 conv2's data-gradient
        # epilogue the extra X reads cost what its statistics pass saves (profiles/README.md r3)
        if self.downsample is None:
            idt = x
            if fused_bwd:
                link = _GradLink()
            out = self.bn1(self.conv1(x, self.bn1, link, in_link if link is not None else None))
        else:
            # the shortcut branch is built AFTER conv1, so autograd (highest sequence number first)
            # runs its backward first and the shortcut conv's data gradient can ride in conv1's
            # data-gradient epilogue (a GEMM residual) instead of a separate add; _GradLink.early
            # keeps either order correct
            # (bn3's `link` stays None: idt is not x here)
            slink = _GradLink() if fused_bwd and SwAVModel.shortcut_grad_link else None
            out = self.bn1(self.conv1(x, self.bn1, slink))
            conv, bn = self.downsample[0], self.downsample[1]
            idt = bn(conv(x, bn, give=slink))
        l2 = _BnBwdLink() if fused_bwd else None
        out = self.bn2(self.conv2(out, self.bn2), bwd_link=l2)
        l3 = _BnBwdLink() if fused_bwd else None
        y = self.bn3(self.conv3(out, self.bn3, bn_link=l2), idt, link, bwd_link=l3)
        if l3 is not None:
            y._dedloc_bn_link = l3
        return y


class ResNet50Trunk(nn.Module):
    pass_workspace = True  # False: per-call BN statistics memsets and counter adds (A/B, tests)

    def __init__(self, layers=(3, 4, 6, 3), zero_init_residual=False, checkpoint_stages: bool = False):
        super().__init__()
        self.inplanes = 64
        self.conv1 = ConvNHWC(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BNAct(64, relu=True)
        self.maxpool = MaxPool3x3s2()
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.checkpoint_stages = checkpoint_stages
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes BNAct
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _make_layer(self, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(ConvNHWC(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                 BNAct(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def alloc_bn_pass(self, x, count: bool = True):
        """One zeroed workspace for every BatchNorm's forward and backward statistics sums of the
        pass over ``x`` (with the BatchNorms' current stat_groups), and one multi-tensor add for their
        num_batches_tracked counters (instead of two memsets and one add launch per BatchNorm; each
        is a ~5 us kernel at b=64).  Returns the per-BatchNorm workspace slices for ``forward``'s
        ``prepared`` (None: the per-call path).  ``count=False``: the caller adds the counters."""
        if not self.pass_workspace or not self.training or self.checkpoint_stages:
            return None
        bns = self._bn_modules()
        G = bns[0].stat_groups
        sizes = [2 * G * m.num_features for m in bns]
        ws = torch.zeros(2 * sum(sizes), dtype=torch.float32, device=x.device)
        out, off = [], 0
        for n in sizes:
            out.append((ws[off:off + n], ws[off + n:off + 2 * n]))
            off += 2 * n
        if count:
            torch._foreach_add_([m.num_batches_tracked for m in bns], G)
        return out

    def _prepare_bn_pass(self, x, prepared=None):
        if prepared is None:
            prepared = self.alloc_bn_pass(x)
        for i, m in enumerate(self._bn_modules()):
            if prepared is None:
                m.count_deferred, m.pass_ws = False, None
            else:
                m.count_deferred, m.pass_ws = True, prepared[i]

    def _bn_modules(self):
        bns = getattr(self, "_bns", None)
        if bns is None:
            bns = self._bns = [m for m in self.modules() if isinstance(m, BNAct)]
        return bns

    def forward(self, x, prepared=None):
        """``prepared``: this pass's BatchNorm workspaces from ``alloc_bn_pass`` (allocated ahead,
        e.g. on another stream); None allocates them here."""
        self._prepare_bn_pass(x, prepared)
        x = self.maxpool(self.bn1(self.conv1(x, self.bn1)))
        for stage in (self.layer1, self.layer2, self.layer3, self.layer4):
            if self.checkpoint_stages and self.training and x.requires_grad:
                x = checkpoint(stage, x, use_reentrant=False)
            else:
                x = stage(x)
        return global_avgpool(x)


class _HeadLinearFn(torch.autograd.Function):
    """y = x W^T (+ b) on the dedloc GEMM kernels (bf16 in/out, fp32 accumulation); the weight and
    bias gradients accumulate in fp32 straight into the parameters' bound ``.grad`` (the flat
    gradient buffer) when there is one, like the conv weight gradients."""

    @staticmethod
    def forward(ctx, x, weight, bias, module):
        wb = module._wb_cache if module._wb_cache is not None else weight.detach().to(torch.bfloat16)
        ctx.save_for_backward(x, wb)
        ctx.module, ctx.has_bias = module, bias is not None
        return torch.ops.dedloc.gemm(x, wb, None if bias is None else bias.detach(), None, False, True, 0)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        m = ctx.module
        dx = torch.ops.dedloc.gemm(dy, wb, None, None, False, False, 0) if ctx.needs_input_grad[0] else None
        dw = db = None
        g = m.weight.grad
        if m.inplace_grad and g is not None and g.dtype == torch.float32 and g.is_contiguous():
            torch.ops.dedloc.gemm_acc_f32(dy, x, g, True, False)
        else:
            dw = torch.zeros(m.weight.shape, dtype=torch.float32, device=dy.device)
            torch.ops.dedloc.gemm_acc_f32(dy, x, dw, True, False)
            dw = dw.to(m.weight.dtype)
        if ctx.has_bias:
            gb = m.bias.grad
            if m.inplace_grad and gb is not None and gb.dtype == torch.float32:
                torch.ops.dedloc.bias_grad(dy, gb, True)
            else:
                db = torch.zeros(m.bias.shape, dtype=torch.float32, device=dy.device)
                torch.ops.dedloc.bias_grad(dy, db, True)
                db = db.to(m.bias.dtype)
        return dx, dw, db, None


class HeadLinear(nn.Linear):
    """``nn.Linear`` (same parameters / keys) on the dedloc GEMM operators (bf16, fp32 accumulation)."""

    inplace_grad = True
    _wb_cache = None  # bf16 weight view set by SwAVModel.forward (the flat buffer's bf16 mirror)

    def forward(self, x):
        return _HeadLinearFn.apply(x.to(torch.bfloat16).contiguous(), self.weight, self.bias, self)


class HeadBN1dReLU(nn.BatchNorm1d):
    """``BatchNorm1d`` + ReLU of the projection MLP (same keys as BatchNorm1d) through the fused BN
    kernels of the trunk: the [N, C] batch is BN over N rows of a 1x1 channels-last image."""

    inplace_grad = True
    stat_groups = 1

    def forward(self, x):
        if not self.training:
            return _bn_eval(self, x, None, True)
        if x.dtype != torch.bfloat16 or x.dim() != 2 or not x.is_contiguous():
            raise ValueError(f"HeadBN1dReLU: expected a contiguous [N, C] bf16 input, got {x.dtype} {tuple(x.shape)}")
        N, C = x.shape
        self.num_batches_tracked.add_(1)
        y = _BNAct.apply(x.view(N, C, 1, 1), self.weight, self.bias, None, self.running_mean, self.running_var,
                         True, self.eps, self.momentum, 1, None, self)
        return y.view(N, C)


class _L2Norm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        y, rinv = torch.ops.dedloc.l2norm_fwd(x, eps)
        ctx.save_for_backward(y, rinv)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, rinv = ctx.saved_tensors
        return torch.ops.dedloc.l2norm_bwd(dy, y, rinv), None


def l2_normalize(x, eps: float = 1e-12):
    """F.normalize(x, p=2, dim=1) of [N, D] rows, D <= 1024 (pool.hip on the GPU)."""
    if x.dim() != 2 or x.shape[1] > 1024:
        raise ValueError(f"l2_normalize: rows of at most 1024 values, got {tuple(x.shape)}")
    return _L2Norm.apply(x.to(torch.bfloat16).contiguous(), eps)


class SwAVPrototypesHead(nn.Module):
    """MLP [2048, 2048, 128] with BN+ReLU, L2 normalisation, prototypes 128 -> 3000 (no bias)
    (vissl swav_prototypes_head.py:61-112; module names and state-dict keys as there).  On the GPU
    every op is a dedloc kernel: the GEMMs, BN1d+ReLU (batchnorm.hip) and the L2 normalisation."""

    def __init__(self, dims: Sequence[int] = (2048, 2048, 128), num_prototypes: int = 3000, use_bn: bool = True):
        super().__init__()
        layers: List[nn.Module] = []
        for i in range(len(dims) - 2):
            layers += [HeadLinear(dims[i], dims[i + 1])]
            layers += [HeadBN1dReLU(dims[i + 1]) if use_bn else nn.ReLU(inplace=True)]
            if use_bn:
                layers += [nn.Identity()]  # the ReLU is fused into the BN kernel (keeps vissl's indices)
        layers += [HeadLinear(dims[-2], dims[-1])]
        self.projection_head = nn.Sequential(*layers)
        self.prototypes0 = HeadLinear(dims[-1], num_prototypes, bias=False)

    def forward(self, x):
        emb = l2_normalize(self.projection_head(x))
        return emb, self.prototypes0(emb)


class SwAVModel(nn.Module):
    def __init__(self, num_prototypes: int = 3000, single_pass_every_crop: bool = True,
                 checkpoint_stages: bool = False, conv_impl: str | None = None):
        super().__init__()
        self.trunk = ResNet50Trunk(checkpoint_stages=checkpoint_stages)
        self.heads = nn.ModuleList([SwAVPrototypesHead(num_prototypes=num_prototypes)])
        self.single_pass_every_crop = single_pass_every_crop
        self._flat = None  # FlatParams with a bf16 mirror (bind_flat)
        if conv_impl not in (None, "hip", "auto"):  # "auto": round-2 configs (it chose MIOpen per shape)
            raise ValueError(f"conv backend must be 'hip' (the hand-written kernels), got {conv_impl!r}")

    # Two concurrent trunk passes (set by a trainer that calls ``after_backward`` after every
    # backward): the resolution groups (2x224 and 6x96 crops) are independent through the trunk, and
    # at b=64 many of their kernels leave most of the chip idle, so the second pass runs on a side
    # stream (forward and, through autograd's per-op streams, backward).  What the passes share is
    # made race-free: the bf16 weights and the data-gradient weights are prepared before the fork;
    # both passes' BatchNorm workspaces and counters are allocated ahead on this stream; the second
    # pass writes its weight / BN-parameter gradients into a buffer of its own (added into the flat
    # gradient by after_backward) and its running-statistics updates into zeroed stand-ins (merged
    # after the join: the update is affine, rm <- (1-m)^G rm + D, so the crop order is kept).
    concurrent_passes = False
    pass_splits = (2, 1)  # concurrent passes per resolution group (_pass_plan; SwavPeer's default)
    # where _trunk_concurrent prepares the data-gradient weights: False = the main stream, ahead of
    # the fork (the default since they are one batched launch: +0.5% over a stream of their own,
    # profiles/r6_swav_dgrad_weights_stream_ab.jsonl; with 41 copy kernels the own stream won +1.8% in
    # round 4), True = a stream of their own, "side" = the first side pass's stream (the layout whose
    # graphed run crashed in round 4 through a self-wait; kept selectable for its test)
    dgrad_weights_stream = False
    # the side passes' running-statistics merge on the weight-preparation stream (1) or on the stream
    # that prepared the weights (0: the main stream by default); a measurement switch
    rs_merge_side = 1
    # a downsample block's shortcut-conv data gradient rides in conv1's data-gradient epilogue (the
    # GEMM residual) instead of an autograd add of two activation-sized tensors (0: the plain add;
    # a measurement switch for bench/swav_step.py --model_attr)
    shortcut_grad_link = 1
    # the data-gradient weights of all convs in one batched transpose launch (0: one permute-copy
    # kernel per conv and parity class; a measurement switch for bench/swav_step.py --model_attr)
    batched_dgrad_weights = 1

    def bind_flat(self, flat):
        """Take the GEMM / conv weights of every forward from ``flat``'s bf16 mirror: one cast
        kernel over the whole flat buffer per iteration instead of one per conv and linear layer."""
        self._flat = flat if getattr(flat, "bf16", None) is not None else None
        self._wb_names = [(m, f"{n}.weight") for n, m in self.named_modules()
                          if isinstance(m, (ConvNHWC, HeadLinear))]
        self._conc = None

    def _conc_state(self, sides: int):
        """Per side pass: a HIP stream, a flat-gradient-shaped buffer for its weight / BN-parameter
        gradients and zeroed running-statistics stand-ins (created once per number of side passes)."""
        c = getattr(self, "_conc", None)
        if c is None or len(c["passes"]) != sides:
            flat = self._flat
            bns = self.trunk._bn_modules()
            passes = []
            # every side pass's gradient buffer as one row of a [sides, n] buffer (after_backward
            # folds all of them into the flat gradient and clears them in one pass)
            gb_all = torch.zeros((sides, flat.grad.numel()), dtype=flat.grad.dtype, device=flat.grad.device)
            for si in range(sides):
                gb = gb_all[si].view_as(flat.grad)
                slots = []
                for n, m in self.trunk.named_modules():
                    if isinstance(m, ConvNHWC):
                        slots.append((m, flat.view(gb, f"trunk.{n}.weight")))
                    elif isinstance(m, BNAct):
                        slots.append((m, (flat.view(gb, f"trunk.{n}.weight"), flat.view(gb, f"trunk.{n}.bias"))))
                rs = torch.zeros(2 * sum(m.num_features for m in bns), dtype=torch.float32, device=gb.device)
                views, off = [], 0
                for m in bns:
                    C = m.num_features
                    views.append((rs[off:off + C], rs[off + C:off + 2 * C]))
                    off += 2 * C
                passes.append({"grad_b": gb, "slots": slots, "rs": rs, "rs_views": views,
                               "stream": torch.cuda.Stream(gb.device)})
            c = self._conc = {"passes": passes, "pending": False, "grad_all": gb_all,
                              "wprep": torch.cuda.Stream(flat.grad.device)}
        return c

    def _pass_plan(self, groups):
        """The trunk passes of one forward: each resolution group, or — ``pass_splits[i]`` > 1 and one
        statistics group per crop — that group cut into ``pass_splits[i]`` passes of whole crops
        (per-crop BatchNorm statistics make the cut exact)."""
        out = []
        for i, (x, g) in enumerate(groups):
            s = self.pass_splits[i] if i < len(self.pass_splits) else 1
            if s > 1 and g > 1 and g % s == 0:
                n = x.shape[0] // s
                out += [(x[j * n:(j + 1) * n], g // s) for j in range(s)]
            else:
                out.append((x, g))
        return out

    def _concurrent_ok(self, passes) -> bool:
        x = passes[0][0]
        return (self.concurrent_passes and len(passes) >= 2 and self._flat is not None
                and x.device.type == "cuda"  # side HIP streams
                and self.training and torch.is_grad_enabled() and ResNet50Trunk.pass_workspace
                and not self.trunk.checkpoint_stages and BNAct.inplace_grad and ConvNHWC.inplace_wgrad
                and all(m.momentum is not None for m in self.trunk._bn_modules())
                and all(g.is_contiguous(memory_format=torch.channels_last) and g.dtype == torch.bfloat16
                        for g, _ in passes))

    @staticmethod
    def _wait(a, b):
        """``a.wait_stream(b)``, skipped when they are the same stream: a stream waiting on an event
        it recorded itself is pointless eagerly, and inside a HIP-graph capture it is an event-record
        node followed by a wait on it on the same captured stream (bench/graph_selfwait_probe.py;
        the round-4 host crash of the graphed iteration had the weight copies on a side pass's stream,
        which made that pass's stream wait on itself)."""
        if a != b:
            a.wait_stream(b)

    def _trunk_concurrent(self, passes):
        c = self._conc_state(len(passes) - 1)
        cur = torch.cuda.current_stream()
        convs = [m for m in self.trunk.modules() if isinstance(m, ConvNHWC)]
        # the data-gradient weights (shared by every pass's backward; one batched transpose launch) on
        # a stream of their own, under the forward passes; each pass's stream waits for them behind
        # its forward
        wprep = (c["passes"][0]["stream"] if self.dgrad_weights_stream == "side" else
                 c["wprep"] if self.dgrad_weights_stream else cur)
        self._wait(wprep, cur)
        with torch.cuda.stream(wprep):
            if self.batched_dgrad_weights:
                _dgrad_weights_all(convs)
            else:
                for m in convs:
                    _dgrad_weights(m, m._wb_cache, m.stride[0], m.padding[0])
        users = [cur] + [sp["stream"] for sp in c["passes"]]
        for m in convs:
            for t in (getattr(m, "_wd_cache", None) or (None, ()))[1] or ():
                if t.numel():
                    for st in users:
                        t.record_stream(st)
        for sp in c["passes"]:
            self._wait(sp["stream"], cur)
        # each pass's zeroed BN workspace on its own stream; every pass's counter increments in one
        # add on the weight stream (training never reads the counters: momentum is set)
        preps = []
        for (x, g), st in zip(passes, users):
            self.set_bn_stat_groups(g)
            with torch.cuda.stream(st):
                preps.append(self.trunk.alloc_bn_pass(x, count=False))
        with torch.cuda.stream(wprep):
            torch._foreach_add_([m.num_batches_tracked for m in self.trunk._bn_modules()],
                                sum(g for _, g in passes))
        self.set_bn_stat_groups(passes[0][1])
        feats = [self.trunk(passes[0][0], preps[0])]
        self._wait(cur, wprep)  # (behind pass 0's forward) its backward reads the data-gradient weights
        bns = self.trunk._bn_modules()
        for (x, g), prep, sp in zip(passes[1:], preps[1:], c["passes"]):
            self.set_bn_stat_groups(g)
            for m, gs in sp["slots"]:
                m._gslot = gs
            for m, r in zip(bns, sp["rs_views"]):
                m._rs_override = r
            try:
                with torch.cuda.stream(sp["stream"]):
                    feats.append(self.trunk(x, prep))
                self._wait(sp["stream"], wprep)
            finally:
                for m, _ in sp["slots"]:
                    m._gslot = None
                for m in bns:
                    m._rs_override = None
        for f, sp in zip(feats[1:], c["passes"]):
            self._wait(cur, sp["stream"])
            f.record_stream(cur)
        # the side passes' running-statistics updates, in crop order, on a stream of their own under
        # the head's forward (nothing in training reads them; SwAVModel.forward joins the stream)
        ms = c["wprep"] if self.rs_merge_side else wprep
        self._wait(ms, cur)
        with torch.cuda.stream(ms), torch.no_grad():
            for (_, g), sp in zip(passes[1:], c["passes"]):
                torch._foreach_mul_([m.running_mean for m in bns], [(1.0 - m.momentum) ** g for m in bns])
                torch._foreach_add_([m.running_mean for m in bns], [v[0] for v in sp["rs_views"]])
                torch._foreach_mul_([m.running_var for m in bns], [(1.0 - m.momentum) ** g for m in bns])
                torch._foreach_add_([m.running_var for m in bns], [v[1] for v in sp["rs_views"]])
                sp["rs"].zero_()
        c["pending"] = True
        c["join"] = ms
        return feats

    def after_backward(self):
        """Add the concurrent side passes' gradients into the flat gradient (after every backward of
        a forward that ran the passes concurrently; a no-op otherwise)."""
        c = getattr(self, "_conc", None)
        if c is not None and c["pending"]:
            # a side pass's backward runs on its stream and ends there (its gradients are written in
            # place, nothing flows back): join it before reading its gradients (this also joins the
            # side streams' work into a HIP-graph capture of the backward)
            cur = torch.cuda.current_stream()
            for sp in c["passes"]:
                self._wait(cur, sp["stream"])
            torch.ops.dedloc.add_slabs_zero_(self._flat.grad, c["grad_all"])
            c["pending"] = False

    def set_bn_stat_groups(self, g: int):
        for m in self.trunk.modules():
            if isinstance(m, BNAct):
                m.stat_groups = g

    def forward(self, crops: List[torch.Tensor]):
        """crops: list of [B, 3, H, W] (channels-last) tensors -> (embeddings, scores) over all crops.

        Equal-resolution crops always run through the trunk as ONE batch.  With
        ``single_pass_every_crop`` (the reference setting) every BatchNorm still normalises each
        crop with that crop's own batch statistics (BNAct statistics groups), which is exactly what
        one trunk pass per crop computes — every other trunk op is per-sample.  Without it, BN
        statistics span the whole resolution group (original SwAV's idx_crops grouping).
        """
        convs = [m for m in self.trunk.modules() if isinstance(m, ConvNHWC)]
        token = object()  # this iteration's weights: the data-gradient weight cache key (_dgrad_weights)
        for m in convs:
            m._wb_cache, m._wb_share, m._wd_token = None, True, token
        flat = self._flat
        if flat is not None and flat.bf16.device == crops[0].device:
            flat.refresh_bf16()
            for m, n in self._wb_names:
                m._wb_cache = flat.w(n)
        try:
            return self._forward(crops)
        finally:
            for m in convs:
                m._wb_cache, m._wb_share = None, False
            for m in self.heads.modules():
                if isinstance(m, HeadLinear):
                    m._wb_cache = None

    def _forward(self, crops):
        groups, i = [], 0
        while i < len(crops):
            j = i
            while j < len(crops) and crops[j].shape[-1] == crops[i].shape[-1]:
                j += 1
            groups.append((join_batch(crops[i:j]),
                           j - i if self.single_pass_every_crop else 1))
            i = j
        passes = self._pass_plan(groups) if self.concurrent_passes else groups
        if self._concurrent_ok(passes):
            feats = self._trunk_concurrent(passes)
        else:
            feats = []
            for x, g in groups:
                self.set_bn_stat_groups(g)
                feats.append(self.trunk(x))
        self.set_bn_stat_groups(1)
        out = self.heads[0](torch.cat(feats))
        c = getattr(self, "_conc", None)
        if c is not None and c.get("join") is not None:  # the running-statistics merge (_trunk_concurrent)
            self._wait(torch.cuda.current_stream(), c["join"])
            c["join"] = None
        return out

    @torch.no_grad()
    def normalize_prototypes(self):
        """NormalizePrototypesHook (swav_hooks.py:63-92): L2-normalise every prototype row."""
        torch.ops.dedloc.row_normalize_(self.heads[0].prototypes0.weight.data)

    def prototype_param_names(self):
        return [n for n, _ in self.named_parameters() if "prototypes" in n]
