"""Implicit-GEMM NHWC convolution kernels (csrc/kernels/conv.hip) vs a plain PyTorch fp32 reference.

Shapes cover every distinct conv of the SwAV ResNet-50 trunk: the 7x7/2
3-channel stem (im2col path), 1x1 reduce/expand, 3x3 stride 1 and stride 2 (parity-class dgrad) and
the 1x1 stride-2 downsample, at small batch and both crop resolutions' spatial sizes.
"""
import pytest
import torch
import torch.nn.functional as F

import dedloc_amd.ops  # noqa: F401

CL = torch.channels_last

# (N, Cin, H, Cout, k, stride, pad)
SHAPES = [
    (2, 3, 32, 64, 7, 2, 3),        # stem (space-to-depth 4x4 conv)
    (2, 3, 33, 64, 7, 2, 3),        # stem, odd size (im2col column GEMM)
    (2, 64, 14, 64, 1, 1, 0),       # layer1 reduce
    (2, 64, 14, 64, 3, 1, 1),       # layer1 3x3
    (2, 64, 14, 256, 1, 1, 0),      # expand / downsample (stride 1)
    (2, 256, 14, 128, 1, 1, 0),
    (2, 128, 14, 128, 3, 2, 1),     # layer2 first block 3x3 stride 2
    (2, 256, 14, 512, 1, 2, 0),     # downsample stride 2
    (3, 512, 6, 512, 3, 2, 1),      # layer4 first block (96-crop spatial 6 -> 3)
    (4, 512, 3, 512, 3, 1, 1),      # layer4 3x3 at 3x3 spatial
    (1, 1024, 7, 2048, 1, 2, 0),    # odd spatial size with stride 2
    (2, 128, 9, 192, 3, 1, 1),      # Cout not a multiple of the 128 tile
]


# 1x1 stride-1 convs and the stem's column GEMM take the tiled GEMM kernels (gemm8 / gemm.hip /
# gemm_small) where their output is wider than 128 columns, conv.hip otherwise
LT_SHAPES = [s for s in SHAPES if s[1] == 3 or (s[4] == 1 and s[5] == 1)]


@pytest.fixture
def hip_kernels():
    """The default dispatch (every conv on the hand-written kernels: conv.hip or the GEMM tiles)."""
    yield


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _data(dev, N, Cin, H, Cout, k, stride, pad, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, Cin, H, H, generator=g).bfloat16().to(dev).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).bfloat16().to(dev)
    w = w.contiguous(memory_format=CL)
    P = (H + 2 * pad - k) // stride + 1
    dy = torch.randn(N, Cout, P, P, generator=g).bfloat16().to(dev).contiguous(memory_format=CL)
    return x, w, dy


def _reference(x, w, dy, stride, pad):
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    y = F.conv2d(xr, wr, stride=stride, padding=pad)
    dx, dw = torch.autograd.grad(y, [xr, wr], dy.float())
    return y.detach(), dx, dw


def test_conv_ops_cpu_match_autograd():
    x, w, dy = _data("cpu", 2, 8, 9, 16, 3, 2, 1)
    y = torch.ops.dedloc.conv2d_fwd(x, w, 2, 1)
    yr, dxr, dwr = _reference(x, w, dy, 2, 1)
    assert _rel(y, yr) < 1e-2
    dx = torch.ops.dedloc.conv2d_dgrad(dy, w, 2, 1, 9, 9)
    assert _rel(dx, dxr) < 1e-2
    dw = torch.zeros(16, 8, 3, 3)
    torch.ops.dedloc.conv2d_wgrad(dy, x, dw, 2, 1)
    assert _rel(dw, dwr) < 1e-5


def test_conv_module_cpu_runs_the_dedloc_operators():
    """No stock-module fallback on the CPU: ConvNHWC runs the dedloc conv operators (their CPU
    implementations) on channels-last bf16, i.e. nn.Conv2d to bf16 rounding, with gradients."""
    from dedloc_amd.models.resnet_swav import ConvNHWC

    m = ConvNHWC(8, 16, 3, stride=2, padding=1, bias=False)
    ref = torch.nn.Conv2d(8, 16, 3, stride=2, padding=1, bias=False)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 8, 9, 9)
    y = m(x)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert "ConvNHWC" in type(y.grad_fn).__name__
    xr = x.bfloat16().float()
    yr = F.conv2d(xr, m.weight.detach().bfloat16().float(), stride=2, padding=1)
    assert _rel(y.float(), yr) < 1e-2
    y.float().sum().backward()
    assert m.weight.grad is not None and torch.isfinite(m.weight.grad).all()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_fwd_gpu(cuda, hip_kernels, shape):
    N, Cin, H, Cout, k, stride, pad = shape
    x, w, dy = _data(cuda, *shape)
    y = torch.ops.dedloc.conv2d_fwd(x, w, stride, pad)
    yr, _, _ = _reference(x, w, dy, stride, pad)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 1e-2, _rel(y, yr)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] % 64 == 0 and s[3] % 64 == 0],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv_dgrad_gpu(cuda, hip_kernels, shape):
    N, Cin, H, Cout, k, stride, pad = shape
    x, w, dy = _data(cuda, *shape, seed=1)
    dx = torch.ops.dedloc.conv2d_dgrad(dy, w, stride, pad, H, H)
    _, dxr, _ = _reference(x, w, dy, stride, pad)
    assert dx.shape == dxr.shape and dx.is_contiguous(memory_format=CL)
    assert _rel(dx, dxr) < 1e-2, _rel(dx, dxr)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_wgrad_gpu(cuda, hip_kernels, shape):
    N, Cin, H, Cout, k, stride, pad = shape
    x, w, dy = _data(cuda, *shape, seed=2)
    _, _, dwr = _reference(x, w, dy, stride, pad)
    base = torch.randn(Cout, Cin, k, k, device=cuda).contiguous(memory_format=CL)
    dw = base.clone()
    torch.ops.dedloc.conv2d_wgrad(dy, x, dw, stride, pad)  # accumulates into the KRSC fp32 buffer
    assert _rel(dw - base, dwr) < 1e-3, _rel(dw - base, dwr)
    dw2 = base.clone().contiguous()  # NCHW-contiguous destination goes through a temporary
    torch.ops.dedloc.conv2d_wgrad(dy, x, dw2, stride, pad)
    assert _rel(dw2 - base, dwr) < 1e-3


@pytest.mark.gpu
def test_conv_wgrad_large_reduction_split_k(cuda, hip_kernels):
    """224-crop stem at batch 4: 50k-pixel reduction split over many workgroups (fp32 atomics)."""
    shape = (4, 3, 224, 64, 7, 2, 3)
    x, w, dy = _data(cuda, *shape, seed=3)
    _, _, dwr = _reference(x, w, dy, 2, 3)
    dw = torch.zeros(64, 3, 7, 7, device=cuda).contiguous(memory_format=CL)
    torch.ops.dedloc.conv2d_wgrad(dy, x, dw, 2, 3)
    assert _rel(dw, dwr) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("H", [96, 224])
def test_stem_space_to_depth_cols_stats_and_wgrad(cuda, H):
    """The 7x7/2 3-channel stem as a 4x4 conv over the space-to-depth image: im2col_stem returns that
    image ([N*H/2*W/2, 16]), which the forward (with the BatchNorm-statistics epilogue, 3 groups) and
    the weight gradient take in place of the input — against fp32 PyTorch."""
    N = 3
    x, w, dy = _data(cuda, N, 3, H, 64, 7, 2, 3, seed=7)
    yr, _, dwr = _reference(x, w, dy, 2, 3)
    cols = torch.ops.dedloc.im2col_stem(x, 7, 7, 2, 3)
    assert cols.shape == (N * (H // 2) ** 2, 16) and cols.dtype == torch.bfloat16
    sums = torch.zeros(2 * N * 64, device=cuda)
    y = torch.ops.dedloc.conv2d_fwd_stats(x, w, 2, 3, sums, N, cols)
    assert _rel(y, yr) < 1e-2, _rel(y, yr)
    yf = y.float().permute(0, 2, 3, 1).reshape(N, -1, 64)
    ref_sums = torch.cat([yf.sum(1), (yf * yf).sum(1)], dim=1).reshape(-1)
    assert _rel(sums, ref_sums) < 1e-4, _rel(sums, ref_sums)
    xs = torch.empty((), dtype=torch.bfloat16, device=cuda).expand(x.shape)  # only the shape is read
    dw = torch.zeros(64, 3, 7, 7, device=cuda).contiguous(memory_format=CL)
    torch.ops.dedloc.conv2d_wgrad(dy, xs, dw, 2, 3, cols)
    assert _rel(dw, dwr) < 1e-3, _rel(dw, dwr)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", LT_SHAPES + [(4, 3, 224, 64, 7, 2, 3)], ids=lambda s: "x".join(map(str, s)))
def test_conv_gemm_route_gpu(cuda, shape):
    """Pointwise convs and the stem's column GEMM on the tiled GEMM kernels (fwd, dgrad, fp32 wgrad
    accumulated with token-split slabs)."""
    N, Cin, H, Cout, k, stride, pad = shape
    x, w, dy = _data(cuda, *shape, seed=4)
    yr, dxr, dwr = _reference(x, w, dy, stride, pad)
    y = torch.ops.dedloc.conv2d_fwd(x, w, stride, pad)
    assert y.is_contiguous(memory_format=CL) and _rel(y, yr) < 1e-2, _rel(y, yr)
    if Cout % 64 == 0 and Cin % 64 == 0:
        dx = torch.ops.dedloc.conv2d_dgrad(dy, w, stride, pad, H, H)
        assert dx.is_contiguous(memory_format=CL) and _rel(dx, dxr) < 1e-2, _rel(dx, dxr)
    base = torch.randn(Cout, Cin, k, k, device=cuda).contiguous(memory_format=CL)
    dw = base.clone()
    torch.ops.dedloc.conv2d_wgrad(dy, x, dw, stride, pad)
    assert _rel(dw - base, dwr) < 1e-3, _rel(dw - base, dwr)


@pytest.mark.gpu
def test_conv_module_grads_land_in_flat_buffer(cuda):
    """ConvNHWC inside FlatParams(autograd, channels_last): dgrad returned, wgrad accumulated in place."""
    from dedloc_amd.models.resnet_swav import ConvNHWC
    from dedloc_amd.utils.flat import FlatParams

    torch.manual_seed(4)
    m = ConvNHWC(64, 128, 3, stride=2, padding=1, bias=False).to(cuda)
    w_ref = m.weight.detach().bfloat16().float().clone()
    flat = FlatParams(m.named_parameters(), device=cuda, with_bf16=False, autograd=True, channels_last=True)
    x = torch.randn(2, 64, 12, 12, device=cuda).bfloat16().contiguous(memory_format=CL).requires_grad_(True)
    for _ in range(2):  # two backward passes accumulate
        y = m(x)
        coef = torch.linspace(-1, 1, y.numel(), device=cuda).view_as(y)
        (y.float() * coef).sum().backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w_ref.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=2, padding=1)
    (yr * coef).sum().backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(flat.view(flat.grad, "weight"), 2 * wr.grad) < 1e-2
    assert _rel(x.grad, 2 * xr.grad) < 1e-2


def _fp32_twin(m, device):
    """The same module as stock PyTorch modules in fp32 (training/swav_eager.py: nn.Conv2d,
    nn.BatchNorm2d, ... with the same parameters and state-dict keys) — the plain PyTorch fp32
    reference of the same ops, sharing no code with the kernels under test."""
    from dedloc_amd.training.swav_eager import eager_twin

    return eager_twin(m, device=device)


@pytest.mark.gpu
def test_resnet_trunk_hip_kernels_match_fp32(cuda):
    """The SwAV trunk's stem + first stage on the hand-written kernels (convs, fused BN, max-pool)
    vs the same module in fp32 PyTorch: forward features agree to bf16 accuracy."""
    from dedloc_amd.models.resnet_swav import SwAVModel
    from dedloc_amd.utils.flat import FlatParams

    torch.manual_seed(5)
    base = SwAVModel(num_prototypes=32)
    x = torch.randn(4, 3, 64, 64, device=cuda).bfloat16().contiguous(memory_format=CL)
    ref = _fp32_twin(base, cuda).train()
    m = base.to(cuda).train()
    FlatParams(m.named_parameters(), device=cuda, with_bf16=False, autograd=True, channels_last=True)
    t, tr = m.trunk, ref.trunk
    with torch.autocast("cuda", dtype=torch.bfloat16):
        feat = t.layer1(t.maxpool(t.bn1(t.conv1(x))))
    fr = tr.layer1(tr.maxpool(tr.relu(tr.bn1(tr.conv1(x.float())))))
    # stem + first stage only: bf16 and fp32 drift apart through random-init conv/BN/ReLU stacks
    # (ReLU sign flips compound), so deeper outputs would test the drift, not the kernels
    assert _rel(feat.float(), fr) < 3e-2, _rel(feat.float(), fr)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,planes,stride,H", [(256, 64, 1, 16), (256, 128, 2, 16), (1024, 512, 2, 8)])
def test_bottleneck_grads_match_fp32(cuda, cin, planes, stride, H):
    """One Bottleneck (incl. the stride-2 downsample variant), identical x and dY: dX and every
    parameter gradient (flat buffer, in-place fp32 wgrad) of the hand-written path match the fp32
    PyTorch module's as closely as stock PyTorch bf16 autocast does.  Through three BN backwards
    (each re-centres the gradient) bf16 rounding alone leaves 5-9e-2 relative difference on the
    gradients — stock bf16 measured 0.071 / 0.072 / 0.073 on dX for these three blocks
    (profiles/bottleneck_bf16_drift_diag.log) — so the bound is relative to that stock-bf16 twin."""
    from dedloc_amd.models.resnet_swav import BNAct, Bottleneck, ConvNHWC
    from dedloc_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    down = None
    if stride != 1 or cin != planes * 4:
        down = torch.nn.Sequential(ConvNHWC(cin, planes * 4, 1, stride=stride, bias=False), BNAct(planes * 4))
    m = Bottleneck(cin, planes, stride, down)
    ref = _fp32_twin(m, cuda).train()
    stock = _fp32_twin(m, cuda).train()
    m = m.to(cuda).train()
    torch.manual_seed(1)
    x = torch.randn(4, cin, H, H, device=cuda).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(4, planes * 4, H // stride, H // stride, device=cuda).bfloat16().contiguous(memory_format=CL)
    flat = FlatParams(m.named_parameters(), device=cuda, with_bf16=False, autograd=True, channels_last=True)
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xx)
    y.backward(dy)
    xr = x.float().requires_grad_(True)
    yr = ref(xr)
    yr.backward(dy.float())
    xs = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ys = stock(xs)
    ys.backward(dy)

    def bound(stock_err):
        # Ill-conditioned sums (a BatchNorm bias gradient: the column sum of a masked random dy,
        # 10-20% relative error even for stock bf16) vary run to run with the order of the fp32
        # atomics that accumulate them (both ours and the previous builds exceeded 1.3x once in
        # six runs, bench/conv_test_repeat.sh); well-conditioned gradients keep the 1.3x bound.
        return 1.3 * stock_err + 5e-3 if stock_err < 0.05 else 1.6 * stock_err

    assert _rel(y.float(), yr) < 1e-2
    assert _rel(xx.grad.float(), xr.grad) < bound(_rel(xs.grad, xr.grad))
    rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
    for n, _ in m.named_parameters():
        ours, theirs = _rel(flat.view(flat.grad, n), rp[n].grad), _rel(sp[n].grad, rp[n].grad)
        assert ours < bound(theirs), (n, ours, theirs)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,planes,stride,H", [(256, 64, 1, 16), (256, 128, 2, 16), (1024, 512, 2, 8)])
def test_bottleneck_grads_deterministic_bn(cuda, monkeypatch, cin, planes, stride, H):
    """The same Bottleneck comparison under DEDLOC_DETERMINISTIC_BN=1 (hygiene): every
    BatchNorm statistic a fixed-order reduction, no epilogue atomics.  Two runs give bitwise-identical
    gradients, and the strict bound (1.3x stock bf16 + 5e-3) holds for EVERY gradient — the 1.6x
    allowance of the default mode only covers run-to-run atomics order in ill-conditioned sums."""
    from dedloc_amd.models.resnet_swav import BNAct, Bottleneck, ConvNHWC
    from dedloc_amd.utils.flat import FlatParams

    monkeypatch.setenv("DEDLOC_DETERMINISTIC_BN", "1")
    torch.manual_seed(0)
    down = None
    if stride != 1 or cin != planes * 4:
        down = torch.nn.Sequential(ConvNHWC(cin, planes * 4, 1, stride=stride, bias=False), BNAct(planes * 4))
    m = Bottleneck(cin, planes, stride, down)
    ref = _fp32_twin(m, cuda).train()
    stock = _fp32_twin(m, cuda).train()
    m = m.to(cuda).train()
    torch.manual_seed(1)
    x = torch.randn(4, cin, H, H, device=cuda).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(4, planes * 4, H // stride, H // stride, device=cuda).bfloat16().contiguous(memory_format=CL)
    flat = FlatParams(m.named_parameters(), device=cuda, with_bf16=False, autograd=True, channels_last=True)
    runs = []
    for _ in range(2):
        flat.grad.zero_()
        xx = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xx)
        y.backward(dy)
        runs.append((flat.grad.clone(), xx.grad.clone()))
    assert torch.equal(runs[0][1], runs[1][1]), "dX differs between two deterministic runs"
    # the weight gradients' conv split-K keeps fp32 atomics (not a BatchNorm statistic): compare BN params bitwise
    bn_names = [n for n, _ in m.named_parameters() if ".bn" in f".{n}" or n.startswith("downsample.1")]
    for n in bn_names:
        assert torch.equal(flat.view(runs[0][0], n), flat.view(runs[1][0], n)), n
    xr = x.float().requires_grad_(True)
    ref(xr).backward(dy.float())
    xs = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ys = stock(xs)
    ys.backward(dy)
    margins = {}
    assert _rel(xx.grad.float(), xr.grad) < 1.3 * _rel(xs.grad, xr.grad) + 5e-3
    rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
    for n, _ in m.named_parameters():
        ours, theirs = _rel(flat.view(flat.grad, n), rp[n].grad), _rel(sp[n].grad, rp[n].grad)
        margins[n] = (round(ours, 5), round(theirs, 5))
        assert ours < 1.3 * theirs + 5e-3, (n, ours, theirs)
    from conftest import record_margin

    record_margin("bottleneck_deterministic_bn", shape=[cin, planes, stride, H], grads=margins)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(64, 512, 7, 512, 3, 1, 1),    # SwAV layer 4, 224 crop: 100 tiles of 72 k-steps
                                   (64, 256, 14, 256, 3, 1, 1),   # layer 3: 196 tiles
                                   (4, 256, 16, 64, 3, 1, 1),     # 256x64 tiles: 4 tiles
                                   (4, 512, 16, 512, 3, 1, 1),    # 32 tiles; BN-backward epilogue fused
                                   (16, 1024, 8, 256, 3, 2, 1)],  # strided: 4 parity-class jobs
                         ids=lambda s: "x".join(map(str, s)))
def test_conv_few_tile_long_k_gpu(cuda, shape):
    """conv.hip launches of fewer tiles than CUs with long reductions (the SwAV b=64 layer-3/4
    shapes): forward, forward with the BatchNorm statistics epilogue, data gradient and the
    BN-backward epilogue against fp32, and bitwise repeatable.  (A split-K form of these launches
    was measured slower in the graphed iteration, whose concurrent passes already fill the chip:
    profiles/r6_conv_splitk_negative.jsonl.)"""
    N, Cin, H, Cout, k, stride, pad = shape
    x, w, dy = _data(cuda, *shape, seed=4)
    yr, dxr, _ = _reference(x, w, dy, stride, pad)
    ys = [torch.ops.dedloc.conv2d_fwd(x, w, stride, pad) for _ in range(3)]
    assert _rel(ys[0], yr) < 1e-2, _rel(ys[0], yr)
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    groups = 2
    sums = torch.zeros(2 * groups * Cout, device=cuda)
    y = torch.ops.dedloc.conv2d_fwd_stats(x, w, stride, pad, sums, groups)
    assert torch.equal(y, ys[0])
    g = y.float().permute(0, 2, 3, 1).reshape(groups, -1, Cout)
    ref = torch.stack([g.sum(1), (g * g).sum(1)], 1).reshape(-1)
    assert _rel(sums, ref) < 1e-4, _rel(sums, ref)
    dxs = [torch.ops.dedloc.conv2d_dgrad(dy, w, stride, pad, H, H) for _ in range(3)]
    assert _rel(dxs[0], dxr) < 1e-2, _rel(dxs[0], dxr)
    assert all(torch.equal(dxs[0], d) for d in dxs[1:])
    # the data gradient prepared for a BN+ReLU backward (mask from the BN input through gamma/beta)
    bx = torch.randn(x.shape, device=cuda).bfloat16().contiguous(memory_format=CL)
    mean = torch.randn(groups, Cin, device=cuda) * 0.1
    rstd = torch.rand(groups, Cin, device=cuda) + 0.5
    gamma, beta = torch.rand(Cin, device=cuda) + 0.5, torch.randn(Cin, device=cuda) * 0.1
    bsums = torch.zeros(2 * groups * Cin, device=cuda)
    gout, fused = torch.ops.dedloc.conv2d_dgrad_bn(dy, w, stride, pad, H, H, None, bx, None, mean, rstd, gamma, beta,
                                                   bsums, groups, None)
    xb = bx.float().permute(0, 2, 3, 1).reshape(groups, -1, Cin)
    pre = (xb - mean[:, None]) * rstd[:, None] * gamma + beta
    gref = dxs[0].float().permute(0, 2, 3, 1).reshape(groups, -1, Cin) * (pre > 0)
    gk = gout.float().permute(0, 2, 3, 1).reshape(groups, -1, Cin)
    if fused:
        assert _rel(gk, gref) < 1e-2, _rel(gk, gref)
        xhat = (xb - mean[:, None]) * rstd[:, None]
        sref = torch.stack([gk.sum(1), (gk * xhat).sum(1)], 1).reshape(-1)
        assert _rel(bsums, sref) < 1e-3, _rel(bsums, sref)
    else:
        assert _rel(gk, dxs[0].float().permute(0, 2, 3, 1).reshape(groups, -1, Cin)) < 1e-6


@pytest.mark.gpu
def test_conv_dgrad_weights_batched_matches_per_conv(cuda):
    """The batched tap-transposed data-gradient weights (one launch for every conv of the trunk,
    SwAVModel's concurrent passes) equal the per-conv op bitwise, class by class."""
    from dedloc_amd.models.resnet_swav import ConvNHWC, ResNet50Trunk

    torch.manual_seed(0)
    convs = [m for m in ResNet50Trunk().modules() if isinstance(m, ConvNHWC) and m.in_channels % 64 == 0]
    ws = [m.weight.detach().bfloat16().to(cuda).contiguous(memory_format=CL) for m in convs]
    st, pd = [m.stride[0] for m in convs], [m.padding[0] for m in convs]
    outs = torch.ops.dedloc.conv2d_dgrad_weights_batched(ws, st, pd)
    i = 0
    for w, s_, p_ in zip(ws, st, pd):
        for r in torch.ops.dedloc.conv2d_dgrad_weights(w, s_, p_):
            o = outs[i]
            i += 1
            assert o.shape == r.shape and torch.equal(o, r), (tuple(w.shape), s_, p_, i)
    assert i == len(outs)


def test_conv_dgrad_weights_batched_cpu():
    ws = [torch.randn(16, 8, 3, 3).bfloat16(), torch.randn(32, 16, 1, 1).bfloat16()]
    outs = torch.ops.dedloc.conv2d_dgrad_weights_batched(ws, [2, 1], [1, 0])
    ref = torch.ops.dedloc.conv2d_dgrad_weights(ws[0], 2, 1) + torch.ops.dedloc.conv2d_dgrad_weights(ws[1], 1, 0)
    assert len(outs) == len(ref) == 5 and all(torch.equal(o, r) for o, r in zip(outs, ref))


def test_conv_fwd_stats_cpu_reference():
    """CPU reference of conv2d_fwd_stats: the conv output and per-group channel sums / sums of
    squares of the stored values, accumulated into `sums`."""
    torch.manual_seed(0)
    x = torch.randn(4, 8, 6, 6).contiguous(memory_format=torch.channels_last)
    w = torch.randn(16, 8, 3, 3)
    sums = torch.ones(2 * 2 * 16)
    y = torch.ops.dedloc.conv2d_fwd_stats(x, w, 1, 1, sums, 2)
    yr = F.conv2d(x, w, padding=1)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-4)
    g = yr.reshape(2, 2, 16, 36)
    ref = torch.stack([g.sum((1, 3)), (g * g).sum((1, 3))], 1).reshape(-1) + 1
    torch.testing.assert_close(sums, ref, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,planes,stride", [(256, 64, 1), (512, 128, 2)])
def test_chained_bottlenecks_grads_match_fp32(cuda, cin, planes, stride):
    """Three chained Bottlenecks (the second and third identity blocks), so every fused backward path
    runs: bn2's backward statistics in conv3's data-gradient epilogue, bn3's in the NEXT block's
    conv1 epilogue (ReLU mask from that conv's input, identity gradient added), and the first
    block's bn3 through its own pass (a downsample block follows nothing here).  dX and every
    parameter gradient against the fp32 PyTorch twin, bounded relative to stock bf16 autocast."""
    from dedloc_amd.models.resnet_swav import BNAct, Bottleneck, ConvNHWC
    from dedloc_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    down = None
    if stride != 1 or cin != planes * 4:
        down = torch.nn.Sequential(ConvNHWC(cin, planes * 4, 1, stride=stride, bias=False), BNAct(planes * 4))
    m = torch.nn.Sequential(Bottleneck(cin, planes, stride, down), Bottleneck(planes * 4, planes),
                            Bottleneck(planes * 4, planes))
    ref = _fp32_twin(m, cuda).train()
    stock = _fp32_twin(m, cuda).train()
    m = m.to(cuda).train()
    H = 16
    torch.manual_seed(1)
    x = torch.randn(8, cin, H, H, device=cuda).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(8, planes * 4, H // stride, H // stride, device=cuda).bfloat16().contiguous(memory_format=CL)
    flat = FlatParams(m.named_parameters(), device=cuda, with_bf16=False, autograd=True, channels_last=True)
    bns = [mod for mod in m.modules() if isinstance(mod, BNAct)]
    ws = torch.zeros(sum(2 * 2 * b.num_features for b in bns), device=cuda)
    off = 0
    for b in bns:  # the trunk's per-pass workspace (fused forward statistics and backward preparation)
        n = 2 * b.num_features
        b.pass_ws, b.count_deferred = (ws[off:off + n], ws[off + n:off + 2 * n]), True
        off += 2 * n
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xx)
    y.backward(dy)
    xr = x.float().requires_grad_(True)
    ref(xr).backward(dy.float())
    xs = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ys = stock(xs)
    ys.backward(dy)

    def bound(stock_err):
        # Ill-conditioned sums (a BatchNorm bias gradient: the column sum of a masked random dy,
        # 10-20% relative error even for stock bf16) vary run to run with the order of the fp32
        # atomics that accumulate them (both ours and the previous builds exceeded 1.3x once in
        # six runs, bench/conv_test_repeat.sh); well-conditioned gradients keep the 1.3x bound.
        return 1.3 * stock_err + 5e-3 if stock_err < 0.05 else 1.6 * stock_err

    assert _rel(xx.grad.float(), xr.grad) < bound(_rel(xs.grad, xr.grad))
    rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
    for n, _ in m.named_parameters():
        ours, theirs = _rel(flat.view(flat.grad, n), rp[n].grad), _rel(sp[n].grad, rp[n].grad)
        assert ours < bound(theirs), (n, ours, theirs)
