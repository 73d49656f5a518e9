"""pool.hip on the GPU against fp32 PyTorch references (SURVEY K17 max-pool, K19 global average
pool, K20 L2 normalisation): forward values and backward gradients on channels-last bf16."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _distinct(N, C, H, W, dev, seed=0):
    # every 3x3 window's values distinct and exact in bf16 (small integers): no tie ambiguity
    g = torch.Generator().manual_seed(seed)
    x = torch.stack([torch.randperm(H * W, generator=g)[: H * W].float() for _ in range(N * C)]).view(N, C, H, W)
    x = (x - H * W / 2) / 4  # quarter steps: exact in bf16 for H*W <= 1024
    return x.to(dev).bfloat16().contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("hw", [(14, 14), (15, 13), (112, 112), (48, 48)])
def test_maxpool_matches_torch(cuda, hw):
    H, W = hw
    N, C = 3, 64
    torch.manual_seed(H * 1000 + W)
    if H * W <= 1024:
        x = _distinct(N, C, H, W, cuda)
    else:  # large planes: random values (ties only among equal values, whose routing is then ambiguous)
        x = torch.randn(N, C, H, W, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    y, arg = torch.ops.dedloc.maxpool_fwd(x)
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    torch.testing.assert_close(y.float(), yr, rtol=0, atol=0)
    dy = torch.randn_like(yr).bfloat16().contiguous(memory_format=torch.channels_last)
    dx = torch.ops.dedloc.maxpool_bwd(dy, arg, H, W)
    yr.backward(dy.float())
    if H * W <= 1024:
        torch.testing.assert_close(dx.float(), xr.grad, rtol=1e-2, atol=1e-2)
    else:  # gradient mass is conserved either way
        torch.testing.assert_close(dx.float().sum((2, 3)), xr.grad.sum((2, 3)), rtol=2e-2, atol=2e-1)


def test_nan_propagates_through_relu_and_maxpool_like_torch(cuda):
    """torch.relu(NaN) and a max-pool window holding a NaN give NaN; the fused BN+ReLU and the max
    pool kernels keep that (a NaN-loss check must see NaNs that arise in the trunk)."""
    N, C, H, W = 2, 64, 8, 8
    x = torch.randn(N, C, H, W, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    x[0, 3, 2, 5] = float("nan")
    y, arg = torch.ops.dedloc.maxpool_fwd(x)
    yr = F.max_pool2d(x.float(), 3, 2, 1)
    assert torch.equal(torch.isnan(y.float()), torch.isnan(yr))
    torch.testing.assert_close(torch.nan_to_num(y.float()), torch.nan_to_num(yr), rtol=0, atol=0)
    g, b = torch.ones(C, device=cuda), torch.zeros(C, device=cuda)
    x2 = torch.randn(N, C, H, W, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    x2[1, 7, 0, 0] = float("nan")
    out = torch.ops.dedloc.bn_fwd(x2, None, g, b, None, None, 1e-5, 0.1, True)[0]
    ref = torch.relu(F.batch_norm(x2.float(), None, None, g, b, training=True, eps=1e-5))
    assert torch.equal(torch.isnan(out.float()), torch.isnan(ref))  # channel 7: NaN statistics


@pytest.mark.parametrize("shape", [(8, 2048, 7, 7), (5, 256, 3, 3), (2, 64, 56, 56)])
def test_avgpool_matches_torch(cuda, shape):
    N, C, H, W = shape
    x = torch.randn(shape, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.ops.dedloc.avgpool_fwd(x)
    torch.testing.assert_close(y.float(), x.float().mean((2, 3)), rtol=1e-2, atol=1e-2)
    dy = torch.randn(N, C, device=cuda).bfloat16()
    dx = torch.ops.dedloc.avgpool_bwd(dy, H, W)
    assert dx.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(dx.float(), (dy.float() / (H * W))[:, :, None, None].expand(N, C, H, W),
                               rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("D", [128, 1000])
def test_l2norm_matches_torch(cuda, D):
    x = torch.randn(512, D, device=cuda).bfloat16()
    y, rinv = torch.ops.dedloc.l2norm_fwd(x, 1e-12)
    xr = x.float().requires_grad_(True)
    yr = F.normalize(xr, dim=1, p=2)
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    dy = torch.randn(512, D, device=cuda).bfloat16()
    dx = torch.ops.dedloc.l2norm_bwd(dy, y, rinv)
    yr.backward(dy.float())
    err = (dx.float() - xr.grad).norm() / xr.grad.norm()
    assert err < 2e-2, err


def test_swav_trunk_uses_native_pools(cuda):
    from dedloc_amd.models.resnet_swav import MaxPool3x3s2, global_avgpool

    x = torch.randn(2, 64, 20, 20, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = MaxPool3x3s2()(x)
    assert y.grad_fn.__class__.__name__ == "_MaxPoolBackward"
    z = global_avgpool(y)
    assert z.shape == (2, 64) and z.grad_fn.__class__.__name__ == "_AvgPoolBackward"
    z.float().sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad.float()).all()


# Conv output + BatchNorm batch statistics (conv2d_fwd_stats): the epilogues of gemm_small (64 / 128
# outputs), gemm8 (N % 256 == 0), conv.hip (3x3 / strided) and the stem column GEMM, plus the
# fallback statistics pass when a tile would straddle two statistics groups (stat_rows not a
# multiple of the tile height).  Reference: fp32 F.conv2d, then per-group sums of the bf16-rounded
# output (the values BN would read back).
@pytest.mark.parametrize("cin,cout,k,stride,hw,groups", [
    (256, 64, 1, 1, 16, 2),     # gemm_small epilogue
    (64, 128, 1, 1, 16, 1),     # gemm_small, TN = 128
    (64, 256, 1, 1, 16, 2),     # gemm8 EPI_STATS
    (128, 512, 1, 1, 8, 2),     # gemm8, 2 N-tiles
    (64, 64, 3, 1, 16, 2),      # conv.hip epilogue
    (128, 256, 1, 2, 16, 2),    # strided 1x1 (downsample) on conv.hip
    (512, 2048, 1, 1, 3, 2),    # 2 x 9 rows per group: fallback statistics pass
    (3, 64, 7, 2, 32, 2),       # stem: im2col + gemm_small epilogue
])
def test_conv_fwd_stats_match_fp32(cuda, cin, cout, k, stride, hw, groups):
    torch.manual_seed(3)
    N = 8
    pad = k // 2
    x = torch.randn(N, cin, hw, hw, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device=cuda) / (cin * k * k) ** 0.5).bfloat16()
    w = w.contiguous(memory_format=torch.channels_last)
    sums = torch.zeros(groups * 2 * cout, device=cuda)
    y = torch.ops.dedloc.conv2d_fwd_stats(x, w, stride, pad, sums, groups)
    y0 = torch.ops.dedloc.conv2d_fwd(x, w, stride, pad)
    assert torch.equal(y, y0)  # the statistics do not change the stored output
    yr = F.conv2d(x.float(), w.float(), stride=stride, padding=pad)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    yg = y.float().reshape(groups, N // groups, cout, -1)
    ref = torch.stack([yg.sum((1, 3)), (yg * yg).sum((1, 3))], 1).reshape(-1)
    torch.testing.assert_close(sums, ref, rtol=1e-4, atol=1e-2)


def test_bottleneck_conv_stats_match_separate_pass(cuda, monkeypatch):
    """A Bottleneck (identity and downsample variants) with the BN statistics from the conv
    epilogues computes what it computes with the separate statistics pass: outputs within bf16
    rounding noise (the sums differ only in fp32 summation order).  Whole random-init trunks are no
    test for this: run-to-run fp32-atomics noise alone grows through their 16 blocks to O(1)
    differences at layer4 (scripts/diag_trunk_paths.py, either path against itself)."""
    from dedloc_amd.models import resnet_swav as rs

    torch.manual_seed(0)
    for cin, planes, stride in ((256, 64, 1), (256, 128, 2)):
        down = None
        if stride != 1 or cin != planes * 4:
            down = torch.nn.Sequential(rs.ConvNHWC(cin, planes * 4, 1, stride=stride, bias=False),
                                       rs.BNAct(planes * 4))
        m = rs.Bottleneck(cin, planes, stride, down).to(cuda).train()
        bns = [mod for mod in m.modules() if isinstance(mod, rs.BNAct)]
        x = torch.randn(4, cin, 16, 16, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
        outs = []
        for with_ws in (True, False):  # pass workspace: statistics from the conv epilogues; none: bn_fwd's pass
            ws = torch.zeros(sum(4 * 2 * b.num_features for b in bns), device=cuda)
            off = 0
            for b in bns:  # the trunk's per-pass workspace, as ResNet50Trunk._prepare_bn_pass lays it out
                n = 2 * 2 * b.num_features
                b.stat_groups = 2
                b.pass_ws = (ws[off:off + n], ws[off + n:off + 2 * n]) if with_ws else None
                b.count_deferred = with_ws
                off += 2 * n
            with torch.no_grad():
                outs.append(m(x).float())
        torch.testing.assert_close(outs[0], outs[1], rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("cin,cout", [(256, 64), (512, 128), (1024, 256)])
def test_conv_dgrad_residual_epilogue(cuda, cin, cout):
    """conv2d_dgrad(..., residual): the 1x1 data gradient plus the identity branch's gradient, added
    in the GEMM epilogue (one rounding), against fp32 PyTorch."""
    torch.manual_seed(5)
    CLF = torch.channels_last
    dy = torch.randn(4, cout, 14, 14, device=cuda).bfloat16().contiguous(memory_format=CLF)
    w = (torch.randn(cout, cin, 1, 1, device=cuda) / cout ** 0.5).bfloat16().contiguous(memory_format=CLF)
    r = torch.randn(4, cin, 14, 14, device=cuda).bfloat16().contiguous(memory_format=CLF)
    dx = torch.ops.dedloc.conv2d_dgrad(dy, w, 1, 0, 14, 14, r)
    ref = torch.nn.grad.conv2d_input((4, cin, 14, 14), w.float(), dy.float()) + r.float()
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("cin,cout,k,stride,N,ymask,res,expect_fused", [
    (64, 256, 1, 1, 4, False, False, True),    # bn2 -> conv3 (1x1 on conv.hip / gemm_small, N=64)
    (256, 1024, 1, 1, 4, False, False, True),  # bn2 -> conv3 (gemm8, N=256)
    (256, 64, 1, 1, 4, True, True, True),      # bn3 -> next conv1 (gemm8, N=256)
    (64, 64, 3, 1, 4, False, False, True),     # bn1 -> conv2 3x3 (conv.hip epilogue, 256x64 tiles)
    (128, 128, 3, 2, 8, False, False, True),   # bn1 -> strided conv2: four parity classes, one workspace
    (64, 64, 3, 2, 4, False, False, False)])   # class rows per group 128: not fused -> prep pass
def test_conv_dgrad_bn_matches_reference(cuda, cin, cout, k, stride, N, ymask, res, expect_fused):
    """conv2d_dgrad_bn (BN+ReLU backward preparation in the data-gradient epilogue; where it reports
    not fused, the plain gradient followed by the separate bn_bwd_prep pass) against plain fp32
    PyTorch: the data gradient (+ residual) masked by the BN+ReLU's live outputs, and the BN
    backward's two per-group column sums."""
    torch.manual_seed(7)
    CLF = torch.channels_last
    G, H = 2, 16
    P = H // stride
    x = (torch.randn(N, cin, H, H, device=cuda) + 0.3).bfloat16().contiguous(memory_format=CLF)
    y = torch.relu(torch.randn(N, cin, H, H, device=cuda)).bfloat16().contiguous(memory_format=CLF) if ymask else None
    w = (torch.randn(cout, cin, k, k, device=cuda) / (cin * k * k) ** 0.5).bfloat16().contiguous(memory_format=CLF)
    dy = torch.randn(N, cout, P, P, device=cuda).bfloat16().contiguous(memory_format=CLF)
    r = torch.randn(N, cin, H, H, device=cuda).bfloat16().contiguous(memory_format=CLF) if res else None
    mean = torch.randn(G, cin, device=cuda) * 0.1 + 0.3
    rstd = torch.rand(G, cin, device=cuda) + 0.5
    gamma, beta = torch.rand(cin, device=cuda) + 0.5, torch.randn(cin, device=cuda) * 0.1
    sums = torch.zeros(G * 2 * cin, device=cuda)
    g, fused = torch.ops.dedloc.conv2d_dgrad_bn(dy, w, stride, k // 2, H, H, r, x, y, mean, rstd, gamma, beta, sums, G)
    assert fused == expect_fused
    if not fused:
        g = torch.ops.dedloc.bn_bwd_prep(g, x, y, mean, rstd, gamma, beta, sums, G)
    # fp32 PyTorch reference
    d = torch.nn.grad.conv2d_input((N, cin, H, H), w.float(), dy.float(), stride=stride, padding=k // 2)
    if r is not None:
        d = d + r.float()
    shp = (G, N // G, cin, H, H)
    xf, mu, rs_ = x.float().reshape(shp), mean.view(G, 1, cin, 1, 1), rstd.view(G, 1, cin, 1, 1)
    if y is not None:
        live = y.float().reshape(shp) > 0
    else:
        live = (xf - mu) * rs_ * gamma.view(1, 1, cin, 1, 1) + beta.view(1, 1, cin, 1, 1) > 0
    gr = torch.where(live, d.reshape(shp), torch.zeros(()))
    sums_ref = torch.stack([gr.sum((1, 3, 4)), (gr * (xf - mu) * rs_).sum((1, 3, 4))], 1).reshape(-1)
    torch.testing.assert_close(g.float(), gr.reshape(N, cin, H, H), rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(sums, sums_ref, rtol=2e-2, atol=2.0)


def test_swav_queue_scores_on_own_gemm(cuda):
    """The SwAV loss's queue-vs-prototype scores run on the own GEMM kernels (bf16 operands, fp32
    accumulation) and match the fp32 product to bf16 operand rounding."""
    from dedloc_amd.models.swav_loss import SwAVLoss

    torch.manual_seed(0)
    loss = SwAVLoss(queue_length=3840, num_prototypes=3000, embedding_dim=128).to(cuda)
    proto = torch.nn.functional.normalize(torch.randn(3000, 128, device=cuda), dim=1)
    s = loss._queue_scores(0, proto)
    ref = loss.queue[0] @ proto.t()
    assert s.dtype == torch.float32 and s.shape == (3840, 3000)
    torch.testing.assert_close(s, ref, rtol=2e-2, atol=2e-2)
