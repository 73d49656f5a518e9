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
