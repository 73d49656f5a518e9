"""Diagnose hip-vs-MIOpen gradient differences on one Bottleneck block (GPU): same input, same upstream
gradient; every parameter gradient and dX compared with an fp32 autograd reference."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from dedloc_amd.models.resnet_swav import Bottleneck, ConvNHWC, ResNet50Trunk  # noqa: E402
from dedloc_amd.utils.flat import FlatParams  # noqa: E402

CL = torch.channels_last
dev = torch.device("cuda")


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def run(mod_factory, x, dy, impl, use_flat):
    torch.manual_seed(0)
    m = mod_factory().to(dev).train()
    for mm in m.modules():
        if isinstance(mm, ConvNHWC):
            mm.native = impl == "hip"
    flat = FlatParams(m.named_parameters(), device=dev, with_bf16=False, autograd=True, channels_last=True) \
        if use_flat else None
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=impl != "fp32"):
        y = m(xx if impl != "fp32" else xx.float())
    y.backward(dy.to(y.dtype))
    grads = {n: (flat.view(flat.grad, n) if flat is not None else p.grad).detach().float().clone()
             for n, p in m.named_parameters()}
    return y.detach().float(), xx.grad.detach().float(), grads


for name, factory, shape in [
        ("block64", lambda: Bottleneck(256, 64), (4, 256, 16, 16)),
        ("stem", lambda: torch.nn.Sequential(ResNet50Trunk().conv1), (4, 3, 64, 64))]:
    torch.manual_seed(1)
    x = torch.randn(*shape, device=dev).bfloat16().contiguous(memory_format=CL)
    with torch.no_grad():
        y0 = factory().to(dev)(x.float())
    dy = torch.randn_like(y0).contiguous(memory_format=CL)
    res = {impl: run(factory, x, dy, impl, flat) for impl, flat in
           (("hip", True), ("miopen", True), ("hip_noflat", False))}
    res["hip_noflat"] = run(factory, x, dy, "hip", False)
    print(f"== {name}: y hip/miopen {rel(res['hip'][0], res['miopen'][0]):.4f} "
          f"dx {rel(res['hip'][1], res['miopen'][1]):.4f}")
    for n in res["hip"][2]:
        print(f"   {n:30s} hip-vs-miopen {rel(res['hip'][2][n], res['miopen'][2][n]):.4f}  "
              f"hip(flat)-vs-hip(noflat) {rel(res['hip'][2][n], res['hip_noflat'][2][n]):.4f}")
