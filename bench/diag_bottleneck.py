"""Diagnostic: where does a Bottleneck's bf16 dX drift from fp32 come from?  Compares the
hand-written path and stock PyTorch bf16 autocast against the fp32 module (same x, dy)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

CL = torch.channels_last


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def twin(m, dev):
    from dedloc_amd.models.resnet_swav import BNAct, ConvNHWC
    ref = copy.deepcopy(m).float().to(dev)
    for mod in ref.modules():
        if isinstance(mod, ConvNHWC):
            mod.forward = lambda x, _m=mod: F.conv2d(x, _m.weight, None, _m.stride, _m.padding)
        if isinstance(mod, BNAct):
            mod.fused = False
    return ref


def main():
    from dedloc_amd.models.resnet_swav import BNAct, Bottleneck, ConvNHWC
    from dedloc_amd.utils.flat import FlatParams
    dev = torch.device("cuda")
    for cin, planes, stride, H in [(256, 64, 1, 16), (256, 128, 2, 16), (1024, 512, 2, 8)]:
        torch.manual_seed(0)
        down = None
        if stride != 1 or cin != planes * 4:
            down = torch.nn.Sequential(ConvNHWC(cin, planes * 4, 1, stride=stride, bias=False), BNAct(planes * 4))
        m = Bottleneck(cin, planes, stride, down)
        ref = twin(m, dev).train()
        stock = twin(m, dev).train()
        m = m.to(dev).train()
        torch.manual_seed(1)
        x = torch.randn(4, cin, H, H, device=dev).bfloat16().contiguous(memory_format=CL)
        dy = torch.randn(4, planes * 4, H // stride, H // stride, device=dev).bfloat16().contiguous(memory_format=CL)
        flat = FlatParams(m.named_parameters(), device=dev, with_bf16=False, autograd=True, channels_last=True)
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
        print(f"cin={cin} planes={planes} stride={stride}: y ours {rel(y, yr):.4f} stock {rel(ys, yr):.4f} | "
              f"dX ours {rel(xx.grad, xr.grad):.4f} stock {rel(xs.grad, xr.grad):.4f}", flush=True)
        rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
        for n, _ in m.named_parameters():
            print(f"   {n:28s} ours {rel(flat.view(flat.grad, n), rp[n].grad):.4f} stock {rel(sp[n].grad, rp[n].grad):.4f}",
                  flush=True)


if __name__ == "__main__":
    main()
