"""How well-conditioned is the SwAV ResNet-50's gradient at init?  Stock bf16 autocast vs fp32 of the
same modules (and this repo's kernels), flat relative gradient error, for several scales of every
Bottleneck's last BatchNorm gamma (bn3.weight; 0 = vissl/torchvision ``zero_init_residual``).

Random-init train-mode BatchNorm ResNets have exploding, chaotic gradients (the parity test's fp32 vs
bf16 comparison came out ~1.3 relative for stock bf16 itself); shrinking the residual branches at
init is the standard remedy and decides which regime a model-level gradient parity test can use.

    python bench/swav_grad_conditioning.py --batch 32 --scales 1,0.3,0.1,0.03
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--scales", default="1,0.3,0.1,0.03")
    args = ap.parse_args()
    from dedloc_amd.models.resnet_swav import Bottleneck, SwAVModel
    from dedloc_amd.training.swav_eager import eager_twin
    from dedloc_amd.utils.flat import FlatParams

    dev = torch.device("cuda", 0)
    CL = torch.channels_last
    bs = args.batch
    g = torch.Generator(device="cpu").manual_seed(1)
    crops = [torch.randn(bs, 3, s, s, generator=g).to(dev).bfloat16().contiguous(memory_format=CL)
             for s, n in ((224, 2), (96, 6)) for _ in range(n)]
    for scale in [float(v) for v in args.scales.split(",")]:
        torch.manual_seed(0)
        model = SwAVModel(num_prototypes=3000)
        model.normalize_prototypes()
        with torch.no_grad():
            for m in model.modules():
                if isinstance(m, Bottleneck):
                    m.bn3.weight.mul_(scale)
        ref = eager_twin(model, device=dev).train()
        stock = eager_twin(model, device=dev).train()
        model.to(dev).train()
        flat = FlatParams(model.named_parameters(), device=dev, with_bf16=True, autograd=True, channels_last=True)
        model.bind_flat(flat)
        model.concurrent_passes = True
        gen = torch.Generator(device="cpu").manual_seed(5)
        emb_r, scores_r = ref([c.float() for c in crops])
        r1 = torch.randn(emb_r.shape, generator=gen).to(dev)
        r2 = torch.randn(scores_r.shape, generator=gen).to(dev)
        ((emb_r * r1).sum() + (scores_r * r2).sum()).backward()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            emb_s, scores_s = stock(crops)
        ((emb_s.float() * r1).sum() + (scores_s.float() * r2).sum()).backward()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            emb, scores = model(crops)
        ((emb.float() * r1).sum() + (scores.float() * r2).sum()).backward()
        model.after_backward()
        torch.cuda.synchronize()
        rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
        names = list(flat.names)
        cat = lambda d: torch.cat([d[n].reshape(-1).float() for n in names])  # noqa: E731
        ours = {n: flat.view(flat.grad, n) for n in names}
        refg = {n: rp[n].grad for n in names}
        stockg = {n: sp[n].grad for n in names}
        per = sorted(((rel(stockg[n], refg[n]), n) for n in names), reverse=True)
        print(json.dumps({"bn3_scale": scale, "batch": bs, "stock_flat_err": rel(cat(stockg), cat(refg)),
                          "ours_flat_err": rel(cat(ours), cat(refg)), "ref_grad_norm": cat(refg).norm().item(),
                          "stock_worst": per[:3], "stock_median_tensor_err": per[len(per) // 2][0]}), flush=True)
        del model, ref, stock, flat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
