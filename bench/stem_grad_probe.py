"""Where does the SwAV stem's BatchNorm-parameter gradient lose precision?  (test_swav_parity_gpu.py's
stem.v group: ours ~1.3x stock bf16's error against fp32, every other parameter group ~1.0x.)

Runs the parity test's setup (b = 32, 2x224 + 6x96 crops, bn3 gammas x 0.03, random projection
loss) for ours, stock bf16 autocast and fp32, and compares against fp32, per crop resolution:
the stem max-pool's input (forward) and its output gradient (backward), the stem BN input, and the
stem BN gamma / beta gradients recomputed from each pipeline's own tensors in fp32.

    python bench/stem_grad_probe.py [--proj_seeds 5,6,7,8]

One JSON line per projection seed (5 is the parity test's).
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--proj_seeds", default="5")
    for seed in [int(v) for v in ap.parse_args().proj_seeds.split(",")]:
        run(seed)
        torch.cuda.empty_cache()


def run(proj_seed):
    from dedloc_amd.models import resnet_swav as rs
    from dedloc_amd.training.swav_eager import eager_twin
    from dedloc_amd.utils.flat import FlatParams

    dev = torch.device("cuda", 0)
    CL = torch.channels_last
    torch.manual_seed(0)
    bs = 32
    model = rs.SwAVModel(num_prototypes=3000)
    model.normalize_prototypes()
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, rs.Bottleneck):
                m.bn3.weight.mul_(0.03)
    ref = eager_twin(model, device=dev).train()
    stock = eager_twin(model, device=dev).train()
    model.to(dev).train()
    flat = FlatParams(model.named_parameters(), device=dev, with_bf16=True, autograd=True, channels_last=True)
    model.bind_flat(flat)
    model.concurrent_passes = True
    g = torch.Generator(device="cpu").manual_seed(1)
    crops = [torch.randn(bs, 3, s, s, generator=g).to(dev).bfloat16().contiguous(memory_format=CL)
             for s, n in ((224, 2), (96, 6)) for _ in range(n)]

    # capture: stem conv output (BN input), max-pool input / output and the output's gradient
    cap = {"ref": [], "stock": [], "ours": []}

    def eager_hooks(twin, key):
        def conv_hook(mod, inp, out):
            cap[key].append({"bnin": out.detach().float()})

        def pool_hook(mod, inp, out):
            d = cap[key][-1]
            d["pin"], d["pout"] = inp[0].detach().float(), out.detach().float()
            out.register_hook(lambda gr, d=d: d.__setitem__("gpout", gr.detach().float()))

        twin.trunk.conv1.register_forward_hook(conv_hook)
        twin.trunk.maxpool.register_forward_hook(pool_hook)

    eager_hooks(ref, "ref")
    eager_hooks(stock, "stock")
    orig_trunk_fwd = rs.ResNet50Trunk.forward

    def trunk_fwd(self, x, prepared=None):
        self._prepare_bn_pass(x, prepared)
        c = self.conv1(x, self.bn1)
        d = {"bnin": c.detach().float()}
        cap["ours"].append(d)
        p_in = self.bn1(c)
        d["pin"] = p_in.detach().float()
        x = self.maxpool(p_in)
        d["pout"] = x.detach().float()
        x.register_hook(lambda gr, d=d: d.__setitem__("gpout", gr.detach().float()))
        for stage in (self.layer1, self.layer2, self.layer3, self.layer4):
            x = stage(x)
        return rs.global_avgpool(x)

    rs.ResNet50Trunk.forward = trunk_fwd
    gen = torch.Generator(device="cpu").manual_seed(proj_seed)
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
    rs.ResNet50Trunk.forward = orig_trunk_fwd

    def by_res(lst, key):  # [224-crop tensors], [96-crop tensors] concatenated along the batch
        out = {}
        for d in lst:
            t = d[key]
            out.setdefault(t.shape[-1], []).append(t)
        return {k: torch.cat(v) for k, v in out.items()}

    rec = {"proj_seed": proj_seed}
    for key in ("bnin", "pin", "pout", "gpout"):
        R = by_res(cap["ref"], key)
        S = by_res(cap["stock"], key)
        O = by_res(cap["ours"], key)
        for hw in R:
            rec[f"{key}@{hw}"] = {"ours": round(rel(O[hw], R[hw]), 5), "stock": round(rel(S[hw], R[hw]), 5)}
    # the stem BN's gamma / beta gradients from each pipeline's own (BN input, max-pool output
    # gradient), recomputed in fp32 with per-crop statistics: isolates the BN + ReLU + max-pool backward
    def bn_param_grads(lst):
        dg, db = 0.0, 0.0
        for d in lst:
            x = d["bnin"]
            n = x.shape[0] // bs
            for i in range(n):
                xi = x[i * bs:(i + 1) * bs]
                mu = xi.mean((0, 2, 3), keepdim=True)
                var = xi.var((0, 2, 3), unbiased=False, keepdim=True)
                xh = (xi - mu) * torch.rsqrt(var + 1e-5)
                y = xh * model.trunk.bn1.weight.detach().float().view(1, -1, 1, 1) + \
                    model.trunk.bn1.bias.detach().float().view(1, -1, 1, 1)
                yr = F.relu(y).requires_grad_(True)
                out = F.max_pool2d(yr, 3, 2, 1)
                (gy,) = torch.autograd.grad(out, yr, d["gpout"][i * bs:(i + 1) * bs])
                gy = gy * (y > 0)
                dg = dg + (gy * xh).sum((0, 2, 3))
                db = db + gy.sum((0, 2, 3))
        return dg, db

    gr_r = bn_param_grads(cap["ref"])
    gr_s = bn_param_grads(cap["stock"])
    gr_o = bn_param_grads(cap["ours"])
    rp, sp = dict(ref.named_parameters()), dict(stock.named_parameters())
    ours_w = flat.view(flat.grad, "trunk.bn1.weight").float()
    ours_b = flat.view(flat.grad, "trunk.bn1.bias").float()
    rec["bn1.weight.grad"] = {"ours": round(rel(ours_w, rp["trunk.bn1.weight"].grad), 5),
                              "stock": round(rel(sp["trunk.bn1.weight"].grad, rp["trunk.bn1.weight"].grad), 5)}
    rec["bn1.bias.grad"] = {"ours": round(rel(ours_b, rp["trunk.bn1.bias"].grad), 5),
                            "stock": round(rel(sp["trunk.bn1.bias"].grad, rp["trunk.bn1.bias"].grad), 5)}
    rec["bn1.weight.grad_recomputed_fp32"] = {"ours": round(rel(gr_o[0], gr_r[0]), 5), "stock": round(rel(gr_s[0], gr_r[0]), 5),
                                              "ref_recomputed_vs_ref_autograd": round(rel(gr_r[0], rp["trunk.bn1.weight"].grad), 6)}
    rec["bn1.bias.grad_recomputed_fp32"] = {"ours": round(rel(gr_o[1], gr_r[1]), 5), "stock": round(rel(gr_s[1], gr_r[1]), 5)}
    rec["ours_kernel_vs_recomputed_from_its_tensors"] = {"weight": round(rel(ours_w, gr_o[0]), 5),
                                                         "bias": round(rel(ours_b, gr_o[1]), 5)}
    rec["stock_autograd_vs_recomputed_from_its_tensors"] = {
        "weight": round(rel(sp["trunk.bn1.weight"].grad, gr_s[0]), 5), "bias": round(rel(sp["trunk.bn1.bias"].grad, gr_s[1]), 5)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
