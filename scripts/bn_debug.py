"""Locate the first BNAct whose batched (statistics-group) output differs from per-crop passes (GPU)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dedloc_amd.models.resnet_swav import BNAct, SwAVModel  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(12)
m1 = SwAVModel(num_prototypes=64, single_pass_every_crop=True).to(dev).train()
m2 = copy.deepcopy(m1)
cl = torch.channels_last
crops = [torch.randn(4, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=cl) for _ in range(2)]
rec1, rec2 = {}, {}


def hook(rec):
    def h(mod, inp, out):
        x = inp[0]
        rec.setdefault(mod._name, []).append((out.detach().float().clone(), tuple(x.shape),
                                              x.is_contiguous(memory_format=cl), len(inp) > 1 and inp[1] is not None,
                                              mod.stat_groups))
    return h


for m, rec in ((m1, rec1), (m2, rec2)):
    for n, mod in m.trunk.named_modules():
        if isinstance(mod, BNAct):
            mod._name = n
            mod.register_forward_hook(hook(rec))
with torch.autocast("cuda", dtype=torch.bfloat16):
    m1(crops)
    for c in crops:
        m2.trunk(c)
for n in rec1:
    o1, shp, clc, res, G = rec1[n][0]
    o2 = torch.cat([r[0] for r in rec2[n]])
    e = ((o1 - o2).norm() / (o2.norm() + 1e-12)).item()
    print(f"{n:35s} in{shp} cl={clc} res={res} G={G} rel={e:.3e}")
    if e > 1e-2:
        break
