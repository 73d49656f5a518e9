"""Diagnostic: per-BatchNorm output differences of the SwAV trunk between runs of the same and of
different statistics paths (conv-epilogue statistics on / off): tells run-to-run noise
(fp32 atomics order) from a path difference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401
from dedloc_amd.models import resnet_swav as rs  # noqa: E402

torch.manual_seed(0)
dev = torch.device("cuda")
m = rs.ResNet50Trunk().to(dev).train()
x = torch.randn(4, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
for mod in m.modules():
    if isinstance(mod, rs.BNAct):
        mod.stat_groups = 2
names = {mod: n for n, mod in m.named_modules() if isinstance(mod, rs.BNAct)}


def run(flag, link=True):
    rs._CONV_STATS = flag
    rs._RES_LINK = link
    acts = {}
    hooks = [mod.register_forward_hook(lambda mod, i, o: acts.__setitem__(names[mod], o.float().clone()))
             for mod in names]
    with torch.no_grad():
        out = m(x).float()
    for h in hooks:
        h.remove()
    return out, acts


runs = {"T1": run(True), "T2": run(True), "F1": run(False), "F2": run(False)}
for a, b in (("T1", "T2"), ("F1", "F2"), ("T1", "F1")):
    print(f"== {a} vs {b}: final max|diff| {(runs[a][0] - runs[b][0]).abs().max().item():.4g}")
    for n in runs[a][1]:
        d = (runs[a][1][n] - runs[b][1][n]).abs().max().item()
        print(f"   {n:28s} {d:.4g}")
