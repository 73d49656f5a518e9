"""Diagnostic: for every ConvNHWC -> BNAct pair of a SwAV trunk pass, compare the BatchNorm
statistics the conv epilogue accumulated (conv2d_fwd_stats) with sums of the conv's stored output
computed in PyTorch; prints one line per conv with the route-relevant shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401
from dedloc_amd.models import resnet_swav as rs  # noqa: E402

torch.manual_seed(0)
dev = torch.device("cuda")
m = rs.ResNet50Trunk().to(dev).train()
orig = torch.ops.dedloc.conv2d_fwd_stats
log = []


def traced(x, w, stride, pad, sums, groups, cols=None):
    before = sums.clone()
    y = orig(x, w, stride, pad, sums, groups, cols)
    torch.cuda.synchronize()
    got = (sums - before).view(groups, 2, -1)
    yg = y.float().reshape(groups, y.shape[0] // groups, y.shape[1], -1)
    ref = torch.stack([yg.sum((1, 3)), (yg * yg).sum((1, 3))], 1)
    err = ((got - ref).norm() / ref.norm()).item()
    log.append((tuple(x.shape), tuple(w.shape), stride, pad, groups, err))
    return y


rs.torch.ops.dedloc.conv2d_fwd_stats = traced  # noqa
for G, res in ((2, 64), (6, 32), (2, 224)):
    for mod in m.modules():
        if isinstance(mod, rs.BNAct):
            mod.stat_groups = G
    x = torch.randn(2 * G, 3, res, res, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    log.clear()
    m(x)
    for e in log:
        print(("BAD " if e[-1] > 1e-3 else "ok  ") + str(e), flush=True)
