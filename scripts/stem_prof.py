"""Profile target: the SwAV stem (7x7/2, 3 -> 64 channels, 128 x 224^2) forward + wgrad through
torch.ops.dedloc, to split im2col from the column GEMM under rocprofv3 --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dedloc_amd.ops  # noqa: E402,F401

CL = torch.channels_last
dev = torch.device("cuda")
x = torch.randn(128, 3, 224, 224, device=dev).bfloat16().contiguous(memory_format=CL)
w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).bfloat16().contiguous(memory_format=CL)
dy = torch.randn(128, 64, 112, 112, device=dev).bfloat16().contiguous(memory_format=CL)
dw = torch.zeros(64, 3, 7, 7, device=dev).contiguous(memory_format=CL)
for _ in range(20):
    torch.ops.dedloc.conv2d_fwd(x, w, 2, 3)
    torch.ops.dedloc.conv2d_wgrad(dy, x, dw, 2, 3)
torch.cuda.synchronize()
print("done", flush=True)
