"""Time the multicrop op alone: 2x224 + 6x96 crops of 64 images, 20 calls each."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from dedloc_amd.data.multicrop import SyntheticMultiCropStream
s = SyntheticMultiCropStream(64, torch.device("cuda"))
for _ in range(3):
    s.next_batch()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(20):
    s.next_batch()
ev1.record()
torch.cuda.synchronize()
print("multicrop_batch_ms", ev0.elapsed_time(ev1) / 20)
