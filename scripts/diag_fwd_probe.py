import sys, os
sys.path[:0] = ['/root/repo', '/root/repo/3d-semantic-segmentation-benchmark_amd']
import torch, pcseg
from pcseg.engine import KernelProbe
from pcseg.synthetic import make_batch
m = pcseg.DGCNNWithColor(num_classes=14, k=20).cuda().train()
pts, labels, lengths = make_batch(32, 4096, seed=1)
x = pts[:, :, :6].contiguous().transpose(1, 2).cuda()
with KernelProbe() as kp:
    out = m(x)
torch.cuda.synchronize()
for k, v in kp.summary().items():
    print(k, v[0], round(v[3]*1e6))
