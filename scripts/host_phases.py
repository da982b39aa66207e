"""Host time per phase of the eager training step (no host sync inside the step), and the
GPU's step time: where the host falls behind the GPU.

usage: python scripts/host_phases.py [model] [prefetch_point: loss|backward|none]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd')]

import torch  # noqa: E402

import bench  # noqa: E402
import pcseg  # noqa: E402
from pcseg.ddp import FlatGradAllReduce  # noqa: E402
from pcseg.optim import FlatAdam  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

model_name = sys.argv[1] if len(sys.argv) > 1 else 'pointnetpp'
point = sys.argv[2] if len(sys.argv) > 2 else 'loss'
name, ctor, kind = bench.WORKLOADS[model_name][:3]
dev = torch.device('cuda', 0)
torch.manual_seed(0)
model = ctor(pcseg).to(dev).train()
grads = FlatGradAllReduce(model)
opt = FlatAdam(grads, lr=1e-3)
pts, labels, lengths = make_batch(32, 4096, seed=7)
x = bench.model_input(pts.to(dev), kind)
lab = (labels.float() if kind == 'chfirst6' else labels).to(dev)
lengths = lengths.to(dev)
prefetch = hasattr(model, 'prefetch_geometry') and point != 'none'
acc = {}


def tick(k, t0):
    t = time.perf_counter()
    acc[k] = acc.get(k, 0.0) + (t - t0)
    return t


def step():
    t = time.perf_counter()
    grads.zero_grad()
    if prefetch and point == 'backward':
        model.prefetch_geometry_in_backward(x)
    t = tick('zero_grad', t)
    out = model(x)
    t = tick('forward', t)
    loss = pcseg.masked_onehot_cross_entropy(bench.logits_of(out), lab, lengths)
    t = tick('loss', t)
    if prefetch and point == 'loss':
        model.prefetch_geometry(x)
        t = tick('prefetch', t)
    loss.backward()
    t = tick('backward', t)
    grads.synchronize()
    opt.step()
    tick('opt', t)


for _ in range(5):
    step()
torch.cuda.synchronize()
acc.clear()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    step()
th = time.perf_counter() - t0
torch.cuda.synchronize()
tg = time.perf_counter() - t0
print(f'{name} prefetch={point}: step {tg / n * 1e3:.3f} ms, host enqueue {th / n * 1e3:.3f} ms')
for k, v in acc.items():
    print(f'  {k:10s} {v / n * 1e3:7.3f} ms/step host')
