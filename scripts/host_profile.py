"""Host-side (Python) profile of the training step: where the enqueue time goes.

usage: python scripts/host_profile.py [model] [batch]
Runs warm-up steps, then cProfile over 10 steps of forward + loss + backward + Adam
(no host sync inside the step), and prints the top functions by own time.
"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd')]

import torch  # noqa: E402

import bench  # noqa: E402
import pcseg  # noqa: E402
from pcseg.ddp import FlatGradAllReduce  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

model_name = sys.argv[1] if len(sys.argv) > 1 else 'pointnetpp'
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
name, ctor, kind = bench.WORKLOADS[model_name][:3]
dev = torch.device('cuda', 0)
model = ctor(pcseg).to(dev).train()
grads = FlatGradAllReduce(model)
from pcseg.optim import FlatAdam  # noqa: E402
opt = FlatAdam(grads, lr=1e-3)
pts, labels, lengths = make_batch(B, 4096, seed=7)
x = bench.model_input(pts.to(dev), kind)
lab = (labels.float() if kind == 'chfirst6' else labels).to(dev)
lengths = lengths.to(dev)
prefetch = hasattr(model, 'prefetch_geometry')


def step():
    grads.zero_grad()
    loss = pcseg.masked_onehot_cross_entropy(bench.logits_of(model(x)), lab, lengths)
    if prefetch:
        model.prefetch_geometry(x)
    loss.backward()
    grads.synchronize()
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f'host enqueue {(t1 - t0) / 10 * 1e3:.3f} ms/step, wall {(t2 - t0) / 10 * 1e3:.3f} ms/step')
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(35)
st.sort_stats('cumtime').print_stats(25)
