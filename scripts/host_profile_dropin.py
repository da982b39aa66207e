"""Host-side (Python) profile of the drop-in harness-A step (bench.run_drop_in: torch.optim.Adam,
zero_grad, forward, criterion, backward, step on the default stream, no prefetch): where the
enqueue time goes.  usage: python scripts/host_profile_dropin.py [model] [batch] [points]"""
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
from pcseg.synthetic import make_batch  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else 'pointnetpp'
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
NPTS = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
name, ctor, kind = bench.WORKLOADS[key][:3]
dev = torch.device('cuda', 0)
torch.manual_seed(0)
model = ctor(pcseg).to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-3)
pts, labels, lengths = make_batch(B, NPTS, seed=2000)
x = bench.model_input(pts.to(dev), kind)
lab = (labels.float() if kind == 'chfirst6' else labels).to(dev)
lengths = lengths.to(dev)


def step():
    opt.zero_grad()
    loss = pcseg.masked_onehot_cross_entropy(bench.logits_of(model(x)), lab, lengths)
    loss.backward()
    opt.step()


def phases():
    """host time of each phase of one step (no sync inside)"""
    t = [time.perf_counter()]
    opt.zero_grad()
    t.append(time.perf_counter())
    out = model(x)
    t.append(time.perf_counter())
    loss = pcseg.masked_onehot_cross_entropy(bench.logits_of(out), lab, lengths)
    t.append(time.perf_counter())
    loss.backward()
    t.append(time.perf_counter())
    opt.step()
    t.append(time.perf_counter())
    return [(b - a) * 1e3 for a, b in zip(t, t[1:])]


for _ in range(5):
    step()
torch.cuda.synchronize()
acc = [0.0] * 5
for _ in range(10):
    torch.cuda.synchronize()
    for i, v in enumerate(phases()):
        acc[i] += v / 10
torch.cuda.synchronize()
print('host ms per phase (zero_grad, forward, criterion, backward, adam): ' + ', '.join(f'{v:.3f}' for v in acc)
      + f'  total {sum(acc):.3f}')
t0 = time.perf_counter()
for _ in range(10):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f'host enqueue {(t1 - t0) / 10 * 1e3:.3f} ms/step, wall {(t2 - t0) / 10 * 1e3:.3f} ms/step')
pr = cProfile.Profile()
# the autograd engine runs the backward of CUDA graphs on its own device thread, where cProfile
# does not look: profile with the backward on this thread instead
with torch.autograd.set_multithreading_enabled(False):
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr.enable()
    for _ in range(10):
        step()
    pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(40)
st.sort_stats('cumtime').print_stats(40)
