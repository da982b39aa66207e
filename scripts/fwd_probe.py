"""PointNet++ forward alone (no backward, no side-stream work): per-kernel HIP-event times of every
probed launch, to compare the pooled top-layer GEMMs with their in-step times."""
import collections
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg.engine import KernelProbe  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

torch.manual_seed(0)
m = pcseg.PointNetpp(14).cuda().train()
pts, _, _ = make_batch(32, 4096, seed=1)
x = pts.cuda()
for _ in range(3):
    with torch.no_grad():
        m(x)
torch.cuda.synchronize()
tot = collections.defaultdict(lambda: [0, 0.0])
for _ in range(5):
    with torch.no_grad():
        with KernelProbe() as kp:
            m(x)
        for name, fl, by, sec in kp.records():
            tot[name][0] += 1
            tot[name][1] += sec
for name, (n, sec) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f'{sec / 5 * 1e3:8.3f} ms/fwd  {n / 5:4.1f}x  {sec / n * 1e6:8.1f} us  {name}')
