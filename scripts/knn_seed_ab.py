"""DGCNN kNN on the model's own features (DGCNNWithColor, B=32, N=4096, k=20): per graph, the
unseeded search vs the search seeded by the previous graph, timed in one process, lists compared
bit for bit."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg import ops  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

B, N, k = 32, 4096, 20
torch.manual_seed(0)
m = pcseg.DGCNNWithColor(14).cuda().train()
pts, _, _ = make_batch(B, N, seed=3)
x = pts[:, :, :6].contiguous().transpose(1, 2).cuda()
feats, graphs = [], []
orig = pcseg.models.EdgeConv.forward_graph


def rec(self, xp, seeds=None, **kw):
    out, idx = orig(self, xp, seeds, **kw)
    feats.append(xp.detach().clone())
    graphs.append(idx)
    return out, idx


pcseg.models.EdgeConv.forward_graph = rec
with torch.no_grad():
    m(x)
pcseg.models.EdgeConv.forward_graph = orig


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for i in range(1, 4):
    f, seeds = feats[i], graphs[i - 1]
    a = ops.knn(f, k)
    b = ops.knn(f, k, seeds=seeds)
    t_plain = timeit(lambda: ops.knn(f, k))
    t_seed = timeit(lambda: ops.knn(f, k, seeds=seeds))
    print(f'graph {i + 1} (F={f.shape[2]}): unseeded {t_plain:8.1f} us  seeded {t_seed:8.1f} us  '
          f'bitwise-equal {torch.equal(a, b)}', flush=True)
