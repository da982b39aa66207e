"""DGCNN kNN launches on the model's own features (DGCNNWithColor, B=32, N=4096, k=20): the
coordinate graph (F = 3) and graphs 2-4 (F = 64, seeded by the previous graph), each also pruned
(pcs_knn_pruned over the Morton order of the xyz), timed with HIP events (the pruned time includes
its norm and tile-summary kernels); the lists are saved under /tmp/knn_lists_<tag>.pt (on the
box, within one call) and compared bit for bit with another tag's (another library, via PCS_LIB).
usage: knn_ab.py <tag> [compare_tag]"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg import ops  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

tag = sys.argv[1]
other = sys.argv[2] if len(sys.argv) > 2 else None
B, N, k = 32, 4096, 20
torch.manual_seed(0)
m = pcseg.DGCNNWithColor(14).cuda().train()
pts, _, _ = make_batch(B, N, seed=3)
x = pts[:, :, :6].contiguous().transpose(1, 2).cuda()
feats, graphs, seedl = [], [], []
orig = pcseg.models.EdgeConv.forward_graph


def rec(self, xp, seeds=None, **kw):
    out, idx = orig(self, xp, seeds, **kw)
    feats.append(xp.detach().clone())
    graphs.append(idx)
    seedl.append(seeds)
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


lists = {}
od = ops.knn_order(feats[0])
t_ord = timeit(lambda: ops.knn_order(feats[0]))
print(f'[{tag}] knn_order {t_ord:8.1f} us', flush=True)
for i in range(4):
    f = feats[i]
    sd = None if i == 0 else graphs[i - 1]
    un = ops.knn(f, k)
    se = ops.knn(f, k, seeds=sd) if sd is not None else un
    pr = ops.knn(f, k, seeds=sd, order=od)
    lists[f'g{i}_unseeded'] = un.cpu()
    lists[f'g{i}_seeded'] = se.cpu()
    lists[f'g{i}_pruned'] = pr.cpu()
    t_un = timeit(lambda: ops.knn(f, k))
    t_se = timeit(lambda: ops.knn(f, k, seeds=sd)) if sd is not None else float('nan')
    t_pr = timeit(lambda: ops.knn(f, k, seeds=sd, order=od))
    t_pu = timeit(lambda: ops.knn(f, k, order=od)) if sd is not None else t_pr
    pu = ops.knn(f, k, order=od)
    print(f'[{tag}] graph {i + 1} (F={f.shape[2]}): unseeded {t_un:8.1f} us  seeded {t_se:8.1f} us  '
          f'pruned+seeded {t_pr:8.1f} us  pruned {t_pu:8.1f} us  seeded==unseeded {torch.equal(un, se)}  '
          f'pruned==unseeded {torch.equal(un, pr)} {torch.equal(un, pu)}', flush=True)
torch.save(lists, f'/tmp/knn_lists_{tag}.pt')          # ~80 MB: box-local, same gpurun call
if other:
    ref = torch.load(f'/tmp/knn_lists_{other}.pt', weights_only=True)
    for key, v in lists.items():
        print(f'[{tag} vs {other}] {key}: bitwise equal {torch.equal(v, ref[key])}', flush=True)
