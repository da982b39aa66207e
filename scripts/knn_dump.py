"""Dump DGCNNWithColor's kNN inputs (xyz and the three 64-wide EdgeConv feature sets) for the
first two clouds of a B=32 bench batch, for the offline tile-pruning analysis
(scripts/knn_prune_study.py).  -> gpurun_out/knn_feats.npz"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             '3d-semantic-segmentation-benchmark_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pcseg  # noqa: E402
from pcseg.synthetic import make_batch  # noqa: E402

B, N = 32, 4096
torch.manual_seed(0)
m = pcseg.DGCNNWithColor(14).cuda().train()
pts, _, _ = make_batch(B, N, seed=3)
x = pts[:, :, :6].contiguous().transpose(1, 2).cuda()
feats, graphs = [], []
orig = pcseg.models.EdgeConv.forward_graph


def rec(self, xp, seeds=None, **kw):
    out, idx = orig(self, xp, seeds, **kw)
    feats.append(xp.detach()[:2].cpu().numpy())
    graphs.append(idx[:2].cpu().numpy())
    return out, idx


pcseg.models.EdgeConv.forward_graph = rec
with torch.no_grad():
    m(x)
os.makedirs('gpurun_out', exist_ok=True)
np.savez_compressed('gpurun_out/knn_feats.npz', **{f'f{i}': f for i, f in enumerate(feats)},
                    **{f'g{i}': g for i, g in enumerate(graphs)}, xyz=pts[:2, :, :3].numpy())
print('saved', [f.shape for f in feats])
